"""MI355X runtime for one MixFormer RGB-T forward: weights, workspace and launch plan.

The per-frame work is a fixed list of libmmt_hip.so launches (the "plan", ~110-130 calls) over
a workspace allocated once per batch size; every call's pointers and shapes are resolved when
the plan is built, so a frame is `for fn, args in plan: fn(*args, stream)` — or one hipGraph
replay (`capture()`), which removes the host launch cost altogether.

HBM layout (B = frames, S = 2B sequences stored modality-major: s = m*B + b, m = 0 RGB / 1 TIR,
ntok = 2*n_t + n_s tokens per sequence, C = 768 for ViT-B):
  X    fp32 [S*ntok][C]      residual stream (patch-embed + pos written straight into it)
  XN   dt   [S*ntok][C]      LayerNorm output = GEMM A operand
  QKV  dt   [S*ntok][3C]     fused qkv Linear output, read in place by the MAM kernel
  AO   dt   [S*ntok][C]      attention output = proj A operand
  HID  dt   [S*ntok][4C]     GELU(fc1) output
  fusion encoder: SRC fp32 / SRCT dt [2][B*n_s][512] (modality-major, i.e. the reference's
  (B, 2*n_s, 512) with the halves as the outer index), head: NHWC maps.
`dt` is the compute dtype (bf16, fp16 or fp32).  Accumulation, softmax and norm statistics are fp32.

Weight preparation (load time, torch on device): casts, Linear/conv weights to [N][K] with
K = (ky, kx, cin) for convs, eval-mode BatchNorm folded into the conv, the six first-level head
convs that read the fused map merged into one GEMM (N = 1344), the MSDA offset and weight
Linears merged (N = 192), fixed position tables and the score-token query constant.
"""
import math

import torch

from . import _lib
from ._lib import LIB, GemmParams, AttnParams, check, MMT_F32, MMT_BF16, MMT_F16

VARIANTS = ("rgbt", "shared", "asym", "asym_online", "asym_ce", "rgb")  # rgb: RGB-only MixFormer (config 1)


LOG2E = 1.4426950408889634


def _ptr(t, off=0):
    return t.data_ptr() + off * t.element_size()


class Dims:
    def __init__(self, sd, variant):
        pre = "backbone_v." if variant == "rgbt" else "backbone."
        self.C = sd[pre + "pos_embed_s"].shape[-1]
        self.H = self.C // 64
        self.depth = 0
        while (pre + "blocks.%d.mlp.fc1.weight" % self.depth) in sd:
            self.depth += 1
        self.nt1 = sd[pre + "pos_embed_t"].shape[1]
        self.ns = sd[pre + "pos_embed_s"].shape[1]
        self.gt = int(round(self.nt1 ** 0.5))
        self.gs = int(round(self.ns ** 0.5))
        self.patch = 16
        self.ht, self.hs = self.gt * self.patch, self.gs * self.patch
        self.n_t = 2 * self.nt1
        self.ntok = self.n_t + self.ns
        self.hidden = sd[pre + "blocks.0.mlp.fc1.weight"].shape[0]
        self.nmod = 1 if variant == "rgb" else 2  # modalities (sequences per frame)
        fusion = self.nmod == 2  # the RGB-only model has no fusion: the head reads the backbone
        self.d_model = sd["fusion_vi.adjust_v.0.weight"].shape[0] if fusion else 512
        self.fusion_layers = 0
        while fusion and ("fusion_vi.fusion_attention.encoder.layers.%d.linear1.weight" % self.fusion_layers) in sd:
            self.fusion_layers += 1
        self.ffn = sd["fusion_vi.fusion_attention.encoder.layers.0.linear1.weight"].shape[0] if fusion else 1024
        self.hc = sd["box_head.conv1_tl.0.weight"].shape[0]
        self.fh = 4 * self.gs


class MixFormerRGBTRuntime:
    """Compiled forward of one of the four hot-path variants on the current CUDA (HIP) device."""

    gemm_impl = 0  # mmt_gemm_params.impl of every plan GEMM (0 = library's choice; A/B knob)
    gemm_splitk = 0  # mmt_gemm_params.splitk of every plan GEMM (0 = library's choice, 1 = off)
    attn_impl = 0  # mmt_attn_params.impl of every plan attention (0 = library's choice; A/B knob)
    SPLITK_FLOATS = 8 << 20  # fp32 split-K partial-tile workspace (32 MiB), shared by every plan GEMM
    SPLITK_TICKETS = 1 << 16

    def __init__(self, state_dict, variant, dtype=torch.bfloat16, device="cuda", fold_ln=None, ce=None, head_dtype=None,
                 ce_mask_count=None):
        """fold_ln (default: on for bf16): the ViT's LayerNorms are folded into the qkv / fc1 GEMMs
        (mmt_gemm_params.ln_fold) and the residual-producing GEMMs also write the bf16 copy of the
        residual stream those GEMMs read, so no LayerNorm launch or normalised tensor remains.
        The fp32 path keeps the explicit LayerNorm kernels."""
        if variant not in VARIANTS:
            raise ValueError("unknown variant %r" % (variant,))
        if dtype not in (torch.bfloat16, torch.float16, torch.float32):
            raise ValueError("dtype must be torch.bfloat16, torch.float16 or torch.float32")
        if dtype == torch.float16 and variant == "asym_ce":
            raise NotImplementedError("candidate elimination runs in bf16 / fp32 (its selection kernels have no fp16 form)")
        if dtype == torch.bfloat16 and variant == "rgb":
            # the RGB-only MixFormer has no fusion (GroupNorm) between backbone and corner head: its score
            # maps carry the backbone's scale (logit std ~8.6 on the golden inputs, ~4 effective soft-argmax
            # positions, against ~2 / hundreds for the RGB-T models), so the bf16 backbone's ~0.5 % token
            # error alone moves its boxes 1.8e-2 (head in fp32) to 2.7e-2 (bf16 head) -- past the north
            # star's 1e-2 (profiles/r03_rgb_dtype.jsonl).  fp16 (1.8e-3, same speed) is its 16-bit type.
            raise ValueError("the RGB-only MixFormer (config 1) runs in fp16 or fp32, not bf16: without the fusion "
                             "stage its boxes leave the 1e-2 bound in bf16 (use torch.float16, the same speed)")
        self.variant = variant
        # candidate elimination (asym_ce): {block: keep ratio}, lib/config/asymmetric_shared_ce/config.py:23-24
        ce = ce if ce is not None else ((3, 6, 9), (0.7, 0.7, 0.7))
        self.ce = dict(zip(ce[0], ce[1])) if variant == "asym_ce" else {}
        # ce_template_mask (candidate_elimination :81-89): None = every template query counts (the
        # tracker); else the number of masked template queries per frame, and forward() takes the
        # [B][2 n_t] mask itself (ce_template_mask), copied into the workspace before the plan runs
        self.ce_mask_count = None if not self.ce or ce_mask_count is None else int(ce_mask_count)
        self.dtype = dtype
        self.cdt = {torch.bfloat16: MMT_BF16, torch.float16: MMT_F16}.get(dtype, MMT_F32)
        # storage type of the corner head's activations and weights (head_dtype; default = dtype)
        self.hdtype = head_dtype or dtype
        if self.hdtype not in (torch.bfloat16, torch.float16, torch.float32):
            raise ValueError("head_dtype must be torch.bfloat16, torch.float16 or torch.float32")
        self.hcdt = {torch.bfloat16: MMT_BF16, torch.float16: MMT_F16}.get(self.hdtype, MMT_F32)
        half = dtype in (torch.bfloat16, torch.float16)
        self.fold_ln = half if fold_ln is None else bool(fold_ln)
        if self.fold_ln and not half:
            raise ValueError("the LayerNorm fold needs the 16-bit (LDS-DMA) GEMM kernels")
        self.device = torch.device(device)
        sd = {k: v.detach() for k, v in state_dict.items()}
        self.d = Dims(sd, variant)
        if self.d.C % 256 or self.d.d_model != 512 or self.d.C // 64 * 64 != self.d.C:
            raise ValueError("unsupported dims C=%d d_model=%d" % (self.d.C, self.d.d_model))
        self.w = {}
        head_dim = self.d.C // self.d.H
        self.q_scale = head_dim ** -0.5 * LOG2E if self.fold_ln else 1.0  # folded into the q weights
        self._prepare(sd)
        self._ws = {}
        self._graphs = {}
        # split-K hand-off buffers: the plan's GEMMs run one after another on one stream, so one
        # slab workspace serves them all; the tickets start at zero and every launch leaves them so
        self._sk_ws = torch.empty(self.SPLITK_FLOATS, device=self.device, dtype=torch.float32)
        self._sk_cnt = torch.zeros(self.SPLITK_TICKETS, device=self.device, dtype=torch.int32)

    # ------------------------------------------------------------------ weights
    def _T(self, x):
        return x.detach().to(self.device, self.dtype).contiguous()

    def _F(self, x):
        return x.detach().to(self.device, torch.float32).contiguous()

    def _TH(self, x):  # head storage type
        return x.detach().to(self.device, self.hdtype).contiguous()

    def _fold(self, sd, name):
        """conv() block (head.py:7-20): Conv3x3 -> BatchNorm2d(eval) -> ReLU, BN folded."""
        w = sd[name + ".0.weight"].double()
        b = sd[name + ".0.bias"].double()
        g, beta = sd[name + ".1.weight"].double(), sd[name + ".1.bias"].double()
        mean, var = sd[name + ".1.running_mean"].double(), sd[name + ".1.running_var"].double()
        s = g / torch.sqrt(var + 1e-5)
        w = w * s.view(-1, 1, 1, 1)
        b = (b - mean) * s + beta
        return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1), b

    def _prepare(self, sd):
        d, W = self.d, self.w
        C = d.C
        pres = ["backbone_v.", "backbone_i."] if self.variant == "rgbt" else ["backbone."]
        single_ln = self.variant in ("rgbt", "rgb")  # norm1 / norm2 (else per-modality norm*_v / norm*_i)
        W["bb"] = []
        for pre in pres:
            bb = {"patch_w": self._T(sd[pre + "patch_embed.proj.weight"].reshape(C, -1)),
                  "patch_b": self._F(sd[pre + "patch_embed.proj.bias"]),
                  "pos": self._F(torch.cat([sd[pre + "pos_embed_t"][0], sd[pre + "pos_embed_t"][0],
                                            sd[pre + "pos_embed_s"][0]], 0)),
                  "blocks": []}
            for i in range(d.depth):
                b = pre + "blocks.%d." % i
                blk = {}
                for nm in ("attn.qkv", "attn.proj", "mlp.fc1", "mlp.fc2"):
                    blk[nm + ".w"] = self._T(sd[b + nm + ".weight"])
                    blk[nm + ".b"] = self._F(sd[b + nm + ".bias"])
                if single_ln:
                    for nm in ("norm1", "norm2"):
                        blk[nm] = (self._F(sd[b + nm + ".weight"]), self._F(sd[b + nm + ".bias"]))
                else:
                    for nm in ("norm1", "norm2"):
                        blk[nm + "_v"] = (self._F(sd[b + nm + "_v.weight"]), self._F(sd[b + nm + "_v.bias"]))
                        blk[nm + "_i"] = (self._F(sd[b + nm + "_i.weight"]), self._F(sd[b + nm + "_i.bias"]))
                if self.fold_ln:
                    # Linear(LayerNorm(x)) = rstd*(x.W' - mu*colsum(W')) + b', W' = W*gamma (per k),
                    # b' = b + W.beta; one (W', colsum, b') per norm (two-stream: this backbone's;
                    # shared: norm*_v / norm*_i -> one GEMM group per modality)
                    norms = ["", ] if single_ln else ["_v", "_i"]
                    for lin, nm in (("attn.qkv", "norm1"), ("mlp.fc1", "norm2")):
                        w64, b64 = sd[b + lin + ".weight"].double(), sd[b + lin + ".bias"].double()
                        if lin == "attn.qkv":
                            # the q rows carry the attention scale * log2(e), so the MAM kernels'
                            # exp2 takes the scores as they come (mmt_attn_params.scale = 1/log2(e))
                            qs = torch.ones(3 * C, dtype=torch.float64, device=w64.device)
                            qs[:C] = self.q_scale
                            w64, b64 = w64 * qs[:, None], b64 * qs
                        fw, fc, fb = [], [], []
                        for suf in norms:
                            gam, bet = sd[b + nm + suf + ".weight"].double(), sd[b + nm + suf + ".bias"].double()
                            wt = self._T(w64 * gam[None, :])
                            fw.append(wt)
                            fc.append(self._F(wt.double().sum(1)))
                            fb.append(self._F(b64 + w64 @ bet))
                        blk[lin + ".fw"], blk[lin + ".fcs"], blk[lin + ".fb"] = fw, fc, fb
                bb["blocks"].append(blk)
            W["bb"].append(bb)
        self._prepare_fusion(sd) if d.nmod == 2 else None
        self._prepare_head(sd)

    def _prepare_fusion(self, sd):
        d, W = self.d, self.w
        C = d.C
        f = "fusion_vi."
        for m in ("v", "i"):
            W["adj_" + m + ".w"] = self._T(sd[f + "adjust_%s.0.weight" % m].reshape(d.d_model, C))
            W["adj_" + m + ".b"] = self._F(sd[f + "adjust_%s.0.bias" % m])
            W["adj_" + m + ".gn"] = (self._F(sd[f + "adjust_%s.1.weight" % m]), self._F(sd[f + "adjust_%s.1.bias" % m]))
        W["adj_cat.w"] = self._T(sd[f + "adjust_cat.0.weight"].reshape(C, 2 * d.d_model))
        W["adj_cat.b"] = self._F(sd[f + "adjust_cat.0.bias"])
        W["adj_cat.gn"] = (self._F(sd[f + "adjust_cat.1.weight"]), self._F(sd[f + "adjust_cat.1.bias"]))
        fa = f + "fusion_attention."
        W["level_embed"] = self._F(sd[fa + "level_embed"])
        W["enc"] = []
        for li in range(d.fusion_layers):
            lp = fa + "encoder.layers.%d." % li
            sa = lp + "self_attn."
            e = {"value.w": self._T(sd[sa + "value_proj.weight"]), "value.b": self._F(sd[sa + "value_proj.bias"]),
                 "offw.w": self._T(torch.cat([sd[sa + "sampling_offsets.weight"], sd[sa + "attention_weights.weight"]], 0)),
                 "offw.b": self._F(torch.cat([sd[sa + "sampling_offsets.bias"], sd[sa + "attention_weights.bias"]], 0)),
                 "out.w": self._T(sd[sa + "output_proj.weight"]), "out.b": self._F(sd[sa + "output_proj.bias"]),
                 "l1.w": self._T(sd[lp + "linear1.weight"]), "l1.b": self._F(sd[lp + "linear1.bias"]),
                 "l2.w": self._T(sd[lp + "linear2.weight"]), "l2.b": self._F(sd[lp + "linear2.bias"])}
            for nm in ("norm1_v", "norm1_i", "norm2_v", "norm2_i"):
                e[nm] = (self._F(sd[lp + nm + ".weight"]), self._F(sd[lp + nm + ".bias"]))
            W["enc"].append(e)
        W["pos_sine"] = self._F(_sine_pos(d.gs, d.d_model))  # [ns][512]
        # The encoder query is src + (pos + level_embed[l]) per modality l (deformable_transformer
        # with_pos_embed), and it only feeds the sampling-offset / attention-weight Linear, so that
        # Linear splits as src.W^T + [(pos + le[l]).W_l^T summed over l + b]: the bracket is a
        # per-cell constant folded here (float64 on the host), added by the GEMM's row-mapped
        # residual, and the query tensor and its add kernel disappear.
        pos64 = _sine_pos(d.gs, d.d_model).double()
        le64 = sd[fa + "level_embed"].detach().cpu().double()
        for li, e in enumerate(W["enc"]):
            sa = fa + "encoder.layers.%d.self_attn." % li
            w64 = torch.cat([sd[sa + "sampling_offsets.weight"], sd[sa + "attention_weights.weight"]], 0)
            b64 = torch.cat([sd[sa + "sampling_offsets.bias"], sd[sa + "attention_weights.bias"]], 0)
            w64, b64 = w64.detach().cpu().double(), b64.detach().cpu().double()
            dm = d.d_model
            pw = sum((pos64 + le64[l]) @ w64[:, l * dm:(l + 1) * dm].t() for l in range(2)) + b64
            e["offw.pos"] = self._F(pw.float())  # [ns][192]

    def _prepare_head(self, sd):
        d, W = self.d, self.w
        C = d.C
        # corner head
        h = "box_head."
        ws, bs = [], []
        for nm in ("conv1_tl", "conv1_br", "adjust1_tl", "adjust1_br", "adjust2_tl", "adjust2_br"):
            w_, b_ = self._fold(sd, h + nm)
            ws.append(w_)
            bs.append(b_)
        W["h0.w"], W["h0.b"] = self._TH(torch.cat(ws, 0)), self._F(torch.cat(bs, 0))
        for nm in ("conv2", "conv3", "conv4"):
            for br in ("tl", "br"):
                w_, b_ = self._fold(sd, h + nm + "_" + br)
                W[nm + "_" + br + ".w"], W[nm + "_" + br + ".b"] = self._TH(w_), self._F(b_)
        for br in ("tl", "br"):
            for nm, idx in (("adjust3", 0), ("adjust3", 1), ("adjust4", 0)):
                w_, b_ = self._fold(sd, h + "%s_%s.%d" % (nm, br, idx))
                W["%s.%d_%s.w" % (nm, idx, br)], W["%s.%d_%s.b" % (nm, idx, br)] = self._TH(w_), self._F(b_)
        c1 = []
        for nm in ("adjust3_tl.2", "adjust3_br.2", "adjust4_tl.1", "adjust4_br.1"):
            c1.append(self._fold(sd, h + nm))
        W["a3c1.w"] = self._TH(torch.stack([c1[0][0][0], c1[1][0][0]]))
        W["a3c1.b"] = self._F(torch.stack([c1[0][1][0], c1[1][1][0]]))
        W["a4c1.w"] = self._TH(torch.stack([c1[2][0][0], c1[3][0][0]]))
        W["a4c1.b"] = self._F(torch.stack([c1[2][1][0], c1[3][1][0]]))
        W["c5.w"] = self._F(torch.stack([sd[h + "conv5_tl.weight"].reshape(-1), sd[h + "conv5_br.weight"].reshape(-1)]))
        W["c5.b"] = self._F(torch.cat([sd[h + "conv5_tl.bias"], sd[h + "conv5_br.bias"]]))
        # score decoder (fp32 throughout: its work is negligible)
        if self.variant == "asym_online":
            s = "score_branch."
            F = self._F
            x0 = torch.nn.functional.layer_norm(sd[s + "score_token"].double().reshape(1, C), (C,),
                                                sd[s + "norm1.weight"].double(), sd[s + "norm1.bias"].double(), 1e-5)
            W["spm.q0"] = F(torch.nn.functional.linear(x0, sd[s + "proj_q.0.weight"].double(),
                                                       sd[s + "proj_q.0.bias"].double()).reshape(C))
            for i in range(2):
                W["spm.kv%d.w" % i] = F(torch.cat([sd[s + "proj_k.%d.weight" % i], sd[s + "proj_v.%d.weight" % i]], 0))
                W["spm.kv%d.b" % i] = F(torch.cat([sd[s + "proj_k.%d.bias" % i], sd[s + "proj_v.%d.bias" % i]], 0))
                W["spm.proj%d.w" % i], W["spm.proj%d.b" % i] = F(sd[s + "proj.%d.weight" % i]), F(sd[s + "proj.%d.bias" % i])
                W["spm.norm2.%d" % i] = (F(sd[s + "norm2.%d.weight" % i]), F(sd[s + "norm2.%d.bias" % i]))
            W["spm.q1.w"], W["spm.q1.b"] = F(sd[s + "proj_q.1.weight"]), F(sd[s + "proj_q.1.bias"])
            n = 0
            while (s + "score_head.layers.%d.weight" % n) in sd:
                W["spm.mlp%d.w" % n] = F(sd[s + "score_head.layers.%d.weight" % n])
                W["spm.mlp%d.b" % n] = F(sd[s + "score_head.layers.%d.bias" % n])
                n += 1
            W["spm.mlp_n"] = n

    # ------------------------------------------------------------------ workspace
    def workspace(self, B):
        if B in self._ws:
            return self._ws[B]
        d = self.d
        dev, dt, f32, ht = self.device, self.dtype, torch.float32, self.hdtype
        S, R, C = d.nmod * B, d.nmod * B * d.ntok, d.C
        ns, dm, hc = d.ns, d.d_model, d.hc
        e = lambda *shape, t=dt: torch.empty(*shape, device=dev, dtype=t)  # noqa: E731
        ws = {
            "B": B,
            "in_t": [e(B, 3, d.ht, d.ht, t=f32) for _ in range(d.nmod)],
            "in_o": [e(B, 3, d.ht, d.ht, t=f32) for _ in range(d.nmod)],
            "in_s": [e(B, 3, d.hs, d.hs, t=f32) for _ in range(d.nmod)],
            "PATCH": e(R, 3 * d.patch * d.patch), "X": e(R, C, t=f32), "XN": e(R, C), "QKV": e(R, 3 * C),
            "AO": e(R, C), "HID": e(R, d.hidden), "XT": e(R, C),
            "LNST": e(R, 2 * (C // 64), t=f32),  # LayerNorm row statistics of XN, per 64 columns
            "Y1": e(2, B * ns, dm, t=f32), "SRC": e(2, B * ns, dm, t=f32), "SRCT": e(2, B * ns, dm),
            "VAL": e(2, B * ns, dm), "OFFW": e(B * ns, 192, t=f32), "MS": e(B * ns, dm),
            "SRC2": e(B * ns, dm, t=f32), "H2": e(2 * B * ns, d.ffn), "Y2": e(B * ns, C, t=f32),
            "FUS": e(B * ns, C, t=f32), "FUST": e(B * ns, C, t=ht),
            "H0": e(B * ns, 2 * hc + hc + hc // 2, t=ht), "X2": e(2, B * ns, hc // 2, t=ht),
            "S1": e(2, B * ns, hc // 2, t=ht), "X3": e(2, B * 4 * ns, hc // 4, t=ht), "S2": e(2, B * 4 * ns, hc // 4, t=ht),
            "X4": e(2, B * 16 * ns, hc // 8, t=ht), "A3a": e(2, B * ns, hc // 4, t=ht), "A3b": e(2, B * ns, hc // 8, t=ht),
            "A3": e(2, B, ns, t=f32), "A4a": e(2, B * 4 * ns, hc // 8, t=ht), "A4": e(2, B, 4 * ns, t=f32),
            "XH": e(R, C, t=ht) if d.nmod == 1 else None,  # RGB-only: the head's input in the head type
            "BOX": e(B, 4, t=f32), "XYXY": e(B, 4, t=f32), "ROIS": e(B, 5, t=f32),
            "MAPS": e(2, B, d.fh * d.fh, t=f32),
        }
        if self.variant == "asym_online":
            ws.update({"ROIT": e(B * 16, C, t=f32), "KV0": e(B * 16, 2 * C, t=f32), "AT": e(B, C, t=f32),
                       "XS": e(B, C, t=f32), "Q1": e(B, C, t=f32), "KV1": e(B * d.n_t, 2 * C, t=f32),
                       "M1": e(B, C, t=f32), "M2": e(B, C, t=f32), "SC": e(B, 1, t=f32)})
        if self.ce:
            nparts = d.H * (2 * d.n_t // 8)  # (bf16 uses 16-query blocks: half of it)
            ws.update({"XC": e(R, C, t=f32), "CEP": e(B * nparts * 2 * ns, t=f32),
                       "CEG": [e(S, ns, t=torch.int32) for _ in self.ce], "CEO": e(S, ns, t=torch.int32),
                       "CEM": [e(B, 2 * ns, t=f32) for _ in self.ce],
                       "CEMASK": torch.ones(B, 2 * d.n_t, device=dev, dtype=torch.uint8)})
        ws["plan"] = self._build_plan(ws, False)
        if self.variant == "asym_online":
            ws["plan_score"] = self._build_plan(ws, True)
            ws["plan_spm"] = []  # the score decoder alone, on ROIS as given (forward with gt_bboxes)
            self._plan_spm(ws["plan_spm"], ws)
        self._ws[B] = ws
        return ws

    # ------------------------------------------------------------------ plan construction
    def _gemm(self, plan, name, *, a, w, c, M, N, K, lda, ldc, bias=None, r=None, ldr=0, c2=None, a1=None,
              k_split=0, act=0, c_f32=0, seg=None, r_mode=0, r_p0=0, r_p1=1, conv=None, r_t=0, dtype=None,
              ln_colsum=None, ln_eps=0.0, c2_copy=0, cmap=None, ln_stats_in=None, ln_stats_out=None, defer=None,
              tile=None):
        """Append one mmt_gemm launch to plan; defer=list: collect (params, dtype) for _gemm_multi instead.
        tile=(impl, splitk): a measured per-entry choice, applied unless an A/B run forces gemm_impl / gemm_splitk."""
        p = GemmParams()
        G = len(a)
        for g in range(G):
            p.a[g] = a[g]
            p.w[g] = w[g]
            p.c[g] = c[g]
            p.bias[g] = bias[g] if bias else None
            p.r[g] = r[g] if r else None
            p.c2[g] = c2[g] if c2 else None
            p.a1[g] = a1[g] if a1 else None
        p.lda, p.ldc, p.ldr = lda, ldc, ldr
        if seg is None:
            p.a_seg_rows, p.a_segs_a, p.a_stride_a, p.a_stride_b = max(M, 1), 1, 0, 0
        else:
            p.a_seg_rows, p.a_segs_a, p.a_stride_a, p.a_stride_b = seg
        p.M, p.N, p.K, p.k_split = M, N, K, k_split
        p.act, p.c_f32 = act, c_f32
        p.r_mode, p.r_p0, p.r_p1 = r_mode, r_p0, r_p1
        if conv:
            p.conv_h, p.conv_up, p.conv_cin, p.conv_k3 = conv
        p.groups = G
        p.r_t = r_t
        p.impl = self.gemm_impl
        if ln_colsum is not None:
            p.ln_fold, p.ln_eps = (2 if ln_stats_in else 1), ln_eps
            for g in range(G):
                p.ln_colsum[g] = ln_colsum[g]
                if ln_stats_in:
                    p.ln_stats_in[g] = ln_stats_in[g]
        if ln_stats_out:
            for g in range(G):
                p.ln_stats_out[g] = ln_stats_out[g]
        p.c2_copy = c2_copy
        if cmap is not None:
            p.c_seg_rows, p.c_seg_pitch = cmap
        p.splitk = self.gemm_splitk
        if tile is not None and self.gemm_impl == 0 and self.gemm_splitk == 0:
            p.impl, p.splitk = tile
        p.sk_ws, p.sk_ws_floats = self._sk_ws.data_ptr(), self._sk_ws.numel()
        p.sk_cnt, p.sk_cnt_n = self._sk_cnt.data_ptr(), self._sk_cnt.numel()
        if defer is not None:
            defer.append((p, self.cdt if dtype is None else dtype))
            return
        plan.append((LIB.mmt_gemm, (ctypes_byref(p), self.cdt if dtype is None else dtype), name, p))

    def _gemm_multi(self, plan, name, items):
        """One mmt_gemm_multi launch of independent problems collected by _gemm(..., defer=items)."""
        dts = {dt for _, dt in items}
        if len(dts) != 1:
            raise ValueError("%s: one dtype per multi-GEMM launch" % name)
        arr = (GemmParams * len(items))(*[q for q, _ in items])
        plan.append((LIB.mmt_gemm_multi, (arr, len(items), dts.pop()), name, arr))

    def _build_plan(self, ws, score):
        plan = []
        xf = self._plan_backbone(plan, ws, None)
        self._plan_tail(plan, ws, score, xf)
        return plan

    def _plan_backbone(self, plan, ws, part, qkv_layers=None):
        """Patch embed + the ViT blocks over the token rows of `part`: None = all rows; "t" = the
        template rows [0, n_t) of every sequence; "s" = the search rows [n_t, ntok).  Template queries
        never attend search keys (the MAM is asymmetric, mixformer.py:61-76), so the "t" pass run once
        per template update followed by "s" passes per frame equals the full forward within rounding (the
        compact passes' GEMMs may take other tile / split-K choices, so fp32 sums can associate differently;
        tests/test_gpu_cache.py holds the boxes to 5e-3), provided each layer's qkv rows persist: qkv_layers gives one [S*ntok][3C] buffer per layer (None: the one
        QKV buffer, reused by every layer).
        A part's activations (X, XN, AO, HID and the LayerNorm statistics) are COMPACT: its nr rows of
        every sequence back to back ([S][nr], modality groups of B sequences), so every GEMM reads and
        writes plain rows (the compact epilogues and the LayerNorm-statistics hand-off apply); only the
        qkv GEMM writes through an output row map into the [S][ntok] per-layer cache, and the attention
        stores its part's rows compact (mmt_attn_params.out_pitch / out_q0)."""
        d, W, B = self.d, self.w, ws["B"]
        C, ntok = d.C, d.ntok
        S = d.nmod * B
        two = self.variant == "rgbt"
        nm_ = d.nmod  # modality groups of the per-modality LayerNorm GEMMs (1 for the RGB-only model)
        P = _ptr
        X, XN, AO, HID = ws["X"], ws["XN"], ws["AO"], ws["HID"]
        cdt = self.cdt
        off, nr = {None: (0, ntok), "t": (0, d.n_t), "s": (d.n_t, d.ns)}[part]
        compact = part is not None
        rp = nr if compact else ntok  # rows per sequence of the activation streams
        R = S * rp

        def at(t, ld, g=0):  # first row of the part in group g's block of B sequences (activations)
            return P(t, (g * B * rp + (0 if compact else off)) * ld)

        def qat(t, g=0):  # the same in the [S][ntok] qkv stream
            return P(t, (g * B * ntok + off) * 3 * C)
        qmap = dict(cmap=(nr, ntok)) if compact else {}  # qkv rows of the part into the [S][ntok] cache

        def rmap(ld):  # after candidate elimination (full forward): the first nr rows of each pitch-ntok sequence
            if compact or nr == ntok:
                return {}
            return dict(seg=(nr, 1 << 30, ntok * ld, 0), cmap=(nr, ntok))
        # --- patch embed (im2col + GEMM, + bias + pos-embed) -> X  (fold: + its bf16 copy XN)
        fold = self.fold_ln
        # the producers of XN (patch embed, proj, fc2) also write its per-64-column row statistics
        # (LNST), which the LayerNorm-folded consumers (qkv, fc1) read instead of summing them in
        # their K loops; not with candidate elimination (the gather moves rows).  The LDS-DMA GEMM takes
        # the hand-off for K = C <= 1024 and producer widths N = C % 64 == 0 only (gemm_glds.hip
        # glds_takes); wider models keep ln_fold 1
        hand = fold and not self.ce and C % 64 == 0 and C <= 1024
        nst = 2 * (C // 64)
        LNST = ws["LNST"]
        plan.append((LIB.mmt_patch_im2col, self._image_args(ws["in_t"], ws["in_o"], ws["in_s"])
                     + (P(ws["PATCH"]), B, d.ht, d.hs, d.patch, cdt), "patch_im2col", None))
        KP = 3 * d.patch * d.patch
        gm = B * nr  # rows per modality group
        pat = lambda g: P(ws["PATCH"], (g * B * ntok + off) * KP)  # noqa: E731  (im2col rows: [S][ntok])
        pseg = dict(seg=(nr, 1 << 30, ntok * KP, 0)) if compact else {}
        cp = dict(c2_copy=1) if fold else {}
        if hand:
            cp["ln_stats_out"] = [at(LNST, nst, 0), at(LNST, nst, 1)] if two else [at(LNST, nst)]
        pos_at = lambda g: P(W["bb"][g]["pos"], off * C)  # noqa: E731  (pos rows of the part)
        if two:
            if fold:
                cp["c2"] = [at(XN, C, 0), at(XN, C, 1)]
            self._gemm(plan, "patch_gemm", a=[pat(0), pat(1)],
                       w=[P(W["bb"][g]["patch_w"]) for g in range(2)], c=[at(X, C, 0), at(X, C, 1)], M=gm, N=C, K=KP,
                       lda=KP, ldc=C, bias=[P(W["bb"][g]["patch_b"]) for g in range(2)],
                       r=[pos_at(g) for g in range(2)], ldr=C, r_mode=1, r_p0=nr, c_f32=1, **cp, **pseg)
        else:
            if fold:
                cp["c2"] = [at(XN, C)]
            self._gemm(plan, "patch_gemm", a=[pat(0)], w=[P(W["bb"][0]["patch_w"])], c=[at(X, C)],
                       M=S * nr, N=C, K=KP, lda=KP, ldc=C, bias=[P(W["bb"][0]["patch_b"])], r=[pos_at(0)], ldr=C,
                       r_mode=1, r_p0=nr, c_f32=1, **cp, **pseg)
        # --- transformer blocks
        if self.ce and part is not None:
            raise NotImplementedError("the template K/V cache is not defined for candidate elimination")
        stage = 0
        for i in range(d.depth):
            gm = B * nr  # rows per modality group (nr shrinks after each elimination stage)
            QKV = ws["QKV"] if qkv_layers is None else qkv_layers[i]
            if two:
                blks = [W["bb"][g]["blocks"][i] for g in range(2)]
                n1 = [blks[0]["norm1"], blks[1]["norm1"]]
                n2 = [blks[0]["norm2"], blks[1]["norm2"]]
                wl = lambda nm: [P(blks[g][nm]) for g in range(2)]  # noqa: E731
                fl = lambda nm: [P(blks[g][nm][0]) for g in range(2)]  # noqa: E731
                rows = lambda t, k: [at(t, k, 0), at(t, k, 1)]  # noqa: E731
                Mg = gm
            else:
                blk = W["bb"][0]["blocks"][i]
                n1 = [blk["norm1"]] * 2 if nm_ == 1 else [blk["norm1_v"], blk["norm1_i"]]
                n2 = [blk["norm2"]] * 2 if nm_ == 1 else [blk["norm2_v"], blk["norm2_i"]]
                wl = lambda nm: [P(blk[nm])]  # noqa: E731
                fl = lambda nm: [P(blk[nm][m]) for m in range(nm_)]  # noqa: E731
                rows = lambda t, k: [at(t, k)]  # noqa: E731
                Mg = S * nr
            rows2 = lambda t, k: [at(t, k, g) for g in range(nm_)]  # noqa: E731  (one group per modality)
            qrows2 = [qat(QKV, g) for g in range(nm_)]
            if fold:  # LayerNorm 1 folded into qkv: A = XN = bf16 copy of the residual stream X
                self._gemm(plan, "qkv", a=rows2(XN, C), w=fl("attn.qkv.fw"), c=qrows2, M=gm, N=3 * C,
                           K=C, lda=C, ldc=3 * C, bias=fl("attn.qkv.fb"), ln_colsum=fl("attn.qkv.fcs"), ln_eps=1e-6,
                           ln_stats_in=rows2(LNST, nst) if hand else None, **(qmap if compact else rmap(C)))
            else:
                plan.append((LIB.mmt_layernorm, (P(X), None, 0, None, P(XN), P(n1[0][0]), P(n1[0][1]), P(n1[1][0]),
                                                 P(n1[1][1]), R, B * rp, C, 1e-6, cdt), "ln1", None))
                self._gemm(plan, "qkv", a=rows(XN, C), w=wl("attn.qkv.w"), c=[qat(QKV, g) for g in range(len(rows(XN, C)))],
                           M=Mg, N=3 * C, K=C, lda=C, ldc=3 * C, bias=wl("attn.qkv.b"), **(qmap if compact else rmap(C)))
            ap = AttnParams()
            ap.qkv, ap.out, ap.S, ap.Bm, ap.ntok, ap.n_t, ap.C, ap.H = P(QKV), P(AO), S, B, ntok, d.n_t, C, d.H
            if compact:  # the part's rows stored compact
                ap.out_pitch, ap.out_q0 = nr, off
            if part is None and nr != ntok:  # after an elimination stage: first nr rows of each sequence
                ap.ntok, ap.tok_pitch = nr, ntok
            ap.asym = 1 if self.variant in ("asym", "asym_online", "asym_ce") else 0
            ap.scale = 1.0 / LOG2E if self.fold_ln else (C // d.H) ** -0.5  # see q_scale
            ap.q_part = {None: 0, "t": 1, "s": 2}[part]
            ap.impl = self.attn_impl
            plan.append((LIB.mmt_mam_attention, (ctypes_byref(ap), cdt), "mam_attention", ap))
            cpx = dict(c2=rows(XN, C), c2_copy=1) if fold else {}
            if hand:
                cpx["ln_stats_out"] = rows(LNST, nst)
            self._gemm(plan, "proj", a=rows(AO, C), w=wl("attn.proj.w"), c=rows(X, C), M=Mg, N=C, K=C, lda=C,
                       ldc=C, bias=wl("attn.proj.b"), r=rows(X, C), ldr=C, c_f32=1, **cpx, **rmap(C))
            if i in self.ce:  # candidate elimination after the attention residual, before the MLP
                k = nr - d.n_t
                keep = math.ceil(self.ce[i] * k)
                if keep < k:
                    nparts = d.H * (2 * d.n_t // (16 if cdt == MMT_BF16 else 8))  # mmt_ce_t2s_attention blocks
                    masked = self.ce_mask_count is not None
                    plan.append((LIB.mmt_ce_t2s_attention_masked,
                                 (P(QKV), P(ws["CEP"]), P(ws["CEMASK"]) if masked else None, B, ntok, d.n_t, k, C, d.H,
                                  ap.scale, cdt), "ce_t2s", None))
                    nq = self.ce_mask_count if masked else 2 * d.n_t  # template queries averaged
                    plan.append((LIB.mmt_ce_select, (P(ws["CEP"]), nparts, B, k, keep, d.ns,
                                                     P(ws["CEG"][stage - 1]) if stage else None, P(ws["CEG"][stage]),
                                                     P(ws["CEO"]), P(ws["CEM"][stage]),
                                                     1.0 / (d.H * nq)), "ce_select", None))
                    Xn = ws["XC"] if X is ws["X"] else ws["X"]
                    plan.append((LIB.mmt_ce_gather, (P(X), P(Xn), P(XN) if fold else None, P(ws["CEO"]), S, ntok,
                                                     d.n_t, keep, d.ns, C, cdt), "ce_gather", None))
                    X = Xn
                    nr = d.n_t + keep
                    ws["CE_FINAL"] = (ws["CEG"][stage], keep)
                    stage += 1
                    Mg = gm = B * nr
                    if not two:
                        Mg = S * nr
            if fold:
                self._gemm(plan, "fc1", a=rows2(XN, C), w=fl("mlp.fc1.fw"), c=rows2(HID, d.hidden), M=gm, N=d.hidden,
                           K=C, lda=C, ldc=d.hidden, bias=fl("mlp.fc1.fb"), act=1, ln_colsum=fl("mlp.fc1.fcs"),
                           ln_eps=1e-6, ln_stats_in=rows2(LNST, nst) if hand else None, **rmap(C))
            else:
                plan.append((LIB.mmt_layernorm, (P(X), None, 0, None, P(XN), P(n2[0][0]), P(n2[0][1]), P(n2[1][0]),
                                                 P(n2[1][1]), R, B * rp, C, 1e-6, cdt), "ln2", None))
                self._gemm(plan, "fc1", a=rows(XN, C), w=wl("mlp.fc1.w"), c=rows(HID, d.hidden), M=Mg, N=d.hidden,
                           K=C, lda=C, ldc=d.hidden, bias=wl("mlp.fc1.b"), act=1, **rmap(C))
            self._gemm(plan, "fc2", a=rows(HID, d.hidden), w=wl("mlp.fc2.w"), c=rows(X, C), M=Mg, N=C, K=d.hidden,
                       lda=d.hidden, ldc=C, bias=wl("mlp.fc2.b"), r=rows(X, C), ldr=C, c_f32=1, **cpx, **rmap(d.hidden))
        return (X, stage)

    def _image_args(self, t, o, s):
        """mmt_patch_im2col's six image pointers (t0, t1, o0, o1, s0, s1); the RGB-only model passes
        NULL for the second modality."""
        if self.d.nmod == 1:
            return (_ptr(t[0]), None, _ptr(o[0]), None, _ptr(s[0]), None)
        return tuple(_ptr(x) for x in list(t) + list(o) + list(s))

    def _plan_tail(self, plan, ws, score, xf=None, spm_kv1=True, compact=False):
        """Fusion, corner head (and score head) on the backbone output's search rows.  xf = (the fp32
        stream holding the backbone output, elimination stages run) from _plan_backbone; compact: the
        search pass of the template K/V cache, whose streams hold only the search rows ([S][ns])."""
        d, W, B = self.d, self.w, ws["B"]
        C, ns, dm = d.C, d.ns, d.d_model
        ntok = ns if compact else d.ntok  # rows per sequence of the backbone output
        t0 = 0 if compact else d.n_t      # its first search row
        R = 2 * B * ntok
        P = _ptr
        X, XN = ws["X"], ws["XN"]
        cdt = self.cdt
        fold = self.fold_ln
        if xf is not None and xf[1] > 0:
            # _recover_search (asymmetric_shared_ce.py:426-447): surviving rows back to their original
            # search positions, zeros where pruned, in the dtype the fusion reads
            XT = XN if fold else ws["XT"]
            gf, kf = ws["CE_FINAL"]
            plan.append((LIB.mmt_ce_recover, (P(xf[0]), P(gf), kf, P(XT), 2 * B, ntok, d.n_t, ns, C, cdt),
                         "ce_recover", None))
            ws["XOUT"] = XT
        elif fold:
            XT = XN  # the last fc2 already wrote the bf16 copy of the backbone output
        else:
            XT = ws["XT"]
            plan.append((LIB.mmt_add_cast, (P(X), None, 0, None, P(XT), d.nmod * B * ntok * C, cdt), "cast_x", None))
        if d.nmod == 1:  # RGB-only: the corner head reads the backbone's search tokens (an NHWC gs x gs
            # image every ntok rows: the conv's image pitch), mixformer_vit/mixformer.py:304-305
            if self.hdtype != self.dtype or not fold:  # the head's own storage type, from the fp32 stream
                XT = ws["XH"]
                plan.append((LIB.mmt_add_cast, (P(X), None, 0, None, P(XT), B * ntok * C, self.hcdt), "cast_head_in",
                             None))
            self._plan_head(plan, ws, score, P(XT, t0 * C), C, None if compact else (max(B * ns, 1), 1, ntok, 0))
            return plan
        # --- fusion: adjust_v / adjust_i (1x1 conv on the search tokens) + GroupNorm
        Y1, SRC, SRCT, VAL = ws["Y1"], ws["SRC"], ws["SRCT"], ws["VAL"]
        Mf = B * ns
        self._gemm(plan, "fusion_adjust", a=[P(XT, t0 * C), P(XT, B * ntok * C + t0 * C)],
                   w=[P(W["adj_v.w"]), P(W["adj_i.w"])], c=[P(Y1), P(Y1, Mf * dm)], M=Mf, N=dm, K=C, lda=C, ldc=dm,
                   bias=[P(W["adj_v.b"]), P(W["adj_i.b"])], seg=None if compact else (ns, 1 << 30, ntok * C, 0), c_f32=1)
        plan.append((LIB.mmt_groupnorm, (P(Y1), P(SRC), P(SRCT), P(W["adj_v.gn"][0]), P(W["adj_v.gn"][1]),
                                         P(W["adj_i.gn"][0]), P(W["adj_i.gn"][1]), 2 * B, B, ns, dm, 32, 1e-5, cdt),
                     "fusion_gn", None))
        for e in W["enc"]:
            # value and the offsets / logits of the query src + pos (src . W^T + the folded per-cell pos
            # term) both read SRCT only: one launch
            vo = []
            self._gemm(plan, "enc_value", a=[P(SRCT)], w=[P(e["value.w"])], c=[P(VAL)], M=2 * Mf, N=dm, K=dm, lda=dm,
                       ldc=dm, bias=[P(e["value.b"])], defer=vo)
            self._gemm(plan, "enc_offw", a=[P(SRCT)], a1=[P(SRCT, Mf * dm)], k_split=dm, w=[P(e["offw.w"])],
                       c=[P(ws["OFFW"])], M=Mf, N=192, K=2 * dm, lda=dm, ldc=192, r=[P(e["offw.pos"])], ldr=192,
                       r_mode=1, r_p0=ns, c_f32=1, defer=vo)
            self._gemm_multi(plan, "enc_value_offw", vo)
            plan.append((LIB.mmt_msda_bimodal, (P(ws["OFFW"]), P(VAL), P(ws["MS"]), B, d.gs, cdt), "msda_bimodal", None))
            self._gemm(plan, "enc_outproj", a=[P(ws["MS"])], w=[P(e["out.w"])], c=[P(ws["SRC2"])], M=Mf, N=dm, K=dm,
                       lda=dm, ldc=dm, bias=[P(e["out.b"])], c_f32=1)
            plan.append((LIB.mmt_layernorm, (P(SRC), P(ws["SRC2"]), Mf, P(SRC), P(SRCT), P(e["norm1_v"][0]),
                                             P(e["norm1_v"][1]), P(e["norm1_i"][0]), P(e["norm1_i"][1]), 2 * Mf, Mf,
                                             dm, 1e-5, cdt), "enc_ln1", None))
            self._gemm(plan, "enc_linear1", a=[P(SRCT)], w=[P(e["l1.w"])], c=[P(ws["H2"])], M=2 * Mf, N=d.ffn, K=dm,
                       lda=dm, ldc=d.ffn, bias=[P(e["l1.b"])], act=2)
            self._gemm(plan, "enc_linear2", a=[P(ws["H2"])], w=[P(e["l2.w"])], c=[P(SRC)], M=2 * Mf, N=dm, K=d.ffn,
                       lda=d.ffn, ldc=dm, bias=[P(e["l2.b"])], r=[P(SRC)], ldr=dm, c_f32=1,
                       # unsplit: as fast as the cost model's 2-way split-K (10.9 vs 11.1 us at B = 1) without its
                       # partial-tile traffic (profiles/r05_splitk_entry_ab.jsonl)
                       tile=(0, 1))
            plan.append((LIB.mmt_layernorm, (P(SRC), None, 0, P(SRC), P(SRCT), P(e["norm2_v"][0]), P(e["norm2_v"][1]),
                                             P(e["norm2_i"][0]), P(e["norm2_i"][1]), 2 * Mf, Mf, dm, 1e-5, cdt),
                         "enc_ln2", None))
        self._gemm(plan, "fusion_adjust_cat", a=[P(SRCT)], a1=[P(SRCT, Mf * dm)], k_split=dm, w=[P(W["adj_cat.w"])],
                   c=[P(ws["Y2"])], M=Mf, N=C, K=2 * dm, lda=dm, ldc=C, bias=[P(W["adj_cat.b"])], c_f32=1)
        plan.append((LIB.mmt_groupnorm, (P(ws["Y2"]), P(ws["FUS"]), P(ws["FUST"]), P(W["adj_cat.gn"][0]),
                                         P(W["adj_cat.gn"][1]), None, None, B, B, ns, C, 32, 1e-5, self.hcdt),
                     "fusion_gn_cat", None))
        self._plan_head(plan, ws, score, P(ws["FUST"]), C, None, spm_kv1)
        return plan

    def _plan_head(self, plan, ws, score, a_ptr, lda, seg, spm_kv1=True):
        """Corner head (head.py:147-212) on the NHWC map at a_ptr (pixel stride lda; seg = the conv
        input's image pitch for the RGB-only model), then the score head."""
        d, W, B = self.d, self.w, ws["B"]
        C, ns = d.C, d.ns
        P = _ptr
        cdt = self.hcdt  # the head's storage type (head_dtype)
        hg = lambda *a, **k: self._gemm(*a, dtype=cdt, **k)  # noqa: E731
        # --- corner head (NHWC implicit-GEMM convs, BN folded, upsampling folded into addressing)
        hc, gs = d.hc, d.gs
        H0 = ws["H0"]
        n0 = 2 * hc + hc + hc // 2
        hg(plan, "head_conv1_adj12", a=[a_ptr], w=[P(W["h0.w"])], c=[P(H0)], M=B * ns, N=n0, K=9 * C,
                   lda=lda, ldc=n0, bias=[P(W["h0.b"])], act=2, conv=(gs, 1, C, 1), seg=seg)
        h2, h4, h8 = hc // 2, hc // 4, hc // 8
        X2, S1, X3, S2, X4 = ws["X2"], ws["S1"], ws["X3"], ws["S2"], ws["X4"]
        br = ("tl", "br")
        hg(plan, "head_conv2", a=[P(H0, g * hc) for g in range(2)], w=[P(W["conv2_%s.w" % b]) for b in br],
                   c=[P(X2, g * B * ns * h2) for g in range(2)], c2=[P(S1, g * B * ns * h2) for g in range(2)],
                   r=[P(H0, 2 * hc + g * h2) for g in range(2)], ldr=n0, r_t=1, M=B * ns, N=h2, K=9 * hc, lda=n0,
                   ldc=h2, bias=[P(W["conv2_%s.b" % b]) for b in br], act=2, conv=(gs, 1, hc, 1))
        # the two pyramid branches are independent of the conv chain past their inputs
        # (head.py:159-197): conv3 beside adjust3[0], conv4 beside adjust4[0] and adjust3[1]
        l3, l4 = [], []
        hg(plan, "head_conv3", a=[P(S1, g * B * ns * h2) for g in range(2)], w=[P(W["conv3_%s.w" % b]) for b in br],
                   c=[P(X3, g * B * 4 * ns * h4) for g in range(2)], c2=[P(S2, g * B * 4 * ns * h4) for g in range(2)],
                   r=[P(H0, 2 * hc + hc + g * h4) for g in range(2)], ldr=n0, r_t=1, r_mode=2, r_p0=2 * gs, r_p1=2,
                   M=B * 4 * ns, N=h4, K=9 * h2, lda=h2, ldc=h4, bias=[P(W["conv3_%s.b" % b]) for b in br], act=2,
                   conv=(2 * gs, 2, h2, 1), defer=l3)
        hg(plan, "head_adjust3_0", a=[P(X2, g * B * ns * h2) for g in range(2)],
                   w=[P(W["adjust3.0_%s.w" % b]) for b in br], c=[P(ws["A3a"], g * B * ns * h4) for g in range(2)],
                   M=B * ns, N=h4, K=9 * h2, lda=h2, ldc=h4, bias=[P(W["adjust3.0_%s.b" % b]) for b in br], act=2,
                   conv=(gs, 1, h2, 1), defer=l3)
        self._gemm_multi(plan, "head_conv3_adjust3_0", l3)
        hg(plan, "head_conv4", a=[P(S2, g * B * 4 * ns * h4) for g in range(2)], w=[P(W["conv4_%s.w" % b]) for b in br],
                   c=[P(X4, g * B * 16 * ns * h8) for g in range(2)], M=B * 16 * ns, N=h8, K=9 * h4, lda=h4, ldc=h8,
                   bias=[P(W["conv4_%s.b" % b]) for b in br], act=2, conv=(4 * gs, 2, h4, 1), defer=l4)
        hg(plan, "head_adjust4_0", a=[P(X3, g * B * 4 * ns * h4) for g in range(2)],
                   w=[P(W["adjust4.0_%s.w" % b]) for b in br], c=[P(ws["A4a"], g * B * 4 * ns * h8) for g in range(2)],
                   M=B * 4 * ns, N=h8, K=9 * h4, lda=h4, ldc=h8, bias=[P(W["adjust4.0_%s.b" % b]) for b in br], act=2,
                   conv=(2 * gs, 1, h4, 1), defer=l4)
        hg(plan, "head_adjust3_1", a=[P(ws["A3a"], g * B * ns * h4) for g in range(2)],
                   w=[P(W["adjust3.1_%s.w" % b]) for b in br], c=[P(ws["A3b"], g * B * ns * h8) for g in range(2)],
                   M=B * ns, N=h8, K=9 * h4, lda=h4, ldc=h8, bias=[P(W["adjust3.1_%s.b" % b]) for b in br], act=2,
                   conv=(gs, 1, h4, 1), defer=l4)
        self._gemm_multi(plan, "head_conv4_adjust4_0_adjust3_1", l4)
        plan.append((LIB.mmt_conv3x3_c1_pair, (P(ws["A3b"]), P(W["a3c1.w"]), P(W["a3c1.b"]), P(ws["A3"]), gs, h8,
                                               P(ws["A4a"]), P(W["a4c1.w"]), P(W["a4c1.b"]), P(ws["A4"]), 2 * gs, h8,
                                               2, B, h8, cdt), "head_adjust3_2_adjust4_1", None))
        plan.append((LIB.mmt_corner_softargmax, (P(X4), P(W["c5.w"]), P(W["c5.b"]), P(ws["A3"]), P(ws["A4"]),
                                                 P(ws["MAPS"]), P(ws["BOX"]), P(ws["XYXY"]), P(ws["ROIS"]) if score else None,
                                                 float(gs), B, d.fh, h8, 4, cdt), "corner_softargmax", None))
        if score:
            self._plan_spm(plan, ws, spm_kv1)

    def _plan_spm_kv1(self, plan, ws, compact=False):
        """K/V of the score decoder's second memory: the first template's tokens of both modalities
        (the template pass computes it once per template update when the K/V cache is used; its stream
        holds only the template rows: compact)."""
        d, W, B, P, C = self.d, self.w, ws["B"], _ptr, self.d.C
        rp = d.n_t if compact else d.ntok
        self._gemm(plan, "spm_kv1", a=[P(ws["X"])], w=[P(W["spm.kv1.w"])], c=[P(ws["KV1"])], M=B * 2 * d.nt1, N=2 * C,
                   K=C, lda=C, ldc=2 * C, bias=[P(W["spm.kv1.b"])], seg=(d.nt1, 2, B * rp * C, rp * C),
                   c_f32=1, dtype=MMT_F32)

    def _plan_spm(self, plan, ws, kv1=True):
        """ScoreDecoder (score_decoder.py:32-66), fp32.  kv1=False: the template memory's K/V are
        already in KV1 (template pass)."""
        d, W, B = self.d, self.w, ws["B"]
        P, C, ns, gs = _ptr, d.C, d.ns, d.gs
        F32 = MMT_F32
        # PrRoIPool(4,4,1.0) on the channels-last fused map -> tokens [B][16][C]
        plan.append((LIB.mmt_prroi_pool_forward, (P(ws["FUS"]), P(ws["ROIS"]), P(ws["ROIT"]), B, C, gs, gs, ns * C, 1,
                                                  gs * C, C, 4, 4, 1.0, 16 * C, 1, C), "spm_prroi", None))
        self._gemm(plan, "spm_kv0", a=[P(ws["ROIT"])], w=[P(W["spm.kv0.w"])], c=[P(ws["KV0"])], M=B * 16, N=2 * C, K=C,
                   lda=C, ldc=2 * C, bias=[P(W["spm.kv0.b"])], c_f32=1, dtype=F32)
        scale = C ** -0.5
        plan.append((LIB.mmt_spm_attention, (P(W["spm.q0"]), 0, P(ws["KV0"]), P(ws["AT"]), B, 16, C, d.H, scale),
                     "spm_attn0", None))
        self._gemm(plan, "spm_proj0", a=[P(ws["AT"])], w=[P(W["spm.proj0.w"])], c=[P(ws["XS"])], M=B, N=C, K=C, lda=C,
                   ldc=C, bias=[P(W["spm.proj0.b"])], c_f32=1, dtype=F32)
        n = W["spm.norm2.0"]
        plan.append((LIB.mmt_layernorm, (P(ws["XS"]), None, 0, P(ws["XS"]), None, P(n[0]), P(n[1]), None, None, B, B, C,
                                         1e-5, F32), "spm_ln0", None))
        self._gemm(plan, "spm_q1", a=[P(ws["XS"])], w=[P(W["spm.q1.w"])], c=[P(ws["Q1"])], M=B, N=C, K=C, lda=C, ldc=C,
                   bias=[P(W["spm.q1.b"])], c_f32=1, dtype=F32)
        # template tokens of both modalities from the fp32 residual stream: [b][m][t]
        if kv1:
            self._plan_spm_kv1(plan, ws)
        plan.append((LIB.mmt_spm_attention, (P(ws["Q1"]), C, P(ws["KV1"]), P(ws["AT"]), B, 2 * d.nt1, C, d.H, scale),
                     "spm_attn1", None))
        self._gemm(plan, "spm_proj1", a=[P(ws["AT"])], w=[P(W["spm.proj1.w"])], c=[P(ws["XS"])], M=B, N=C, K=C, lda=C,
                   ldc=C, bias=[P(W["spm.proj1.b"])], c_f32=1, dtype=F32)
        n = W["spm.norm2.1"]
        plan.append((LIB.mmt_layernorm, (P(ws["XS"]), None, 0, P(ws["XS"]), None, P(n[0]), P(n[1]), None, None, B, B, C,
                                         1e-5, F32), "spm_ln1", None))
        src = ws["XS"]
        nl = W["spm.mlp_n"]
        for i in range(nl):
            last = i == nl - 1
            dst = ws["SC"] if last else (ws["M1"] if i % 2 == 0 else ws["M2"])
            N = W["spm.mlp%d.w" % i].shape[0]
            self._gemm(plan, "spm_mlp%d" % i, a=[P(src)], w=[P(W["spm.mlp%d.w" % i])], c=[P(dst)], M=B, N=N, K=C,
                       lda=C, ldc=N, bias=[P(W["spm.mlp%d.b" % i])], act=0 if last else 2, c_f32=1, dtype=F32)
            src = dst

    # ------------------------------------------------------------------ execution
    def run_plan(self, plan, stream=None):
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        for fn, args, name, _keep in plan:
            st = fn(*args, s)
            if st != 0:
                check(st, name)

    def load_inputs(self, ws, template, online_template, search):
        for dst, src in zip(ws["in_t"] + ws["in_o"] + ws["in_s"], list(template) + list(online_template) + list(search)):
            if src.shape != dst.shape:
                raise ValueError("input shape %s, expected %s" % (tuple(src.shape), tuple(dst.shape)))
            dst.copy_(src, non_blocking=True)

    def forward(self, template, online_template, search, run_score_head=False, use_graph=False, ce_template_mask=None):
        """template / online_template / search: [rgb, tir] lists of (B,3,H,W) fp32 device tensors.
        ce_template_mask: (B, 2 n_t) bool template-query mask of the candidate elimination (a runtime
        built with ce_mask_count; each row must select that many queries).
        Returns (boxes_cxcywh (B,4) fp32, scores (B,) fp32 or None) — views of the workspace."""
        B = template[0].shape[0]
        ws = self.workspace(B)
        score = bool(run_score_head) and self.variant == "asym_online"
        self.load_inputs(ws, template, online_template, search)
        if (ce_template_mask is None) != (self.ce_mask_count is None):
            raise ValueError("ce_template_mask must be given exactly when the runtime was built with ce_mask_count")
        if ce_template_mask is not None:
            m = ws["CEMASK"]
            if tuple(ce_template_mask.shape) != tuple(m.shape):
                raise ValueError("ce_template_mask shape %s, expected %s" % (tuple(ce_template_mask.shape), tuple(m.shape)))
            m.copy_(ce_template_mask.to(device=m.device, dtype=torch.uint8), non_blocking=True)
        if use_graph:
            g = self._graphs.get((B, score))
            if g is None:
                g = self.capture(B, score)
            g.replay()
        else:
            self.run_plan(ws["plan_score"] if score else ws["plan"])
        return ws["BOX"], (ws["SC"].view(-1) if score else None)

    def score_on_boxes(self, B, boxes_xyxy):
        """The score decoder (score_decoder.py:32-66) on caller boxes (xyxy normalised to the search
        crop) after forward() of batch B: ROIs = [b, box * feature size] into the workspace, then the
        ScoreDecoder plan.  Not a reference entry point: the reference's forward drops gt_bboxes
        (asymmetric_shared_online.py:374) and always scores the predicted box, as model.forward does."""
        ws = self.workspace(B)
        gs = float(self.d.gs)
        rois = ws["ROIS"]
        rois[:, 0] = torch.arange(B, device=rois.device, dtype=rois.dtype)
        rois[:, 1:] = boxes_xyxy.reshape(B, 4).to(rois.dtype) * gs
        self.run_plan(ws["plan_spm"])
        return ws["SC"].view(-1)

    # ------------------------------------------------------------------ template K/V cache
    def cache_workspace(self, B):
        """Workspace of batch B plus the template K/V cache (the RGB MixFormer's
        set_online / forward_test, mixformer_vit/mixformer.py:308-323, which the RGB-T models
        lack, reference defect D2): one qkv buffer per layer, whose template rows the template
        pass ("plan_t") fills once per template update and whose search rows each frame's pass
        ("plan_s"; "plan_s_score" with the score head) fills before the layer's attention reads
        all of them.  Template queries attend template keys only, so template + search passes
        reproduce the full forward (same kernels, same per-row arithmetic)."""
        ws = self.workspace(B)
        if "plan_t" not in ws:
            d = self.d
            ws["QKVL"] = [torch.empty(d.nmod * B * d.ntok, 3 * d.C, device=self.device, dtype=self.dtype)
                          for _ in range(d.depth)]
            ws["plan_t"] = []
            self._plan_backbone(ws["plan_t"], ws, "t", ws["QKVL"])
            if self.variant == "asym_online":  # the score head's template K/V: once per template update
                self._plan_spm_kv1(ws["plan_t"], ws, compact=True)
            for score in ((False, True) if self.variant == "asym_online" else (False,)):
                plan = []
                self._plan_backbone(plan, ws, "s", ws["QKVL"])
                self._plan_tail(plan, ws, score, spm_kv1=False, compact=True)
                ws["plan_s_score" if score else "plan_s"] = plan
        return ws

    def set_template(self, template, online_template):
        """Template pass: template + online template ([rgb, tir] lists of (B,3,h,h) fp32 device
        tensors) through the backbone, filling the per-layer K/V cache (and the final template
        token states the score head reads)."""
        B = template[0].shape[0]
        ws = self.cache_workspace(B)
        for dst, src in zip(ws["in_t"] + ws["in_o"], list(template) + list(online_template)):
            if src.shape != dst.shape:
                raise ValueError("input shape %s, expected %s" % (tuple(src.shape), tuple(dst.shape)))
            dst.copy_(src, non_blocking=True)
        self.run_plan(ws["plan_t"])

    def forward_search(self, search, run_score_head=False):
        """Search pass against the cached template (set_template first, same batch size): boxes
        (B,4) cxcywh and scores as forward() returns them."""
        B = search[0].shape[0]
        ws = self.cache_workspace(B)
        score = bool(run_score_head) and self.variant == "asym_online"
        for dst, src in zip(ws["in_s"], list(search)):
            if src.shape != dst.shape:
                raise ValueError("input shape %s, expected %s" % (tuple(src.shape), tuple(dst.shape)))
            dst.copy_(src, non_blocking=True)
        self.run_plan(ws["plan_s_score"] if score else ws["plan_s"])
        return ws["BOX"], (ws["SC"].view(-1) if score else None)

    def plan_for_inputs(self, template, online_template, search, run_score_head=False, part=None):
        """The plan of batch B with its patch staging reading the given device tensors directly
        (zero-copy: for frames already resident in HBM, e.g. written there by the preprocessing).
        part None: the full forward; "t": the template pass (search may be None); "s": the search
        pass against the cache (template / online_template may be None)."""
        B = (search if part == "s" else template)[0].shape[0]
        ws = self.workspace(B) if part is None else self.cache_workspace(B)
        score = bool(run_score_head) and self.variant == "asym_online"
        key = {None: "plan", "t": "plan_t", "s": "plan_s"}[part]
        base = ws[key + "_score" if score and part != "t" else key]
        fn, args, name, keep = base[0]
        assert name == "patch_im2col"
        if part == "t":
            search = ws["in_s"]
        elif part == "s":
            template, online_template = ws["in_t"], ws["in_o"]
        srcs = list(template) + list(online_template) + list(search)
        for src, dst in zip(srcs, ws["in_t"] + ws["in_o"] + ws["in_s"]):
            if src.shape != dst.shape or src.dtype != torch.float32 or not src.is_contiguous() or src.device != dst.device:
                raise ValueError("zero-copy inputs must be contiguous fp32 %s tensors on %s" % (tuple(dst.shape), dst.device))
        n = self.d.nmod
        new_args = self._image_args(srcs[:n], srcs[n:2 * n], srcs[2 * n:]) + args[6:]
        return [(fn, new_args, name, srcs)] + base[1:]

    def capture_plan(self, plan):
        """Record an arbitrary plan as one hipGraph (returned; caller keeps the inputs alive)."""
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self.run_plan(plan)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.run_plan(plan)
        return g

    def capture(self, B, score=False):
        """Record the plan of batch B as one hipGraph (inputs are the workspace's static buffers)."""
        ws = self.workspace(B)
        plan = ws["plan_score"] if score else ws["plan"]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self.run_plan(plan)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.run_plan(plan)
        self._graphs[(B, score)] = g
        return g


def ctypes_byref(p):
    import ctypes
    return ctypes.byref(p)


def _sine_pos(g, c):
    """PositionEmbeddingSine(c/2, normalize=True) on a g x g all-valid map, flattened to
    [g*g][c] (position_encoding.py:34-54)."""
    npf = c // 2
    ones = torch.ones(1, g, g)
    y = ones.cumsum(1, dtype=torch.float32)
    x = ones.cumsum(2, dtype=torch.float32)
    eps, scale = 1e-6, 2 * math.pi
    y = (y - 0.5) / (y[:, -1:, :] + eps) * scale
    x = (x - 0.5) / (x[:, :, -1:] + eps) * scale
    dim_t = torch.arange(npf, dtype=torch.float32)
    dim_t = 10000 ** (2 * (dim_t // 2) / npf)
    px = x[:, :, :, None] / dim_t
    py = y[:, :, :, None] / dim_t
    px = torch.stack((px[:, :, :, 0::2].sin(), px[:, :, :, 1::2].cos()), dim=4).flatten(3)
    py = torch.stack((py[:, :, :, 0::2].sin(), py[:, :, :, 1::2].cos()), dim=4).flatten(3)
    return torch.cat((py, px), dim=3).reshape(g * g, c)
