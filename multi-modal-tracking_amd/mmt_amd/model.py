"""Drop-in MixFormer RGB-T models: the reference's `build_*` builders, module tree and state_dict
names, with the forward running on libmmt_hip.so (mmt_amd.runtime).

Boundary: lib/models/mixformer_vit_rgbt/__init__.py:1-2 (build_mixformer_vit_rgbt,
build_mixformer_vit_rgbt_shared), asymmetric_shared.py:408 (build_asymmetric_shared),
asymmetric_shared_online.py:430 (build_asymmetric_shared_online_score).  `build_*(cfg, train)`
returns an nn.Module whose state_dict keys equal the reference's (so
`load_state_dict(torch.load(ckpt)["net"], strict=True)` works, lib/test/tracker/mixformer_vit_rgbt.py:17)
and whose `forward(template, online_template, search, run_score_head=False, gt_bboxes=None,
return_features=False)` returns `({"pred_boxes": (B,1,4)[, "pred_scores": (B,)]}, (B,1,4))`.

The nn.Linear / nn.Conv2d / norm modules below are parameter containers only: they are never
called.  The forward is the fixed HIP launch plan; the first call after construction, `.to()` /
`.cuda()` or `load_state_dict` prepares device weights from the module's own parameters (call
`refresh_kernels()` after editing parameters in place).  There is no PyTorch fallback: without a
HIP device and libmmt_hip.so the forward raises.

Scope: inference (eval) of the hot path.  Fusion class Attention_Fusion_Bimodal_LNSpecific and
head CORNER_UP only; the reference's other fusion/head classes are ablations
out of scope.  Deviation D1: the fusion width follows MODEL.HIDDEN_DIM instead of the reference's
hard-coded 768, so ViT-L (HIDDEN_DIM 1024) builds; for ViT-B both are 768.
"""
import math
import os

import torch
import torch.nn as nn

# ----------------------------------------------------------------------------- parameter containers
class PatchEmbed(nn.Module):
    def __init__(self, patch_size=16, in_chans=3, embed_dim=768):
        super().__init__()
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = nn.Identity()


class Attention(nn.Module):
    """MAM parameters (mixformer.py:37-50): fused qkv Linear + proj."""

    def __init__(self, dim, num_heads):
        super().__init__()
        self.num_heads = num_heads
        self.scale = (dim // num_heads) ** -0.5
        self.qkv = nn.Linear(dim, dim * 3)
        self.proj = nn.Linear(dim, dim)


class Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(hidden, dim)


class Block(nn.Module):
    """Pre-LN block (mixformer.py:113-139); `shared` = per-modality LNs (mixformer_shared.py:121-141)."""

    def __init__(self, dim, num_heads, mlp_ratio=4.0, shared=False):
        super().__init__()
        ln = lambda: nn.LayerNorm(dim, eps=1e-6)  # noqa: E731
        if shared:
            self.norm1_v, self.norm1_i = ln(), ln()
        else:
            self.norm1 = ln()
        self.attn = Attention(dim, num_heads)
        if shared:
            self.norm2_v, self.norm2_i = ln(), ln()
        else:
            self.norm2 = ln()
        self.mlp = Mlp(dim, int(dim * mlp_ratio))


class VisionTransformer(nn.Module):
    """Backbone container (mixformer.py:152-229): patch embed, blocks, fixed sin-cos pos-embeds."""

    def __init__(self, img_size_s, img_size_t, embed_dim, depth, num_heads, shared):
        super().__init__()
        self.pos_drop = nn.Dropout(0.0)
        self.patch_embed = PatchEmbed(16, 3, embed_dim)
        self.blocks = nn.Sequential(*[Block(embed_dim, num_heads, 4.0, shared) for _ in range(depth)])
        self.grid_size_s, self.grid_size_t = img_size_s // 16, img_size_t // 16
        self.pos_embed_s = nn.Parameter(torch.zeros(1, self.grid_size_s ** 2, embed_dim), requires_grad=False)
        self.pos_embed_t = nn.Parameter(torch.zeros(1, self.grid_size_t ** 2, embed_dim), requires_grad=False)
        if self.pos_embed_s.device.type != "meta":
            from .synthetic import sincos_pos_embed
            with torch.no_grad():
                self.pos_embed_s.copy_(torch.from_numpy(sincos_pos_embed(embed_dim, self.grid_size_s))[None])
                self.pos_embed_t.copy_(torch.from_numpy(sincos_pos_embed(embed_dim, self.grid_size_t))[None])


class MSDeformAttn_Bimodal(nn.Module):
    """ms_deform_attn_bimodal.py:31-81 parameters (8 heads, 2 levels, 4 points)."""

    def __init__(self, d_model=512, n_levels=2, n_heads=8, n_points=4):
        super().__init__()
        self.im2col_step = 64
        self.d_model, self.n_levels, self.n_heads, self.n_points = d_model, n_levels, n_heads, n_points
        self.sampling_offsets = nn.Linear(2 * d_model, n_heads * n_levels * n_points * 2)
        self.attention_weights = nn.Linear(2 * d_model, n_heads * n_levels * n_points)
        self.value_proj = nn.Linear(d_model, d_model)
        self.output_proj = nn.Linear(d_model, d_model)


class DeformableTransformerEncoderLayer(nn.Module):
    """deformable_encoder_lnspecific.py:111-160 parameters."""

    def __init__(self, d_model, d_ffn):
        super().__init__()
        self.self_attn = MSDeformAttn_Bimodal(d_model)
        self.dropout1 = nn.Dropout(0.1)
        self.norm1_v, self.norm1_i = nn.LayerNorm(d_model), nn.LayerNorm(d_model)
        self.linear1 = nn.Linear(d_model, d_ffn)
        self.dropout2 = nn.Dropout(0.1)
        self.linear2 = nn.Linear(d_ffn, d_model)
        self.dropout3 = nn.Dropout(0.1)
        self.norm2_v, self.norm2_i = nn.LayerNorm(d_model), nn.LayerNorm(d_model)


class DeformableTransformerEncoder(nn.Module):
    def __init__(self, d_model, d_ffn, num_layers):
        super().__init__()
        self.layers = nn.ModuleList([DeformableTransformerEncoderLayer(d_model, d_ffn) for _ in range(num_layers)])
        self.num_layers = num_layers


class DeformableAttentionFusion_LNSpecific(nn.Module):
    def __init__(self, d_model=512, num_encoder_layers=2, num_feature_levels=2):
        super().__init__()
        self.d_model, self.nhead = d_model, 8
        self.encoder = DeformableTransformerEncoder(d_model, 4 * d_model, num_encoder_layers)
        self.level_embed = nn.Parameter(torch.zeros(num_feature_levels, d_model))


class Attention_Fusion_Bimodal_LNSpecific(nn.Module):
    """fusion_utils.py:243-268 parameters."""

    def __init__(self, channels_num, d_model=512, num_feature_levels=2, num_encoder_layers=2):
        super().__init__()
        self.adjust_v = nn.Sequential(nn.Conv2d(channels_num, d_model, 1), nn.GroupNorm(32, d_model))
        self.adjust_i = nn.Sequential(nn.Conv2d(channels_num, d_model, 1), nn.GroupNorm(32, d_model))
        self.fusion_attention = DeformableAttentionFusion_LNSpecific(d_model, num_encoder_layers, num_feature_levels)
        self.adjust_cat = nn.Sequential(nn.Conv2d(2 * d_model, channels_num, 1), nn.GroupNorm(32, channels_num))


class FrozenBatchNorm2d(nn.Module):
    """lib/models/mixformer_cvt/utils.py:21-57: fixed statistics and affine (buffers); eps 1e-5 inside the
    rsqrt as the reference's.  The inference runtime folds it into the conv; training's head on the HIP ops
    computes it with mmt_batchnorm_relu in eval mode (train.HipOps.bn_relu)."""

    eps = 1e-5

    def __init__(self, n):
        super().__init__()
        self.register_buffer("weight", torch.ones(n))
        self.register_buffer("bias", torch.zeros(n))
        self.register_buffer("running_mean", torch.zeros(n))
        self.register_buffer("running_var", torch.ones(n))

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        state_dict.pop(prefix + "num_batches_tracked", None)  # utils.py:37-45
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                                      error_msgs)

    def forward(self, x):  # utils.py:47-57
        scale = self.weight.reshape(1, -1, 1, 1) * (self.running_var.reshape(1, -1, 1, 1) + self.eps).rsqrt()
        return x * scale + (self.bias.reshape(1, -1, 1, 1) - self.running_mean.reshape(1, -1, 1, 1) * scale)


def conv(cin, cout, freeze_bn=False):
    """head.py:7-20: Conv3x3(bias) -> BN -> ReLU."""
    return nn.Sequential(nn.Conv2d(cin, cout, 3, 1, 1, bias=True),
                         FrozenBatchNorm2d(cout) if freeze_bn else nn.BatchNorm2d(cout), nn.ReLU(inplace=True))


class Pyramid_Corner_Predictor(nn.Module):
    """head.py:98-145 parameters (CORNER_UP)."""

    def __init__(self, inplanes=768, channel=384, feat_sz=80, stride=4, freeze_bn=False):
        super().__init__()
        self.feat_sz, self.stride, self.img_sz = feat_sz, stride, feat_sz * stride
        for br in ("tl", "br"):
            setattr(self, "conv1_" + br, conv(inplanes, channel, freeze_bn))
            setattr(self, "conv2_" + br, conv(channel, channel // 2, freeze_bn))
            setattr(self, "conv3_" + br, conv(channel // 2, channel // 4, freeze_bn))
            setattr(self, "conv4_" + br, conv(channel // 4, channel // 8, freeze_bn))
            setattr(self, "conv5_" + br, nn.Conv2d(channel // 8, 1, kernel_size=1))
            setattr(self, "adjust1_" + br, conv(inplanes, channel // 2, freeze_bn))
            setattr(self, "adjust2_" + br, conv(inplanes, channel // 4, freeze_bn))
            setattr(self, "adjust3_" + br, nn.Sequential(conv(channel // 2, channel // 4, freeze_bn),
                                                          conv(channel // 4, channel // 8, freeze_bn),
                                                          conv(channel // 8, 1, freeze_bn)))
            setattr(self, "adjust4_" + br, nn.Sequential(conv(channel // 4, channel // 8, freeze_bn),
                                                          conv(channel // 8, 1, freeze_bn)))


class MLP(nn.Module):
    def __init__(self, input_dim, hidden_dim, output_dim, num_layers):
        super().__init__()
        self.num_layers = num_layers
        h = [hidden_dim] * (num_layers - 1)
        self.layers = nn.ModuleList(nn.Linear(n, k) for n, k in zip([input_dim] + h, h + [output_dim]))


class ScoreDecoder(nn.Module):
    """score_decoder.py:12-30 parameters (SPM)."""

    def __init__(self, num_heads=12, hidden_dim=768, nlayer_head=3, pool_size=4):
        super().__init__()
        self.num_heads, self.pool_size = num_heads, pool_size
        self.score_head = MLP(hidden_dim, hidden_dim, 1, nlayer_head)
        self.scale = hidden_dim ** -0.5
        self.proj_q = nn.ModuleList(nn.Linear(hidden_dim, hidden_dim) for _ in range(2))
        self.proj_k = nn.ModuleList(nn.Linear(hidden_dim, hidden_dim) for _ in range(2))
        self.proj_v = nn.ModuleList(nn.Linear(hidden_dim, hidden_dim) for _ in range(2))
        self.proj = nn.ModuleList(nn.Linear(hidden_dim, hidden_dim) for _ in range(2))
        self.norm1 = nn.LayerNorm(hidden_dim)
        self.norm2 = nn.ModuleList(nn.LayerNorm(hidden_dim) for _ in range(2))
        self.score_token = nn.Parameter(torch.zeros(1, 1, hidden_dim))


# ----------------------------------------------------------------------------- HIP-backed models
class _HipTracker(nn.Module):
    """Common forward: prepares mmt_amd.runtime from this module's parameters, runs the plan
    (inference); in train() mode under autograd, mmt_amd.train.module_forward."""

    variant = None
    train_ops = None  # None = mmt_amd.train.HipOps (the product); tests on CPU inject a stand-in
    drop_path_rate = 0.1  # the backbone's stochastic depth in training (mixformer.py:311, :324)

    def __init__(self, head_type="CORNER_UP"):
        super().__init__()
        self.head_type = head_type
        self._rt = None
        self._online_batch = None
        self.compute_dtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "f16": torch.float16}.get(
            os.environ.get("MMT_DTYPE", "bf16"), torch.float32)
        self.use_hip_graph = True
        self.register_load_state_dict_post_hook(lambda m, keys: m.refresh_kernels())

    def refresh_kernels(self):
        self._rt = None
        self._online_batch = None

    def set_compute_dtype(self, dtype):
        self.compute_dtype = dtype
        self.refresh_kernels()
        return self

    def _apply(self, fn, *args, **kwargs):
        self._rt = None
        self._online_batch = None
        return super()._apply(fn, *args, **kwargs)

    def _runtime(self, device):
        if self._rt is None:
            from .runtime import MixFormerRGBTRuntime
            sd = self.state_dict()
            with torch.cuda.device(device):
                self._rt = MixFormerRGBTRuntime(sd, self.variant, dtype=self.compute_dtype, device=device)
        return self._rt

    def forward(self, template, online_template, search, run_score_head=False, gt_bboxes=None, return_features=False):
        for nm, x in (("template", template), ("online_template", online_template), ("search", search)):
            if not isinstance(x, (list, tuple)) or len(x) != 2:
                raise ValueError("%s must be a list [rgb, tir] of (B,3,H,W) tensors" % nm)
        dev = search[0].device
        if self.training and torch.is_grad_enabled():
            # training (the reference actor, DDP + SyncBN wrap this module unchanged): autograd over
            # the HIP ops of mmt_amd.train; `train_ops` may be replaced only by test stand-ins
            from .train import HipOps, module_forward
            ops = self.train_ops or HipOps
            if ops is HipOps and dev.type != "cuda":
                raise RuntimeError("the MI355X forward needs the inputs on the HIP device (got %s); there is no CPU path"
                                   % dev)
            return module_forward(self, template, online_template, search, ops, run_score_head=run_score_head,
                                  gt_bboxes=gt_bboxes)
        if dev.type != "cuda":
            raise RuntimeError("the MI355X forward needs the inputs on the HIP device (got %s); there is no CPU path" % dev)
        rt = self._runtime(dev)
        # gt_bboxes is accepted and ignored, as in the reference: asymmetric_shared_online.py:374 calls
        # forward_head(search, template, run_score_head) without it, so the score head always pools the
        # predicted box (pooling given boxes is the runtime's separate score_on_boxes API)
        score = bool(run_score_head) and self.variant == "asym_online"
        with torch.cuda.device(dev):
            box, sc = rt.forward(template, online_template, search, run_score_head=score,
                                 use_graph=self.use_hip_graph, ce_template_mask=getattr(self, "_mask", None))
            B = box.shape[0]
            coord = box.clone().view(B, 1, 4)
            out = {"pred_boxes": coord}
            if score:
                out["pred_scores"] = sc.clone()
            if not return_features:
                return out, coord
            ws = rt.workspace(B)
            d = rt.d
            # backbone output rows (candidate elimination: the recovered rows the fusion reads)
            X = ws.get("XOUT", ws["X"]).view(2, B, d.ntok, d.C)[:, :, d.n_t:].float()
            feats = X.permute(0, 1, 3, 2).reshape(2, B, d.C, d.gs, d.gs).clone()
            fused = ws["FUS"].view(B, d.ns, d.C).permute(0, 2, 1).reshape(B, d.C, d.gs, d.gs).clone()
            return out, coord, feats[0], feats[1], fused

    # ------------------------------------------------------------------ template K/V cache
    # The RGB MixFormer's online API (lib/models/mixformer_vit/mixformer.py:308-323: set_online
    # caches the template tokens' qkv in every block, forward_test runs only the search tokens),
    # defined for the RGB-T models whose own versions are broken (reference defect D2).  Both
    # take [rgb, tir] lists; the result equals forward() on the same template / search.
    def set_online(self, template, online_template):
        for nm, x in (("template", template), ("online_template", online_template)):
            if not isinstance(x, (list, tuple)) or len(x) != 2:
                raise ValueError("%s must be a list [rgb, tir] of (B,3,H,W) tensors" % nm)
        dev = template[0].device
        if dev.type != "cuda":
            raise RuntimeError("the MI355X forward needs the inputs on the HIP device (got %s); there is no CPU path" % dev)
        rt = self._runtime(dev)
        with torch.cuda.device(dev):
            rt.set_template(template, online_template)
        self._online_batch = template[0].shape[0]

    def forward_test(self, search, run_score_head=False, gt_bboxes=None):
        if not isinstance(search, (list, tuple)) or len(search) != 2:
            raise ValueError("search must be a list [rgb, tir] of (B,3,H,W) tensors")
        if getattr(self, "_online_batch", None) != search[0].shape[0]:
            raise RuntimeError("forward_test needs set_online() with the same batch size first")
        dev = search[0].device
        rt = self._runtime(dev)
        score = bool(run_score_head) and self.variant == "asym_online"
        with torch.cuda.device(dev):
            box, sc = rt.forward_search(search, run_score_head=score)
            coord = box.clone().view(-1, 1, 4)
            out = {"pred_boxes": coord}
            if score:
                out["pred_scores"] = sc.clone()
            return out, coord


class MixFormer_RGBT(_HipTracker):
    """Two-stream model (mixformer.py:352-432)."""

    variant = "rgbt"

    def __init__(self, backbone, box_head, fusion_vi, head_type="CORNER_UP"):
        super().__init__(head_type)
        self.backbone_v = backbone[0]
        self.backbone_i = backbone[1]
        self.fusion_vi = fusion_vi
        self.box_head = box_head


class MixFormer_RGBT_Shared(_HipTracker):
    """Shared backbone with per-modality LNs (mixformer_shared.py:386-424)."""

    variant = "shared"

    def __init__(self, backbone, box_head, fusion_vi, head_type="CORNER_UP"):
        super().__init__(head_type)
        self.backbone = backbone
        self.fusion_vi = fusion_vi
        self.box_head = box_head


class MixFormer_RGBT_Asymmetric(MixFormer_RGBT_Shared):
    """Cross-modal asymmetric MAM (asymmetric_shared.py:336-368)."""

    variant = "asym"


class MixFormer_RGBT_CE(MixFormer_RGBT_Shared):
    """Asymmetric model with candidate elimination (asymmetric_shared_ce.py:543-608): the search
    tokens are pruned to ceil(keep * n) after the attention of the CE_LOC blocks (by the template
    queries' mean attention) and restored as zero tokens after the last block.  Same parameters as
    the asymmetric model."""

    variant = "asym_ce"

    def __init__(self, backbone, box_head, fusion_vi, head_type="CORNER_UP", ce_loc=(3, 6, 9),
                 ce_keep_ratio=(0.7, 0.7, 0.7)):
        super().__init__(backbone, box_head, fusion_vi, head_type)
        if len(ce_loc) != len(ce_keep_ratio):
            raise ValueError("CE_LOC and CE_KEEP_RATIO differ in length")
        self.ce_loc, self.ce_keep_ratio = tuple(int(i) for i in ce_loc), tuple(float(r) for r in ce_keep_ratio)

    def _runtime(self, device):
        if self._rt is None:
            from .runtime import MixFormerRGBTRuntime
            keep = self.ce_keep_ratio if self._keep_override is None else (self._keep_override,) * len(self.ce_loc)
            with torch.cuda.device(device):
                self._rt = MixFormerRGBTRuntime(self.state_dict(), self.variant, dtype=self.compute_dtype,
                                                device=device, ce=(self.ce_loc, keep), ce_mask_count=self._mask_count)
        return self._rt

    _keep_override = None
    _mask_count = None  # template queries per frame the CE mean averages (None: all of them)
    _mask = None

    def forward(self, template, online_template, search, run_score_head=False, gt_bboxes=None, ce_template_mask=None,
                ce_keep_rate=None, return_features=False):
        """asymmetric_shared_ce.py:557-587 signature.  ce_keep_rate (the actor's keep-rate schedule,
        actors/mixformer_rgbt.py:70-89) replaces every CE layer's keep ratio; >= 1 disables the
        elimination (asymmetric_shared_ce.py:249-252).  ce_template_mask: None (the tracker) or the
        (B, 2 n_t) bool mask of generate_mask_cond (lib/utils/ce_utils.py:14-38; CTR_POINT selects
        the centre token of each of the four 8x8 templates) that the training actor passes
        (actors/mixformer_rgbt.py:67-90): the elimination then averages the template->search attention
        over the masked template queries only (candidate_elimination :81-89).  As in the reference
        (attn[mask].view(bs, hn, -1, ...)) every frame must select the same number of queries."""
        if self.training and torch.is_grad_enabled():
            raise NotImplementedError("training forward of asymmetric_shared_ce (candidate elimination with autograd) "
                                      "is not built; its inference forward runs under eval() / no_grad()")
        count = None
        if ce_template_mask is not None:
            m = torch.as_tensor(ce_template_mask).to(torch.bool)
            B, n_q = search[0].shape[0], 2 * self.backbone.pos_embed_t.shape[1] * 2
            if tuple(m.shape) != (B, n_q):
                raise ValueError("ce_template_mask shape %s, expected (%d, %d) (template queries [q_mt_V ; q_mt_I])"
                                 % (tuple(m.shape), B, n_q))
            counts = m.sum(1).cpu()
            if not bool((counts == counts[0]).all()) or int(counts[0]) == 0:
                raise ValueError("ce_template_mask must select the same nonzero number of template queries in every "
                                 "frame (the reference views attn[mask] as (bs, heads, -1, L))")
            count = None if int(counts[0]) == n_q else int(counts[0])  # all selected == no mask
            if count is not None:
                ce_template_mask = m
        rate = None if ce_keep_rate is None else float(ce_keep_rate)
        if rate != self._keep_override or count != self._mask_count:
            self._keep_override = rate
            self._mask_count = count
            self.refresh_kernels()
        self._mask = ce_template_mask if count is not None else None
        try:
            return super().forward(template, online_template, search, run_score_head=run_score_head,
                                   gt_bboxes=gt_bboxes, return_features=return_features)
        finally:
            self._mask = None

    def set_online(self, template, online_template):
        raise NotImplementedError("the template K/V cache is not defined for candidate elimination")


class MixFormer_RGBT_OnlineScore(_HipTracker):
    """Asymmetric model + score prediction module (asymmetric_shared_online.py:337-413)."""

    variant = "asym_online"

    def __init__(self, backbone, box_head, fusion_vi, score_branch, head_type="CORNER_UP"):
        super().__init__(head_type)
        self.backbone = backbone
        self.fusion_vi = fusion_vi
        self.box_head = box_head
        self.score_branch = score_branch


class MixFormer(_HipTracker):
    """RGB-only MixFormer (lib/models/mixformer_vit/mixformer.py:285-337; BASELINE config 1): one ViT
    with the same MAM, the corner head straight on its search tokens, no fusion.  forward takes
    single (B,3,H,W) tensors (5-D inputs squeezed, :296-301) and returns ({"pred_boxes"}, coord);
    set_online / forward_test are the reference's template-cache API (:308-321)."""

    variant = "rgb"

    def __init__(self, backbone, box_head, head_type="CORNER_UP"):
        super().__init__(head_type)
        self.backbone = backbone
        self.box_head = box_head
        # 16-bit default fp16, not bf16: without the fusion between backbone and head this model's
        # boxes move 2.7e-2 from the reference's in bf16 and 1.8e-3 in fp16 on the golden inputs, at
        # the same speed (profiles/r02_head_dtype_ab.jsonl); MMT_DTYPE / set_compute_dtype override
        if "MMT_DTYPE" not in os.environ:
            self.compute_dtype = torch.float16

    @staticmethod
    def _one(x, nm):
        if isinstance(x, (list, tuple)):
            raise ValueError("%s: the RGB-only MixFormer takes a (B,3,H,W) tensor, not a list" % nm)
        return x.squeeze(0) if x.dim() == 5 else x

    def _device(self, x):
        if x.device.type != "cuda":
            raise RuntimeError("the MI355X forward needs the inputs on the HIP device (got %s); there is no CPU path"
                               % x.device)
        return x.device

    def forward(self, template, online_template, search, run_score_head=False, gt_bboxes=None):
        t, o, s = self._one(template, "template"), self._one(online_template, "online_template"), self._one(search, "search")
        if self.training and torch.is_grad_enabled():
            raise NotImplementedError("training the RGB-only MixFormer is outside the RGB-T hot path (inference only)")
        dev = self._device(s)
        rt = self._runtime(dev)
        with torch.cuda.device(dev):
            box, _ = rt.forward([t], [o], [s], use_graph=self.use_hip_graph)
            coord = box.clone().view(box.shape[0], 1, 4)
        return {"pred_boxes": coord}, coord

    def set_online(self, template, online_template):
        t, o = self._one(template, "template"), self._one(online_template, "online_template")
        dev = self._device(t)
        rt = self._runtime(dev)
        with torch.cuda.device(dev):
            rt.set_template([t], [o])
        self._online_batch = t.shape[0]

    def forward_test(self, search, run_score_head=True, gt_bboxes=None):
        s = self._one(search, "search")
        if self._online_batch != s.shape[0]:
            raise RuntimeError("forward_test needs set_online() with the same batch size first")
        dev = self._device(s)
        rt = self._runtime(dev)
        with torch.cuda.device(dev):
            box, _ = rt.forward_search([s])
            coord = box.clone().view(-1, 1, 4)
        return {"pred_boxes": coord}, coord



# ----------------------------------------------------------------------------- builders
def _vit_spec(cfg):
    if cfg.MODEL.VIT_TYPE == "large_patch16":
        return 1024, 24, 16
    if cfg.MODEL.VIT_TYPE == "base_patch16":
        return 768, 12, 12
    raise KeyError("VIT_TYPE shoule set to 'large_patch16' or 'base_patch16'")


def _check_cfg(cfg):
    if cfg.MODEL.FUSION_CLASS != "Attention_Fusion_Bimodal_LNSpecific":
        raise NotImplementedError("FUSION_CLASS %r: only Attention_Fusion_Bimodal_LNSpecific (the hot path) is "
                                  "implemented on MI355X" % cfg.MODEL.FUSION_CLASS)
    if cfg.MODEL.HEAD_TYPE != "CORNER_UP":
        raise NotImplementedError("HEAD_TYPE %r: only CORNER_UP is implemented on MI355X" % cfg.MODEL.HEAD_TYPE)


def _backbone(cfg, shared):
    dim, depth, heads = _vit_spec(cfg)
    vit = VisionTransformer(cfg.DATA.SEARCH.SIZE, cfg.DATA.TEMPLATE.SIZE, dim, depth, heads, shared)
    return vit


def _head(cfg):
    channel = getattr(cfg.MODEL, "HEAD_DIM", 384)
    freeze_bn = getattr(cfg.MODEL, "HEAD_FREEZE_BN", False)
    return Pyramid_Corner_Predictor(cfg.MODEL.HIDDEN_DIM, channel, int(cfg.DATA.SEARCH.SIZE / 4), 4, freeze_bn)


def _fusion(cfg):
    return Attention_Fusion_Bimodal_LNSpecific(cfg.MODEL.HIDDEN_DIM, 512, 2, cfg.MODEL.FUSION_LAYERS)


def _load_checkpoint(path, key):
    ck = torch.load(path, map_location="cpu", weights_only=True)
    return ck[key] if key in ck else ck


def _load_mae(vit, cfg, shared):
    """MAE backbone init (mixformer.py:335-347 / mixformer_shared.py:358-382)."""
    if not (cfg.MODEL.BACKBONE.PRETRAINED and cfg.MODEL.BACKBONE.PRETRAINED_PATH):
        return
    new = {}
    for k, v in _load_checkpoint(cfg.MODEL.BACKBONE.PRETRAINED_PATH, "model").items():
        if "pos_embed" in k or "mask_token" in k:
            continue
        if shared and ("norm1" in k or "norm2" in k) and k.startswith("blocks."):
            n = "norm1" if "norm1" in k else "norm2"
            new[k.replace(n, n + "_v")] = v
            new[k.replace(n, n + "_i")] = v
        else:
            new[k] = v
    vit.load_state_dict(new, strict=False)


def _load_rgb_tracker(model, path, two_stream):
    """RGB MixFormer checkpoint duplicated into both modalities (mixformer.py:449-468,
    mixformer_shared.py:479-506)."""
    new = {}
    for k, v in _load_checkpoint(path, "net").items():
        if "pos_embed" in k or "mask_token" in k:
            continue
        if "backbone" in k:
            if two_stream:
                new[k.replace("backbone", "backbone_v")] = v
                new[k.replace("backbone", "backbone_i")] = v
            elif "norm1" in k or "norm2" in k:
                n = "norm1" if "norm1" in k else "norm2"
                new[k.replace(n, n + "_v")] = v
                new[k.replace(n, n + "_i")] = v
            else:
                new[k] = v
        else:
            new[k] = v
    model.load_state_dict(new, strict=False)


def build_mixformer_vit_rgbt(cfg, train=True):
    _check_cfg(cfg)
    bv, bi = _backbone(cfg, False), _backbone(cfg, False)
    if train:
        _load_mae(bv, cfg, False)
        _load_mae(bi, cfg, False)
    model = MixFormer_RGBT([bv, bi], _head(cfg), _fusion(cfg), cfg.MODEL.HEAD_TYPE)
    if train and getattr(cfg.MODEL, "RGBT_PRETRAINED_PATH", ""):
        _load_rgb_tracker(model, cfg.MODEL.RGBT_PRETRAINED_PATH, True)
    return model


def build_mixformer_vit_rgbt_shared(cfg, train=True):
    _check_cfg(cfg)
    bb = _backbone(cfg, True)
    if train:
        _load_mae(bb, cfg, True)
    model = MixFormer_RGBT_Shared(bb, _head(cfg), _fusion(cfg), cfg.MODEL.HEAD_TYPE)
    if train and getattr(cfg.MODEL, "RGBT_PRETRAINED_PATH", ""):
        _load_rgb_tracker(model, cfg.MODEL.RGBT_PRETRAINED_PATH, False)
    return model


def build_asymmetric_shared(cfg, train=True):
    _check_cfg(cfg)
    bb = _backbone(cfg, True)
    if train:
        _load_mae(bb, cfg, True)
    model = MixFormer_RGBT_Asymmetric(bb, _head(cfg), _fusion(cfg), cfg.MODEL.HEAD_TYPE)
    if train and getattr(cfg.MODEL, "RGBT_PRETRAINED_PATH", ""):
        _load_rgb_tracker(model, cfg.MODEL.RGBT_PRETRAINED_PATH, False)
    return model


def build_asymmetric_shared_online_score(cfg, train=True):
    _check_cfg(cfg)
    bb = _backbone(cfg, True)
    if train:
        _load_mae(bb, cfg, True)
    sb = ScoreDecoder(pool_size=4, hidden_dim=cfg.MODEL.HIDDEN_DIM, num_heads=cfg.MODEL.HIDDEN_DIM // 64)
    model = MixFormer_RGBT_OnlineScore(bb, _head(cfg), _fusion(cfg), sb, cfg.MODEL.HEAD_TYPE)
    if train:
        for key in ("SCORE_PRETRAINED_PATH", "TRACKER_PRETRAINED_PATH"):
            path = getattr(cfg.MODEL, key, "")
            if path:
                model.load_state_dict(_load_checkpoint(path, "net"), strict=False)
    return model


def build_asymmetric_shared_ce(cfg, train=True):
    """build_asymmetric_shared_ce (asymmetric_shared_ce.py:611-675); MODEL.BACKBONE.CE_LOC /
    CE_KEEP_RATIO as lib/config/asymmetric_shared_ce/config.py:23-24."""
    _check_cfg(cfg)
    bb = _backbone(cfg, True)
    if train:
        _load_mae(bb, cfg, True)
    ce_loc = getattr(cfg.MODEL.BACKBONE, "CE_LOC", None) or (3, 6, 9)
    ce_keep = getattr(cfg.MODEL.BACKBONE, "CE_KEEP_RATIO", None) or (0.7, 0.7, 0.7)
    model = MixFormer_RGBT_CE(bb, _head(cfg), _fusion(cfg), cfg.MODEL.HEAD_TYPE, ce_loc, ce_keep)
    if train and getattr(cfg.MODEL, "RGBT_PRETRAINED_PATH", ""):
        _load_rgb_tracker(model, cfg.MODEL.RGBT_PRETRAINED_PATH, False)
    return model


def build_mixformer_vit(cfg, train=True):
    """build_mixformer_vit (lib/models/mixformer_vit/mixformer.py:341-366): RGB-only MixViT with the
    CORNER_UP head (experiments/mixformer_vit/baseline.yaml); MODEL.RGB_PRETRAINED_PATH as there."""
    if cfg.MODEL.HEAD_TYPE != "CORNER_UP":
        raise NotImplementedError("HEAD_TYPE %r: only CORNER_UP is implemented on MI355X" % cfg.MODEL.HEAD_TYPE)
    bb = _backbone(cfg, False)
    if train:
        _load_mae(bb, cfg, False)
    model = MixFormer(bb, _head(cfg), cfg.MODEL.HEAD_TYPE)
    path = getattr(cfg.MODEL, "RGB_PRETRAINED_PATH", "")
    if train and path:
        model.load_state_dict({k: v for k, v in _load_checkpoint(path, "net").items()
                               if "pos_embed" not in k and "mask_token" not in k}, strict=False)
    return model


BUILDERS = {"rgbt": build_mixformer_vit_rgbt, "shared": build_mixformer_vit_rgbt_shared,
            "asym": build_asymmetric_shared, "asym_online": build_asymmetric_shared_online_score,
            "asym_ce": build_asymmetric_shared_ce, "rgb": build_mixformer_vit}


def hot_path_cfg(vit="base_patch16", search=320, template=128, fusion_layers=2, hidden=None):
    """Config of BASELINE.json configs 2-5 (experiments/mixformer_vit_rgbt/attention_lasher_newfusion_2layer.yaml
    with the search size overridden)."""
    from .config import default_cfg
    cfg = default_cfg("asymmetric_shared_online")
    cfg.MODEL.VIT_TYPE = vit
    cfg.MODEL.HIDDEN_DIM = hidden or (1024 if vit == "large_patch16" else 768)
    cfg.MODEL.HEAD_TYPE = "CORNER_UP"
    cfg.MODEL.FUSION_CLASS = "Attention_Fusion_Bimodal_LNSpecific"
    cfg.MODEL.FUSION_LAYERS = fusion_layers
    cfg.MODEL.BACKBONE.PRETRAINED = False
    cfg.MODEL.RGBT_PRETRAINED_PATH = ""
    cfg.DATA.SEARCH.SIZE = cfg.TEST.SEARCH_SIZE = search
    cfg.DATA.TEMPLATE.SIZE = cfg.TEST.TEMPLATE_SIZE = template
    return cfg


def reference_state_dict_shapes(variant, hidden=768, depth=12, search=320, template=128, fusion_layers=2):
    """(name, shape) of the reference state_dict, built on the meta device (no memory)."""
    vit = {768: "base_patch16", 1024: "large_patch16"}[hidden]
    cfg = hot_path_cfg(vit, search, template, fusion_layers)
    with torch.device("meta"):
        m = BUILDERS[variant](cfg, train=False)
    return [(k, list(v.shape)) for k, v in m.state_dict().items()]
