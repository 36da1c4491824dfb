"""Training step of the two-stream MixFormer RGB-T tracker on the MI355X (BASELINE
config 4): forward with autograd, the reference's box loss, backward, data-parallel gradient
all-reduce over RCCL (DistributedDataParallel) and the AdamW update with the reference's parameter
groups and gradient clipping.

Reference: lib/train/train_script_mixformer.py:105-140 (DDP, SyncBN, MixFormerRGBTActor),
lib/train/actors/mixformer_rgbt.py:33-168 (forward pass, CIoU + L1 loss on xyxy boxes),
lib/utils/box_ops.py:100-152 (ciou_loss), lib/train/base_functions.py:362-400 (rgbt strategy:
parameter groups with per-group lr multipliers, pos_embed frozen), lib/train/trainers/
ltr_trainer.py (clip_grad_norm_ with TRAIN.GRAD_CLIP_NORM).

What runs where.  The ViT backbones (≈ 85 % of the step's FLOPs) run on libmmt_hip.so through two
autograd Functions: every Linear (patch embed as a GEMM on the unfolded patches, qkv, proj, fc1,
fc2) forward and backward on the LDS-DMA bf16 GEMM (dX = dY W and dW = dY^T X after bf16
transposes, fp32 accumulation, fp32 master weights), and the MAM attention forward (throughput
kernel, log-sum-exp kept) and backward (mmt_mam_attention_bwd).  The fusion encoder's Linears
(value / offset / weight / output projections, FFN) take the same GEMM op, and its deformable
sampling runs on mmt_ms_deform_attn_forward / _backward (mmt_amd.functional.MSDeformAttnFunction,
the reference's MSDeformAttnFunction).  Clipping + AdamW is mmt_adamw_step (mmt_amd.optim.HipAdamW,
three launches over every parameter, writing the bf16 copies of the backbone weights the GEMMs
read).  The backbone LayerNorms run on mmt_layernorm / mmt_layernorm_bwd (_HipLayerNorm), and each
block's MLP is one autograd Function whose GELU and GELU backward live in GEMM epilogues (_HipMlp); the
fusion encoder's LayerNorms take the same kernels, and the fusion's adjust_* 1x1 convs + GroupNorms run on
token rows as the HIP GEMM + mmt_groupnorm / mmt_groupnorm_bwd.  The residual adds and the corner head run as
PyTorch-ROCm ops on the same
module tree (`nn.Conv2d`, `nn.GroupNorm`, `SyncBatchNorm` under DDP), in bf16 autocast like the
reference's AMP path.  The backbone ops are injected (`ops`), so the data-parallel plumbing can be exercised on CPU
with stand-in ops in tests; the product's ops are `HipOps` and have no CPU path.
"""
import math
import time

import torch
import torch.nn.functional as F

from .model import FrozenBatchNorm2d

LOG2E = 1.4426950408889634


# ----------------------------------------------------------------------------- HIP backbone ops
_CONSTS = {}


def _const(key, device, make):
    """Small constant tensors built on the host once per device and reused (no host-to-device copy
    inside a step, so the step can be captured in a hipGraph)."""
    k = key + (str(device),)
    if k not in _CONSTS:
        v = make()
        _CONSTS[k] = tuple(t.to(device) for t in v) if isinstance(v, tuple) else v.to(device)
    return _CONSTS[k]


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _transpose(x, rows, cols, ld_out=None, ones_row=False):
    """[rows][cols] bf16 -> [cols][ld_out] (mmt_transpose_bf16); columns rows..ld_out-1 are zero
    (the GEMM's K must be a multiple of 8).  ones_row: 8 more rows, the first all ones over the
    `rows` columns (so a GEMM against it also yields the row sums of its other operand), the rest zero."""
    from ._lib import LIB, check
    ld_out = ld_out or rows
    out = torch.empty(cols + (8 if ones_row else 0), ld_out, device=x.device, dtype=torch.bfloat16)
    # the kernel writes the padding columns and the ones-row block itself (fill 1 / 2): one launch
    fill = 2 if ones_row else (1 if ld_out > rows else 0)
    check(LIB.mmt_transpose_bf16(x.data_ptr(), out.data_ptr(), rows, cols, cols, ld_out, 1, 0, 0, fill, _stream()),
          "mmt_transpose_bf16")
    return out


# The Linear backward reads dY, X and W as they are (MN-major GEMM operands, ds_read_b64_tr_b16) instead
# of transposed copies; False: the transposing form (A/B knob, tools/train_ab.py)
MN_MAJOR = True
# The two-stream backbones in lockstep with grouped GEMMs (backbone_forward_pair); False: one after the
# other (A/B knob, tools/train_ab.py)
PAIR = True
_SPLITK = {}  # device -> (slab workspace, arrival tickets) of the dW GEMMs' split-K (stream-ordered: one set)


def _splitk_ws(dev):
    """The split-K workspace of the current stream (GEMMs on one stream run one after another, so one slab and one
    ticket array per stream; the backward's side stream has its own)."""
    key = (str(dev), torch.cuda.current_stream(dev).cuda_stream)
    ws = _SPLITK.get(key)
    if ws is None:
        ws = _SPLITK[key] = (torch.empty(32 << 20, device=dev, dtype=torch.float32),
                             torch.zeros(1 << 16, device=dev, dtype=torch.int32))
    return ws


# The pair backward's weight-gradient GEMMs on a side stream, beside the input-gradient GEMMs on the main stream
# (round 6): the two are independent, so the second fills the CUs the first leaves idle in its last round of tiles
# (the N = 768 GEMMs of the backbone run 1.55 rounds of 512 tile slots).  Measured no faster in an interleaved A/B
# (tools/train_ab.py --only hip,single_stream: 569-576 dual vs 574-580 single samples/s, profiles/r06aa_train_ab.jsonl),
# so off: an A/B knob.
DUAL_STREAM = False
_SIDE = {}


def _side_stream(dev):
    s = _SIDE.get(str(dev))
    if s is None:
        s = _SIDE[str(dev)] = torch.cuda.Stream(device=dev)
    return s


# Per-step GEMM accounting for bench.py's train_step.roofline: None, or a dict that every GEMM launch of the
# step adds to while it is set (one eager step: "flops" = 2 M N K per group, "bytes" = the launch's algorithmic
# HBM bytes -- each operand read once, the output written once, bias / residual / second output included --
# and "launches").  Host-side bookkeeping only; the launches themselves are unchanged.
GEMM_ACCOUNT = None


def _account(M, N, K, G, a_bytes, w_bytes, c_bytes, extra_bytes=0):
    acc = GEMM_ACCOUNT
    if acc is not None:
        acc["flops"] = acc.get("flops", 0.0) + 2.0 * M * N * K * G
        acc["bytes"] = acc.get("bytes", 0.0) + G * (M * K * a_bytes + N * K * w_bytes + M * N * c_bytes) + extra_bytes
        acc["launches"] = acc.get("launches", 0) + 1


def _gemm(a, w, M, N, K, bias=None, out_f32=False, act=0, r=None, c2=None, c2_copy=0, c=None, ldc=None, a_t=0,
          w_t=0, ldw=0, lda=None, splitk=False, impl=0, row_scale=None, row_scale_div=1, nsk=0):
    """C[M][N] = A[M][K] W[N][K]^T (+ bias), bf16 operands, fp32 accumulation (mmt_gemm); act / r (bf16,
    [M][N]) / c2 / c2_copy as mmt_gemm_params (act 1 GELU, 5 GELU backward against r; c2_copy 2: c2 = the
    pre-activation; 3: the last 8 columns to c2 [M][8]; 4: column N - 8 alone to c2 [M]); c / ldc: a
    preallocated output and its pitch;
    a_t / w_t / ldw / lda: MN-major operands (A^T [K][lda], W^T [K][ldw]); splitk: with a split-K
    workspace (the cost model may split K over workgroups; nsk >= 1 forces the slice count, A/B tools).
    Grouped form (the two-stream backbones in lockstep): a and w (and bias / r / c2 / c) tuples, one entry
    per group, one launch; without c the output is one [groups * M][N] tensor, group g on rows g M ..."""
    from ._lib import LIB, GemmParams, MMT_BF16, check
    grouped = isinstance(a, tuple)
    A, W = (a, w) if grouped else ((a,), (w,))
    G = len(A)
    if c is None:
        c = torch.empty(G * M, N, device=A[0].device, dtype=torch.float32 if out_f32 else torch.bfloat16)
        cs = c.split(M) if grouped else (c,)
    else:
        cs = c if grouped else (c,)
    bs = bias if grouped else (bias,)
    p = GemmParams()
    for g in range(G):
        p.a[g], p.w[g], p.c[g] = A[g].data_ptr(), W[g].data_ptr(), cs[g].data_ptr()
        p.bias[g] = bs[g].data_ptr() if bs is not None and bs[g] is not None else None
    p.lda, p.ldc = lda or K, ldc or N
    p.a_t, p.w_t, p.ldw, p.impl = a_t, w_t, ldw, impl
    if splitk:
        ws, cnt = _splitk_ws(A[0].device)
        p.sk_ws, p.sk_ws_floats, p.sk_cnt, p.sk_cnt_n = ws.data_ptr(), ws.numel(), cnt.data_ptr(), cnt.numel()
        p.splitk = nsk
    p.a_seg_rows, p.a_segs_a = M, 1
    p.M, p.N, p.K, p.groups, p.c_f32 = M, N, K, G, 1 if out_f32 else 0
    p.act = act
    if r is not None:  # bf16 (act 5's pre-activation) or the fp32 residual stream
        rs = r if grouped else (r,)
        for g in range(G):
            p.r[g] = rs[g].data_ptr()
        p.ldr, p.r_t = N, 0 if rs[0].dtype == torch.float32 else 1
    if row_scale is not None:  # one per-row scale vector, indexed by the row within a group
        if G > 1:
            raise ValueError("row_scale with grouped operands")
        p.row_scale, p.row_scale_div = row_scale.data_ptr(), row_scale_div
    if c2 is not None:
        for g, t in enumerate(c2 if grouped else (c2,)):
            p.c2[g] = t.data_ptr()
        p.c2_copy = c2_copy
    check(LIB.mmt_gemm(p, MMT_BF16, _stream()), "mmt_gemm")
    if GEMM_ACCOUNT is not None:
        extra = G * N * 4 if bias is not None else 0
        if r is not None:
            extra += G * M * N * (r if not grouped else r[0]).element_size()
        if c2 is not None:
            t2 = c2 if not grouped else c2[0]
            extra += G * t2.numel() * t2.element_size()
        _account(M, N, K, G, 2, 2, 4 if out_f32 else 2, extra)
    return c


def _bf16_weight(w):
    """The bf16 copy of an fp32 master weight HipAdamW's update wrote (same values), else a fresh cast."""
    sh = getattr(w, "_mmt_bf16", None)
    if sh is None and w._base is not None:  # a reshaped conv weight (patch embed, 1x1 adjust convs)
        sh = getattr(w._base, "_mmt_bf16", None)
    if sh is not None and sh[1] == w._version and sh[0].numel() == w.numel():
        return sh[0].view(w.shape)
    return w.detach().to(torch.bfloat16).contiguous()


def _weight_grads(dy, x, M, N, K):
    """dW [N][K] and db [N] of y = x W^T + b from one GEMM: dy^T [x | 1] (a row of ones appended to the
    transposed activations gives the bias gradient as output column K; fp32 accumulation).  The GEMM
    writes dW contiguous and the bias column alone as a contiguous [N] vector behind it (c2_copy 4), so
    autograd takes both as the parameters' .grad as they are (round 5: a strided db column was cloned by
    AccumulateGrad, ~100 small copy launches per training step)."""
    buf = torch.empty(N * (K + 1), device=dy.device, dtype=torch.float32)
    dw, db = buf[:N * K].view(N, K), buf[N * K:]
    if MN_MAJOR and M % 8 == 0:  # dY [M][N] and X [M][K] read as they are (a_t, w_t 2: the ones column)
        _gemm(dy, x, N, K + 8, M, out_f32=True, c=dw, ldc=K, c2=db, c2_copy=4, a_t=1, w_t=2, ldw=K, lda=N,
              splitk=True)
        return dw, db
    Mp = (M + 7) // 8 * 8  # contraction over tokens, zero-padded to the GEMM's K granule
    _gemm(_transpose(dy, M, N, Mp), _transpose(x, M, K, Mp, ones_row=True), N, K + 8, Mp, out_f32=True,
          c=dw, ldc=K, c2=db, c2_copy=4)
    return dw, db


def _dx(dy, wb, M, N, K, act=0, r=None):
    """dX [M][K] = dY [M][N] W [N][K] (bf16 out; act 5: times GELU'(r))."""
    if MN_MAJOR:  # W read MN-major as it is
        return _gemm(dy, wb, M, K, N, act=act, r=r, w_t=1, ldw=K)
    return _gemm(dy, _transpose(wb, N, K), M, K, N, act=act, r=r)


class _HipLinear(torch.autograd.Function):
    """y = x W^T + b (nn.Linear) with bf16 operands; x [M][K] bf16, W [N][K] fp32 master, b [N]; y bf16,
    or fp32 straight from the GEMM's accumulators (out_f32: the residual-stream adds, no cast pass)."""

    @staticmethod
    def forward(ctx, x, w, b, out_f32=False):
        M, K = x.shape
        N = w.shape[0]
        x = x.contiguous()
        wb = _bf16_weight(w)  # bf16 shadow written by HipAdamW's update (same values)
        y = _gemm(x, wb, M, N, K, bias=b.detach().float().contiguous(), out_f32=out_f32)
        ctx.save_for_backward(x, wb)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wb = ctx.saved_tensors
        M, K = x.shape
        N = wb.shape[0]
        dy = dy.to(torch.bfloat16).contiguous()
        dx = _dx(dy, wb, M, N, K) if ctx.needs_input_grad[0] else None
        # dW and the bias gradient from one GEMM: x^T carries an extra row of ones, so output column
        # K of dy^T [x | 1] is sum_m dy[m][n] (the same bf16 dy, fp32 accumulation; no reduce kernel)
        dw, db = _weight_grads(dy, x, M, N, K)
        return dx, dw, db, None


class _HipMlp(torch.autograd.Function):
    """timm Mlp of the ViT blocks (mixformer.py:136-139): y = fc2(GELU(fc1(x))) with x [M][C] bf16, y [M][C]
    fp32 (the residual branch).  fc1 runs with the GELU epilogue and also stores its pre-activation (bf16,
    c2_copy 2); the backward's dX GEMM of fc2 multiplies by GELU'(pre-activation) in its epilogue (act 5),
    so neither the activation nor its gradient is a separate pass."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        M, C = x.shape
        F4 = w1.shape[0]
        x = x.contiguous()
        wb1, wb2 = _bf16_weight(w1), _bf16_weight(w2)
        hp = torch.empty(M, F4, device=x.device, dtype=torch.bfloat16)
        h = _gemm(x, wb1, M, F4, C, bias=b1.detach(), act=1, c2=hp, c2_copy=2)
        y = _gemm(h, wb2, M, C, F4, bias=b2.detach(), out_f32=True)
        ctx.save_for_backward(x, wb1, wb2, h, hp)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wb1, wb2, h, hp = ctx.saved_tensors
        M, C = x.shape
        F4 = wb1.shape[0]
        dy = dy.to(torch.bfloat16).contiguous()
        dhp = _dx(dy, wb2, M, C, F4, act=5, r=hp)  # d(pre-activation), bf16
        dw2, db2 = _weight_grads(dy, h, M, C, F4)
        dx = _dx(dhp, wb1, M, F4, C) if ctx.needs_input_grad[0] else None
        dw1, db1 = _weight_grads(dhp, x, M, F4, C)
        return dx, dw1, db1, dw2, db2


def _scaled_bf16(dy, keep, rows_per):
    """keep[m // rows_per] * dy in bf16, one pass (the residual branch's gradient under stochastic depth)."""
    if keep is None:
        return dy.to(torch.bfloat16).contiguous()
    from ._lib import LIB, MMT_BF16, check
    dy = dy.float().contiguous()
    out = torch.empty(dy.shape, device=dy.device, dtype=torch.bfloat16)
    cols = dy.shape[-1]
    check(LIB.mmt_scale_rows_cast(dy.data_ptr(), keep.float().contiguous().data_ptr(), rows_per, out.data_ptr(),
                                  dy.numel() // cols, cols, MMT_BF16, _stream()), "mmt_scale_rows_cast")
    return out


class _HipLinearResidual(torch.autograd.Function):
    """x + keep * (a W^T + b) in one GEMM (fp32 residual stream x [M][N] as the epilogue's R, keep [B] the
    per-sample stochastic-depth scale over blocks of M / B rows as its row_scale, or None): the block's
    proj + DropPath + residual add (mixformer.py:136-137) without the addcmul pass; the backward hands
    the stream gradient through and scales + casts the branch gradient in one pass."""

    @staticmethod
    def forward(ctx, x, a, w, b, keep):
        M, K = a.shape
        N = w.shape[0]
        a = a.contiguous()
        wb = _bf16_weight(w)
        rows = M // keep.shape[0] if keep is not None else 1
        y = _gemm(a, wb, M, N, K, bias=b.detach(), out_f32=True, r=x.detach().reshape(M, N),
                  row_scale=keep, row_scale_div=rows)
        ctx.save_for_backward(a, wb, keep)
        ctx.rows = rows
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dout):
        a, wb, keep = ctx.saved_tensors
        M, K = a.shape
        N = wb.shape[0]
        dy = _scaled_bf16(dout.reshape(M, N), keep, ctx.rows)
        da = _dx(dy, wb, M, N, K) if ctx.needs_input_grad[1] else None
        dw, db = _weight_grads(dy, a, M, N, K)
        return dout, da, dw, db, None


class _HipMlpResidual(torch.autograd.Function):
    """x + keep * fc2(GELU(fc1(xn))) (the block's MLP branch + DropPath + residual, mixformer.py:138-139):
    _HipMlp with the residual add and the per-sample scale in fc2's epilogue."""

    @staticmethod
    def forward(ctx, x, xn, w1, b1, w2, b2, keep):
        M, C = xn.shape
        F4 = w1.shape[0]
        xn = xn.contiguous()
        wb1, wb2 = _bf16_weight(w1), _bf16_weight(w2)
        rows = M // keep.shape[0] if keep is not None else 1
        hp = torch.empty(M, F4, device=xn.device, dtype=torch.bfloat16)
        h = _gemm(xn, wb1, M, F4, C, bias=b1.detach(), act=1, c2=hp, c2_copy=2)
        y = _gemm(h, wb2, M, C, F4, bias=b2.detach(), out_f32=True, r=x.detach().reshape(M, C), row_scale=keep,
                  row_scale_div=rows)
        ctx.save_for_backward(xn, wb1, wb2, h, hp, keep)
        ctx.rows = rows
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dout):
        xn, wb1, wb2, h, hp, keep = ctx.saved_tensors
        M, C = xn.shape
        F4 = wb1.shape[0]
        dy = _scaled_bf16(dout.reshape(M, C), keep, ctx.rows)
        dhp = _dx(dy, wb2, M, C, F4, act=5, r=hp)
        dw2, db2 = _weight_grads(dy, h, M, C, F4)
        dxn = _dx(dhp, wb1, M, F4, C) if ctx.needs_input_grad[1] else None
        dw1, db1 = _weight_grads(dhp, xn, M, F4, C)
        return dout, dxn, dw1, db1, dw2, db2, None


# -- the two-stream backbones in lockstep: the RGB rows [0, M) and the TIR rows [M, 2M) of one stacked
# operand, each modality with its own weights, as one grouped GEMM (groups 2) per Linear and per gradient.
# One modality's dW GEMM (768-3080 output columns, K = the 8448 tokens of 16 pairs) is a 42-168 tile grid on
# 256 CUs; the pair fills the chip twice as well (tools/dw_split_ab.py: 250-425 TFLOP/s at one group, 390-595
# at two; the step 417 -> 462 samples/s, profiles/r04_train_pair_ab.jsonl).
class _Beside:
    """Runs work on the device's side stream beside the calling (main) stream: run(fn, ...) makes the side stream
    wait for everything issued on the main stream so far, then issues fn there; leaving the block makes the main
    stream wait for the side stream.  Every tensor the side work reads or writes must be allocated on the main
    stream and stay referenced until the block ends (so no block is recycled while the side stream uses it).
    Captured in a hipGraph as a fork / join.  With DUAL_STREAM False (or on the host) run() calls fn inline."""

    def __init__(self, dev):
        self.on = DUAL_STREAM and MN_MAJOR and torch.device(dev).type == "cuda"
        self.dev = dev

    def __enter__(self):
        if self.on:
            self.main, self.side = torch.cuda.current_stream(self.dev), _side_stream(self.dev)
        return self

    def run(self, fn, *a, **kw):
        if not self.on:
            return fn(*a, **kw)
        self.side.wait_stream(self.main)
        with torch.cuda.stream(self.side):
            return fn(*a, **kw)

    def __exit__(self, *exc):
        if self.on:
            self.main.wait_stream(self.side)
        return False


def _halves(t, M):
    return t[:M], t[M:]


def _wg2_bufs(dev, N, K):
    """The two modalities' [dW | db] buffers of _weight_grads2 (allocated on the calling stream)."""
    return [torch.empty(N * (K + 1), device=dev, dtype=torch.float32) for _ in range(2)]


def _weight_grads2(dy, x, M, N, K, bufs=None):
    """_weight_grads of both modalities (dy [2M][N], x [2M][K]) in one launch: ((dW, db) RGB, (dW, db) TIR).
    bufs: preallocated _wg2_bufs (the dual-stream backward allocates on the main stream)."""
    bufs = bufs if bufs is not None else _wg2_bufs(dy.device, N, K)
    dws = tuple(b[:N * K].view(N, K) for b in bufs)
    dbs = tuple(b[N * K:] for b in bufs)
    if not (MN_MAJOR and M % 8 == 0):
        return [_weight_grads(u, v, M, N, K) for u, v in zip(_halves(dy, M), _halves(x, M))]
    _gemm(_halves(dy, M), _halves(x, M), N, K + 8, M, out_f32=True, c=dws, ldc=K, c2=dbs, c2_copy=4, a_t=1,
          w_t=2, ldw=K, lda=N, splitk=True)
    return [(dws[0], dbs[0]), (dws[1], dbs[1])]


def _dx2(dy, wbs, M, N, K, act=0, r=None):
    """_dx of both modalities: dX [2M][K] = dY [2M][N] W_m [N][K] per half (bf16; act 5 with r [2M][N])."""
    rr = _halves(r, M) if r is not None else None
    if MN_MAJOR:
        return _gemm(_halves(dy, M), wbs, M, K, N, act=act, r=rr, w_t=1, ldw=K)
    return _gemm(_halves(dy, M), tuple(_transpose(w, N, K) for w in wbs), M, K, N, act=act, r=rr)


class _HipLinear2(torch.autograd.Function):
    """_HipLinear for the two modalities: x [2M][K] bf16 (RGB rows first), weights (w0, b0) / (w1, b1)."""

    @staticmethod
    def forward(ctx, x, w0, b0, w1, b1, out_f32=False):
        M2, K = x.shape
        M, N = M2 // 2, w0.shape[0]
        x = x.contiguous()
        wbs = (_bf16_weight(w0), _bf16_weight(w1))
        y = _gemm(_halves(x, M), wbs, M, N, K, bias=(b0.detach().float(), b1.detach().float()), out_f32=out_f32)
        ctx.save_for_backward(x, *wbs)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wb0, wb1 = ctx.saved_tensors
        M2, K = x.shape
        M, N = M2 // 2, wb0.shape[0]
        dy = dy.to(torch.bfloat16).contiguous()
        with _Beside(dy.device) as side:
            (dw0, db0), (dw1, db1) = side.run(_weight_grads2, dy, x, M, N, K, bufs=_wg2_bufs(dy.device, N, K))
            dx = _dx2(dy, (wb0, wb1), M, N, K) if ctx.needs_input_grad[0] else None
        return dx, dw0, db0, dw1, db1, None


def _residual_gemm2(a, wbs, bs, x, keep, M, N, K, rows):
    """x + keep * (a W_m^T + b_m) for both halves, fp32 [2M][N]: one grouped launch without stochastic depth;
    with it one launch per modality (the row scale is one vector indexed by the row within a group; a
    per-group index and so one launch measured no faster: 458.6 vs 462.1 samples/s on the step)."""
    xr = x.detach().reshape(2 * M, N)
    if keep is None:
        return _gemm(_halves(a, M), wbs, M, N, K, bias=bs, out_f32=True, r=_halves(xr, M))
    y = torch.empty(2 * M, N, device=a.device, dtype=torch.float32)
    B = keep.shape[0] // 2
    for m, (am, ym, xm) in enumerate(zip(_halves(a, M), _halves(y, M), _halves(xr, M))):
        _gemm(am, wbs[m], M, N, K, bias=bs[m], out_f32=True, r=xm, c=ym, row_scale=keep[m * B:(m + 1) * B],
              row_scale_div=rows)
    return y


class _HipLinearResidual2(torch.autograd.Function):
    """_HipLinearResidual for the two modalities: x [2B][ntok][N] fp32, a [2M][K], keep [2B] or None."""

    @staticmethod
    def forward(ctx, x, a, w0, b0, w1, b1, keep):
        M2, K = a.shape
        M, N = M2 // 2, w0.shape[0]
        a = a.contiguous()
        wbs = (_bf16_weight(w0), _bf16_weight(w1))
        rows = M2 // keep.shape[0] if keep is not None else 1
        y = _residual_gemm2(a, wbs, (b0.detach(), b1.detach()), x, keep, M, N, K, rows)
        ctx.save_for_backward(a, *wbs, keep)
        ctx.rows = rows
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dout):
        a, wb0, wb1, keep = ctx.saved_tensors
        M2, K = a.shape
        M, N = M2 // 2, wb0.shape[0]
        dy = _scaled_bf16(dout.reshape(M2, N), keep, ctx.rows)
        with _Beside(dy.device) as side:
            (dw0, db0), (dw1, db1) = side.run(_weight_grads2, dy, a, M, N, K, bufs=_wg2_bufs(dy.device, N, K))
            da = _dx2(dy, (wb0, wb1), M, N, K) if ctx.needs_input_grad[1] else None
        return dout, da, dw0, db0, dw1, db1, None


class _HipMlpResidual2(torch.autograd.Function):
    """_HipMlpResidual for the two modalities: fc1 (GELU epilogue, pre-activation stored) as one grouped GEMM,
    fc2 + DropPath + residual as _residual_gemm2, the backward's four GEMMs grouped."""

    @staticmethod
    def forward(ctx, x, xn, w10, b10, w20, b20, w11, b11, w21, b21, keep):
        M2, C = xn.shape
        M, F4 = M2 // 2, w10.shape[0]
        xn = xn.contiguous()
        wb1 = (_bf16_weight(w10), _bf16_weight(w11))
        wb2 = (_bf16_weight(w20), _bf16_weight(w21))
        rows = M2 // keep.shape[0] if keep is not None else 1
        hp = torch.empty(M2, F4, device=xn.device, dtype=torch.bfloat16)
        h = _gemm(_halves(xn, M), wb1, M, F4, C, bias=(b10.detach(), b11.detach()), act=1, c2=_halves(hp, M),
                  c2_copy=2)
        y = _residual_gemm2(h, wb2, (b20.detach(), b21.detach()), x, keep, M, C, F4, rows)
        ctx.save_for_backward(xn, *wb1, *wb2, h, hp, keep)
        ctx.rows = rows
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dout):
        xn, wb10, wb11, wb20, wb21, h, hp, keep = ctx.saved_tensors
        M2, C = xn.shape
        M, F4 = M2 // 2, wb10.shape[0]
        dy = _scaled_bf16(dout.reshape(M2, C), keep, ctx.rows)
        with _Beside(dy.device) as side:
            (dw20, db20), (dw21, db21) = side.run(_weight_grads2, dy, h, M, C, F4, bufs=_wg2_bufs(dy.device, C, F4))
            dhp = _dx2(dy, (wb20, wb21), M, C, F4, act=5, r=hp)
            (dw10, db10), (dw11, db11) = side.run(_weight_grads2, dhp, xn, M, F4, C, bufs=_wg2_bufs(dy.device, F4, C))
            dxn = _dx2(dhp, (wb10, wb11), M, F4, C) if ctx.needs_input_grad[1] else None
        return dout, dxn, dw10, db10, dw20, db20, dw11, db11, dw21, db21, None


class _HipMamAttention(torch.autograd.Function):
    """MAM softmax attention (mixformer.py:52-78) over qkv [S][ntok][3C] bf16 -> [S][ntok][C] bf16:
    the registered ops mmt::mam_attention_forward (with log-sum-exp) / mmt::mam_attention_backward."""

    @staticmethod
    def forward(ctx, qkv, n_t, heads):
        from .ops import mam_attention_forward
        qkv = qkv.contiguous()
        out, lse = mam_attention_forward(qkv, n_t, heads)
        ctx.save_for_backward(qkv, out, lse)
        ctx.n_t, ctx.heads = n_t, heads
        return out

    @staticmethod
    def backward(ctx, dout):
        from .ops import mam_attention_backward
        qkv, out, lse = ctx.saved_tensors
        return mam_attention_backward(qkv, out, dout, lse, ctx.n_t, ctx.heads), None, None


def _ln_fwd(ctx, x, w0, b0, w1, b1, rows0, eps, out_f32):
    """mmt_layernorm of x (fp32, last dim C) -> [rows][C] bf16 (fp32 with out_f32); saves what _ln_bwd needs."""
    from ._lib import LIB, MMT_BF16, check
    C = x.shape[-1]
    x2 = x.reshape(-1, C).contiguous()
    rows = x2.shape[0]
    two = w1 is not None  # (LayerNorm parameters are contiguous fp32 leaves)
    out = torch.empty(rows, C, device=x.device, dtype=torch.float32 if out_f32 else torch.bfloat16)
    check(LIB.mmt_layernorm(x2.data_ptr(), None, 0, out.data_ptr() if out_f32 else None,
                            None if out_f32 else out.data_ptr(), w0.data_ptr(), b0.data_ptr(),
                            w1.data_ptr() if two else None, b1.data_ptr() if two else None, rows,
                            rows0 if two else rows, C, eps, MMT_BF16, _stream()), "mmt_layernorm")
    ctx.save_for_backward(x2, w0, w1 if two else w0)
    ctx.two, ctx.rows0, ctx.eps, ctx.shape = two, rows0, eps, x.shape
    return out


def _ln_bwd(ctx, dy, dres=None):
    """(dx, dgamma0, dbeta0, dgamma1, dbeta1) of _ln_fwd's LayerNorm; dres (fp32, the input's shape): a second
    gradient of the input, added in the same kernel (mmt_layernorm_bwd_add)."""
    from ._lib import LIB, MMT_BF16, MMT_F32, check
    x2, g0, g1 = ctx.saved_tensors
    rows, C = x2.shape
    dy = dy.reshape(rows, C).contiguous()
    code = {torch.bfloat16: MMT_BF16, torch.float32: MMT_F32}[dy.dtype]
    sets = 4 if ctx.two else 2
    nws = (rows + 31) // 32 * 4 * C
    # dgamma / dbeta in their own small tensor: AccumulateGrad keeps them as .grad, and views into the
    # dx / workspace buffer would hold its rows * C floats alive until the next zero_grad
    buf = torch.empty(rows * C + nws, device=x2.device, dtype=torch.float32)
    dx, ws = buf[:rows * C].view(rows, C), buf[rows * C:]
    dgb = torch.empty(sets, C, device=x2.device, dtype=torch.float32)
    args = (x2.data_ptr(), dy.data_ptr(), code, g0.data_ptr(), g1.data_ptr() if ctx.two else None)
    tail = (dx.data_ptr(), dgb.data_ptr(), 0, ws.data_ptr(), ws.numel(), rows, ctx.rows0 if ctx.two else rows, C,
            ctx.eps, _stream())
    if dres is None:
        check(LIB.mmt_layernorm_bwd(*args, *tail), "mmt_layernorm_bwd")
    else:
        dres = dres.reshape(rows, C).float().contiguous()
        check(LIB.mmt_layernorm_bwd_add(*args, dres.data_ptr(), *tail), "mmt_layernorm_bwd_add")
    dx = dx.view(ctx.shape)
    if ctx.two:
        return dx, dgb[0], dgb[1], dgb[2], dgb[3]
    return dx, dgb[0], dgb[1], None, None


class _HipLayerNorm(torch.autograd.Function):
    """nn.LayerNorm over the last dim of the fp32 residual stream -> bf16 (the next Linear's operand; fp32
    with out_f32), rows in alternating blocks of rows0 with (w0, b0) / (w1, b1) (the per-modality
    norm*_v / norm*_i: the shared backbone's [rgb; tir] halves, or the fusion encoder's [v; i] token
    halves of every sequence) or all rows with (w0, b0): forward mmt_layernorm, backward
    mmt_layernorm_bwd (dx, dgamma / dbeta from the saved fp32 input; statistics recomputed)."""

    @staticmethod
    def forward(ctx, x, w0, b0, w1, b1, rows0, eps, out_f32=False):
        return _ln_fwd(ctx, x, w0, b0, w1, b1, rows0, eps, out_f32).view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        return (*_ln_bwd(ctx, dy), None, None, None)


class _HipLayerNormPass(torch.autograd.Function):
    """_HipLayerNorm (bf16 out) that also hands its input through as a second output.  A pre-LN block's residual
    stream x feeds both the LayerNorm and the residual op (x + f(LN(x)), mixformer.py:136-139), so autograd would
    sum the two gradients of x with one more elementwise pass over the [rows][C] fp32 stream (24 per training
    step); the consumers take the pass-through instead, and the backward adds its gradient inside the LayerNorm
    backward kernel (mmt_layernorm_bwd_add)."""

    @staticmethod
    def forward(ctx, x, w0, b0, w1, b1, rows0, eps):
        return _ln_fwd(ctx, x, w0, b0, w1, b1, rows0, eps, False).view(x.shape), x

    @staticmethod
    def backward(ctx, dy, dres):
        return (*_ln_bwd(ctx, dy, dres), None, None)


class _HipGroupNorm(torch.autograd.Function):
    """nn.GroupNorm over channels-last fp32 [n][P][C] (the fusion's adjust_* GroupNorms on token rows):
    forward mmt_groupnorm, backward mmt_groupnorm_bwd (statistics recomputed from the saved input)."""

    @staticmethod
    def forward(ctx, x, w, b, groups, eps):
        from ._lib import LIB, MMT_F32, check
        n, P, C = x.shape
        x = x.contiguous()
        out = torch.empty_like(x)
        check(LIB.mmt_groupnorm(x.data_ptr(), out.data_ptr(), None, w.data_ptr(), b.data_ptr(), None, None, n, n, P,
                                C, groups, eps, MMT_F32, _stream()), "mmt_groupnorm")
        ctx.save_for_backward(x, w)
        ctx.groups, ctx.eps = groups, eps
        return out

    @staticmethod
    def backward(ctx, dy):
        from ._lib import LIB, check
        x, w = ctx.saved_tensors
        n, P, C = x.shape
        dy = dy.float().contiguous()
        buf = torch.empty(n * P * C + n * 2 * C, device=x.device, dtype=torch.float32)
        dx, ws = buf[:n * P * C].view(n, P, C), buf[n * P * C:]
        dgb = torch.empty(2, C, device=x.device, dtype=torch.float32)  # separate from dx (see _HipLayerNorm)
        check(LIB.mmt_groupnorm_bwd(x.data_ptr(), dy.data_ptr(), w.data_ptr(), dx.data_ptr(), dgb.data_ptr(), 0,
                                    ws.data_ptr(), ws.numel(), n, P, C, ctx.groups, ctx.eps, _stream()),
              "mmt_groupnorm_bwd")
        return dx, dgb[0], dgb[1], None, None


def _conv_gemm(x, wr, B, H, Cin, Cout, bias=None, flip=False, up=1):
    """NHWC 3x3 / pad-1 convolution as the implicit-GEMM conv mode of mmt_gemm: y [B*H*H][Cout] bf16 =
    im2col(x) wr^T (+ bias), x [B][H][H][Cin] bf16 (square maps), wr [Cout][(ky*3 + kx)*Cin + ci] bf16;
    flip: the taps read in reverse order (conv_k3 2: the convolution with the flipped kernel); up: x is
    [B][H/up][H/up][Cin] and the conv runs on its nearest upsampling (conv_up: the map never materialised)."""
    from ._lib import LIB, GemmParams, MMT_BF16, check
    M = B * H * H
    y = torch.empty(M, Cout, device=x.device, dtype=torch.bfloat16)
    p = GemmParams()
    p.a[0], p.w[0], p.c[0] = x.data_ptr(), wr.data_ptr(), y.data_ptr()
    p.bias[0] = bias.data_ptr() if bias is not None else None
    p.lda, p.ldc = Cin, Cout
    p.a_seg_rows, p.a_segs_a = M, 1
    p.M, p.N, p.K, p.groups = M, Cout, 9 * Cin, 1
    p.conv_h, p.conv_up, p.conv_cin, p.conv_k3 = H, up, Cin, 2 if flip else 1
    check(LIB.mmt_gemm(p, MMT_BF16, _stream()), "mmt_gemm (conv)")
    # implicit GEMM: the input map is read once (B (H/up)^2 Cin), not the im2col matrix
    _account(M, Cout, 9 * Cin, 1, 0, 2, 2, M // (up * up) * Cin * 2 + (Cout * 4 if bias is not None else 0))
    return y


class _HipBatchNormReLU(torch.autograd.Function):
    """nn.BatchNorm2d -> nn.ReLU of a conv() block (head.py:7-20) on an NHWC bf16 map [B][H][W][C]
    (mmt_batchnorm_relu / _bwd): batch statistics in training (running statistics updated in place with the
    module's momentum) or the running statistics in eval, affine + ReLU in one pass; the backward recomputes
    the ReLU mask and x-hat from the saved input and per-channel coefficients."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, training, C):
        from ._lib import LIB, check
        if x.dtype != torch.bfloat16 or not x.is_contiguous():
            raise ValueError("HIP batch norm: contiguous NHWC bf16 maps")
        pitch = x.shape[-1]  # C valid channels of `pitch` (the 1-channel maps are padded to 8)
        M = x.numel() // pitch
        y = torch.empty_like(x)
        save = torch.empty(4, C, device=x.device, dtype=torch.float32)
        nws = int(LIB.mmt_batchnorm_ws_floats(M, C))
        ws = torch.empty(nws, device=x.device, dtype=torch.float32) if training else None
        ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        check(LIB.mmt_batchnorm_relu(x.data_ptr(), y.data_ptr(), M, C, pitch, ptr(weight), ptr(bias), ptr(running_mean),
                                     ptr(running_var), float(momentum), float(eps), int(training), 1, save.data_ptr(),
                                     ptr(ws), nws if training else 0, _stream()), "mmt_batchnorm_relu")
        ctx.save_for_backward(x, weight, save)
        ctx.training, ctx.nws, ctx.C = training, nws, C
        return y

    @staticmethod
    def backward(ctx, dy):
        from ._lib import LIB, check
        x, weight, save = ctx.saved_tensors
        C, pitch = ctx.C, x.shape[-1]
        M = x.numel() // pitch
        dy = dy.to(torch.bfloat16).contiguous()
        dx = torch.empty_like(x)
        dgb = torch.empty(2, C, device=x.device, dtype=torch.float32)
        ws = torch.empty(ctx.nws, device=x.device, dtype=torch.float32)
        check(LIB.mmt_batchnorm_relu_bwd(x.data_ptr(), dy.data_ptr(), dx.data_ptr(), M, C, pitch,
                                         weight.data_ptr() if weight is not None else None, save.data_ptr(),
                                         int(ctx.training), 1, dgb.data_ptr(), ws.data_ptr(), ctx.nws, _stream()),
              "mmt_batchnorm_relu_bwd")
        # weight / bias may be None (affine=False) or buffers (FrozenBatchNorm2d): no gradient for those
        dw = dgb[0] if ctx.needs_input_grad[1] else None
        db = dgb[1] if ctx.needs_input_grad[2] else None
        return dx, dw, db, None, None, None, None, None, None


class _HipCornerScore(torch.autograd.Function):
    """One corner branch's score map in the training step (head.py:191-192): conv5 (Conv2d(48, 1, 1), in fp32 as
    HEAD_SCORE_FP32) + up4(adjust3) + up2(adjust4) -> (B, fh*fh) fp32, forward and backward on
    mmt_corner_score_train / _bwd.  x4 (B, fh, fh, c4) bf16 NHWC; a3 / a4 (B, fh/4, fh/4, 1) / (B, fh/2, fh/2, 1)
    bf16 views (the HIP BatchNorm's 8-channel rows: pixel stride = their stride(2)).  Replaces aten's fp32
    F.linear through hipBLASLt (~175 us a launch), two nearest upsamplings and two adds, and their backward."""

    @staticmethod
    def forward(ctx, x4, w5, b5, a3, a4):
        from ._lib import LIB, check
        B, fh, _, c4 = x4.shape
        if x4.dtype != torch.bfloat16 or not x4.is_contiguous() or a3.dtype != torch.bfloat16 or a4.dtype != torch.bfloat16:
            raise ValueError("HIP corner score: contiguous bf16 NHWC x4, bf16 adjust maps")
        if a3.shape[:3] != (B, fh // 4, fh // 4) or a4.shape[:3] != (B, fh // 2, fh // 2):
            raise ValueError("HIP corner score: adjust maps of fh/4 and fh/2")
        for a in (a3, a4):  # channel 0 of pixel-strided rows: (B, h, w, 1) views, or the padded 8-channel rows
            if a.shape[3] not in (1, a.stride(2)) or a.stride(1) != a.stride(2) * a.shape[2] or a.stride(0) != a.stride(1) * a.shape[1]:
                raise ValueError("HIP corner score: adjust maps must be pixel-strided rows")
        w = w5.detach().reshape(-1).float().contiguous()
        b = b5.detach().reshape(-1).float().contiguous()
        out = torch.empty(B, fh * fh, device=x4.device, dtype=torch.float32)
        check(LIB.mmt_corner_score_train(x4.data_ptr(), w.data_ptr(), b.data_ptr(), a3.data_ptr(), a3.stride(2),
                                         a4.data_ptr(), a4.stride(2), out.data_ptr(), B, fh, c4, _stream()),
              "mmt_corner_score_train")
        ctx.save_for_backward(x4, w)
        ctx.wshape, ctx.c3, ctx.c4 = w5.shape, a3.shape[3], a4.shape[3]
        return out

    @staticmethod
    def backward(ctx, dsm):
        from ._lib import LIB, check
        x4, w = ctx.saved_tensors
        B, fh, _, c4 = x4.shape
        dsm = dsm.float().contiguous()
        dx4 = torch.empty_like(x4)
        # (padded rows: the kernel writes channel 0 and zeroes the padding channels)
        da3 = torch.empty(B, fh // 4, fh // 4, ctx.c3, device=x4.device, dtype=torch.bfloat16)
        da4 = torch.empty(B, fh // 2, fh // 2, ctx.c4, device=x4.device, dtype=torch.bfloat16)
        dw = torch.empty(c4 + 1, device=x4.device, dtype=torch.float32)
        ws = torch.empty(int(LIB.mmt_corner_score_train_ws_floats(B, fh, c4)), device=x4.device, dtype=torch.float32)
        check(LIB.mmt_corner_score_train_bwd(dsm.data_ptr(), x4.data_ptr(), w.data_ptr(), dx4.data_ptr(), da3.data_ptr(),
                                             ctx.c3, da4.data_ptr(), ctx.c4, dw.data_ptr(), dw[c4:].data_ptr(),
                                             ws.data_ptr(), B, fh, c4, _stream()), "mmt_corner_score_train_bwd")
        return dx4, dw[:c4].view(ctx.wshape), dw[c4:], da3, da4


def _conv_wprep(convs):
    """The bf16 operand layouts of 3x3 convs [(weight [Cout][Cin][3][3] fp32, bias or None)] in one launch
    (mmt_conv3x3_wprep): per conv (wf [Cp][9 Cin] forward, wb [Cin][9 Cp] dX, bp [Cp] fp32 padded bias),
    Cp = Cout rounded up to 8, views of one bf16 and one fp32 buffer."""
    from ._lib import LIB, ConvWprep, WPREP_MAX, check
    out = []
    for i in range(0, len(convs), WPREP_MAX):
        part = convs[i:i + WPREP_MAX]
        dims = [(w.shape[0], (w.shape[0] + 7) // 8 * 8, w.shape[1]) for w, _ in part]
        dev = part[0][0].device
        wbuf = torch.empty(sum(2 * cp * 9 * cin for _, cp, cin in dims), device=dev, dtype=torch.bfloat16)
        bbuf = torch.empty(sum(cp for _, cp, _ in dims), device=dev, dtype=torch.float32)
        items = (ConvWprep * len(part))()
        ow = ob = 0
        keep = []
        for j, ((w, b), (cout, cp, cin)) in enumerate(zip(part, dims)):
            w = w.detach().contiguous()
            b = b.detach().float().contiguous() if b is not None else None
            keep += [w, b]
            n = cp * 9 * cin
            wf, wb, bp = wbuf[ow:ow + n].view(cp, 9 * cin), wbuf[ow + n:ow + 2 * n].view(cin, 9 * cp), bbuf[ob:ob + cp]
            ow, ob = ow + 2 * n, ob + cp
            items[j] = ConvWprep(w.data_ptr(), b.data_ptr() if b is not None else None, wf.data_ptr(), wb.data_ptr(),
                                 bp.data_ptr(), cout, cp, cin, 0)
            out.append((wf, wb, bp))
        check(LIB.mmt_conv3x3_wprep(items, len(part), _stream()), "mmt_conv3x3_wprep")
    return out


class _HipConv3x3(torch.autograd.Function):
    """nn.Conv2d(Cin, Cout, 3, padding=1) of the corner head's conv() blocks (lib/models/mixformer_cvt/head.py:
    7-20) on NHWC bf16 maps, all three products on the LDS-DMA GEMM: the forward and dX as implicit-GEMM
    convs (dX = the 3x3 conv of dY with the kernel flipped -- taps read in reverse, conv_k3 2 -- and Cin / Cout
    swapped), dW and the bias
    gradient as one GEMM over pixels against the im2col of X (mmt_im2col3x3_bf16; `_weight_grads`).  Replaces
    MIOpen's igemm forward / backward-data / backward-weights kernels, whose backward did not replay
    correctly from a captured hipGraph.
    up (round 6): the conv of the nearest upsampling (x up) of x, the map never materialised (forward: the GEMM's
    conv_up addressing; dX: the flipped conv at the upsampled size, then the up x up block sums,
    mmt_upsample_sum_bf16; dW: im2col of the upsampled map, mmt_im2col3x3_up_bf16).  keep_pad: Cout < 8 outputs
    stay in their 8-channel rows (padding channels 0) for the next HIP op, instead of a sliced view whose
    backward zero-fills and copies."""

    @staticmethod
    def forward(ctx, x, w, b, up=1, keep_pad=False, prep=None):
        B, H, W, Cin = x.shape
        Cout = w.shape[0]
        if H != W or Cin % 8 or w.shape[2:] != (3, 3) or x.dtype != torch.bfloat16 or up not in (1, 2, 4):
            raise ValueError("HIP conv3x3: square NHWC bf16 maps, input channels multiple of 8, 3x3 kernels, up 1/2/4")
        Cp = (Cout + 7) // 8 * 8  # output channels padded to the GEMM's N granule (the 48 -> 1 adjust convs)
        x = x.contiguous()
        # the weight's two bf16 layouts and the padded bias: given (one launch for the whole head, _conv_wprep)
        # or made here
        wf, wb, bp = prep if prep is not None else _conv_wprep([(w, b)])[0]
        if wf.shape != (Cp, 9 * Cin) or wb.shape != (Cin, 9 * Cp):
            raise ValueError("HIP conv3x3: prepared weights of another conv")
        Ho = H * up
        y = _conv_gemm(x, wf, B, Ho, Cin, Cp, bias=bp, up=up)
        ctx.save_for_backward(x, wb)
        ctx.up, ctx.wshape = up, w.shape
        y = y.view(B, Ho, Ho, Cp)
        return y if (Cp == Cout or keep_pad) else y[..., :Cout]

    @staticmethod
    def backward(ctx, dy):
        from ._lib import LIB, check
        x, wb = ctx.saved_tensors
        up = ctx.up
        B, H, W, Cin = x.shape
        Ho = H * up
        Cout = ctx.wshape[0]
        Cp = (Cout + 7) // 8 * 8
        if dy.shape[-1] != Cp:  # a sliced output: back to the padded rows
            dyp = torch.zeros(B, Ho, Ho, Cp, device=dy.device, dtype=torch.bfloat16)
            dyp[..., :Cout] = dy
            dy = dyp
        else:  # padded rows (keep_pad): the padding channels' gradient multiplies zero weights
            dy = dy.to(torch.bfloat16).contiguous()
        dx = None
        if ctx.needs_input_grad[0]:  # the flipped-tap conv of dY with W as [Cin][ky][kx][Cout] (no flip copy)
            dxu = _conv_gemm(dy, wb, B, Ho, Cp, Cin, flip=True).view(B, Ho, Ho, Cin)
            if up == 1:
                dx = dxu
            else:
                dx = torch.empty_like(x)
                check(LIB.mmt_upsample_sum_bf16(dxu.data_ptr(), dx.data_ptr(), B, H, W, Cin, up, _stream()),
                      "mmt_upsample_sum_bf16")
        # dW against the channel-major im2col: the GEMM writes [Cout][Cin][3][3], the parameter's layout
        M = B * Ho * Ho
        col = torch.empty(M, 9 * Cin, device=x.device, dtype=torch.bfloat16)
        check(LIB.mmt_im2col3x3_cm_bf16(x.data_ptr(), col.data_ptr(), B, Ho, Ho, Cin, up, _stream()),
              "mmt_im2col3x3_cm_bf16")
        dw, db = _weight_grads(dy.view(M, Cp), col, M, Cp, 9 * Cin)
        return dx, dw[:Cout].view(ctx.wshape), db[:Cout], None, None, None


class _HipMSDABimodal(torch.autograd.Function):
    """The middle of MSDeformAttn_Bimodal in the training step (ms_deform_attn_bimodal.py:97-128; 8 heads, 2 levels,
    4 points, 64 channels per head), from the bf16 outputs of value_proj and the [sampling_offsets |
    attention_weights] Linear to the bf16 input of output_proj, on mmt_msda_bimodal_train_fwd / _bwd: softmax of the
    attention logits, sampling locations ref + off / hw, the bilinear sampling sum, and their backward (grad_value
    by the deterministic per-pixel gather) -- the arithmetic of F.softmax(aw.float()), ref + off.float() / wh and
    MSDeformAttnFunction on value.float(), with the casts those imply.  value (B, 2 nq, 512), offw (B, nq, >= 192)
    bf16 with the offsets in columns [0, 128) and the logits in [128, 192) (row pitch = its last stride); ref
    (nq, 2) fp32 (the device-computed reference points) -> (B, nq, 512) bf16."""

    @staticmethod
    def forward(ctx, value, offw, ref, hw):
        from ._lib import LIB, check
        B, nq = offw.shape[0], hw * hw
        if value.dtype != torch.bfloat16 or tuple(value.shape) != (B, 2 * nq, 512) or offw.dtype != torch.bfloat16 \
                or offw.shape[1:] != (nq, 192):
            raise ValueError("HIP MSDA (training): bf16 value (B, 2 nq, 512) and offsets | logits (B, nq, 192)")
        if ref.dtype != torch.float32 or tuple(ref.shape) != (nq, 2):
            raise ValueError("HIP MSDA (training): fp32 reference points (nq, 2)")
        value, offw, ref = value.contiguous(), offw.contiguous(), ref.contiguous()
        out = torch.empty(B, nq, 512, device=value.device, dtype=torch.bfloat16)
        check(LIB.mmt_msda_bimodal_train_fwd(value.data_ptr(), offw.data_ptr(), 192, offw[..., 128:].data_ptr(), 192,
                                             ref.data_ptr(), out.data_ptr(), B, hw, _stream()),
              "mmt_msda_bimodal_train_fwd")
        ctx.save_for_backward(value, offw, ref)
        ctx.hw = hw
        return out

    @staticmethod
    def backward(ctx, gout):
        from ._lib import LIB, check
        value, offw, ref = ctx.saved_tensors
        gout = gout.to(torch.bfloat16).contiguous()
        gv, gow = torch.empty_like(value), torch.empty_like(offw)
        check(LIB.mmt_msda_bimodal_train_bwd(value.data_ptr(), offw.data_ptr(), 192, offw[..., 128:].data_ptr(), 192,
                                             ref.data_ptr(), gout.data_ptr(), gv.data_ptr(), gow.data_ptr(),
                                             gow[..., 128:].data_ptr(), offw.shape[0], ctx.hw, _stream()),
              "mmt_msda_bimodal_train_bwd")
        return gv, gow, None, None


_DROP_RNG = {}  # device -> int64 [2] {seed, counter} of the encoder's dropout draws (csrc/fusion_train.hip)


def _drop_rng(device):
    """The device's dropout key {seed, counter}: the seed drawn from torch's default generator at first use (so
    torch.manual_seed makes runs repeatable), the counter advanced once per training forward (_drop_advance)."""
    st = _DROP_RNG.get(str(device))
    if st is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        st = _DROP_RNG[str(device)] = torch.tensor([seed, 0], dtype=torch.int64).to(device)
    return st


class _HipSearchTokens(torch.autograd.Function):
    """The two backbones' search tokens as the fusion's adjust Linears read them (mixformer.py:256-259 ->
    fusion_utils.py:270-275): x (2B, ntok, C) fp32 (RGB sequences first) -> rows [n_t, ntok) as bf16 (2B, ns, C),
    one pass (mmt_ft_rows_cast); backward: the stream's gradient with zero template rows, one pass (replaces the
    slice / transpose / reshape / cast chain and its zero-filling slice backwards)."""

    @staticmethod
    def forward(ctx, x, n_t):
        from ._lib import LIB, check
        S, ntok, C = x.shape
        x = x.contiguous()
        out = torch.empty(S, ntok - n_t, C, device=x.device, dtype=torch.bfloat16)
        check(LIB.mmt_ft_rows_cast(x.data_ptr(), out.data_ptr(), S, ntok, n_t, ntok - n_t, C, _stream()),
              "mmt_ft_rows_cast")
        ctx.args = (S, ntok, n_t, C)
        return out

    @staticmethod
    def backward(ctx, d):
        from ._lib import LIB, check
        S, ntok, n_t, C = ctx.args
        d = d.to(torch.bfloat16).contiguous()
        dx = torch.empty(S, ntok, C, device=d.device, dtype=torch.float32)
        check(LIB.mmt_ft_rows_cast_bwd(d.data_ptr(), dx.data_ptr(), S, ntok, n_t, ntok - n_t, C, _stream()),
              "mmt_ft_rows_cast_bwd")
        return dx, None


class _HipGroupNorm2(torch.autograd.Function):
    """The fusion's adjust_v / adjust_i GroupNorms (fusion_utils.py:252-268) on the stacked modalities' rows
    x (2B, P, C) fp32 (RGB first), each half with its own affine -> (RGB (B, P, C), TIR (B, P, C)) as two tensors
    (so the cat that follows hands each its gradient as a view); backward: one dx buffer for both halves."""

    @staticmethod
    def forward(ctx, x, w0, b0, w1, b1, groups, eps):
        from ._lib import LIB, MMT_F32, check
        n2, P, C = x.shape
        B = n2 // 2
        x = x.contiguous()
        outs = []
        for h, (w, b) in enumerate(((w0, b0), (w1, b1))):
            o = torch.empty(B, P, C, device=x.device, dtype=torch.float32)
            check(LIB.mmt_groupnorm(x[h * B:].data_ptr(), o.data_ptr(), None, w.data_ptr(), b.data_ptr(), None, None, B,
                                    B, P, C, groups, eps, MMT_F32, _stream()), "mmt_groupnorm")
            outs.append(o)
        ctx.save_for_backward(x, w0, w1)
        ctx.groups, ctx.eps = groups, eps
        return outs[0], outs[1]

    @staticmethod
    def backward(ctx, dv, di):
        from ._lib import LIB, check
        x, w0, w1 = ctx.saved_tensors
        n2, P, C = x.shape
        B = n2 // 2
        dx = torch.empty_like(x)
        dgb = torch.empty(2, 2, C, device=x.device, dtype=torch.float32)
        ws = torch.empty(B * 2 * C, device=x.device, dtype=torch.float32)
        for h, (dy, w) in enumerate(((dv, w0), (di, w1))):
            dy = dy.float().contiguous() if dy is not None else torch.zeros(B, P, C, device=x.device)
            check(LIB.mmt_groupnorm_bwd(x[h * B:].data_ptr(), dy.data_ptr(), w.data_ptr(), dx[h * B:].data_ptr(),
                                        dgb[h].data_ptr(), 0, ws.data_ptr(), ws.numel(), B, P, C, ctx.groups, ctx.eps,
                                        _stream()), "mmt_groupnorm_bwd")
        return dx, dgb[0, 0], dgb[0, 1], dgb[1, 0], dgb[1, 1], None, None


class _HipQueryPrep(torch.autograd.Function):
    """The encoder layer's inputs from its fp32 stream src (B, 2 nq, d) and the level-embedded positions lpos
    (1, 2 nq, d) (deformable_encoder_lnspecific.py:131-136, ms_deform_attn_bimodal.py:97-105): q_bi = the bimodal
    query cat(chunk(src + lpos, 2, 1), 2) in bf16 (B, nq, 2 d), src in bf16 (value_proj's operand) and src handed
    through for the residual -- one pass (mmt_ft_query_prep); the backward sums the three gradients of src and
    reduces lpos's over the batch in one pass (mmt_ft_query_prep_bwd)."""

    @staticmethod
    def forward(ctx, src, lpos):
        from ._lib import LIB, check
        B, n2, d = src.shape
        src, lp = src.contiguous(), lpos.detach().contiguous()
        qbi = torch.empty(B, n2 // 2, 2 * d, device=src.device, dtype=torch.bfloat16)
        srcb = torch.empty(B, n2, d, device=src.device, dtype=torch.bfloat16)
        check(LIB.mmt_ft_query_prep(src.data_ptr(), lp.data_ptr(), qbi.data_ptr(), srcb.data_ptr(), B, n2 // 2, d,
                                    _stream()), "mmt_ft_query_prep")
        ctx.set_materialize_grads(False)
        ctx.shape = (B, n2, d)
        return qbi, srcb, src

    @staticmethod
    def backward(ctx, dqbi, dsrcb, dthrough):
        from ._lib import LIB, check
        B, n2, d = ctx.shape
        dev = (dqbi if dqbi is not None else dsrcb).device
        z = lambda shp: torch.zeros(shp, device=dev, dtype=torch.bfloat16)  # noqa: E731 (an unused output)
        dqbi = dqbi.to(torch.bfloat16).contiguous() if dqbi is not None else z((B, n2 // 2, 2 * d))
        dsrcb = dsrcb.to(torch.bfloat16).contiguous() if dsrcb is not None else z((B, n2, d))
        dt = dthrough.float().contiguous() if dthrough is not None else None
        dsrc = torch.empty(B, n2, d, device=dev, dtype=torch.float32)
        dlpos = torch.empty(1, n2, d, device=dev, dtype=torch.float32)
        check(LIB.mmt_ft_query_prep_bwd(dqbi.data_ptr(), dsrcb.data_ptr(), dt.data_ptr() if dt is not None else None,
                                        dsrc.data_ptr(), dlpos.data_ptr(), B, n2 // 2, d, _stream()),
              "mmt_ft_query_prep_bwd")
        return dsrc, dlpos


class _HipDropResidual(torch.autograd.Function):
    """x + Dropout(y) of the encoder layer's branches (deformable_encoder_lnspecific.py:139-148): x the fp32 stream
    (B, rows, d), y the bf16 branch (B, rows, d), or with dup its (B, rows / 2, d) unique rows repeated on both halves
    (the bimodal query's output_proj, cat([y, y], 1)); p: the module's dropout rate when training, else 0 (one
    pass, mmt_ft_drop_residual; backward: x's gradient handed through, y's one pass)."""

    @staticmethod
    def forward(ctx, x, y, p, salt, dup):
        from ._lib import LIB, check
        B, rows, d = x.shape
        x, y = x.contiguous(), y.to(torch.bfloat16).contiguous()
        rng = _drop_rng(x.device) if p > 0 else None
        out = torch.empty_like(x)
        check(LIB.mmt_ft_drop_residual(x.data_ptr(), y.data_ptr(), out.data_ptr(),
                                       rng.data_ptr() if rng is not None else None, salt, float(p), B, rows, d, int(dup),
                                       _stream()), "mmt_ft_drop_residual")
        ctx.p, ctx.salt, ctx.dup, ctx.yshape = p, salt, dup, y.shape
        return out

    @staticmethod
    def backward(ctx, dout):
        from ._lib import LIB, check
        dout = dout.float().contiguous()
        B, rows, d = dout.shape
        rng = _drop_rng(dout.device) if ctx.p > 0 else None
        dy = torch.empty(ctx.yshape, device=dout.device, dtype=torch.bfloat16)
        check(LIB.mmt_ft_drop_residual_bwd(dout.data_ptr(), dy.data_ptr(), rng.data_ptr() if rng is not None else None,
                                           ctx.salt, float(ctx.p), B, rows, d, int(ctx.dup), _stream()),
              "mmt_ft_drop_residual_bwd")
        return dout, dy, None, None, None


class _HipEncoderFFN(torch.autograd.Function):
    """x + Dropout3(linear2(Dropout2(ReLU(linear1(x))))) of the encoder layer (deformable_encoder_lnspecific.py:
    145-148; forward_ffn), x the fp32 stream (M, d): linear1 with the ReLU epilogue, the hidden dropout one pass
    (mmt_ft_relu_drop), linear2, the residual dropout-add one pass (mmt_ft_drop_residual); backward: the branch's
    dropout backward, linear2's products, the hidden dropout + ReLU backward in one pass, linear1's dX GEMM with
    the stream gradient added in its epilogue (fp32: the branch gradient is not rounded to bf16 before the add)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, p2, p3, salt):
        from ._lib import LIB, check
        M, d = x.shape
        F_ = w1.shape[0]
        x = x.contiguous()
        xb = x.to(torch.bfloat16)
        wb1, wb2 = _bf16_weight(w1), _bf16_weight(w2)
        h = _gemm(xb, wb1, M, F_, d, bias=b1.detach(), act=2)  # relu(linear1(x)) in bf16
        rng = _drop_rng(x.device) if (p2 > 0 or p3 > 0) else None
        if p2 > 0:
            hd = torch.empty_like(h)
            check(LIB.mmt_ft_relu_drop(h.data_ptr(), hd.data_ptr(), rng.data_ptr(), salt + 1, float(p2), h.numel(),
                                       _stream()), "mmt_ft_relu_drop")
        else:
            hd = h
        y = _gemm(hd, wb2, M, d, F_, bias=b2.detach())
        out = torch.empty_like(x)
        check(LIB.mmt_ft_drop_residual(x.data_ptr(), y.data_ptr(), out.data_ptr(),
                                       rng.data_ptr() if (rng is not None and p3 > 0) else None, salt + 2, float(p3),
                                       1, M, d, 0, _stream()), "mmt_ft_drop_residual")
        ctx.save_for_backward(xb, wb1, wb2, h, hd)
        ctx.p2, ctx.p3, ctx.salt = p2, p3, salt
        return out

    @staticmethod
    def backward(ctx, dout):
        from ._lib import LIB, check
        xb, wb1, wb2, h, hd = ctx.saved_tensors
        M, d = xb.shape
        F_ = wb1.shape[0]
        dout = dout.float().contiguous()
        rng = _drop_rng(dout.device) if (ctx.p2 > 0 or ctx.p3 > 0) else None
        dy = torch.empty(M, d, device=dout.device, dtype=torch.bfloat16)
        check(LIB.mmt_ft_drop_residual_bwd(dout.data_ptr(), dy.data_ptr(),
                                           rng.data_ptr() if (rng is not None and ctx.p3 > 0) else None, ctx.salt + 2,
                                           float(ctx.p3), 1, M, d, 0, _stream()), "mmt_ft_drop_residual_bwd")
        dhd = _dx(dy, wb2, M, d, F_)
        dw2, db2 = _weight_grads(dy, hd, M, d, F_)
        dh = torch.empty_like(dhd)
        check(LIB.mmt_ft_relu_drop_bwd(dhd.data_ptr(), h.data_ptr(), dh.data_ptr(),
                                       rng.data_ptr() if (rng is not None and ctx.p2 > 0) else None, ctx.salt + 1,
                                       float(ctx.p2), dh.numel(), _stream()), "mmt_ft_relu_drop_bwd")
        dw1, db1 = _weight_grads(dh, xb, M, F_, d)
        dx = None
        if ctx.needs_input_grad[0]:  # dX = dh W1 + the stream gradient (fp32 epilogue residual)
            if MN_MAJOR:
                dx = _gemm(dh, wb1, M, d, F_, r=dout, out_f32=True, w_t=1, ldw=d)
            else:
                dx = _gemm(dh, _transpose(wb1, F_, d), M, d, F_, r=dout, out_f32=True)
        return dx, dw1, db1, dw2, db2, None, None, None


class _HipLinearCat(torch.autograd.Function):
    """Two nn.Linear layers on the same input as one GEMM (the bimodal query's sampling_offsets and
    attention_weights, ms_deform_attn_bimodal.py:99-100): y = x [W0; W1]^T + [b0; b1] (bf16 x (M, K) -> bf16
    (M, N0 + N1)); one dX GEMM (the two input gradients summed in its K loop) and one dW GEMM, whose rows are the
    two weights' gradients."""

    @staticmethod
    def forward(ctx, x, w0, b0, w1, b1):
        M, K = x.shape
        N0, N1 = w0.shape[0], w1.shape[0]
        x = x.contiguous()
        wb = torch.cat([_bf16_weight(w0), _bf16_weight(w1)], 0)
        bias = torch.cat([b0.detach().float(), b1.detach().float()], 0)
        y = _gemm(x, wb, M, N0 + N1, K, bias=bias)
        ctx.save_for_backward(x, wb)
        ctx.n0 = N0
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wb = ctx.saved_tensors
        M, K = x.shape
        N = wb.shape[0]
        dy = dy.to(torch.bfloat16).contiguous()
        dx = _dx(dy, wb, M, N, K) if ctx.needs_input_grad[0] else None
        dw, db = _weight_grads(dy, x, M, N, K)
        n0 = ctx.n0
        return dx, dw[:n0], db[:n0], dw[n0:], db[n0:]


class _HipCornerBoxes(torch.autograd.Function):
    """Both corners' soft-argmax (head.py:200-212) and the normalisation (head.py:176-177): score maps (B, fh*fh)
    fp32 -> xyxy (B, 4) in [0, 1] (mmt_corner_boxes; backward mmt_corner_boxes_bwd, the softmax backward of the
    expectations' gradient)."""

    @staticmethod
    def forward(ctx, s_tl, s_br, fh, stride, img_sz):
        from ._lib import LIB, check
        B = s_tl.shape[0]
        s_tl, s_br = s_tl.float().contiguous(), s_br.float().contiguous()
        xyxy = torch.empty(B, 4, device=s_tl.device, dtype=torch.float32)
        stats = torch.empty(B, 2, 4, device=s_tl.device, dtype=torch.float32)
        check(LIB.mmt_corner_boxes(s_tl.data_ptr(), s_br.data_ptr(), xyxy.data_ptr(), stats.data_ptr(), B, fh,
                                   float(stride), float(img_sz), _stream()), "mmt_corner_boxes")
        ctx.save_for_backward(s_tl, s_br, stats)
        ctx.args = (fh, float(stride), float(img_sz))
        return xyxy

    @staticmethod
    def backward(ctx, dxyxy):
        from ._lib import LIB, check
        s_tl, s_br, stats = ctx.saved_tensors
        fh, stride, img_sz = ctx.args
        dxyxy = dxyxy.float().contiguous()
        d_tl, d_br = torch.empty_like(s_tl), torch.empty_like(s_br)
        check(LIB.mmt_corner_boxes_bwd(s_tl.data_ptr(), s_br.data_ptr(), stats.data_ptr(), dxyxy.data_ptr(),
                                       d_tl.data_ptr(), d_br.data_ptr(), s_tl.shape[0], fh, stride, img_sz, _stream()),
              "mmt_corner_boxes_bwd")
        return d_tl, d_br, None, None, None


class _HipBoxLoss(torch.autograd.Function):
    """box_loss (MixFormerRGBTActor.compute_losses, actors/mixformer_rgbt.py:127-168; CIoU of box_ops.py:100-152)
    in one launch each way: pred cxcywh (B, 4), gt xywh (B, 4) -> (loss, ciou loss, l1, mean iou) as a (4,) fp32
    tensor; only the loss (entry 0) carries a gradient (mmt_box_loss / _bwd)."""

    @staticmethod
    def forward(ctx, pred, gt, iou_w, l1_w):
        from ._lib import LIB, check
        pred, gt = pred.float().reshape(-1, 4).contiguous(), gt.detach().float().reshape(-1, 4).contiguous()
        out = torch.empty(4, device=pred.device, dtype=torch.float32)
        check(LIB.mmt_box_loss(pred.data_ptr(), gt.data_ptr(), out.data_ptr(), pred.shape[0], float(iou_w), float(l1_w),
                               _stream()), "mmt_box_loss")
        ctx.save_for_backward(pred, gt)
        ctx.w = (float(iou_w), float(l1_w))
        return out

    @staticmethod
    def backward(ctx, dout):
        from ._lib import LIB, check
        pred, gt = ctx.saved_tensors
        dout = dout.float().contiguous()
        dpred = torch.empty_like(pred)
        check(LIB.mmt_box_loss_bwd(pred.data_ptr(), gt.data_ptr(), dout.data_ptr(), dpred.data_ptr(), pred.shape[0],
                                   *ctx.w, _stream()), "mmt_box_loss_bwd")
        return dpred, None, None, None


class _HipAddUp(torch.autograd.Function):
    """bf16(up(a) + b) on NHWC bf16 maps (mmt_add_up_bf16; up 1 = a plain add): the corner head's pyramid adds
    (head.py:187-189) at the lower of their two resolutions; backward: db = dout, da = its up x up block sums."""

    @staticmethod
    def forward(ctx, a, b, up):
        from ._lib import LIB, check
        B, H, W, C = b.shape
        if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or a.shape != (B, H // up, W // up, C):
            raise ValueError("HIP add_up: bf16 NHWC maps, a at 1/up of b")
        a, b = a.contiguous(), b.contiguous()
        out = torch.empty_like(b)
        check(LIB.mmt_add_up_bf16(a.data_ptr(), b.data_ptr(), out.data_ptr(), B, H, W, C, up, _stream()), "mmt_add_up_bf16")
        ctx.up, ctx.ashape = up, a.shape
        return out

    @staticmethod
    def backward(ctx, dout):
        from ._lib import LIB, check
        dout = dout.to(torch.bfloat16).contiguous()
        if ctx.up == 1:
            return dout, dout, None
        B, H, W, C = dout.shape
        da = torch.empty(ctx.ashape, device=dout.device, dtype=torch.bfloat16)
        check(LIB.mmt_upsample_sum_bf16(dout.data_ptr(), da.data_ptr(), B, H // ctx.up, W // ctx.up, C, ctx.up, _stream()),
              "mmt_upsample_sum_bf16")
        return da, dout, None


def _adjust_tokens(ops, seq, tok):
    """nn.Sequential(Conv2d 1x1, GroupNorm) of the fusion (fusion_utils.py:252-268) on token rows
    tok [B][P][Cin] -> [B][P][Cout] fp32: the 1x1 conv as ops.linear (HIP GEMM) and ops.group_norm."""
    conv, gn = seq[0], seq[1]
    B, P, Cin = tok.shape
    w = conv.weight.view(conv.weight.shape[0], Cin)
    y = ops.linear(tok.reshape(B * P, Cin).to(ops.dtype).contiguous(), w, conv.bias, out_f32=True)
    return ops.group_norm(y.view(B, P, -1), gn.weight, gn.bias, gn.num_groups, gn.eps)


def _mlp(ops, x, mlp):
    """timm Mlp (fc1 -> GELU -> fc2) of a block on x [M][C] in ops.dtype -> fp32: ops.mlp when the ops
    provide one (HipOps: fused GELU epilogues), else two ops.linear calls around aten's GELU."""
    fn = getattr(ops, "mlp", None)
    if fn is not None:
        return fn(x, mlp.fc1.weight, mlp.fc1.bias, mlp.fc2.weight, mlp.fc2.bias)
    h = ops.linear(x, mlp.fc1.weight, mlp.fc1.bias)
    h = F.gelu(h) if h.dtype == ops.dtype else F.gelu(h.float()).to(ops.dtype)  # bf16 in/out, fp32 math
    return ops.linear(h, mlp.fc2.weight, mlp.fc2.bias, out_f32=True)


def _layer_norm_pass(ops, x, a, b=None, eps=1e-6):
    """(_layer_norm(ops, x, a, b, eps), x'), x' = x for the residual op: with HipOps the pass-through output of
    the LayerNorm node (_HipLayerNormPass), so the two gradients of x are summed inside its backward kernel."""
    fn = getattr(ops, "layer_norm_pass", None)
    if fn is not None:
        return fn(x, a.weight, a.bias, eps, b.weight if b is not None else None, b.bias if b is not None else None)
    return _layer_norm(ops, x, a, b, eps), x


def _layer_norm(ops, x, a, b=None, eps=1e-6):
    """LayerNorm of the fp32 stream x to ops.dtype: norm module a on every row, or a on the first half of
    the rows and b on the second (per-modality norms of the shared backbone).  ops.layer_norm when the
    ops provide one (HipOps: the HIP kernels), else aten's (stand-in ops of the CPU tests)."""
    ln = getattr(ops, "layer_norm", None)
    if ln is not None:
        return ln(x, a.weight, a.bias, eps, b.weight if b is not None else None, b.bias if b is not None else None)
    C = x.shape[-1]
    if b is None:
        return F.layer_norm(x, (C,), a.weight, a.bias, eps).to(ops.dtype)
    h = x.shape[0] // 2
    return torch.cat([F.layer_norm(x[:h], (C,), a.weight, a.bias, eps),
                      F.layer_norm(x[h:], (C,), b.weight, b.bias, eps)], 0).to(ops.dtype)


class HipOps:
    """The backbone's matrix work on libmmt_hip.so (bf16 in, bf16 out)."""

    dtype = torch.bfloat16  # activation dtype of the GEMM / attention operands

    @staticmethod
    def layer_norm(x, w0, b0, eps, w1=None, b1=None, rows0=None, out_f32=False):
        """x [2h or n, ..., C] fp32 -> bf16 (fp32 with out_f32); (w1, b1) given: rows of the second half of
        dim 0 take them, or alternate blocks of rows0 rows when rows0 is given."""
        if w1 is not None and rows0 is None:
            rows0 = x.numel() // x.shape[-1] // 2
        return _HipLayerNorm.apply(x, w0, b0, w1, b1, rows0 or 0, eps, out_f32)

    @staticmethod
    def layer_norm_pass(x, w0, b0, eps, w1=None, b1=None):
        """(layer_norm(x, ...) in bf16, x passed through for the residual op) (_HipLayerNormPass)."""
        rows0 = x.numel() // x.shape[-1] // 2 if w1 is not None else 0
        return _HipLayerNormPass.apply(x, w0, b0, w1, b1, rows0, eps)

    @staticmethod
    def linear(x, weight, bias, out_f32=False):
        return _HipLinear.apply(x, weight, bias, out_f32)

    @staticmethod
    def group_norm(x, w, b, groups, eps):
        """GroupNorm over channels-last x [n][P][C] fp32 (_HipGroupNorm)."""
        return _HipGroupNorm.apply(x, w, b, groups, eps)

    @staticmethod
    def mlp(x, w1, b1, w2, b2):
        """fc2(GELU(fc1(x))), x [M][C] bf16 -> fp32 (_HipMlp)."""
        return _HipMlp.apply(x, w1, b1, w2, b2)

    @staticmethod
    def linear_residual(x, a, weight, bias, keep):
        """x + keep * Linear(a) (fp32 x, bf16 a, keep [B] per-sample scale or None) (_HipLinearResidual)."""
        return _HipLinearResidual.apply(x, a, weight, bias, keep)

    @staticmethod
    def mlp_residual(x, xn, w1, b1, w2, b2, keep):
        """x + keep * Mlp(xn) (_HipMlpResidual)."""
        return _HipMlpResidual.apply(x, xn, w1, b1, w2, b2, keep)

    @staticmethod
    def linear2(x, w0, b0, w1, b1, out_f32=False):
        """Linear of the stacked modalities, rows [0, M) with (w0, b0) and [M, 2M) with (w1, b1) (_HipLinear2)."""
        return _HipLinear2.apply(x, w0, b0, w1, b1, out_f32)

    @staticmethod
    def linear_residual2(x, a, w0, b0, w1, b1, keep):
        """linear_residual of the stacked modalities (_HipLinearResidual2; keep [2B] or None)."""
        return _HipLinearResidual2.apply(x, a, w0, b0, w1, b1, keep)

    @staticmethod
    def mlp_residual2(x, xn, p0, p1, keep):
        """mlp_residual of the stacked modalities; p0 / p1 = (w1, b1, w2, b2) of each (_HipMlpResidual2)."""
        return _HipMlpResidual2.apply(x, xn, *p0, *p1, keep)

    @staticmethod
    def mam_attention(qkv, n_t, heads):
        return _HipMamAttention.apply(qkv, n_t, heads)

    @staticmethod
    def mam_attention_asym(qkv, Bh, n_t, heads):
        return asym_attention_from_mam(HipOps.mam_attention, qkv, Bh, n_t, heads)

    @staticmethod
    def conv3x3(x, w, b, up=1, keep_pad=False, prep=None):
        """The corner head's 3x3 convolutions on NHWC maps (_HipConv3x3), operands cast to bf16 (autocast runs
        the nearest upsampling of the pyramid inputs in fp32); up: of the nearest upsampling of x (not
        materialised); keep_pad: 1-channel outputs in their 8-channel rows; prep: the weight layouts from
        conv_wprep (else made per call)."""
        return _HipConv3x3.apply(x.to(torch.bfloat16), w, b, up, keep_pad, prep)

    @staticmethod
    def conv_wprep(convs):
        """[(weight, bias)] of 3x3 convs -> their bf16 operand layouts, one launch (_conv_wprep)."""
        return _conv_wprep(convs)

    @staticmethod
    def add_up(a, b, up):
        """bf16(up(a) + b) on NHWC bf16 maps (_HipAddUp)."""
        return _HipAddUp.apply(a, b, up)

    @staticmethod
    def corner_score(x4, conv5, a3, a4):
        """conv5 (fp32) + up4(adjust3) + up2(adjust4) of one corner branch -> (B, fh*fh) fp32 (_HipCornerScore)."""
        return _HipCornerScore.apply(x4.contiguous(), conv5.weight, conv5.bias, a3, a4)

    @staticmethod
    def bn_relu(x, bn):
        """bn (nn.BatchNorm2d) then ReLU on an NHWC bf16 map (_HipBatchNormReLU), with the module's training /
        eval semantics: batch statistics when training or not tracking, running statistics updated (and
        num_batches_tracked advanced) when training and tracking."""
        if isinstance(bn, FrozenBatchNorm2d):  # fixed statistics and affine (buffers): eval semantics
            C = bn.weight.shape[0]
            x = x.to(torch.bfloat16)
            padded = x.shape[-1] != C  # 8-channel rows in: padded rows out
            if not padded and C % 8:
                x = F.pad(x, (0, (C + 7) // 8 * 8 - C))
            y = _HipBatchNormReLU.apply(x.contiguous(), bn.weight, bn.bias, bn.running_mean, bn.running_var, 0.0,
                                        bn.eps, False, C)
            return y if (padded or y.shape[-1] == C) else y[..., :C]
        training = bn.training or not bn.track_running_stats
        update = bn.training and bn.track_running_stats
        if update:
            if _BN_TRACKED is not None:  # head_forward_nhwc: one multi-tensor add for the whole head
                _BN_TRACKED.append(bn.num_batches_tracked)
            else:
                bn.num_batches_tracked.add_(1)
        keep = update or not training
        C = bn.num_features
        x = x.to(torch.bfloat16)
        padded = x.shape[-1] != C  # 8-channel rows in (a keep_pad conv): padded rows out, padding channels 0
        if not padded and C % 8:  # the 1-channel maps: 8-channel rows, padding channels ignored (autograd slices dy back)
            x = F.pad(x, (0, (C + 7) // 8 * 8 - C))
        y = _HipBatchNormReLU.apply(x.contiguous(), bn.weight, bn.bias, bn.running_mean if keep else None,
                                    bn.running_var if keep else None, bn.momentum, bn.eps, training, C)
        return y if (padded or y.shape[-1] == C) else y[..., :C]

    @staticmethod
    def corner_boxes(s_tl, s_br, fh, stride, img_sz):
        """Both corners' soft-argmax, normalised: (B, fh*fh) fp32 maps -> xyxy (B, 4) (_HipCornerBoxes)."""
        return _HipCornerBoxes.apply(s_tl, s_br, fh, stride, img_sz)

    @staticmethod
    def box_loss(pred_cxcywh, gt_xywh, iou_weight=2.0, l1_weight=5.0):
        """box_loss on mmt_box_loss (_HipBoxLoss): (loss, {"ciou", "l1", "iou"})."""
        out = _HipBoxLoss.apply(pred_cxcywh.view(-1, 4), gt_xywh, iou_weight, l1_weight)
        st = out.detach()
        return out[0], {"ciou": st[1], "l1": st[2], "iou": st[3]}

    @staticmethod
    def msda_bimodal(value, offw, ref, hw):
        """The bimodal MSDA middle of the training step, bf16 in / out (_HipMSDABimodal)."""
        return _HipMSDABimodal.apply(value, offw, ref, hw)

    @staticmethod
    def encoder_layer(layer, src, lpos, ref_q, hw, li):
        """One deformable encoder layer of the training step on the fused HIP ops (_encoder_layer_hip)."""
        return _encoder_layer_hip(layer, src, lpos, ref_q, hw, li)

    @staticmethod
    def ms_deform_attn(value, hw, loc, aw):
        """MSDeformAttnFunction (ms_deform_attn_func.py:22-38) on mmt_ms_deform_attn_forward / _backward,
        fp32 as the reference op; L levels of hw x hw."""
        from .functional import MSDeformAttnFunction
        L = loc.shape[3]
        shapes, starts = _const(("msda_levels", hw, L), value.device,
                                lambda: (torch.tensor([[hw, hw]] * L, dtype=torch.long),
                                         torch.arange(L, dtype=torch.long) * (hw * hw)))
        return MSDeformAttnFunction.apply(value, shapes, starts, loc, aw, 64)


def asym_attention_from_mam(mam, qkv, Bh, n_t, heads):
    """Cross-modal asymmetric MAM (asymmetric_shared.py:55-104) composed from two standard MAM
    attentions, so that training reuses the standard kernel pair (forward with log-sum-exp,
    mmt_mam_attention_bwd) and autograd routes the gradients back into qkv:
      - template queries of every sequence attend its own template keys: the standard attention of
        the sequence itself, template rows kept;
      - search queries of modality m attend [template_V | template_I | search_m]: the standard
        attention of the built sequence [tV | tI | s_m] with 2 n_t "template" rows, search rows kept.
    qkv: (2 Bh, ntok, 3C), RGB sequences first.  The discarded rows cost extra arithmetic (about 1.6x
    the attention FLOPs of the fused inference kernel) but no accuracy: their outputs get zero
    gradients, which contribute nothing to dq / dk / dv."""
    ntok = qkv.shape[1]
    own = mam(qkv, n_t, heads)
    t_v, t_i = qkv[:Bh, :n_t], qkv[Bh:, :n_t]
    tt = torch.cat([t_v, t_i], 1)  # (Bh, 2 n_t, 3C)
    built = torch.cat([torch.cat([tt, qkv[:Bh, n_t:]], 1), torch.cat([tt, qkv[Bh:, n_t:]], 1)], 0)
    cross = mam(built.contiguous(), 2 * n_t, heads)
    return torch.cat([own[:, :n_t], cross[:, 2 * n_t:]], 1)


# ----------------------------------------------------------------------------- forward
DROP_PATH_RATE = 0.1  # get_mixformer_vit drop_path_rate (mixformer.py:311, :324); timm linear per-block schedule


def _residual(x, y, p, training):
    """x + DropPath(y) (timm DropPath in mixformer.py:136-139: per-sample stochastic depth, survivors
    scaled by 1/(1-p)) as one fused multiply-add per element (torch.addcmul with the per-sample keep /
    (1 - p) scale) instead of three elementwise passes."""
    if not training or p <= 0.0:
        return x + y
    keep = y.new_empty((y.shape[0],) + (1,) * (y.dim() - 1)).bernoulli_(1.0 - p)
    return torch.addcmul(x, y, keep.div_(1.0 - p))


def _keep(x, p, training):
    """Per-sample DropPath scale (survivors 1 / (1 - p), others 0) for the fused residual GEMMs, or None."""
    if not training or p <= 0.0:
        return None
    return torch.empty(x.shape[0], device=x.device, dtype=torch.float32).bernoulli_(1.0 - p).div_(1.0 - p)


def _keeps(x, ps, training):
    """_keep for a list of rates at once (the residual branches of every block): one bernoulli draw and one
    division over [len(ps)][batch] instead of two small launches per branch (round 5: 44 per training step).
    Entries with rate 0 (or eval) are None, as _keep's."""
    live = [i for i, p in enumerate(ps) if training and p > 0.0]
    out = [None] * len(ps)
    if not live:
        return out
    q = _const(("keep_q", tuple(ps[i] for i in live)), x.device,
               lambda: torch.tensor([[1.0 - ps[i]] for i in live], dtype=torch.float32))
    k = torch.empty(len(live), x.shape[0], device=x.device, dtype=torch.float32).bernoulli_(q.expand(-1, x.shape[0]))
    k.div_(q)
    for j, i in enumerate(live):
        out[i] = k[j]
    return out


def _branch_residual(ops, x, a, lin, p, training):
    """x + DropPath(lin(a)) for the block's attention projection: one fused GEMM with HipOps."""
    fn = getattr(ops, "linear_residual", None)
    if fn is not None:
        return fn(x, a, lin.weight, lin.bias, _keep(x, p, training))
    B, ntok, C = x.shape
    return _residual(x, ops.linear(a, lin.weight, lin.bias, out_f32=True).view(B, ntok, C), p, training)


def _mlp_residual(ops, x, xn, mlp, p, training):
    """x + DropPath(Mlp(xn)): one fused autograd node with HipOps."""
    fn = getattr(ops, "mlp_residual", None)
    if fn is not None:
        return fn(x, xn, mlp.fc1.weight, mlp.fc1.bias, mlp.fc2.weight, mlp.fc2.bias, _keep(x, p, training))
    return _residual(x, _mlp(ops, xn, mlp).view(x.shape), p, training)


def _patches(x, p=16):
    """(B, C, H, W) -> (B, (H/p)(W/p), C p p): F.unfold(x, p, stride=p).transpose(1, 2) for non-overlapping
    patches (channel-major, then kernel row, kernel column; patches row-major), as one copy (aten's
    unfold launches one im2col kernel per sample)."""
    B, C, H, W = x.shape
    return x.view(B, C, H // p, p, W // p, p).permute(0, 2, 4, 1, 3, 5).reshape(B, (H // p) * (W // p), C * p * p)


def backbone_forward(bb, t, o, s, ops, drop_path_rate=DROP_PATH_RATE):
    """VisionTransformer.forward (mixformer.py:231-259) for one modality: returns the search
    features (B, C, gs, gs) fp32.  Tokens [template | online | search], pre-LN blocks; in training
    mode the blocks' residual branches use stochastic depth (mixformer.py:129-138)."""
    B = t.shape[0]
    C = bb.pos_embed_s.shape[-1]
    H = C // 64
    gt, gs = bb.grid_size_t, bb.grid_size_s
    ntok, n_t = 2 * gt * gt + gs * gs, 2 * gt * gt
    patches = torch.cat([_patches(x) for x in (t, o, s)], 1)  # (B, ntok, 3*256)
    w = bb.patch_embed.proj.weight
    x = ops.linear(patches.reshape(B * ntok, -1).to(ops.dtype), w.reshape(w.shape[0], -1), bb.patch_embed.proj.bias,
                   out_f32=True)
    pos = torch.cat([bb.pos_embed_t, bb.pos_embed_t, bb.pos_embed_s], 1)
    x = x.view(B, ntok, C) + pos
    depth = len(bb.blocks)
    for li, blk in enumerate(bb.blocks):
        dp = drop_path_rate * li / max(depth - 1, 1)
        xn, xr = _layer_norm_pass(ops, x, blk.norm1)
        qkv = ops.linear(xn.view(B * ntok, C), blk.attn.qkv.weight, blk.attn.qkv.bias).view(B, ntok, 3 * C)
        a = ops.mam_attention(qkv, n_t, H).view(B * ntok, C)
        x = _branch_residual(ops, xr, a, blk.attn.proj, dp, bb.training)
        xn, xr = _layer_norm_pass(ops, x, blk.norm2)
        x = _mlp_residual(ops, xr, xn.view(B * ntok, C), blk.mlp, dp, bb.training)
    xs = x[:, n_t:]
    return xs.transpose(1, 2).reshape(B, C, gs, gs)


def backbone_forward_pair(bv, bi, t, o, s, ops, drop_path_rate=DROP_PATH_RATE, tokens=False):
    """backbone_forward of the two-stream model's RGB (bv) and TIR (bi) backbones in lockstep, the
    modalities stacked on the batch ([rgb; tir], t / o / s pairs of (B, 3, H, W)): the same math per
    modality (mixformer.py:231-259, own weights, own norms, own DropPath draws), but every Linear and
    every gradient GEMM one grouped launch for both, and one attention / LayerNorm launch over 2B
    sequences.  Returns (s_v, s_i), each (B, C, gs, gs) fp32."""
    B = t[0].shape[0]
    C = bv.pos_embed_s.shape[-1]
    H = C // 64
    gt, gs = bv.grid_size_t, bv.grid_size_s
    ntok, n_t = 2 * gt * gt + gs * gs, 2 * gt * gt
    patches = torch.cat([_patches(torch.cat(x, 0)) for x in (t, o, s)], 1)  # (2B, ntok, 3*256)
    wv, wi = bv.patch_embed.proj.weight, bi.patch_embed.proj.weight
    x = ops.linear2(patches.reshape(2 * B * ntok, -1).to(ops.dtype), wv.reshape(wv.shape[0], -1),
                    bv.patch_embed.proj.bias, wi.reshape(wi.shape[0], -1), bi.patch_embed.proj.bias, out_f32=True)
    pos = torch.stack([torch.cat([bb.pos_embed_t, bb.pos_embed_t, bb.pos_embed_s], 1) for bb in (bv, bi)], 0)
    x = (x.view(2, B, ntok, C) + pos).view(2 * B, ntok, C)
    depth = len(bv.blocks)
    M2 = 2 * B * ntok
    keeps = _keeps(x, [drop_path_rate * (i // 2) / max(depth - 1, 1) for i in range(2 * depth)], bv.training)
    for li, (kv, ki) in enumerate(zip(bv.blocks, bi.blocks)):
        keep = keeps[2 * li]
        xn, xr = _layer_norm_pass(ops, x, kv.norm1, ki.norm1)
        qkv = ops.linear2(xn.view(M2, C), kv.attn.qkv.weight, kv.attn.qkv.bias, ki.attn.qkv.weight,
                          ki.attn.qkv.bias).view(2 * B, ntok, 3 * C)
        a = ops.mam_attention(qkv, n_t, H).view(M2, C)
        x = ops.linear_residual2(xr, a, kv.attn.proj.weight, kv.attn.proj.bias, ki.attn.proj.weight,
                                 ki.attn.proj.bias, keep)
        keep = keeps[2 * li + 1]
        xn, xr = _layer_norm_pass(ops, x, kv.norm2, ki.norm2)
        mp = [(k.mlp.fc1.weight, k.mlp.fc1.bias, k.mlp.fc2.weight, k.mlp.fc2.bias) for k in (kv, ki)]
        x = ops.mlp_residual2(xr, xn.view(M2, C), mp[0], mp[1], keep)
    if tokens:  # the search tokens as bf16 rows (2B, ns, C), RGB first, for the fusion's token-row adjust
        return _HipSearchTokens.apply(x, n_t), None
    xs = x[:, n_t:].transpose(1, 2).reshape(2 * B, C, gs, gs)
    return xs[:B], xs[B:]


def _backbones_rgbt(net, template, online_template, search, ops, dpr, tokens=False):
    """(s_v, s_i) of the two-stream model: the lockstep pair when the ops provide grouped Linears (HipOps),
    else one backbone after the other.  tokens (lockstep pair only): (the search tokens of both as bf16 rows (2B, ns,
    C), RGB first, None) instead of two (B, C, gs, gs) maps (fusion_forward takes either)."""
    if PAIR and getattr(ops, "linear2", None) is not None:
        return backbone_forward_pair(net.backbone_v, net.backbone_i, template, online_template, search, ops, dpr,
                                     tokens=tokens)
    return (backbone_forward(net.backbone_v, template[0], online_template[0], search[0], ops, dpr),
            backbone_forward(net.backbone_i, template[1], online_template[1], search[1], ops, dpr))


def backbone_forward_stacked(bb, t, o, s, ops, asym=False, drop_path_rate=DROP_PATH_RATE):
    """Shared-backbone forward with the modalities stacked on the batch ([rgb; tir], 2B):
    mixformer_shared.py:143-159, :253-282 (per-modality LayerNorms, shared weights, standard MAM) or,
    asym, asymmetric_shared.py:137-154, :236-266 (cross-modal MAM).  Returns the search features
    (2B, C, gs, gs) and the first template's tokens (2B, gt*gt, C) (the score decoder's memory)."""
    B2 = t.shape[0]
    Bh = B2 // 2
    C = bb.pos_embed_s.shape[-1]
    H = C // 64
    gt, gs = bb.grid_size_t, bb.grid_size_s
    ntok, n_t = 2 * gt * gt + gs * gs, 2 * gt * gt
    patches = torch.cat([_patches(x) for x in (t, o, s)], 1)
    w = bb.patch_embed.proj.weight
    x = ops.linear(patches.reshape(B2 * ntok, -1).to(ops.dtype), w.reshape(w.shape[0], -1), bb.patch_embed.proj.bias,
                   out_f32=True)
    pos = torch.cat([bb.pos_embed_t, bb.pos_embed_t, bb.pos_embed_s], 1)
    x = x.view(B2, ntok, C) + pos
    depth = len(bb.blocks)

    def ln2(x, a, b):  # norm*_v on the RGB half, norm*_i on the TIR half (and x passed through)
        return _layer_norm_pass(ops, x, a, b)

    for li, blk in enumerate(bb.blocks):
        dp = drop_path_rate * li / max(depth - 1, 1)
        xn, xr = ln2(x, blk.norm1_v, blk.norm1_i)
        qkv = ops.linear(xn.view(B2 * ntok, C), blk.attn.qkv.weight, blk.attn.qkv.bias).view(B2, ntok, 3 * C)
        a = ops.mam_attention_asym(qkv, Bh, n_t, H) if asym else ops.mam_attention(qkv, n_t, H)
        x = _branch_residual(ops, xr, a.reshape(B2 * ntok, C), blk.attn.proj, dp, bb.training)
        xn, xr = ln2(x, blk.norm2_v, blk.norm2_i)
        x = _mlp_residual(ops, xr, xn.view(B2 * ntok, C), blk.mlp, dp, bb.training)
    return x[:, n_t:].transpose(1, 2).reshape(B2, C, gs, gs), x[:, :gt * gt]


def _sine_pos(B, C, H, W, device):
    """PositionEmbeddingSine(C/2, normalize=True) on an all-valid mask (position_encoding.py:34-54)."""
    npf = C // 2
    ones = torch.ones(B, H, W, device=device)
    y = ones.cumsum(1)
    x = ones.cumsum(2)
    y = (y - 0.5) / (y[:, -1:, :] + 1e-6) * (2 * math.pi)
    x = (x - 0.5) / (x[:, :, -1:] + 1e-6) * (2 * math.pi)
    dim_t = 10000 ** (2 * (torch.arange(npf, device=device, dtype=torch.float32) // 2) / npf)
    px, py = x[..., None] / dim_t, y[..., None] / dim_t
    px = torch.stack((px[..., 0::2].sin(), px[..., 1::2].cos()), dim=4).flatten(3)
    py = torch.stack((py[..., 0::2].sin(), py[..., 1::2].cos()), dim=4).flatten(3)
    return torch.cat((py, px), dim=3).permute(0, 3, 1, 2)


def _ref_points(H, W, B, L, device):
    """get_reference_points (deformable_encoder_lnspecific.py:170-186), valid ratios 1."""
    ry, rx = torch.meshgrid(torch.linspace(0.5, H - 0.5, H, device=device), torch.linspace(0.5, W - 0.5, W, device=device),
                            indexing="ij")
    ref = torch.stack((rx.reshape(-1) / W, ry.reshape(-1) / H), -1)
    ref = torch.cat([ref] * L, 0)[None].expand(B, -1, -1)
    return ref[:, :, None].expand(B, ref.shape[1], L, 2)


def fusion_forward(fu, s_v, s_i, ops):
    """Attention_Fusion_Bimodal_LNSpecific.forward (fusion_utils.py:270-279) with the deformable
    encoder (deformable_encoder_lnspecific.py:131-160) and MSDeformAttn_Bimodal
    (ms_deform_attn_bimodal.py:83-130)."""
    tokens = getattr(ops, "group_norm", None) is not None  # adjust_* on token rows (HIP GEMM + GroupNorm)
    if s_i is None:  # both modalities' search tokens as bf16 rows (2B, ns, C) (_backbones_rgbt tokens=True)
        b, P, Cin = s_v.shape[0] // 2, s_v.shape[1], s_v.shape[2]
        h = w = int(round(P ** 0.5))
        if not tokens or h * w != P or getattr(ops, "linear2", None) is None:
            raise ValueError("fusion_forward: token-row inputs need the grouped token-row adjust (HipOps), square maps")
        cv, ci = fu.adjust_v[0], fu.adjust_i[0]
        y = ops.linear2(s_v.view(2 * b * P, Cin), cv.weight.view(cv.weight.shape[0], Cin), cv.bias,
                        ci.weight.view(ci.weight.shape[0], Cin), ci.bias, out_f32=True)
        gv, gi = fu.adjust_v[1], fu.adjust_i[1]
        if (gv.num_groups, gv.eps) != (gi.num_groups, gi.eps):
            raise ValueError("fusion_forward: the two adjust GroupNorms differ in groups / eps")
        av, ai = _HipGroupNorm2.apply(y.view(2 * b, P, -1), gv.weight, gv.bias, gi.weight, gi.bias, gv.num_groups,
                                      gv.eps)
        d = av.shape[2]
        src = torch.cat([av, ai], 1)
    elif tokens:
        b, _, h, w = s_v.shape
        av = _adjust_tokens(ops, fu.adjust_v, s_v.flatten(2).transpose(1, 2))
        ai = _adjust_tokens(ops, fu.adjust_i, s_i.flatten(2).transpose(1, 2))
        d = av.shape[2]
        src = torch.cat([av, ai], 1)
    else:
        b, _, h, w = s_v.shape
        av, ai = fu.adjust_v(s_v), fu.adjust_i(s_i)
        d = av.shape[1]
        src = torch.cat([av.flatten(2).transpose(1, 2), ai.flatten(2).transpose(1, 2)], 1)
    fa = fu.fusion_attention
    # the sine table depends on the shapes only: built once per shape and device (~20 small launches per step,
    # round 5).  The reference points stay computed on the device: they sit on pixel centres, where the bilinear
    # sampling's location gradient is discontinuous, and the host's linspace differs from the device's in the last
    # ulp -- enough to move the training gradients 0.17 -> 0.64 (relative L2) from the fp32 CPU reference in
    # test_module_forward_training_gpu_grads
    pos = _const(("sine_pos", b, d, h, w), s_v.device,
                 lambda: _sine_pos(b, d, h, w, "cpu").flatten(2).transpose(1, 2).contiguous())
    nl = 2 * h * w

    def lin(mod, x):  # the encoder's nn.Linear layers on the backbone's GEMM op (bf16 operands, as autocast)
        y = ops.linear(x.reshape(-1, x.shape[-1]).to(ops.dtype).contiguous(), mod.weight, mod.bias)
        return y.view(*x.shape[:-1], -1)

    sa0 = fa.encoder.layers[0].self_attn if len(fa.encoder.layers) else None
    fused_msda = (getattr(ops, "encoder_layer", None) is not None and sa0 is not None and h == w and
                  (sa0.n_heads, sa0.n_levels, sa0.n_points, d) == (8, 2, 4, 512) and h * w <= 484)
    if fused_msda:  # the reference points of the nl / 2 unique queries, one level: (h w, 2), computed on the
        # device as _ref_points does (its values, to the last ulp) once per shape
        ref_q = _const(("ref_q", h, w), s_v.device, lambda: _ref_points(h, w, 1, 2, s_v.device)[0, :h * w, 0, :].contiguous())
    else:
        ref = _ref_points(h, w, b, 2, s_v.device)
    # the level-embedded positions; the fused layers take them once (1, 2 nq, d), the batch rows being equal
    p1 = pos[:1] if fused_msda else pos
    lpos = torch.cat([p1 + fa.level_embed[0].view(1, 1, -1), p1 + fa.level_embed[1].view(1, 1, -1)], 1)
    if fused_msda:  # round 6: every encoder layer on the fused HIP ops
        if any(m.training and m.p > 0 for m in fa.encoder.modules() if isinstance(m, torch.nn.Dropout)):
            _drop_rng(src.device)[1:].add_(1)  # this step's dropout draws (one captured add)
        for li, layer in enumerate(fa.encoder.layers):
            src = ops.encoder_layer(layer, src, lpos, ref_q, h, li)
    for layer in (fa.encoder.layers if not fused_msda else ()):
        sa = layer.self_attn
        query = src + lpos
        q_bi = torch.cat(torch.chunk(query, 2, 1), dim=2)
        value = lin(sa.value_proj, src).view(b, nl, sa.n_heads, d // sa.n_heads)
        # The reference repeats the bimodal query's offsets / weights on both halves of its nl queries
        # (ms_deform_attn_bimodal.py:113-118), and the two halves' reference points are the same cells, so both
        # halves sample identically: sample the nl / 2 unique queries once and repeat the projected output
        # (autograd of the repeat sums the halves' gradients, exactly the gradient of the reference's repeat).
        off = lin(sa.sampling_offsets, q_bi).view(b, nl // 2, sa.n_heads, sa.n_levels, sa.n_points, 2)
        aw = lin(sa.attention_weights, q_bi).view(b, nl // 2, sa.n_heads, sa.n_levels * sa.n_points)
        aw = F.softmax(aw.float(), -1).view(b, nl // 2, sa.n_heads, sa.n_levels, sa.n_points)
        wh = _const(("loc_norm", w, h), src.device, lambda: torch.tensor([w, h], dtype=torch.float32))
        loc = ref[:, :nl // 2, None, :, None, :] + off.float() / wh
        src2 = lin(sa.output_proj, ops.ms_deform_attn(value.float().contiguous(), h, loc.contiguous(), aw.contiguous()))
        src2 = torch.cat([src2, src2], 1)
        src = src + layer.dropout1(src2)
        src = _ln_halves(ops, src, layer.norm1_v, layer.norm1_i)
        src = src + layer.dropout3(lin(layer.linear2, layer.dropout2(F.relu(lin(layer.linear1, src)))))
        src = _ln_halves(ops, src, layer.norm2_v, layer.norm2_i)
    o_v, o_i = torch.chunk(src, 2, 1)
    if tokens:  # channel concat on token rows, then back to NCHW for the corner head's convolutions
        y = _adjust_tokens(ops, fu.adjust_cat, torch.cat([o_v, o_i], 2))
        return y.transpose(1, 2).reshape(b, -1, h, w)
    o_v = o_v.permute(0, 2, 1).reshape(b, -1, h, w)
    o_i = o_i.permute(0, 2, 1).reshape(b, -1, h, w)
    return fu.adjust_cat(torch.cat([o_v, o_i], 1))


def _encoder_layer_hip(layer, src, lpos, ref_q, hw, li):
    """DeformableTransformerEncoderLayer.forward (deformable_encoder_lnspecific.py:131-148) with
    MSDeformAttn_Bimodal (ms_deform_attn_bimodal.py:83-130) on the fused HIP ops: the bimodal query and the bf16
    value operand in one pass (_HipQueryPrep), value_proj, [sampling_offsets | attention_weights] as one GEMM
    (_HipLinearCat), the sampling (_HipMSDABimodal), output_proj, the duplicated-halves dropout-residual
    (_HipDropResidual), norm1, the FFN with its dropouts and residual (_HipEncoderFFN), norm2.  src (B, 2 nq, d)
    fp32 -> fp32.  Dropout draws: salts 8 li + 1 .. 8 li + 3."""
    sa = layer.self_attn
    B, n2, d = src.shape
    M = B * n2
    drop = lambda m: m.p if m.training else 0.0  # noqa: E731
    qbi, srcb, src = _HipQueryPrep.apply(src, lpos)
    value = HipOps.linear(srcb.view(M, d), sa.value_proj.weight, sa.value_proj.bias).view(B, n2, d)
    offw = _HipLinearCat.apply(qbi.view(M // 2, 2 * d), sa.sampling_offsets.weight, sa.sampling_offsets.bias,
                               sa.attention_weights.weight, sa.attention_weights.bias).view(B, n2 // 2, -1)
    ms = HipOps.msda_bimodal(value, offw, ref_q, hw)
    src2 = HipOps.linear(ms.view(M // 2, d), sa.output_proj.weight, sa.output_proj.bias).view(B, n2 // 2, d)
    src = _HipDropResidual.apply(src, src2, drop(layer.dropout1), 8 * li + 1, True)
    src = _ln_halves(HipOps, src, layer.norm1_v, layer.norm1_i)
    src = _HipEncoderFFN.apply(src.view(M, d), layer.linear1.weight, layer.linear1.bias, layer.linear2.weight,
                               layer.linear2.bias, drop(layer.dropout2), drop(layer.dropout3), 8 * li + 1)
    return _ln_halves(HipOps, src.view(B, n2, d), layer.norm2_v, layer.norm2_i)


def _ln_halves(ops, src, nv, ni):
    """The LN-specific encoder's norms (deformable_encoder_lnspecific.py:94-148): nv on the first half of
    every sequence's tokens, ni on the second, fp32 -> fp32 (ops.layer_norm's alternating row groups; the
    aten path chunks and concatenates)."""
    ln = getattr(ops, "layer_norm", None)
    if ln is not None:
        return ln(src, nv.weight, nv.bias, nv.eps, ni.weight, ni.bias, rows0=src.shape[1] // 2, out_f32=True)
    s1, s2 = torch.chunk(src, 2, 1)
    return torch.cat([nv(s1), ni(s2)], 1)


def _soft_argmax(score_map, stride):
    """head.py:200-212, coord grids :138-145 (x = stride * col, y = stride * row)."""
    B, _, H, W = score_map.shape

    def grids():
        idx = torch.arange(0, H).view(-1, 1) * stride
        return idx.repeat((H, 1)).view((H * W,)).float(), idx.repeat((1, H)).view((H * W,)).float()
    coord_x, coord_y = _const(("softargmax", H, W, stride), score_map.device, grids)  # (shape constants: cached)
    prob = F.softmax(score_map.float().view(-1, H * W), dim=1)
    return (coord_x * prob).sum(1), (coord_y * prob).sum(1)


def _hip_bn_ok(bn):
    """The conv() block norms the HIP batch norm computes with the module's own semantics: BatchNorm2d with a
    momentum, SyncBatchNorm when its statistics are local (eval, or a process group of one rank: SyncBatchNorm
    then runs F.batch_norm itself), and FrozenBatchNorm2d (fixed statistics and affine, lib/models/mixformer_cvt/
    utils.py:21-57)."""
    if isinstance(bn, FrozenBatchNorm2d):
        return True
    if type(bn) is torch.nn.SyncBatchNorm:
        if bn.momentum is None:
            return False
        if not bn.training:
            return True
        import torch.distributed as dist
        pg = bn.process_group
        return not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(pg) == 1
    return type(bn) is torch.nn.BatchNorm2d and bn.momentum is not None


_BN_TRACKED = None  # head_forward_nhwc: the num_batches_tracked counters its batch norms advance, added at its end

HEAD_SCORE_FP32 = True  # head_forward_nhwc: the 48 -> 1 conv5 in fp32 (False: bf16 under autocast, as aten's path)


def head_forward_nhwc(hd, x, ops):
    """head_forward with NHWC maps and the 3x3 convolutions on ops.conv3x3 (HIP): _head_forward_nhwc, with the
    HIP batch norms' num_batches_tracked advances gathered into one multi-tensor add at the end."""
    global _BN_TRACKED
    outer, _BN_TRACKED = _BN_TRACKED, ([] if getattr(ops, "bn_relu", None) is not None else None)
    try:
        out = _head_forward_nhwc(hd, x, ops)
        if _BN_TRACKED:
            torch._foreach_add_(_BN_TRACKED, 1)
    finally:
        _BN_TRACKED = outer
    return out


def _head_forward_nhwc(hd, x, ops):
    """head_forward with NHWC maps and the 3x3 convolutions on ops.conv3x3 (HIP): every conv() block =
    conv (HIP) -> BatchNorm2d + ReLU on ops.bn_relu (HIP, the module's statistics semantics and running-stat
    updates); SyncBatchNorm (its RCCL statistics), FrozenBatchNorm2d and the 1-channel maps call the modules
    on the NCHW map as the reference runs them.  Nearest upsampling, the pyramid adds, the 48 -> 1 1x1 convs
    and the soft-argmax stay PyTorch ops (head.py:147-212)."""
    nchw = lambda t: t.permute(0, 3, 1, 2)  # noqa: E731
    nhwc = lambda t: t.permute(0, 2, 3, 1)  # noqa: E731

    bn_relu = getattr(ops, "bn_relu", None)
    # every 3x3 conv's bf16 weight layouts in one launch (round 6; the weights are fixed within the step)
    convs = [m for m in hd.modules() if isinstance(m, torch.nn.Conv2d) and m.kernel_size == (3, 3)]
    wprep = getattr(ops, "conv_wprep", None)
    prep = dict(zip(map(id, convs), wprep([(m.weight, m.bias) for m in convs]))) if wprep is not None and convs else {}
    conv3x3 = lambda m, t, **kw: ops.conv3x3(t, m.weight, m.bias, prep=prep[id(m)], **kw) if id(m) in prep \
        else ops.conv3x3(t, m.weight, m.bias, **kw)  # noqa: E731

    def block(seq, t):  # conv(): Conv2d 3x3 + BN + ReLU (head.py:7-20)
        y = conv3x3(seq[0], t.contiguous())
        bn = seq[1]
        if bn_relu is not None and type(seq[2]) is torch.nn.ReLU and _hip_bn_ok(bn):
            return bn_relu(y, bn)  # HIP batch norm + ReLU on the NHWC map
        # SyncBatchNorm in a process group of more than one rank (its RCCL statistics) and cumulative-average
        # BatchNorm (momentum None): the module on a contiguous NCHW map as the reference runs it (MIOpen's
        # batch norm on the channels-last view of a bf16 map crashed in train mode: DESIGN.md §7)
        return nhwc(seq[2](bn(nchw(y).contiguous()))).contiguous()

    def c1(mod, t):  # Conv2d(48, 1, 1) on channels-last rows
        if not HEAD_SCORE_FP32:
            return F.linear(t, mod.weight.view(mod.weight.shape[0], -1), mod.bias)
        # fp32 (autocast off): the score map feeds the soft-argmax directly, and conv5's output is its largest
        # term, so its bf16 rounding was the largest single error on the corners (tools/head_stage_error.py)
        with torch.autocast(t.device.type, enabled=False):
            return F.linear(t.float(), mod.weight.view(mod.weight.shape[0], -1).float(), mod.bias.float())

    def up(t, f):
        return nhwc(F.interpolate(nchw(t), scale_factor=f))

    xh = nhwc(x).to(torch.bfloat16).contiguous()
    coords, maps = [], {}
    boxes = getattr(ops, "corner_boxes", None)  # both soft-argmaxes + normalisation in one op (round 6)
    score, add_up = getattr(ops, "corner_score", None), getattr(ops, "add_up", None)
    fused = score is not None and add_up is not None and HEAD_SCORE_FP32 and bn_relu is not None
    for br in ("tl", "br"):
        g = lambda n: getattr(hd, n + "_" + br)  # noqa: E731
        x1 = block(g("conv1"), xh)
        x2 = block(g("conv2"), x1)
        a3, a4 = g("adjust3"), g("adjust4")
        if fused and all(_hip_bn_ok(m[1]) and type(m[2]) is torch.nn.ReLU
                         for m in (g("conv3"), g("conv4"), a3[2], a4[1])):
            # round 6: the pyramid's nearest upsamplings folded into the convolutions that consume them (exact:
            # nearest upsampling commutes with the add of two maps at one resolution, and rounding the fp32 sum to
            # bf16 before or after upsampling gives the same values), the adds on HIP, the 1-channel maps kept in
            # their 8-channel rows, and conv5 + up4(adjust3) + up2(adjust4) in one HIP op
            def blk(seq, t, up=1, keep_pad=False):
                return bn_relu(conv3x3(seq[0], t, up=up, keep_pad=keep_pad), seq[1])
            x3 = blk(g("conv3"), add_up(block(g("adjust1"), xh), x2, 1), up=2)  # conv3(up2(adjust1 + x2))
            x4 = blk(g("conv4"), add_up(block(g("adjust2"), xh), x3, 2), up=2)  # conv4(up2(up2(adjust2) + x3))
            m3 = blk(a3[2], block(a3[1], block(a3[0], x2)), keep_pad=True)
            m4 = blk(a4[1], block(a4[0], x3), keep_pad=True)
            fh = x4.shape[1]
            sm = score(x4, g("conv5"), m3, m4)  # (B, fh * fh) fp32 (padded rows in)
            maps[br] = sm
            if boxes is None:
                coords += list(_soft_argmax(sm.view(-1, 1, fh, fh), hd.stride))
            continue
        x3 = block(g("conv3"), up(block(g("adjust1"), xh), 2) + up(x2, 2))
        x4 = block(g("conv4"), up(block(g("adjust2"), xh), 4) + up(x3, 2))
        m3, m4 = block(a3[2], block(a3[1], block(a3[0], x2))), block(a4[1], block(a4[0], x3))
        if score is not None and HEAD_SCORE_FP32 and m3.dtype == torch.bfloat16 and m4.dtype == torch.bfloat16:
            fh = x4.shape[1]
            sm = score(x4, g("conv5"), m3, m4).view(-1, 1, fh, fh)  # (B, 1, fh, fh) fp32
            coords += list(_soft_argmax(sm, hd.stride))
            continue
        sm = c1(g("conv5"), x4) + up(m3, 4) + up(m4, 2)
        coords += list(_soft_argmax(nchw(sm), hd.stride))
    if boxes is not None and len(maps) == 2:
        fh = int(round(maps["tl"].shape[1] ** 0.5))
        return boxes(maps["tl"], maps["br"], fh, hd.stride, hd.img_sz)
    if len(coords) < 4:  # the fused path ran for one branch only: that branch's soft-argmax now
        for br in ("tl", "br"):
            if br in maps:
                fh = int(round(maps[br].shape[1] ** 0.5))
                c = list(_soft_argmax(maps[br].view(-1, 1, fh, fh), hd.stride))
                coords = c + coords if br == "tl" else coords + c
    return torch.stack(coords, dim=1) / hd.img_sz


def head_forward(hd, x, ops=None):
    """Pyramid_Corner_Predictor.forward / get_score_map (head.py:147-212) -> (B, 4) xyxy in [0, 1].  With ops
    providing conv3x3 (HipOps) the convolutions run on the HIP GEMM (head_forward_nhwc)."""
    if getattr(ops, "conv3x3", None) is not None:
        return head_forward_nhwc(hd, x, ops)
    up = lambda t, f: F.interpolate(t, scale_factor=f)  # noqa: E731
    coords = []
    for br in ("tl", "br"):
        g = lambda n: getattr(hd, n + "_" + br)  # noqa: E731
        x1 = g("conv1")(x)
        x2 = g("conv2")(x1)
        x3 = g("conv3")(up(g("adjust1")(x), 2) + up(x2, 2))
        x4 = g("conv4")(up(g("adjust2")(x), 4) + up(x3, 2))
        sm = g("conv5")(x4) + up(g("adjust3")(x2), 4) + up(g("adjust4")(x3), 2)
        coords += list(_soft_argmax(sm, hd.stride))
    return torch.stack(coords, dim=1) / hd.img_sz


def _token_rows(ops):
    """The backbones hand the fusion bf16 token rows (HipOps: the lockstep pair and the token-row adjust)."""
    return PAIR and TOKEN_ROWS and all(getattr(ops, n, None) is not None for n in ("linear2", "group_norm"))


TOKEN_ROWS = True  # False: NCHW search maps between backbone and fusion (the pre-round-6 chain; A/B knob)


def forward_boxes(net, template, online_template, search, ops):
    """MixFormer_RGBT.forward (mixformer.py:366-395) + forward_box_head (:419-432): pred_boxes
    (B, 1, 4) cxcywh.  Stochastic depth at the module's drop_path_rate (as module_forward)."""
    dpr = getattr(net, "drop_path_rate", DROP_PATH_RATE)
    s_v, s_i = _backbones_rgbt(net, template, online_template, search, ops, dpr, tokens=_token_rows(ops))
    with torch.autocast(s_v.device.type, dtype=torch.bfloat16, enabled=s_v.device.type == "cuda"):
        fused = fusion_forward(net.fusion_vi, s_v, s_i, ops)
        xyxy = head_forward(net.box_head, fused, ops)
    x0, y0, x1, y1 = xyxy.float().unbind(-1)
    return torch.stack([(x0 + x1) / 2, (y0 + y1) / 2, (x1 - x0), (y1 - y0)], -1).view(-1, 1, 4)


def module_forward(net, template, online_template, search, ops, run_score_head=False, gt_bboxes=None):
    """The drop-in module's forward with autograd (net.train() under grad mode; what the reference's
    MixFormerRGBTActor calls, actors/mixformer_rgbt.py:82-98, possibly wrapped in DDP + SyncBN,
    train_script_mixformer.py:105-110): MixFormer_RGBT.forward (mixformer.py:366-395),
    mixformer_shared.py:400-424, asymmetric_shared.py:349-368 and asymmetric_shared_online.py:351-413
    (score head on the predicted boxes: gt_bboxes is accepted and ignored, as the reference's forward
    drops it at asymmetric_shared_online.py:374).  Returns
    ({"pred_boxes": (B,1,4)[, "pred_scores": (B,)]}, (B,1,4))."""
    variant = net.variant
    dpr = getattr(net, "drop_path_rate", DROP_PATH_RATE)
    if variant == "rgbt":
        s_v, s_i = _backbones_rgbt(net, template, online_template, search, ops, dpr, tokens=_token_rows(ops))
        tok = None
    elif variant in ("shared", "asym", "asym_online"):
        feats, tok = backbone_forward_stacked(net.backbone, torch.cat(template, 0), torch.cat(online_template, 0),
                                              torch.cat(search, 0), ops, asym=variant != "shared", drop_path_rate=dpr)
        s_v, s_i = feats.chunk(2, 0)
    else:
        raise NotImplementedError("training forward of %s (candidate elimination with autograd) is not built; "
                                  "its inference forward runs under eval() / no_grad()" % variant)
    with torch.autocast(s_v.device.type, dtype=torch.bfloat16, enabled=s_v.device.type == "cuda"):
        fused = fusion_forward(net.fusion_vi, s_v, s_i, ops)
        xyxy = head_forward(net.box_head, fused, ops)
    x0, y0, x1, y1 = xyxy.float().unbind(-1)
    coord = torch.stack([(x0 + x1) / 2, (y0 + y1) / 2, (x1 - x0), (y1 - y0)], -1).view(-1, 1, 4)
    out = {"pred_boxes": coord}
    if run_score_head and variant == "asym_online":
        B = coord.shape[0]
        gt = tok.shape[1]
        g = int(round(gt ** 0.5))
        C = tok.shape[-1]
        t_v, t_i = tok[:B].transpose(1, 2).reshape(B, C, g, g), tok[B:].transpose(1, 2).reshape(B, C, g, g)
        templ = torch.cat([t_v, t_i], 2)
        # box_cxcywh_to_xyxy(outputs_coord.clone()) (asymmetric_shared_online.py:408-409)
        xc, yc, w, h = coord.clone().view(-1, 4).unbind(-1)
        rois = torch.stack([xc - 0.5 * w, yc - 0.5 * h, xc + 0.5 * w, yc + 0.5 * h], -1)
        out["pred_scores"] = score_decoder_forward(net.score_branch, fused.float(), templ.float(), rois.float())
    return out, coord


# ----------------------------------------------------------------------------- loss / optimizer
def ciou_loss(b1, b2):
    """lib/utils/box_ops.py:100-152 for equal-length (N, 4) xyxy sets: (mean(1 - ciou), iou).  The x and y terms
    are computed as (N, 2) pairs with the reference's operations in its order (same values; round 5: half the small
    launches of the scalar-column form, forward and backward)."""
    wh1, wh2 = b1[:, 2:] - b1[:, :2], b2[:, 2:] - b2[:, :2]
    c1, c2 = (b1[:, :2] + b1[:, 2:]) / 2.0, (b2[:, :2] + b2[:, 2:]) / 2.0
    lo1, hi1 = c1 - wh1 / 2, c1 + wh1 / 2
    lo2, hi2 = c2 - wh2 / 2, c2 + wh2 / 2
    iwh = torch.clamp(torch.min(hi1, hi2) - torch.max(lo1, lo2), min=0)
    inter = iwh[:, 0] * iwh[:, 1]
    ewh = torch.clamp(torch.max(hi1, hi2) - torch.min(lo1, lo2), min=0) ** 2
    d2 = (c2 - c1) ** 2
    inter_diag = d2[:, 0] + d2[:, 1]
    c_diag = ewh[:, 0] + ewh[:, 1]
    union = wh1[:, 0] * wh1[:, 1] + wh2[:, 0] * wh2[:, 1] - inter
    u = inter_diag / c_diag
    iou = inter / union
    v = (4 / (math.pi ** 2)) * torch.pow(torch.atan(wh2[:, 0] / wh2[:, 1]) - torch.atan(wh1[:, 0] / wh1[:, 1]), 2)
    with torch.no_grad():
        alpha = (iou > 0.5).float() * v / (1 - iou + v)
    cious = torch.clamp(iou - u - alpha * v, min=-1.0, max=1.0)
    return torch.mean(1 - cious), iou


def box_loss(pred_cxcywh, gt_xywh, iou_weight=2.0, l1_weight=5.0):
    """MixFormerRGBTActor.compute_losses (actors/mixformer_rgbt.py:127-168)."""
    p = pred_cxcywh.view(-1, 4)
    pred = torch.cat([p[:, :2] - 0.5 * p[:, 2:], p[:, :2] + 0.5 * p[:, 2:]], -1)
    gt = torch.cat([gt_xywh[:, :2], gt_xywh[:, :2] + gt_xywh[:, 2:]], -1).clamp(min=0.0, max=1.0)
    ciou, iou = ciou_loss(pred, gt)
    l1 = F.l1_loss(pred, gt)
    return iou_weight * ciou + l1_weight * l1, {"ciou": ciou.detach(), "l1": l1.detach(), "iou": iou.detach().mean()}


def param_groups(net, lr):
    """base_functions.py:362-400 (rgbt strategy): pos_embed frozen; backbone_i 0.1 lr, backbone_v
    0.02 lr, box_head 0.02 lr, fusion 1.0 lr except sampling_offsets / reference_points 0.1 lr."""
    named = list(net.named_parameters())
    for n, p in named:
        p.requires_grad = "pos_embed" not in n
    proj = ("reference_points", "sampling_offsets")
    sel = lambda f: [p for n, p in named if p.requires_grad and f(n)]  # noqa: E731
    return [
        {"params": sel(lambda n: "backbone_i" in n), "lr": 0.1 * lr},
        {"params": sel(lambda n: "backbone_v" in n), "lr": 0.02 * lr},
        {"params": sel(lambda n: "box_head" in n), "lr": 0.02 * lr},
        {"params": sel(lambda n: "fusion_vi" in n and not any(k in n for k in proj))},
        {"params": sel(lambda n: "fusion_vi" in n and any(k in n for k in proj)), "lr": 0.1 * lr},
    ]


def synthetic_batch(B, device, generator=None, template=128, search=320):
    """LaSOT-shaped synthetic pairs: N(0,1) images, search box label xywh with the
    centre at 0.5 +- 0.1 and the size in [0.1, 0.5] (normalised to the search crop)."""
    g = generator
    t = [torch.randn(B, 3, template, template, generator=g).to(device) for _ in range(2)]
    o = [torch.randn(B, 3, template, template, generator=g).to(device) for _ in range(2)]
    s = [torch.randn(B, 3, search, search, generator=g).to(device) for _ in range(2)]
    wh = 0.1 + 0.4 * torch.rand(B, 2, generator=g)
    c = 0.5 + 0.2 * (torch.rand(B, 2, generator=g) - 0.5)
    return t, o, s, torch.cat([c - wh / 2, wh], 1).to(device)


# GradBucketAllReduce: bucket all-reduces issued asynchronously and joined after the backward (False: each joined
# at its launch, the form measured before round 6's end; A/B tools only)
ALLREDUCE_ASYNC = True


class GradBucketAllReduce:
    """Data-parallel gradient averaging (what DistributedDataParallel's reducer does for the reference,
    train_script_mixformer.py:104-110, run_training_ddp.py:94) issued by the step itself on its own
    stream, so that the whole DDP step can be captured as one hipGraph (RCCL collectives record into a
    graph; DDP's reducer does host-side bookkeeping that does not).

    Buckets: the trainable parameters in reverse registration order (the order their gradients appear in
    the backward), cut at `cap_bytes` of fp32 (one ViT block's parameters by default, ~27 MB at ViT-B).
    A post-accumulate-grad hook on every parameter counts a bucket's arrivals; the last one launches the
    bucket's all-reduce at once, asynchronously (the process group's stream), so a block's exchange overlaps
    the backward of the blocks below it; finish() joins them in launch order and copies the averages back.
    A bucket is one flat buffer (the gradients concatenated, divided by the world size, in fp32 or
    rounded to bf16 with compress="bf16") and one all-reduce; the parameters' .grad then become views of the
    averaged fp32 bucket (bf16 buckets: one multi-tensor copy back into the fp32 .grad tensors).  finish() launches buckets whose parameters did not all receive a gradient, in bucket
    order (every rank runs the same graph, so every rank launches the same sequence)."""

    def __init__(self, params, world, group=None, cap_bytes=None, compress="none"):
        import torch.distributed as dist
        if compress not in (None, "none", "bf16"):
            raise ValueError("grad_compress: 'bf16' or 'none'")
        self.dist, self.group, self.world = dist, group, world
        self.dtype = torch.bfloat16 if compress == "bf16" else None
        params = [p for p in params if p.requires_grad][::-1]
        cap = cap_bytes or 25 * 2 ** 20
        self.buckets, cur, size = [], [], 0
        for p in params:
            if cur and size + p.numel() * 4 > cap:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += p.numel() * 4
        if cur:
            self.buckets.append(cur)
        self.bucket_of = {}
        for i, b in enumerate(self.buckets):
            for p in b:
                self.bucket_of[id(p)] = i
        self.handles = [p.register_post_accumulate_grad_hook(self._arrived) for p in params]
        self.begin()

    def begin(self):
        self.left = [len(b) for b in self.buckets]
        self.done = [False] * len(self.buckets)
        self.pending = []  # (work, flat bucket, its .grad tensors) of the launched, not yet joined all-reduces

    def _arrived(self, p):
        i = self.bucket_of[id(p)]
        self.left[i] -= 1
        if self.left[i] == 0:
            self._launch(i)

    def _launch(self, i):
        self.done[i] = True
        ps = [p for p in self.buckets[i] if p.grad is not None]
        grads = [p.grad for p in ps]
        if not grads:
            return
        flat = torch.cat([g.reshape(-1) for g in grads])
        if self.dtype is not None:
            flat = flat.to(self.dtype)
        if self.world > 1:
            flat.div_(self.world)
        # asynchronous: the collective runs on the process group's own stream (RCCL: after an event on the step's
        # stream), so the backward of the blocks below keeps the step's stream busy meanwhile; finish() joins it
        work = self.dist.all_reduce(flat, group=self.group, async_op=ALLREDUCE_ASYNC)
        self.pending.append((work, flat, ps, grads))

    def finish(self):
        for i in range(len(self.buckets)):
            if not self.done[i]:
                self._launch(i)
        for work, flat, ps, grads in self.pending:  # in launch order: the step's stream waits, then the averages
            if work is not None:
                work.wait()
            views = [v.view_as(g) for v, g in zip(flat.split([g.numel() for g in grads]), grads)]
            if self.dtype is None:  # fp32 buckets: the parameters' .grad become views of the averaged bucket (no copy)
                for p, v in zip(ps, views):
                    p.grad = v
            else:  # bf16 buckets: the averages rounded back into the fp32 .grad tensors
                torch._foreach_copy_(grads, views)
        self.pending = []

    def remove(self):
        for h in self.handles:
            h.remove()


class TrainStep:
    """One optimisation step: forward, loss, backward, (data-parallel gradient all-reduce), clip, AdamW.

    net: the two-stream model (mmt_amd.model.build_mixformer_vit_rgbt) on the device.
    ddp: False (one process), True (GradBucketAllReduce over the default process group: bucketed RCCL
    all-reduce launched from the backward's gradient hooks, capturable with the rest of the step), or
    "torch" (torch.nn.parallel.DistributedDataParallel around the step's module, the reference's wrap;
    eager only).  grad_compress: "none" (fp32 buckets, the reference's semantics, the default) or "bf16"
    (buckets rounded to bf16: half the bytes on the links, an explicit numerics deviation)."""

    def __init__(self, net, ops, lr=1e-4, weight_decay=1e-4, grad_clip=0.1, iou_weight=2.0, l1_weight=5.0,
                 ddp=False, grad_compress="none"):
        self.net = net
        self.ops = ops
        self.grad_clip, self.iou_weight, self.l1_weight = grad_clip, iou_weight, l1_weight
        self._captured_hparams = None
        self.reducer = None
        # on the device: clip + AdamW as three launches over every parameter (mmt_amd.optim.HipAdamW,
        # which also keeps the bf16 copies of the backbone Linear weights the GEMMs read); on the
        # host (stand-in ops in tests): torch.optim.AdamW + clip_grad_norm_
        groups = param_groups(net, lr)
        if next(net.parameters()).is_cuda:
            from .optim import HipAdamW
            shadow = [m.weight for m in net.modules()
                      if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d)) and m.weight.requires_grad]
            self.opt = HipAdamW(groups, lr=lr, weight_decay=weight_decay, shadow=shadow, set_to_none=True)
        else:
            self.opt = torch.optim.AdamW(groups, lr=lr, weight_decay=weight_decay)
        self.hip_opt = next(net.parameters()).is_cuda
        if ddp and next(net.parameters()).is_cuda:  # train_script_mixformer.py:105
            net = self.net = torch.nn.SyncBatchNorm.convert_sync_batchnorm(net)
        if grad_compress not in (None, "none", "bf16"):
            raise ValueError("grad_compress: 'bf16' or 'none'")
        # Gradient all-reduce over RCCL (xGMI rings): buckets of one ViT block's gradients (about 27 MiB of
        # fp32 for ViT-B), so a block's all-reduce starts as soon as its backward is done and overlaps the
        # next block's, in ~12 buckets per backbone instead of a 25 MiB cut through the layers.
        blocks = [m for m in net.modules() if type(m).__name__ in ("Block", "Block_Shared", "Block_Asym")]
        cap_mb = max((sum(p.numel() for p in b.parameters()) for b in blocks), default=0) * 4 / 2 ** 20
        cap_mb = cap_mb if cap_mb > 0 else 25
        if ddp == "torch":
            self.model = torch.nn.parallel.DistributedDataParallel(_Wrapped(net, ops), broadcast_buffers=False,
                                                                   bucket_cap_mb=cap_mb)
            if grad_compress == "bf16":
                from torch.distributed.algorithms.ddp_comm_hooks import default_hooks
                self.model.register_comm_hook(None, default_hooks.bf16_compress_hook)
        elif ddp:
            import torch.distributed as dist
            # replicas start from rank 0's parameters and buffers (DDP's construction-time broadcast)
            with torch.no_grad():
                for t in list(net.parameters()) + list(net.buffers()):
                    dist.broadcast(t, 0)
            self.reducer = GradBucketAllReduce(net.parameters(), dist.get_world_size(),
                                               cap_bytes=int(cap_mb * 2 ** 20), compress=grad_compress)
            self.model = _Wrapped(net, ops)
        else:
            self.model = _Wrapped(net, ops)

    def backward(self, t, o, s, gt_xywh):
        """Forward, loss and backward; under DDP the gradient all-reduce runs inside backward()."""
        self.opt.zero_grad(set_to_none=True)  # autograd then hands each fresh gradient over as .grad
        if self.reducer is not None:
            self.reducer.begin()
        pred = self.model(t, o, s)
        loss_fn = getattr(self.ops, "box_loss", None) or box_loss  # HipOps: one launch each way
        loss, stats = loss_fn(pred, gt_xywh, self.iou_weight, self.l1_weight)
        loss.backward()
        if self.reducer is not None:
            self.reducer.finish()
        stats["loss"] = loss.detach()
        return stats

    def apply(self):
        """Gradient clipping (TRAIN.GRAD_CLIP_NORM) and the AdamW update."""
        if self.hip_opt:
            self.opt.step(self.grad_clip)
            return
        if self.grad_clip > 0:
            torch.nn.utils.clip_grad_norm_(self.net.parameters(), self.grad_clip)
        self.opt.step()

    def __call__(self, t, o, s, gt_xywh):
        stats = self.backward(t, o, s, gt_xywh)
        self.apply()
        return stats

    def capture(self, t, o, s, gt_xywh, warmup=2):
        """Record the whole step -- forward, loss, backward, clip + AdamW -- as one hipGraph on the static
        input tensors t / o / s / gt_xywh (single process, HIP ops: every kernel of the step is then
        libmmt_hip.so's or PyTorch's own, none of MIOpen's convolutions).  `warmup` eager steps on a side
        stream first (they update the weights like any step).  replay() then runs one step on whatever
        was copied into the static inputs, with no Python issue cost.  The learning rates and weight decay
        are those at capture time, and so are grad_clip and the loss weights.  With ddp=True the
        bucketed RCCL all-reduces are captured too (GradBucketAllReduce); a torch DDP wrapper
        (ddp="torch") cannot be captured."""
        if not self.hip_opt or isinstance(self.model, torch.nn.parallel.DistributedDataParallel):
            raise RuntimeError("TrainStep.capture: HIP training step without the torch DDP wrapper only")
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self(t, o, s, gt_xywh)
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        self.opt.zero_grad(set_to_none=True)
        # With a process group, its watchdog thread polls the events of earlier (eager) collectives; in the
        # default global capture mode such a query from another thread fails the capture ("operation not
        # permitted when stream is capturing") and the watchdog aborts the process.  thread_local mode
        # forbids unsafe calls on the capturing thread only; kernels launched onto the captured stream from
        # any thread (the autograd worker's) are recorded either way.
        # The watchdog also keeps the eager collectives of the warm-up steps in its list until its next poll
        # (every ~100 ms), and a query of such a work's event once the process group's stream has joined the
        # capture fails the same way (hipErrorCapturedEvent, seen once in the one-rank test): the device is
        # drained and the watchdog given a few polls to retire them before the capture starts.
        mode = "global"
        if self.reducer is not None:
            torch.cuda.synchronize()
            time.sleep(0.5)
            mode = "thread_local"
        with torch.cuda.graph(self.graph, capture_error_mode=mode):
            self.graph_stats = self(t, o, s, gt_xywh)
        self.static_inputs = (t, o, s, gt_xywh)
        self._captured_hparams = self._hparams()
        return self.graph_stats

    def _hparams(self):
        return ([(g.get("lr"), g.get("weight_decay"), tuple(g.get("betas", ())), g.get("eps")) for g in self.opt.param_groups]
                + [("grad_clip", self.grad_clip), ("iou_weight", self.iou_weight), ("l1_weight", self.l1_weight)])

    def replay(self, t=None, o=None, s=None, gt_xywh=None):
        """One captured step; given inputs are first copied into the static ones (device copies).  The
        captured AdamW launches carry the learning rates / weight decays of capture time as kernel arguments,
        so a changed optimizer hyper-parameter (an LR scheduler step) raises instead of replaying stale
        values: capture() again after changing them."""
        if self._captured_hparams is None:
            raise RuntimeError("TrainStep.replay: call capture() first")
        if self._hparams() != self._captured_hparams:
            raise RuntimeError("TrainStep.replay: optimizer hyper-parameters changed since capture "
                               "(%s -> %s); call capture() again" % (self._captured_hparams, self._hparams()))
        if t is not None:
            st, so, ss, sg = self.static_inputs
            for dst, src in zip(st + so + ss, t + o + s):
                dst.copy_(src)
            sg.copy_(gt_xywh)
        self.graph.replay()
        return self.graph_stats


class _Wrapped(torch.nn.Module):
    """nn.Module view of forward_boxes (DDP needs a module whose forward runs the graph)."""

    def __init__(self, net, ops):
        super().__init__()
        self.net = net
        self.ops = ops

    def forward(self, t, o, s):
        return forward_boxes(self.net, t, o, s, self.ops)


# ----------------------------------------------------------------------------- score-head training
def score_decoder_forward(sb, search_feat, template_feat, box_xyxy):
    """ScoreDecoder.forward (lib/models/mixformer_cvt/score_decoder.py:32-66) with autograd; the ROI
    features come from PrRoIPool on libmmt_hip.so (mmt_amd.functional.prroi_pool2d, whose backward
    is mmt_prroi_pool_backward / _coor_backward).  search_feat (b,C,h,w) fp32, template_feat
    (b,C,2*ht,wt), box_xyxy (b,4) normalised -> logits (b,)."""
    from .functional import prroi_pool2d
    b, c, h, w = search_feat.shape
    H = sb.num_heads
    bb = (box_xyxy.clone() * w).view(-1, 4).float()
    rois = torch.cat([torch.arange(bb.shape[0], dtype=torch.float32, device=bb.device).view(-1, 1), bb], 1)
    x = sb.norm1(sb.score_token.expand(b, -1, -1))
    roi = prroi_pool2d(search_feat.float().contiguous(), rois.contiguous(), sb.pool_size, sb.pool_size, 1.0)
    mem = [roi.flatten(2).transpose(1, 2), template_feat.float().flatten(2).transpose(1, 2)]
    for i in range(2):
        q = sb.proj_q[i](x).view(b, -1, H, c // H).transpose(1, 2)
        k = sb.proj_k[i](mem[i]).view(b, -1, H, c // H).transpose(1, 2)
        v = sb.proj_v[i](mem[i]).view(b, -1, H, c // H).transpose(1, 2)
        a = torch.softmax(q @ k.transpose(-1, -2) * sb.scale, dim=-1)
        x = (a @ v).transpose(1, 2).reshape(b, -1, c)
        x = sb.norm2[i](sb.proj[i](x))
    n = len(sb.score_head.layers)
    for i, layer in enumerate(sb.score_head.layers):
        x = layer(x)
        if i < n - 1:
            x = F.relu(x)
    return x.view(-1)


class ScoreTrainStep:
    """The TRAIN.TRAIN_SCORE stage of the online-score model (asymmetric_shared_online): only the
    parameters whose name contains "score" learn (base_functions.py:300-308), the loss is
    BCEWithLogits(pred_scores, labels) * TRAIN.SCORE_WEIGHT (train_script_mixformer.py:138-140,
    actors/mixformer_rgbt.py:150-152), clip TRAIN.GRAD_CLIP_NORM, AdamW (lr 1e-4, wd 1e-4).

    The frozen trunk (backbone, fusion, box head) runs on the HIP inference runtime `rt` (no
    autograd is needed through it); its search feature, template tokens and predicted boxes feed
    the score decoder, which runs with autograd.  The reference builds the ROI from the predicted
    boxes (asymmetric_shared_online.py:398-413: forward_head is called without gt_bboxes)."""

    def __init__(self, net, rt, lr=1e-4, weight_decay=1e-4, grad_clip=0.1, score_weight=1.0):
        self.net, self.rt = net, rt
        for n, p in net.named_parameters():
            p.requires_grad = "score" in n
        self.params = [p for n, p in net.named_parameters() if "score" in n]
        self.opt = torch.optim.AdamW([{"params": self.params}], lr=lr, weight_decay=weight_decay)
        self.grad_clip, self.score_weight = grad_clip, score_weight
        self.loss_fn = torch.nn.BCEWithLogitsLoss()

    @torch.no_grad()
    def trunk(self, t, o, s):
        """-> search feature (B,C,gs,gs), template feature (B,C,2*gt,gt), boxes xyxy (B,4)."""
        rt, d = self.rt, self.rt.d
        box, _ = rt.forward(t, o, s, run_score_head=False)
        B = box.shape[0]
        ws = rt.workspace(B)
        fused = ws["FUS"].view(B, d.ns, d.C).permute(0, 2, 1).reshape(B, d.C, d.gs, d.gs).float()
        X = ws["X"].view(2, B, d.ntok, d.C)[:, :, :d.nt1]  # first template's tokens, RGB then TIR
        templ = torch.cat([X[0], X[1]], 1).transpose(1, 2).reshape(B, d.C, 2 * d.gt, d.gt).float()
        cx, cy, w, h = box.float().unbind(-1)
        xyxy = torch.stack([cx - 0.5 * w, cy - 0.5 * h, cx + 0.5 * w, cy + 0.5 * h], -1)
        return fused.clone(), templ.clone(), xyxy

    def backward(self, t, o, s, labels):
        self.opt.zero_grad(set_to_none=True)
        fused, templ, xyxy = self.trunk(t, o, s)
        scores = score_decoder_forward(self.net.score_branch, fused, templ, xyxy)
        loss = self.loss_fn(scores, labels.float().view(-1)) * self.score_weight
        loss.backward()
        return {"loss": loss.detach(), "scores": scores.detach()}

    def apply(self):
        if self.grad_clip > 0:
            torch.nn.utils.clip_grad_norm_(self.params, self.grad_clip)
        self.opt.step()

    def __call__(self, t, o, s, labels):
        stats = self.backward(t, o, s, labels)
        self.apply()
        return stats
