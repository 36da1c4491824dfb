"""torch.library registration of the native ops: namespace `mmt`.

The reference binds its two native ops through pybind modules (MultiScaleDeformableAttention,
ops/src/vision.cpp:13-16; _prroi_pooling, prroi_pooling_gpu.c:22-113) that torch's tracer cannot see.
Here every native op of the drop-in is a `torch.library.custom_op` over libmmt_hip.so with a fake
(meta) kernel, so FakeTensor / torch.compile / torch.export trace through them, and the differentiable
ones carry `register_autograd` formulas built from the registered backward ops:

  mmt::ms_deform_attn_forward / _backward       mmt_ms_deform_attn_forward / _backward (fp32 / fp64;
                                                ms_deform_attn_func.py:22-38)
  mmt::prroi_pool_forward / _backward / _coor_backward
                                                mmt_prroi_pool_* (fp32; prroi_pool/functional.py:38-76)
  mmt::mam_attention_forward / _backward        mmt_mam_attention (with log-sum-exp) / mmt_mam_attention_bwd
                                                (bf16, the training form of mixformer.py:52-78)

Each *_forward op has its backward registered (register_autograd over the *_backward ops), so
autograd, FakeTensor and torch.compile see one op per native call.
The implementations raise on non-CUDA or non-contiguous tensors as the reference's AT_ASSERTM does;
there is no CPU path.
"""
import torch

from ._lib import LIB, AttnBwdParams, AttnParams, MMT_BF16, MMT_F32, MMT_F64, check

_DT = {torch.float32: MMT_F32, torch.float64: MMT_F64}


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _need(t, name, dtypes):
    if not t.is_cuda:
        raise RuntimeError("%s must be a CUDA tensor" % name)
    if not t.is_contiguous():
        raise RuntimeError("%s tensor has to be contiguous" % name)
    if dtypes and t.dtype not in dtypes:
        raise RuntimeError("%s: unsupported dtype %s" % (name, t.dtype))


# ------------------------------------------------------------------------------------------- MSDA
@torch.library.custom_op("mmt::ms_deform_attn_forward", mutates_args=())
def ms_deform_attn_forward(value: torch.Tensor, spatial_shapes: torch.Tensor, level_start_index: torch.Tensor,
                           sampling_loc: torch.Tensor, attn_weight: torch.Tensor) -> torch.Tensor:
    """value (N,S,M,D), spatial_shapes (L,2) int64, level_start_index (L) int64, sampling_loc
    (N,Lq,M,L,P,2), attn_weight (N,Lq,M,L,P) -> (N,Lq,M*D)  (ms_deform_attn_cuda.cu:20-80)."""
    for t, nm in ((value, "value"), (sampling_loc, "sampling_loc"), (attn_weight, "attn_weight")):
        _need(t, nm, (torch.float32, torch.float64))
    for t, nm in ((spatial_shapes, "spatial_shapes"), (level_start_index, "level_start_index")):
        _need(t, nm, (torch.int64,))
    if not (value.dtype == sampling_loc.dtype == attn_weight.dtype):
        raise RuntimeError("value / sampling_loc / attn_weight dtypes differ")
    N, S, M, D = value.shape
    _, Lq, _, L, P, _ = sampling_loc.shape
    out = torch.empty(N, Lq, M * D, device=value.device, dtype=value.dtype)
    check(LIB.mmt_ms_deform_attn_forward(value.data_ptr(), spatial_shapes.data_ptr(), level_start_index.data_ptr(),
                                         sampling_loc.data_ptr(), attn_weight.data_ptr(), out.data_ptr(), N, S, M, D,
                                         Lq, L, P, _DT[value.dtype], _stream()), "mmt_ms_deform_attn_forward")
    return out


@ms_deform_attn_forward.register_fake
def _(value, spatial_shapes, level_start_index, sampling_loc, attn_weight):
    N, S, M, D = value.shape
    return value.new_empty(N, sampling_loc.shape[1], M * D)


@torch.library.custom_op("mmt::ms_deform_attn_backward", mutates_args=())
def ms_deform_attn_backward(value: torch.Tensor, spatial_shapes: torch.Tensor, level_start_index: torch.Tensor,
                            sampling_loc: torch.Tensor, attn_weight: torch.Tensor,
                            grad_output: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(grad_value, grad_sampling_loc, grad_attn_weight)  (ms_deform_attn_cuda.cu:83-153)."""
    grad_output = grad_output.contiguous().to(value.dtype)
    N, S, M, D = value.shape
    _, Lq, _, L, P, _ = sampling_loc.shape
    gv, gl, ga = torch.empty_like(value), torch.empty_like(sampling_loc), torch.empty_like(attn_weight)
    check(LIB.mmt_ms_deform_attn_backward(value.data_ptr(), spatial_shapes.data_ptr(), level_start_index.data_ptr(),
                                          sampling_loc.data_ptr(), attn_weight.data_ptr(), grad_output.data_ptr(),
                                          gv.data_ptr(), gl.data_ptr(), ga.data_ptr(), N, S, M, D, Lq, L, P,
                                          _DT[value.dtype], _stream()), "mmt_ms_deform_attn_backward")
    return gv, gl, ga


@ms_deform_attn_backward.register_fake
def _(value, spatial_shapes, level_start_index, sampling_loc, attn_weight, grad_output):
    return torch.empty_like(value), torch.empty_like(sampling_loc), torch.empty_like(attn_weight)


def _msda_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _msda_backward(ctx, grad):
    value, shapes, starts, loc, aw = ctx.saved_tensors
    gv, gl, ga = ms_deform_attn_backward(value, shapes, starts, loc, aw, grad)
    return gv, None, None, gl, ga


ms_deform_attn_forward.register_autograd(_msda_backward, setup_context=_msda_setup)


# --------------------------------------------------------------------------------------- PrRoIPool
@torch.library.custom_op("mmt::prroi_pool_forward", mutates_args=())
def prroi_pool_forward(features: torch.Tensor, rois: torch.Tensor, pooled_height: int, pooled_width: int,
                       spatial_scale: float) -> torch.Tensor:
    """features (B,C,H,W) fp32, rois (R,5) fp32 -> (R,C,ph,pw)  (prroi_pooling_gpu.c:22-50)."""
    _need(features, "features", (torch.float32,))
    _need(rois, "rois", (torch.float32,))
    B, C, H, W = features.shape
    R = rois.shape[0]
    ph, pw = int(pooled_height), int(pooled_width)
    out = torch.empty(R, C, ph, pw, device=features.device, dtype=torch.float32)
    check(LIB.mmt_prroi_pool_forward(features.data_ptr(), rois.data_ptr(), out.data_ptr(), R, C, H, W, C * H * W,
                                     H * W, W, 1, ph, pw, float(spatial_scale), C * ph * pw, ph * pw, 1, _stream()),
          "mmt_prroi_pool_forward")
    return out


@prroi_pool_forward.register_fake
def _(features, rois, pooled_height, pooled_width, spatial_scale):
    return features.new_empty(rois.shape[0], features.shape[1], pooled_height, pooled_width)


@torch.library.custom_op("mmt::prroi_pool_backward", mutates_args=())
def prroi_pool_backward(features: torch.Tensor, rois: torch.Tensor, grad_output: torch.Tensor, pooled_height: int,
                        pooled_width: int, spatial_scale: float) -> torch.Tensor:
    """grad_features (B,C,H,W); `features` gives the shape only (prroi_pooling_gpu.c:52-80)."""
    _need(rois, "rois", (torch.float32,))
    B, C, H, W = features.shape
    g = grad_output.contiguous().float()
    gf = torch.empty(B, C, H, W, device=rois.device, dtype=torch.float32)
    check(LIB.mmt_prroi_pool_backward(rois.data_ptr(), g.data_ptr(), gf.data_ptr(), B, rois.shape[0], C, H, W,
                                      int(pooled_height), int(pooled_width), float(spatial_scale), _stream()),
          "mmt_prroi_pool_backward")
    return gf


@prroi_pool_backward.register_fake
def _(features, rois, grad_output, pooled_height, pooled_width, spatial_scale):
    return torch.empty_like(features, dtype=torch.float32)


@torch.library.custom_op("mmt::prroi_pool_coor_backward", mutates_args=())
def prroi_pool_coor_backward(features: torch.Tensor, rois: torch.Tensor, output: torch.Tensor, grad_output: torch.Tensor,
                             pooled_height: int, pooled_width: int, spatial_scale: float) -> torch.Tensor:
    """grad_rois (R,5), column 0 = 0 (prroi_pooling_gpu.c:82-113)."""
    _need(features, "features", (torch.float32,))
    _need(rois, "rois", (torch.float32,))
    B, C, H, W = features.shape
    g = grad_output.contiguous().float()
    gr = torch.empty_like(rois)
    check(LIB.mmt_prroi_pool_coor_backward(features.data_ptr(), rois.data_ptr(), output.data_ptr(), g.data_ptr(),
                                           gr.data_ptr(), rois.shape[0], C, H, W, int(pooled_height), int(pooled_width),
                                           float(spatial_scale), _stream()), "mmt_prroi_pool_coor_backward")
    return gr


@prroi_pool_coor_backward.register_fake
def _(features, rois, output, grad_output, pooled_height, pooled_width, spatial_scale):
    return torch.empty_like(rois)


def _prroi_setup(ctx, inputs, output):
    features, rois, ph, pw, sc = inputs
    ctx.params = (ph, pw, sc)
    ctx.save_for_backward(features, rois, output)


def _prroi_backward(ctx, grad):
    features, rois, out = ctx.saved_tensors
    ph, pw, sc = ctx.params
    gf = prroi_pool_backward(features, rois, grad, ph, pw, sc) if ctx.needs_input_grad[0] else None
    gr = prroi_pool_coor_backward(features, rois, out, grad, ph, pw, sc) if ctx.needs_input_grad[1] else None
    return gf, gr, None, None, None


prroi_pool_forward.register_autograd(_prroi_backward, setup_context=_prroi_setup)


# ---------------------------------------------------------------------------------- MAM attention
@torch.library.custom_op("mmt::mam_attention_forward", mutates_args=())
def mam_attention_forward(qkv: torch.Tensor, n_t: int, heads: int) -> tuple[torch.Tensor, torch.Tensor]:
    """qkv [S][ntok][3C] bf16 (the fused qkv Linear output) -> (out [S][ntok][C] bf16, lse [S][H][ntok]
    fp32 log2-sum-exp2 of the scaled scores); template queries [0, n_t) attend template keys, search
    queries all keys (mixformer.py:52-78)."""
    _need(qkv, "qkv", (torch.bfloat16,))
    S, ntok, C3 = qkv.shape
    C = C3 // 3
    out = torch.empty(S, ntok, C, device=qkv.device, dtype=torch.bfloat16)
    lse = torch.empty(S, heads, ntok, device=qkv.device, dtype=torch.float32)
    p = AttnParams()
    p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym = qkv.data_ptr(), out.data_ptr(), S, S, ntok, n_t, C, heads, 0
    p.scale, p.impl, p.lse = (C // heads) ** -0.5, 0, lse.data_ptr()
    check(LIB.mmt_mam_attention(p, MMT_BF16, _stream()), "mmt_mam_attention")
    return out, lse


@mam_attention_forward.register_fake
def _(qkv, n_t, heads):
    S, ntok, C3 = qkv.shape
    return qkv.new_empty(S, ntok, C3 // 3), qkv.new_empty(S, heads, ntok, dtype=torch.float32)


@torch.library.custom_op("mmt::mam_attention_backward", mutates_args=())
def mam_attention_backward(qkv: torch.Tensor, out: torch.Tensor, dout: torch.Tensor, lse: torch.Tensor, n_t: int,
                           heads: int) -> torch.Tensor:
    """dL/dqkv [S][ntok][3C] bf16 (deterministic, mmt_mam_attention_bwd)."""
    _need(qkv, "qkv", (torch.bfloat16,))
    S, ntok, C3 = qkv.shape
    C = C3 // 3
    dout = dout.to(torch.bfloat16).contiguous()
    delta = torch.empty_like(lse)
    dqkv = torch.empty_like(qkv)
    p = AttnBwdParams()
    p.qkv, p.out, p.dout, p.lse, p.delta, p.dqkv = (qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(),
                                                    delta.data_ptr(), dqkv.data_ptr())
    p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym, p.scale = S, S, ntok, n_t, C, heads, 0, (C // heads) ** -0.5
    check(LIB.mmt_mam_attention_bwd(p, MMT_BF16, _stream()), "mmt_mam_attention_bwd")
    return dqkv


@mam_attention_backward.register_fake
def _(qkv, out, dout, lse, n_t, heads):
    return torch.empty_like(qkv)


def _mam_setup(ctx, inputs, output):
    qkv, n_t, heads = inputs
    out, lse = output
    ctx.args = (n_t, heads)
    ctx.save_for_backward(qkv, out, lse)


def _mam_backward(ctx, dout, dlse):
    qkv, out, lse = ctx.saved_tensors
    n_t, heads = ctx.args
    return mam_attention_backward(qkv, out, dout, lse, n_t, heads), None, None


mam_attention_forward.register_autograd(_mam_backward, setup_context=_mam_setup)


def mam_attention(qkv, n_t, heads):
    """Differentiable MAM attention output (bf16): mmt::mam_attention_forward's first output."""
    return mam_attention_forward(qkv.contiguous(), n_t, heads)[0]


def ms_deform_attn(value, spatial_shapes, level_start_index, sampling_loc, attn_weight):
    """Differentiable MSDA (MSDeformAttnFunction.apply without im2col_step)."""
    return ms_deform_attn_forward(value, spatial_shapes, level_start_index, sampling_loc, attn_weight)


def prroi_pool2d(features, rois, pooled_height, pooled_width, spatial_scale):
    """Differentiable PrRoIPool2D (fp32)."""
    return prroi_pool_forward(features, rois, int(pooled_height), int(pooled_width), float(spatial_scale))
