"""Autograd drop-ins for the reference's two native ops, over libmmt_hip.so.

  MSDeformAttnFunction   lib/models/mixformer_vit_rgbt/deformable_attention/ops/functions/
                         ms_deform_attn_func.py:22-38 (forward / backward through the pybind module
                         MultiScaleDeformableAttention, ops/src/vision.cpp:13-16)
  PrRoIPool2DFunction    external/PreciseRoIPooling/pytorch/prroi_pool/functional.py:38-76
                         (_prroi_pooling.prroi_pooling_{forward,backward,coor_backward}_cuda,
                         prroi_pooling_gpu.c:22-113); `prroi_pool2d` = its apply, as there

Same argument meaning, dtype rules (MSDA fp32 / fp64; PrRoIPool fp32) and error behaviour (a
non-contiguous or non-CUDA tensor raises, as the reference's AT_ASSERTM); `im2col_step` is accepted
and ignored (the HIP kernels take the whole batch in one launch).  No CPU path: the HIP library is
required."""
import torch

from ._lib import LIB, MMT_F32, MMT_F64, check


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _need(t, name, dtypes):
    if not t.is_cuda:
        raise RuntimeError("%s must be a CUDA tensor" % name)
    if not t.is_contiguous():
        raise RuntimeError("%s tensor has to be contiguous" % name)
    if dtypes and t.dtype not in dtypes:
        raise RuntimeError("%s: unsupported dtype %s" % (name, t.dtype))


_DT = {torch.float32: MMT_F32, torch.float64: MMT_F64}


class MSDeformAttnFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, value, value_spatial_shapes, value_level_start_index, sampling_locations, attention_weights,
                im2col_step=64):
        for t, nm in ((value, "value"), (sampling_locations, "sampling_loc"), (attention_weights, "attn_weight")):
            _need(t, nm, (torch.float32, torch.float64))
        for t, nm in ((value_spatial_shapes, "spatial_shapes"), (value_level_start_index, "level_start_index")):
            _need(t, nm, (torch.int64,))
        if not (value.dtype == sampling_locations.dtype == attention_weights.dtype):
            raise RuntimeError("value / sampling_loc / attn_weight dtypes differ")
        N, S, M, D = value.shape
        _, Lq, _, L, P, _ = sampling_locations.shape
        out = torch.empty(N, Lq, M * D, device=value.device, dtype=value.dtype)
        check(LIB.mmt_ms_deform_attn_forward(value.data_ptr(), value_spatial_shapes.data_ptr(),
                                             value_level_start_index.data_ptr(), sampling_locations.data_ptr(),
                                             attention_weights.data_ptr(), out.data_ptr(), N, S, M, D, Lq, L, P,
                                             _DT[value.dtype], _stream()), "mmt_ms_deform_attn_forward")
        ctx.save_for_backward(value, value_spatial_shapes, value_level_start_index, sampling_locations,
                              attention_weights)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        value, shapes, starts, loc, aw = ctx.saved_tensors
        grad_output = grad_output.contiguous().to(value.dtype)
        N, S, M, D = value.shape
        _, Lq, _, L, P, _ = loc.shape
        gv = torch.empty_like(value)
        gl = torch.empty_like(loc)
        ga = torch.empty_like(aw)
        check(LIB.mmt_ms_deform_attn_backward(value.data_ptr(), shapes.data_ptr(), starts.data_ptr(), loc.data_ptr(),
                                              aw.data_ptr(), grad_output.data_ptr(), gv.data_ptr(), gl.data_ptr(),
                                              ga.data_ptr(), N, S, M, D, Lq, L, P, _DT[value.dtype], _stream()),
              "mmt_ms_deform_attn_backward")
        return gv, None, None, gl, ga, None


class PrRoIPool2DFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, features, rois, pooled_height, pooled_width, spatial_scale):
        ctx.dtypes = (features.dtype, rois.dtype)  # gradients go back in the inputs' dtypes
        features = features.contiguous().float()
        rois = rois.contiguous().float()
        _need(features, "features", (torch.float32,))
        _need(rois, "rois", (torch.float32,))
        B, C, H, W = features.shape
        R = rois.shape[0]
        ph, pw, sc = int(pooled_height), int(pooled_width), float(spatial_scale)
        out = torch.empty(R, C, ph, pw, device=features.device, dtype=torch.float32)
        check(LIB.mmt_prroi_pool_forward(features.data_ptr(), rois.data_ptr(), out.data_ptr(), R, C, H, W, C * H * W,
                                         H * W, W, 1, ph, pw, sc, C * ph * pw, ph * pw, 1, _stream()),
              "mmt_prroi_pool_forward")
        ctx.params = (ph, pw, sc)
        ctx.save_for_backward(features, rois, out)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        features, rois, out = ctx.saved_tensors
        ph, pw, sc = ctx.params
        B, C, H, W = features.shape
        R = rois.shape[0]
        g = grad_output.contiguous().float()
        gf = gr = None
        # needs_input_grad, not the saved copies' requires_grad: forward's .float() copies of
        # non-fp32 inputs are made with grad mode off and never require grad
        if ctx.needs_input_grad[0]:
            gf = torch.empty_like(features)
            check(LIB.mmt_prroi_pool_backward(rois.data_ptr(), g.data_ptr(), gf.data_ptr(), B, R, C, H, W, ph, pw, sc,
                                              _stream()), "mmt_prroi_pool_backward")
            gf = gf.to(ctx.dtypes[0])
        if ctx.needs_input_grad[1]:
            gr = torch.empty_like(rois)
            check(LIB.mmt_prroi_pool_coor_backward(features.data_ptr(), rois.data_ptr(), out.data_ptr(), g.data_ptr(),
                                                   gr.data_ptr(), R, C, H, W, ph, pw, sc, _stream()),
                  "mmt_prroi_pool_coor_backward")
            gr = gr.to(ctx.dtypes[1])
        return gf, gr, None, None, None


prroi_pool2d = PrRoIPool2DFunction.apply


class PrRoIPool2D(torch.nn.Module):
    """external/PreciseRoIPooling/pytorch/prroi_pool/prroi_pool.py:19-31."""

    def __init__(self, pooled_height, pooled_width, spatial_scale):
        super().__init__()
        self.pooled_height = int(pooled_height)
        self.pooled_width = int(pooled_width)
        self.spatial_scale = float(spatial_scale)

    def forward(self, features, rois):
        return prroi_pool2d(features, rois, self.pooled_height, self.pooled_width, self.spatial_scale)

    def extra_repr(self):
        return "kernel_size=({pooled_height}, {pooled_width}), spatial_scale={spatial_scale}".format(**self.__dict__)
