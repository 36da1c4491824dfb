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
required.  The native calls are the torch.library ops of mmt_amd.ops (namespace `mmt`), so
FakeTensor / torch.compile see them as registered ops."""
import torch

from . import ops


class MSDeformAttnFunction(torch.autograd.Function):
    """forward / backward = the registered ops mmt::ms_deform_attn_forward / _backward."""

    @staticmethod
    def forward(ctx, value, value_spatial_shapes, value_level_start_index, sampling_locations, attention_weights,
                im2col_step=64):
        out = ops.ms_deform_attn_forward(value, value_spatial_shapes, value_level_start_index, sampling_locations,
                                         attention_weights)
        ctx.save_for_backward(value, value_spatial_shapes, value_level_start_index, sampling_locations,
                              attention_weights)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        value, shapes, starts, loc, aw = ctx.saved_tensors
        gv, gl, ga = ops.ms_deform_attn_backward(value, shapes, starts, loc, aw, grad_output)
        return gv, None, None, gl, ga, None


class PrRoIPool2DFunction(torch.autograd.Function):
    """forward / backward = mmt::prroi_pool_forward / _backward / _coor_backward; fp32 arithmetic,
    gradients returned in the inputs' dtypes."""

    @staticmethod
    def forward(ctx, features, rois, pooled_height, pooled_width, spatial_scale):
        ctx.dtypes = (features.dtype, rois.dtype)
        features = features.contiguous().float()
        rois = rois.contiguous().float()
        ph, pw, sc = int(pooled_height), int(pooled_width), float(spatial_scale)
        out = ops.prroi_pool_forward(features, rois, ph, pw, sc)
        ctx.params = (ph, pw, sc)
        ctx.save_for_backward(features, rois, out)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        features, rois, out = ctx.saved_tensors
        ph, pw, sc = ctx.params
        gf = gr = None
        # needs_input_grad, not the saved copies' requires_grad: forward's .float() copies of
        # non-fp32 inputs are made with grad mode off and never require grad
        if ctx.needs_input_grad[0]:
            gf = ops.prroi_pool_backward(features, rois, grad_output, ph, pw, sc).to(ctx.dtypes[0])
        if ctx.needs_input_grad[1]:
            gr = ops.prroi_pool_coor_backward(features, rois, out, grad_output, ph, pw, sc).to(ctx.dtypes[1])
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
