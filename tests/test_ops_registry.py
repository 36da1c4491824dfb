"""torch.library registration of the native ops (mmt_amd/ops.py): every op exists
under torch.ops.mmt, its fake kernel gives the reference op's output shapes and dtypes under
FakeTensorMode (what torch.compile / torch.export trace with), and the *_forward ops carry a
registered autograd formula.  CPU-only: no kernel runs here (GPU: tests/test_gpu_ops_registry.py)."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

import mmt_amd.ops  # noqa: F401  (registers the ops)

OPS = ["ms_deform_attn_forward", "ms_deform_attn_backward", "prroi_pool_forward", "prroi_pool_backward",
       "prroi_pool_coor_backward", "mam_attention_forward", "mam_attention_backward"]


@pytest.mark.parametrize("name", OPS)
def test_op_registered(name):
    assert hasattr(torch.ops.mmt, name)
    assert torch._C._dispatch_has_kernel_for_dispatch_key("mmt::" + name, "Meta")  # the fake kernel


@pytest.mark.parametrize("name", ["ms_deform_attn_forward", "prroi_pool_forward", "mam_attention_forward"])
def test_forward_ops_have_autograd(name):
    assert torch._C._dispatch_has_kernel_for_dispatch_key("mmt::" + name, "Autograd")


def test_fake_shapes():
    with FakeTensorMode():
        v = torch.empty(2, 100, 8, 32)
        loc = torch.empty(2, 50, 8, 2, 4, 2)
        aw = torch.empty(2, 50, 8, 2, 4)
        sh, st = torch.empty(2, 2, dtype=torch.long), torch.empty(2, dtype=torch.long)
        out = torch.ops.mmt.ms_deform_attn_forward(v, sh, st, loc, aw)
        assert out.shape == (2, 50, 256) and out.dtype == torch.float32
        gv, gl, ga = torch.ops.mmt.ms_deform_attn_backward(v, sh, st, loc, aw, out)
        assert gv.shape == v.shape and gl.shape == loc.shape and ga.shape == aw.shape
        f, r = torch.empty(2, 768, 20, 20), torch.empty(3, 5)
        o = torch.ops.mmt.prroi_pool_forward(f, r, 4, 4, 1.0)
        assert o.shape == (3, 768, 4, 4)
        assert torch.ops.mmt.prroi_pool_backward(f, r, o, 4, 4, 1.0).shape == f.shape
        assert torch.ops.mmt.prroi_pool_coor_backward(f, r, o, o, 4, 4, 1.0).shape == r.shape
        q = torch.empty(4, 528, 2304, dtype=torch.bfloat16)
        a, lse = torch.ops.mmt.mam_attention_forward(q, 128, 12)
        assert a.shape == (4, 528, 768) and a.dtype == torch.bfloat16 and lse.shape == (4, 12, 528)
        assert torch.ops.mmt.mam_attention_backward(q, a, a, lse, 128, 12).shape == q.shape


def test_cpu_tensors_raise():
    with pytest.raises(RuntimeError, match="CUDA"):
        torch.ops.mmt.prroi_pool_forward(torch.zeros(1, 4, 8, 8), torch.zeros(1, 5), 2, 2, 1.0)
