"""Diagnostic: where a GEMM output deviates from the torch reference (rows/cols of bad elements)."""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-tracking_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
from test_gpu_ops import _gemm  # noqa: E402


def case(dt, M, N, K, impl):
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / math.sqrt(K)
    b = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    Ad, Wd, bd, Rd = A.to(dt).cuda(), W.to(dt).cuda(), b.cuda(), R.cuda()
    out = torch.full((M, N), float("nan"), device="cuda")
    _gemm([Ad.data_ptr()], [Wd.data_ptr()], [out.data_ptr()], M, N, K, K, N, dt, bias=[bd.data_ptr()],
          r=[Rd.data_ptr()], ldr=N, c_f32=1, impl=impl)
    torch.cuda.synchronize()
    ref = A.to(dt).float() @ W.to(dt).float().t() + b + R
    e = (out.cpu() - ref).abs()
    e[torch.isnan(e)] = 1e9
    bad = (e > 1e-2).nonzero()
    print(dt, M, N, K, impl, "maxerr", e.max().item(), "nbad", len(bad),
          "rows", sorted(set(bad[:, 0].tolist()))[:20], "cols", sorted(set(bad[:, 1].tolist()))[:20], flush=True)


for rep in range(2):
    for dt in (torch.float32, torch.bfloat16):
        for (M, N, K) in [(300, 200, 192), (1056, 2304, 768), (128, 128, 64), (77, 192, 1024)]:
            case(dt, M, N, K, -1)
