"""Per-kernel parity of libmmt_hip.so on the GPU against fp32/fp64 references (oracle or torch CPU).

Tolerances: fp32 kernels 1e-4..1e-5 relative to the reference magnitude; bf16 kernels ~1e-2
(operands rounded to bf16, fp32 accumulation)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

DT = {"f32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}


def _code(dt):
    """mmt dtype code of a torch dtype (MMT_F32 / MMT_BF16 / MMT_F16)."""
    L = _lib()
    return {torch.bfloat16: L.MMT_BF16, torch.float16: L.MMT_F16}.get(dt, L.MMT_F32)


def _lib():
    from mmt_amd import _lib
    return _lib


def _gemm(a, w, c, M, N, K, lda, ldc, dtype, **kw):
    L = _lib()
    p = _gemm_params(a, w, c, M, N, K, lda, ldc, **kw)
    L.check(L.LIB.mmt_gemm(p, _code(dtype),
                           torch.cuda.current_stream().cuda_stream), "mmt_gemm")


def _gemm_params(a, w, c, M, N, K, lda, ldc, **kw):
    L = _lib()
    p = L.GemmParams()
    G = len(a)
    for g in range(G):
        p.a[g] = a[g]
        p.w[g] = w[g]
        p.c[g] = c[g]
        p.bias[g] = kw["bias"][g] if kw.get("bias") else None
        p.r[g] = kw["r"][g] if kw.get("r") else None
        p.c2[g] = kw["c2"][g] if kw.get("c2") else None
        p.a1[g] = kw["a1"][g] if kw.get("a1") else None
    p.lda, p.ldc, p.ldr = lda, ldc, kw.get("ldr", 0)
    seg = kw.get("seg")
    p.a_seg_rows, p.a_segs_a, p.a_stride_a, p.a_stride_b = seg if seg else (M, 1, 0, 0)
    p.M, p.N, p.K, p.k_split = M, N, K, kw.get("k_split", 0)
    p.act, p.c_f32 = kw.get("act", 0), kw.get("c_f32", 0)
    p.r_mode, p.r_p0, p.r_p1 = kw.get("r_mode", 0), kw.get("r_p0", 0), kw.get("r_p1", 1)
    if kw.get("conv"):
        p.conv_h, p.conv_up, p.conv_cin, p.conv_k3 = kw["conv"]
    p.groups = G
    p.r_t = kw.get("r_t", 0)
    p.impl = kw.get("impl", 0)
    p.c2_copy = kw.get("c2_copy", 0)
    if kw.get("sk"):  # (splitk, slab workspace, tickets)
        n, ws, cnt = kw["sk"]
        p.splitk, p.sk_ws, p.sk_ws_floats, p.sk_cnt, p.sk_cnt_n = n, ws.data_ptr(), ws.numel(), cnt.data_ptr(), cnt.numel()
    return p


def _tol(dt):
    return 2e-2 if dt != torch.float32 else 2e-5


@pytest.mark.parametrize("dname", ["f32", "bf16", "fp16"])
@pytest.mark.parametrize("M,N,K,act", [(300, 200, 192, 0), (1056, 2304, 768, 0), (128, 128, 64, 1), (77, 192, 1024, 2),
                                       (1056, 3072, 768, 1)])  # the last: fc1 shape, packed GELU epilogue
def test_gemm_plain(dname, M, N, K, act):
    dt = DT[dname]
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / math.sqrt(K)
    b = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    Ad, Wd = A.to(dt).cuda(), W.to(dt).cuda()
    bd, Rd = b.cuda(), R.cuda()  # held: a temporary's memory could be recycled before the launch
    out = torch.empty(M, N, device="cuda")
    _gemm([Ad.data_ptr()], [Wd.data_ptr()], [out.data_ptr()], M, N, K, K, N, dt, bias=[bd.data_ptr()],
          r=[Rd.data_ptr()], ldr=N, act=act, c_f32=1)
    torch.cuda.synchronize()
    ref = A.to(dt).float() @ W.to(dt).float().t() + b
    ref = {0: ref, 1: F.gelu(ref), 2: F.relu(ref)}[act] + R
    err = (out.cpu() - ref).abs().max().item()
    assert err <= 1e-3 * ref.abs().max().item() + 1e-4, err


@pytest.mark.parametrize("dname", ["f32", "bf16", "fp16"])
def test_gemm_groups_segments_ksplit(dname):
    dt = DT[dname]
    g = torch.Generator().manual_seed(1)
    # A rows come from segments of 5 rows spaced 9 rows apart (like search tokens after templates),
    # K split over two sources; two groups with their own weights / outputs.
    M, N, K, ks = 20, 96, 64, 32
    src0 = torch.randn(2, 40, ks, generator=g)
    src1 = torch.randn(2, 40, ks, generator=g)
    W = torch.randn(2, N, K, generator=g) / 8
    outs = torch.zeros(2, M, N, device="cuda", dtype=dt)
    s0, s1, Wd = src0.to(dt).cuda(), src1.to(dt).cuda(), W.to(dt).cuda()
    _gemm([s0[0].data_ptr() + 4 * ks * s0.element_size(), s0[1].data_ptr() + 4 * ks * s0.element_size()],
          [Wd[0].data_ptr(), Wd[1].data_ptr()], [outs[0].data_ptr(), outs[1].data_ptr()], M, N, K, ks, N, dt,
          a1=[s1[0].data_ptr() + 4 * ks * s1.element_size(), s1[1].data_ptr() + 4 * ks * s1.element_size()],
          k_split=ks, seg=(5, 1 << 40, 9 * ks, 0))
    torch.cuda.synchronize()
    for grp in range(2):
        rows = [4 + 9 * (r // 5) + r % 5 for r in range(M)]
        A = torch.cat([src0[grp, rows], src1[grp, rows]], 1).to(dt).float()
        ref = A @ W[grp].to(dt).float().t()
        err = (outs[grp].float().cpu() - ref).abs().max().item()
        assert err <= _tol(dt) * ref.abs().max().item(), (grp, err)


@pytest.mark.parametrize("impl", [-1, 1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("M,N,K", [(528, 768, 768), (77, 200, 64), (300, 136, 192), (1056, 256, 3072), (300, 136, 200),
                                   (4224, 1160, 256)])
def test_gemm_bf16_tile_paths(impl, M, N, K):
    """Every bf16 GEMM kernel (impl: register-staged / LDS-DMA 128x128, 128x64 K-split, 64x64
    K-split, 256x128 / 128x256, 256x256 with its four-pass epilogue) on ragged M/N, odd K-step counts (the K-split's empty last step), a
    grid of more than 512 workgroups (the grouped tile order of large grids), and each epilogue:
    GELU + fp32 residual into an fp32 C; bf16 C + C2 = C + bf16 residual (r_t) with a modulo row
    map; two groups with segmented rows and a split K source."""
    g = torch.Generator().manual_seed(M * 7 + N + K)
    A = torch.randn(2, M, K, generator=g)
    W = torch.randn(2, N, K, generator=g) / math.sqrt(K)
    b = torch.randn(2, N, generator=g)
    R = torch.randn(2, M, N, generator=g)
    Ab, Wb = A.bfloat16(), W.bfloat16()
    Ad, Wd, bd, Rd = Ab.cuda(), Wb.cuda(), b.cuda(), R.cuda()
    ref = torch.einsum("gmk,gnk->gmn", Ab.float(), Wb.float()) + b[:, None]
    # (1) GELU + fp32 residual, fp32 out, two groups
    out = torch.empty(2, M, N, device="cuda")
    _gemm([Ad[0].data_ptr(), Ad[1].data_ptr()], [Wd[0].data_ptr(), Wd[1].data_ptr()],
          [out[0].data_ptr(), out[1].data_ptr()], M, N, K, K, N, torch.bfloat16,
          bias=[bd[0].data_ptr(), bd[1].data_ptr()], r=[Rd[0].data_ptr(), Rd[1].data_ptr()], ldr=N, act=1, c_f32=1,
          impl=impl)
    torch.cuda.synchronize()
    r1 = F.gelu(ref) + R
    err = (out.cpu() - r1).abs().max().item()
    assert err <= 1e-3 * r1.abs().max().item() + 1e-4, err
    # (2) bf16 out + C2 with a bf16 residual read at row m % 5
    Rt = R[0, :5].bfloat16().cuda()
    c1 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    c2 = torch.empty_like(c1)
    _gemm([Ad[0].data_ptr()], [Wd[0].data_ptr()], [c1.data_ptr()], M, N, K, K, N, torch.bfloat16,
          bias=[bd[0].data_ptr()], r=[Rt.data_ptr()], ldr=N, r_t=1, r_mode=1, r_p0=5, c2=[c2.data_ptr()], impl=impl)
    torch.cuda.synchronize()
    rr = Rt.float().cpu()[torch.arange(M) % 5]
    tol = 1e-2 * (ref[0].abs().max().item() + 4)
    assert (c1.float().cpu() - ref[0]).abs().max().item() <= tol
    assert (c2.float().cpu() - (ref[0] + rr)).abs().max().item() <= tol
    # (3) segmented rows (runs of 7 rows, 3 per A block) + K split between two sources
    if K >= 128:
        ks = (K // 2) // 8 * 8 + 8 if K % 128 else K // 2  # both sources use row stride lda = ks (k_split % 8 == 0)
        src0 = torch.randn(2, M + 64, ks, generator=g).bfloat16()
        src1 = torch.randn(2, M + 64, ks, generator=g).bfloat16()
        s0, s1 = src0.cuda(), src1.cuda()
        o3 = torch.empty(2, M, N, device="cuda")
        _gemm([s0[0].data_ptr(), s0[1].data_ptr()], [Wd[0].data_ptr(), Wd[1].data_ptr()],
              [o3[0].data_ptr(), o3[1].data_ptr()], M, N, K, ks, N, torch.bfloat16, c_f32=1, impl=impl,
              a1=[s1[0].data_ptr(), s1[1].data_ptr()], k_split=ks, seg=(7, 3, 8 * ks, 0))
        torch.cuda.synchronize()
        # segment seg: rows (seg % 3) * 8 + (m % 7) of source block seg // 3 (a_stride_b = 0)
        rows = [(m // 7 % 3) * 8 + m % 7 for m in range(M)]
        for grp in range(2):
            Ag = torch.cat([src0[grp, rows].float(), src1[grp, rows, :K - ks].float()], 1)
            r3 = Ag @ Wb[grp].float().t()
            e3 = (o3[grp].cpu() - r3).abs().max().item()
            assert e3 <= 1e-3 * r3.abs().max().item() + 1e-4, (grp, e3)


@pytest.mark.parametrize("impl", [-1, 0, 1, 2, 3, 4, 5, 6, 7, 8])
def test_gemm_gelu_backward_and_preact_epilogues(impl):
    """The training MLP's epilogues: act 1 with c2_copy 2 (C = GELU(acc + b), C2 = acc + b in bf16) and
    act 5 (C = (acc + b) * GELU'(R), R bf16); 16-bit LDS-DMA kernels only (impl -1, the register-staged
    kernel, rejects both)."""
    L = _lib()
    M, N, K = 528, 768, 256
    g = torch.Generator().manual_seed(impl + 40)
    A = torch.randn(M, K, generator=g).bfloat16()
    W = (torch.randn(N, K, generator=g) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, generator=g)
    R = (torch.randn(M, N, generator=g) * 2).bfloat16()
    Ad, Wd, bd, Rd = A.cuda(), W.cuda(), b.cuda(), R.cuda()
    pre = A.float() @ W.float().t() + b
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    c2 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    p = _gemm_params([Ad.data_ptr()], [Wd.data_ptr()], [c.data_ptr()], M, N, K, K, N, bias=[bd.data_ptr()], act=1,
                     c2=[c2.data_ptr()], c2_copy=2, impl=impl)
    st = torch.cuda.current_stream().cuda_stream
    rc = L.LIB.mmt_gemm(p, L.MMT_BF16, st)
    if impl == -1:
        assert rc == -10000
    else:
        L.check(rc, "gemm act1 c2_copy2")
        torch.cuda.synchronize()
        assert (c2.float().cpu() - pre).abs().max().item() <= 2e-2 * pre.abs().max().item()
        gel = F.gelu(pre)
        assert (c.float().cpu() - gel).abs().max().item() <= 2e-2 * gel.abs().max().item()
    c5 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    p5 = _gemm_params([Ad.data_ptr()], [Wd.data_ptr()], [c5.data_ptr()], M, N, K, K, N, bias=[bd.data_ptr()], act=5,
                      r=[Rd.data_ptr()], ldr=N, r_t=1, impl=impl)
    rc = L.LIB.mmt_gemm(p5, L.MMT_BF16, st)
    if impl == -1:
        assert rc == -10000
        return
    L.check(rc, "gemm act5")
    torch.cuda.synchronize()
    r = R.float().requires_grad_(True)
    F.gelu(r).backward(torch.ones_like(r))
    ref = pre * r.grad
    assert (c5.float().cpu() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()


@pytest.mark.parametrize("impl", [0, 8])
@pytest.mark.parametrize("c_f32", [1, 0])
def test_gemm_row_scale_residual(impl, c_f32):
    """row_scale (the training step's per-sample stochastic depth on a residual branch, mixformer.py:136-139):
    C = R + keep[m // div] * (A W^T + b), as an fp32 C with its bf16 copy (the compact residual epilogue) or a bf16
    C (the general epilogue), two groups, a partial last row tile; impl 0 / 8 (the 128x128 two-per-CU tile)."""
    L = _lib()
    M, N, K, div = 1100, 768, 768, 275
    g = torch.Generator().manual_seed(impl * 2 + c_f32)
    A = torch.randn(2, M, K, generator=g).bfloat16()
    W = (torch.randn(2, N, K, generator=g) / math.sqrt(K)).bfloat16()
    b = torch.randn(2, N, generator=g)
    R = torch.randn(2, M, N, generator=g)
    keep = torch.tensor([0.0, 1.25, 1.25, 0.0], dtype=torch.float32)
    Ad, Wd, bd, Rd, kd = A.cuda(), W.cuda(), b.cuda(), R.cuda(), keep.cuda()
    c = torch.empty(2, M, N, device="cuda", dtype=torch.float32 if c_f32 else torch.bfloat16)
    c2 = torch.empty(2, M, N, device="cuda", dtype=torch.bfloat16)
    kw = dict(c2=[c2[0].data_ptr(), c2[1].data_ptr()], c2_copy=1) if c_f32 else {}
    p = _gemm_params([Ad[0].data_ptr(), Ad[1].data_ptr()], [Wd[0].data_ptr(), Wd[1].data_ptr()],
                     [c[0].data_ptr(), c[1].data_ptr()], M, N, K, K, N, bias=[bd[0].data_ptr(), bd[1].data_ptr()],
                     r=[Rd[0].data_ptr(), Rd[1].data_ptr()], ldr=N, c_f32=c_f32, impl=impl, **kw)
    p.row_scale, p.row_scale_div = kd.data_ptr(), div
    L.check(L.LIB.mmt_gemm(p, L.MMT_BF16, torch.cuda.current_stream().cuda_stream), "gemm row_scale")
    torch.cuda.synchronize()
    sc = keep[torch.arange(M) // div][None, :, None]
    ref = R + sc * (torch.einsum("gmk,gnk->gmn", A.float(), W.float()) + b[:, None])
    err = (c.float().cpu() - ref).abs().max().item()
    assert err <= (1e-3 if c_f32 else 1e-2) * ref.abs().max().item() + 1e-4, err
    if c_f32:
        assert torch.equal(c2.cpu(), c.cpu().bfloat16())


@pytest.mark.parametrize("impl", [-1, 0, 1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("splitk", [0, 3])
@pytest.mark.parametrize("N,K,M", [(768, 3072, 776), (3072, 768, 1024), (256, 2112, 264)])
@pytest.mark.parametrize("mode", [3, 4])
def test_gemm_column_split_epilogue(impl, splitk, N, K, M, mode):
    """c2_copy 3 (the training dW GEMM, dy^T [x | 1]): output columns [0, M - 8) go to C with pitch
    M - 8, the last 8 columns (the bias gradient, then zeros) to C2 [rows][8]; c2_copy 4: only column M - 8
    (the bias gradient) to C2 as a contiguous [rows] vector; fp32 outputs.  Every 16-bit LDS-DMA configuration,
    with and without split-K (impl -1 rejects the mode)."""
    if splitk and impl in (5, 7, 8):
        pytest.skip("forced impl 5 / 7 / 8 take no split-K")
    L = _lib()
    g = torch.Generator().manual_seed(N + K + impl)
    A = torch.randn(N, K, generator=g).bfloat16()  # dy^T
    X = torch.randn(M, K, generator=g)  # [x | 1]^T: rows M - 8 ones, M - 7.. zeros
    X[M - 8] = 1.0
    X[M - 7:] = 0.0
    Xb = X.bfloat16()
    Ad, Xd = A.cuda(), Xb.cuda()
    buf = torch.full((N * M + 64,), float("nan"), device="cuda")
    nb = 8 if mode == 3 else 1
    dw, db8 = buf[:N * (M - 8)].view(N, M - 8), buf[N * (M - 8):N * (M - 8) + N * nb].view(N, nb)
    kw = {}
    if splitk:
        kw["sk"] = (splitk, torch.empty(8 << 20, device="cuda"), torch.zeros(1 << 16, device="cuda", dtype=torch.int32))
    p = _gemm_params([Ad.data_ptr()], [Xd.data_ptr()], [dw.data_ptr()], N, M, K, K, M - 8, c_f32=1,
                     c2=[db8.data_ptr()], c2_copy=mode, impl=impl, **kw)
    rc = L.LIB.mmt_gemm(p, L.MMT_BF16, torch.cuda.current_stream().cuda_stream)
    if impl == -1:
        assert rc == -10000
        return
    L.check(rc, "gemm c2_copy %d" % mode)
    torch.cuda.synchronize()
    ref = A.float() @ Xb.float().t()
    got = torch.cat([dw.cpu(), db8.cpu()], 1)
    err = (got - ref[:, :M - 8 + nb]).abs().max().item()
    assert err <= 1e-3 * ref.abs().max().item() + 1e-4, err
    if mode == 3:
        assert torch.equal(db8[:, 1:].cpu(), torch.zeros(N, 7))
    else:  # nothing written past the vector
        assert torch.isnan(buf[N * (M - 8) + N:].cpu()).all()
    if splitk:
        assert int(kw["sk"][2].abs().sum()) == 0


def _mn_major(p, a_t, w_t, ldw):
    p.a_t, p.w_t, p.ldw = a_t, w_t, ldw
    return p


@pytest.mark.parametrize("impl", [0, 1, 8])
@pytest.mark.parametrize("splitk", [0, 3])
@pytest.mark.parametrize("M,N,K,act", [(1056, 768, 2304, 0), (200, 136, 1000, 5), (4224, 3072, 768, 5), (96, 64, 72, 0)])
def test_gemm_mn_major_w(impl, splitk, M, N, K, act):
    """w_t 1 (the Linear backward's dX = dY W): W given MN-major as W^T [K][ldw] and read with
    ds_read_b64_tr_b16; plain and GELU-backward (act 5) epilogues, K tails (K % 64 != 0), row / column
    tails, split-K (impl 8's register hand-off: bit-identical to impl 1's split); every launch repeats bitwise;
    impl -1 / 2 reject the mode."""
    L = _lib()
    g = torch.Generator().manual_seed(M + N + K + act)
    A = torch.randn(M, K, generator=g).bfloat16()
    Wt = (torch.randn(K, N + 8, generator=g) / math.sqrt(K)).bfloat16()  # pitch N + 8 (ldw > N)
    b = torch.randn(N, generator=g)
    R = (torch.randn(M, N, generator=g) * 2).bfloat16()
    Ad, Wd, bd, Rd = A.cuda(), Wt.cuda(), b.cuda(), R.cuda()
    kw = {"r": [Rd.data_ptr()], "ldr": N, "r_t": 1} if act == 5 else {}
    if splitk:
        kw["sk"] = (splitk, torch.empty(8 << 20, device="cuda"), torch.zeros(1 << 16, device="cuda", dtype=torch.int32))
    outs = []
    for rep in range(2):
        c = torch.full((M, N), float("nan"), device="cuda")
        p = _mn_major(_gemm_params([Ad.data_ptr()], [Wd.data_ptr()], [c.data_ptr()], M, N, K, K, N, bias=[bd.data_ptr()],
                                   act=act, c_f32=1, impl=impl, **kw), 0, 1, N + 8)
        L.check(L.LIB.mmt_gemm(p, L.MMT_BF16, torch.cuda.current_stream().cuda_stream), "gemm w_t 1")
        torch.cuda.synchronize()
        outs.append(c.cpu())
    ref = A.float() @ Wt[:, :N].float() + b
    if act == 5:
        r = R.float().requires_grad_(True)
        F.gelu(r).backward(torch.ones_like(r))
        ref = ref * r.grad
    err = (outs[0] - ref).abs().max().item()
    assert err <= 2e-3 * ref.abs().max().item() + 1e-4, err
    assert torch.equal(outs[0], outs[1])
    if splitk:
        assert int(kw["sk"][2].abs().sum()) == 0
    if splitk and impl == 8:  # the same slices on the one-per-CU tile
        c = torch.full((M, N), float("nan"), device="cuda")
        p = _mn_major(_gemm_params([Ad.data_ptr()], [Wd.data_ptr()], [c.data_ptr()], M, N, K, K, N, bias=[bd.data_ptr()],
                                   act=act, c_f32=1, impl=1, **kw), 0, 1, N + 8)
        L.check(L.LIB.mmt_gemm(p, L.MMT_BF16, torch.cuda.current_stream().cuda_stream), "gemm w_t 1")
        torch.cuda.synchronize()
        assert torch.equal(outs[0], c.cpu())
    for bad in (-1, 2):
        p = _mn_major(_gemm_params([Ad.data_ptr()], [Wd.data_ptr()], [c.data_ptr()], M, N, K, K, N, c_f32=1, impl=bad),
                      0, 1, N + 8)
        assert L.LIB.mmt_gemm(p, L.MMT_BF16, torch.cuda.current_stream().cuda_stream) == -10000


@pytest.mark.parametrize("impl", [0, 1, 8])
@pytest.mark.parametrize("splitk", [0, 4])
@pytest.mark.parametrize("M,Kx,T", [(768, 768, 8448), (2304, 768, 1000), (136, 200, 520), (3072, 768, 4224)])
def test_gemm_mn_major_dw(impl, splitk, M, Kx, T):
    """a_t 1 + w_t 2 + c2_copy 3: the Linear backward's dW / db = dY^T [X | 1] straight from dY [T][M] and
    X [T][Kx] (both MN-major, no transposed copies): dW [M][Kx] contiguous, db in column 0 of C2 [M][8],
    columns 1..7 zero; T (the contraction) not a multiple of 64; split-K (impl 8's register hand-off: bit-identical
    to impl 1's split); bitwise repeatable."""
    L = _lib()
    g = torch.Generator().manual_seed(M + Kx + T)
    dY = torch.randn(T, M, generator=g).bfloat16()
    X = torch.randn(T, Kx, generator=g).bfloat16()
    dYd, Xd = dY.cuda(), X.cuda()
    kw = {}
    if splitk:
        kw["sk"] = (splitk, torch.empty(16 << 20, device="cuda"), torch.zeros(1 << 16, device="cuda", dtype=torch.int32))
    outs = []
    for rep in range(2):
        buf = torch.full((M * (Kx + 8),), float("nan"), device="cuda")
        dw, db8 = buf[:M * Kx].view(M, Kx), buf[M * Kx:].view(M, 8)
        p = _mn_major(_gemm_params([dYd.data_ptr()], [Xd.data_ptr()], [dw.data_ptr()], M, Kx + 8, T, M, Kx, c_f32=1,
                                   c2=[db8.data_ptr()], c2_copy=3, impl=impl, **kw), 1, 2, Kx)
        L.check(L.LIB.mmt_gemm(p, L.MMT_BF16, torch.cuda.current_stream().cuda_stream), "gemm a_t 1 w_t 2")
        torch.cuda.synchronize()
        outs.append(buf.cpu())
    dw, db8 = outs[0][:M * Kx].view(M, Kx), outs[0][M * Kx:].view(M, 8)
    ref_w = dY.float().t() @ X.float()
    ref_b = dY.float().sum(0)
    assert (dw - ref_w).abs().max().item() <= 2e-3 * ref_w.abs().max().item() + 1e-4
    assert (db8[:, 0] - ref_b).abs().max().item() <= 2e-3 * ref_b.abs().max().item() + 1e-4
    assert torch.equal(db8[:, 1:], torch.zeros(M, 7))
    assert torch.equal(outs[0], outs[1])
    if splitk:
        assert int(kw["sk"][2].abs().sum()) == 0
    if splitk and impl == 8:  # the same slices on the one-per-CU tile
        buf = torch.full((M * (Kx + 8),), float("nan"), device="cuda")
        dw, db8 = buf[:M * Kx].view(M, Kx), buf[M * Kx:].view(M, 8)
        p = _mn_major(_gemm_params([dYd.data_ptr()], [Xd.data_ptr()], [dw.data_ptr()], M, Kx + 8, T, M, Kx, c_f32=1,
                                   c2=[db8.data_ptr()], c2_copy=3, impl=1, **kw), 1, 2, Kx)
        L.check(L.LIB.mmt_gemm(p, L.MMT_BF16, torch.cuda.current_stream().cuda_stream), "gemm a_t 1 w_t 2")
        torch.cuda.synchronize()
        assert torch.equal(outs[0], buf.cpu())


@pytest.mark.parametrize("impl", [1, 2, 3, 4, 6])
@pytest.mark.parametrize("splitk", [2, 3, 5])
@pytest.mark.parametrize("M,N,K", [(528, 768, 3072), (77, 200, 1024), (400, 192, 640)])
def test_gemm_splitk(impl, splitk, M, N, K):
    """Split-K over workgroups (slices summed in slice order by the last-arriving workgroup): matches
    the reference, repeats bitwise across launches (no dependence on arrival order), handles an
    in-place fp32 residual (C = R, the residual stream's X += ...) and a bf16 C2 copy, and leaves
    every ticket at zero."""
    g = torch.Generator().manual_seed(M + N + K + splitk)
    A = torch.randn(2, M, K, generator=g).bfloat16()
    W = (torch.randn(2, N, K, generator=g) / math.sqrt(K)).bfloat16()
    b = torch.randn(2, N, generator=g)
    X0 = torch.randn(2, M, N, generator=g)
    Ad, Wd, bd = A.cuda(), W.cuda(), b.cuda()
    ws = torch.empty(8 << 20, device="cuda")
    cnt = torch.zeros(1 << 16, device="cuda", dtype=torch.int32)
    ref = torch.einsum("gmk,gnk->gmn", A.float(), W.float()) + b[:, None] + X0
    outs = []
    for rep in range(3):
        X = X0.cuda()
        c2 = torch.empty(2, M, N, device="cuda", dtype=torch.bfloat16)
        _gemm([Ad[0].data_ptr(), Ad[1].data_ptr()], [Wd[0].data_ptr(), Wd[1].data_ptr()],
              [X[0].data_ptr(), X[1].data_ptr()], M, N, K, K, N, torch.bfloat16,
              bias=[bd[0].data_ptr(), bd[1].data_ptr()], r=[X[0].data_ptr(), X[1].data_ptr()], ldr=N, c_f32=1,
              c2=[c2[0].data_ptr(), c2[1].data_ptr()], c2_copy=1, impl=impl, sk=(splitk, ws, cnt))
        torch.cuda.synchronize()
        outs.append((X.cpu(), c2.cpu()))
    err = (outs[0][0] - ref).abs().max().item()
    assert err <= 1e-3 * ref.abs().max().item() + 1e-4, err
    assert torch.equal(outs[0][1], outs[0][0].bfloat16())
    for X, c2 in outs[1:]:
        assert torch.equal(X, outs[0][0]) and torch.equal(c2, outs[0][1])
    assert int(cnt.abs().sum()) == 0


def test_gemm_splitk_conv():
    """Split-K on the implicit-GEMM 3x3 conv (K = 9 * 96 = 864, a zero-filled K tail)."""
    B, h, cin, cout = 2, 20, 96, 48
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, cin, h, h, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(9 * cin)
    b = torch.randn(cout, generator=g)
    xin = x.permute(0, 2, 3, 1).contiguous().bfloat16().cuda()
    wk = w.permute(0, 2, 3, 1).reshape(cout, -1).contiguous().bfloat16().cuda()
    bd = b.cuda()
    ws = torch.empty(8 << 20, device="cuda")
    cnt = torch.zeros(1 << 16, device="cuda", dtype=torch.int32)
    ref = F.relu(F.conv2d(x.bfloat16().float(), w.bfloat16().float(), b, padding=1))
    for impl, n in ((1, 4), (3, 3), (2, 2)):
        out = torch.empty(B * h * h, cout, device="cuda")
        _gemm([xin.data_ptr()], [wk.data_ptr()], [out.data_ptr()], B * h * h, cout, 9 * cin, cin, cout, torch.bfloat16,
              bias=[bd.data_ptr()], act=2, conv=(h, 1, cin, 1), c_f32=1, impl=impl, sk=(n, ws, cnt))
        torch.cuda.synchronize()
        o = out.cpu().reshape(B, h, h, cout).permute(0, 3, 1, 2)
        assert (o - ref).abs().max().item() <= 1e-3 * ref.abs().max().item() + 1e-4, (impl, n)
    assert int(cnt.abs().sum()) == 0


@pytest.mark.parametrize("dname", ["bf16", "fp16"])
@pytest.mark.parametrize("impl", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("M,N,K", [(528, 2304, 768), (300, 136, 512)])
def test_gemm_layernorm_fold(dname, impl, M, N, K):
    """Linear(LayerNorm(x)) as one GEMM (ln_fold): A = bf16 rows of x with a nonzero mean, W' =
    W * gamma, colsum / bias' precomputed as the runtime does; two groups (modalities) with their
    own gamma / beta.  Also the producer side: c2_copy writes the bf16 copy of an fp32 C + R."""
    L = _lib()
    dt = DT[dname]
    g = torch.Generator().manual_seed(M + K)
    x = torch.randn(2, M, K, generator=g) * 2 + 0.7
    W = torch.randn(N, K, generator=g) / math.sqrt(K)
    b = torch.randn(N, generator=g)
    gam = 1 + 0.3 * torch.randn(2, K, generator=g)
    bet = 0.2 * torch.randn(2, K, generator=g)
    xb = x.to(dt)
    Wp = (W[None] * gam[:, None, :]).to(dt)                      # [2][N][K]
    colsum = Wp.float().sum(-1).contiguous()                         # [2][N]
    bp = (b[None] + torch.einsum("nk,gk->gn", W, bet)).contiguous()  # [2][N]
    xd, Wd, cd, bd = xb.cuda(), Wp.cuda(), colsum.cuda(), bp.cuda()
    out = torch.empty(2, M, N, device="cuda")
    p = L.GemmParams()
    for q in range(2):
        p.a[q], p.w[q], p.c[q], p.bias[q], p.ln_colsum[q] = (xd[q].data_ptr(), Wd[q].data_ptr(), out[q].data_ptr(),
                                                             bd[q].data_ptr(), cd[q].data_ptr())
    p.lda, p.ldc = K, N
    p.a_seg_rows, p.a_segs_a = M, 1
    p.M, p.N, p.K, p.c_f32, p.groups, p.impl, p.ln_fold, p.ln_eps = M, N, K, 1, 2, impl, 1, 1e-6
    L.check(L.LIB.mmt_gemm(p, _code(dt), torch.cuda.current_stream().cuda_stream), "gemm_ln")
    torch.cuda.synchronize()
    for q in range(2):
        ref = F.layer_norm(xb[q].float(), (K,), gam[q], bet[q], 1e-6) @ W.t() + b
        err = (out[q].cpu() - ref).abs().max().item()
        assert err <= 1e-2 * ref.abs().max().item(), (q, err)
    # producer: C (fp32) = A W^T + bias + R and C2 = bf16 copy of C
    R = torch.randn(M, N, generator=g)
    Rd = R.cuda()
    c1 = torch.empty(M, N, device="cuda")
    c2 = torch.empty(M, N, device="cuda", dtype=dt)
    _gemm([xd[0].data_ptr()], [Wd[0].data_ptr()], [c1.data_ptr()], M, N, K, K, N, dt,
          bias=[bd[0].data_ptr()], r=[Rd.data_ptr()], ldr=N, c_f32=1, c2=[c2.data_ptr()], impl=impl, c2_copy=1)
    torch.cuda.synchronize()
    ref = xb[0].float() @ Wp[0].float().t() + bp[0] + R
    assert (c1.cpu() - ref).abs().max().item() <= 1e-3 * ref.abs().max().item() + 1e-4
    assert torch.equal(c2.cpu(), c1.cpu().to(dt))


@pytest.mark.parametrize("dname", ["bf16", "fp16"])
@pytest.mark.parametrize("pimpl,cimpl", [(1, 1), (2, 3), (3, 2), (0, 0), (6, 5), (5, 6), (8, 0), (0, 8)])
def test_gemm_layernorm_stats_handoff(dname, pimpl, cimpl):
    """ln_stats_out / ln_fold 2: a producer GEMM (C fp32 = A W^T + b + R, C2 = its 16-bit copy) also
    writes the per-64-column row statistics of C2; the LayerNorm-folded consumer reads them instead
    of summing its A fragments.  Equal to the in-loop statistics (ln_fold 1) up to fp32 summation
    order, and to Linear(LayerNorm(C2)) in fp32."""
    L = _lib()
    dt = DT[dname]
    g = torch.Generator().manual_seed(7)
    M, K0, C, N = 300, 256, 768, 1152
    x = torch.randn(M, K0, generator=g).to(dt)
    W0 = (torch.randn(C, K0, generator=g) / math.sqrt(K0)).to(dt)
    b0 = torch.randn(C, generator=g)
    R = torch.randn(M, C, generator=g) * 3 + 0.5
    W = torch.randn(N, C, generator=g) / math.sqrt(C)
    b = torch.randn(N, generator=g)
    gam, bet = 1 + 0.3 * torch.randn(C, generator=g), 0.2 * torch.randn(C, generator=g)
    Wp = (W * gam[None]).to(dt)
    colsum, bp = Wp.float().sum(-1).contiguous(), (b + W @ bet).contiguous()
    xd, W0d, b0d, Rd, Wd, cd, bd = [t.cuda() for t in (x, W0, b0, R, Wp, colsum, bp)]
    c1 = torch.empty(M, C, device="cuda")
    c2 = torch.empty(M, C, device="cuda", dtype=dt)
    stats = torch.full((M, 2 * (C // 64)), float("nan"), device="cuda")
    p = L.GemmParams()
    p.a[0], p.w[0], p.c[0], p.c2[0], p.bias[0], p.r[0] = (xd.data_ptr(), W0d.data_ptr(), c1.data_ptr(), c2.data_ptr(),
                                                          b0d.data_ptr(), Rd.data_ptr())
    p.ln_stats_out[0] = stats.data_ptr()
    p.lda, p.ldc, p.ldr, p.a_seg_rows, p.a_segs_a = K0, C, C, M, 1
    p.M, p.N, p.K, p.c_f32, p.groups, p.impl, p.c2_copy = M, C, K0, 1, 1, pimpl, 1
    L.check(L.LIB.mmt_gemm(p, _code(dt), torch.cuda.current_stream().cuda_stream), "producer")
    torch.cuda.synchronize()
    v = c2.float().cpu().reshape(M, C // 64, 64)
    ref_st = torch.stack([v.sum(-1), (v * v).sum(-1)], -1).reshape(M, -1)
    assert torch.allclose(stats.cpu(), ref_st, rtol=1e-5, atol=1e-3), (stats.cpu() - ref_st).abs().max()
    outs = []
    for mode in (1, 2):
        out = torch.empty(M, N, device="cuda")
        q = L.GemmParams()
        q.a[0], q.w[0], q.c[0], q.bias[0], q.ln_colsum[0] = c2.data_ptr(), Wd.data_ptr(), out.data_ptr(), bd.data_ptr(), cd.data_ptr()
        if mode == 2:
            q.ln_stats_in[0] = stats.data_ptr()
        q.lda, q.ldc, q.a_seg_rows, q.a_segs_a = C, N, M, 1
        q.M, q.N, q.K, q.c_f32, q.groups, q.ln_fold, q.ln_eps = M, N, C, 1, 1, mode, 1e-6
        q.impl = 0 if cimpl == 8 and mode == 1 else cimpl  # (impl 8 folds handed-in statistics only)
        L.check(L.LIB.mmt_gemm(q, _code(dt), torch.cuda.current_stream().cuda_stream), "consumer")
        torch.cuda.synchronize()
        outs.append(out.cpu())
    ref = F.layer_norm(c2.float().cpu(), (C,), gam, bet, 1e-6) @ W.t() + b
    for o in outs:
        assert (o - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()
    assert (outs[0] - outs[1]).abs().max().item() <= 1e-4 * ref.abs().max().item()


@pytest.mark.parametrize("dname,impl", [("f32", 0), ("bf16", -1), ("bf16", 1), ("bf16", 2), ("bf16", 3), ("bf16", 5), ("bf16", 6),
                                        ("fp16", 1), ("fp16", -1)])
@pytest.mark.parametrize("h,up,cin,cout", [(20, 1, 64, 96), (40, 2, 32, 48), (10, 1, 16, 200), (20, 1, 96, 48), (80, 4, 48, 32)])
def test_conv3x3_implicit_gemm(dname, impl, h, up, cin, cout):
    """3x3/pad-1 conv as implicit GEMM on every kernel (impl); K = 9*cin is not a multiple of the
    64-deep K-step for cin = 16 / 32 / 96 (zero-filled K tail)."""
    dt = DT[dname]
    B = 2
    g = torch.Generator().manual_seed(h + cin)
    hi = h // up
    x = torch.randn(B, cin, hi, hi, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(9 * cin)
    b = torch.randn(cout, generator=g)
    res = torch.randn(B, cout, hi, hi, generator=g)  # residual at the input resolution, read upsampled
    xin = x.permute(0, 2, 3, 1).contiguous().to(dt).cuda()
    wk = w.permute(0, 2, 3, 1).reshape(cout, -1).contiguous().to(dt).cuda()
    rr = res.permute(0, 2, 3, 1).contiguous().cuda()
    out = torch.empty(B * h * h, cout, device="cuda", dtype=dt)
    out2 = torch.empty_like(out)
    bd = b.cuda()
    _gemm([xin.data_ptr()], [wk.data_ptr()], [out.data_ptr()], B * h * h, cout, 9 * cin, cin, cout, dt,
          bias=[bd.data_ptr()], act=2, conv=(h, up, cin, 1), c2=[out2.data_ptr()], r=[rr.data_ptr()], ldr=cout,
          r_mode=2, r_p0=h, r_p1=up, impl=impl)
    torch.cuda.synchronize()
    xu = F.interpolate(x.to(dt).float(), scale_factor=up) if up > 1 else x.to(dt).float()
    ref = F.relu(F.conv2d(xu, w.to(dt).float(), b, padding=1))
    ref2 = ref + (F.interpolate(res, scale_factor=up) if up > 1 else res)
    o = out.float().cpu().reshape(B, h, h, cout).permute(0, 3, 1, 2)
    o2 = out2.float().cpu().reshape(B, h, h, cout).permute(0, 3, 1, 2)
    tol = _tol(dt) * ref2.abs().max().item() + 1e-5
    assert (o - ref).abs().max().item() <= tol
    assert (o2 - ref2).abs().max().item() <= tol


def _multi_problems(dt, mode):
    """Independent problems for mmt_gemm_multi: mode "conv" = the corner head's conv4 / adjust4[0] /
    adjust3[1] shapes at batch 1 (2 groups each, upsampled input and residual on one), "gemm" = the
    fusion encoder's value Linear (bf16 out, bias) beside its offset / logit Linear (K split over two
    operands, fp32 out, row-mapped residual)."""
    g = torch.Generator().manual_seed(11 if mode == "conv" else 12)
    keep, probs = [], []

    def T(*shape, scale=1.0, dtype=None):
        t = (torch.randn(*shape, generator=g) * scale).to(dtype or dt).cuda()
        keep.append(t)
        return t
    if mode == "conv":
        for h, up, cin, cout, res in ((80, 2, 96, 48, False), (40, 1, 96, 48, True), (20, 1, 96, 48, False)):
            hi = h // up
            xs = [T(hi * hi, cin) for _ in range(2)]
            ws = [T(cout, 9 * cin, scale=1 / math.sqrt(9 * cin)) for _ in range(2)]
            bs = [T(cout, dtype=torch.float32) for _ in range(2)]
            outs = [torch.zeros(h * h, cout, device="cuda", dtype=dt) for _ in range(2)]
            keep += outs
            kw = dict(bias=[b.data_ptr() for b in bs], act=2, conv=(h, up, cin, 1))
            if res:
                rs = [T(h * h, cout, dtype=torch.float32) for _ in range(2)]
                o2 = [torch.zeros_like(outs[0]) for _ in range(2)]
                keep += o2
                kw.update(r=[r.data_ptr() for r in rs], c2=[o.data_ptr() for o in o2], ldr=cout)
                outs += o2
            probs.append(((h * h, cout, 9 * cin, cin, cout), [x.data_ptr() for x in xs], [w.data_ptr() for w in ws],
                          [o.data_ptr() for o in outs[:2]], kw, outs))
    else:
        Mf, dm = 400, 512
        src = T(2 * Mf, dm)
        wv, bv = T(dm, dm, scale=dm ** -0.5), T(dm, dtype=torch.float32)
        val = torch.zeros(2 * Mf, dm, device="cuda", dtype=dt)
        wo, pos = T(192, 2 * dm, scale=(2 * dm) ** -0.5), T(400, 192, dtype=torch.float32)
        offw = torch.zeros(Mf, 192, device="cuda")
        keep += [val, offw]
        probs.append(((2 * Mf, dm, dm, dm, dm), [src.data_ptr()], [wv.data_ptr()], [val.data_ptr()],
                      dict(bias=[bv.data_ptr()]), [val]))
        probs.append(((Mf, 192, 2 * dm, dm, 192), [src.data_ptr()], [wo.data_ptr()], [offw.data_ptr()],
                      dict(a1=[src.data_ptr() + Mf * dm * src.element_size()], k_split=dm, r=[pos.data_ptr()], ldr=192,
                           r_mode=1, r_p0=400, c_f32=1), [offw]))
    return probs, keep


@pytest.mark.parametrize("dname", ["bf16", "fp16", "f32"])
@pytest.mark.parametrize("mode", ["conv", "gemm"])
def test_gemm_multi_matches_single_launches(dname, mode):
    """mmt_gemm_multi (several independent problems in one launch, the head's conv chains and the
    encoder's value / offset Linears) writes exactly what one mmt_gemm per problem writes for the
    same forced tile shape (impl 1-4; 16-bit: one multi-problem launch, fp32: the per-problem
    fallback), and the auto choice agrees within the tile shapes' fp32 summation order."""
    L = _lib()
    dt = DT[dname]
    probs, keep = _multi_problems(dt, mode)
    st = torch.cuda.current_stream().cuda_stream

    def run(impl, multi):
        for *_, outs in probs:
            for o in outs:
                o.zero_()
        ps = [_gemm_params(a, w, c, *shape, impl=impl, **kw) for shape, a, w, c, kw, _ in probs]
        if multi:
            arr = (L.GemmParams * len(ps))(*ps)
            L.check(L.LIB.mmt_gemm_multi(arr, len(ps), _code(dt), st), "mmt_gemm_multi")
        else:
            for p in ps:
                L.check(L.LIB.mmt_gemm(p, _code(dt), st), "mmt_gemm")
        torch.cuda.synchronize()
        return [o.float().cpu().clone() for *_, outs in probs for o in outs]
    for impl in ((1, 2, 3, 4) if dt != torch.float32 else (0,)):
        single, multi = run(impl, False), run(impl, True)
        for a, b in zip(single, multi):
            assert torch.equal(a, b), impl
    ref, multi = run(0, False), run(0, True)
    for a, b in zip(ref, multi):
        assert (a - b).abs().max().item() <= _tol(dt) * max(1.0, a.abs().max().item())


def test_gemm_multi_rejects_bad_counts():
    L = _lib()
    arr = (L.GemmParams * 5)()
    st = torch.cuda.current_stream().cuda_stream
    for n in (0, 5):
        assert L.LIB.mmt_gemm_multi(arr, n, L.MMT_BF16, st) == -10000  # MMT_EBADARG


def _attn_ref(qkv, S, Bm, ntok, n_t, C, H, asym):
    d = C // H
    q, k, v = qkv.view(S, ntok, 3, H, d).permute(2, 0, 3, 1, 4).unbind(0)
    out = torch.empty(S, H, ntok, d)
    sc = d ** -0.5
    for s in range(S):
        out[s, :, :n_t] = torch.softmax(q[s, :, :n_t] @ k[s, :, :n_t].transpose(-1, -2) * sc, -1) @ v[s, :, :n_t]
        if asym:
            b = s % Bm
            kk = torch.cat([k[b, :, :n_t], k[b + Bm, :, :n_t], k[s, :, n_t:]], 1)
            vv = torch.cat([v[b, :, :n_t], v[b + Bm, :, :n_t], v[s, :, n_t:]], 1)
        else:
            kk, vv = k[s], v[s]
        out[s, :, n_t:] = torch.softmax(q[s, :, n_t:] @ kk.transpose(-1, -2) * sc, -1) @ vv
    return out.permute(0, 2, 1, 3).reshape(S, ntok, C)


ATTN_BF16_IMPLS = [4, 8, 17, 21, 22]


@pytest.mark.parametrize("dname,impl", [("f32", 0), ("bf16", 0)] + [("bf16", i) for i in ATTN_BF16_IMPLS]
                         + [("fp16", i) for i in (0, 4, 8)])
@pytest.mark.parametrize("asym", [0, 1])
@pytest.mark.parametrize("Bm,ntok,n_t,H", [(1, 528, 128, 12), (2, 100, 36, 2), (1, 70, 8, 1), (1, 864, 288, 2)])
def test_mam_attention(dname, impl, asym, Bm, ntok, n_t, H):
    """impl = key groups of the bf16 kernel (2 / 4); (1, 864, 288) is the ViT-L 192/384 shape
    (14 / 18 key tiles: more tiles than ring slots)."""
    dt = DT[dname]
    L = _lib()
    S, C = 2 * Bm, 64 * H
    g = torch.Generator().manual_seed(ntok + asym)
    qkv = torch.randn(S, ntok, 3 * C, generator=g)
    qd = qkv.to(dt).cuda()
    out = torch.empty(S, ntok, C, device="cuda", dtype=dt)
    p = L.AttnParams()
    p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym, p.scale = qd.data_ptr(), out.data_ptr(), S, Bm, ntok, n_t, C, H, asym, 0.125
    p.impl = impl
    L.check(L.LIB.mmt_mam_attention(p, _code(dt),
                                    torch.cuda.current_stream().cuda_stream), "attn")
    torch.cuda.synchronize()
    ref = _attn_ref(qkv.to(dt).float(), S, Bm, ntok, n_t, C, H, asym)
    err = (out.float().cpu() - ref).abs().max().item()
    assert err <= (1.5e-2 if dt != torch.float32 else 2e-5), err


@pytest.mark.parametrize("dname,impl", [("f32", 0), ("bf16", 0)] + [("bf16", i) for i in ATTN_BF16_IMPLS]
                         + [("fp16", i) for i in (0, 4, 8)])
def test_mam_attention_rescale_branch(dname, impl):
    """Online-softmax rescale forced: one key per query block carries a huge score in a late tile
    (bf16: and in a different key group than the first tile, so the group merge rescales)."""
    dt = DT[dname]
    L = _lib()
    S, Bm, ntok, n_t, H, C = 2, 1, 528, 128, 1, 64
    g = torch.Generator().manual_seed(9)
    qkv = torch.randn(S, ntok, 3 * C, generator=g) * 0.5
    qkv[:, 500, C:2 * C] = qkv[:, 300, :C] * 6  # key 500 aligned with query 300
    qd = qkv.to(dt).cuda()
    out = torch.empty(S, ntok, C, device="cuda", dtype=dt)
    p = L.AttnParams()
    p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym, p.scale = qd.data_ptr(), out.data_ptr(), S, Bm, ntok, n_t, C, H, 0, 0.125
    p.impl = impl
    L.check(L.LIB.mmt_mam_attention(p, _code(dt),
                                    torch.cuda.current_stream().cuda_stream), "attn")
    torch.cuda.synchronize()
    ref = _attn_ref(qkv.to(dt).double(), S, Bm, ntok, n_t, C, H, 0).float()
    assert (out.float().cpu() - ref).abs().max().item() < (1.5e-2 if dt != torch.float32 else 5e-5)


@pytest.mark.parametrize("impl", [0, 4, 8, 17, 21, 22])
@pytest.mark.parametrize("asym", [0, 1])
def test_mam_attention_prescaled_q(impl, asym):
    """The runtime's convention (bf16): q arrives multiplied by scale * log2(e) (folded into the qkv
    weights) and mmt_attn_params.scale = 1 / log2(e); both bf16 kernels must give softmax(q k^T * scale) v."""
    L = _lib()
    Bm, ntok, n_t, H = 3, 528, 128, 4
    S, C = 2 * Bm, 64 * H
    g = torch.Generator().manual_seed(77 + asym)
    qkv = torch.randn(S, ntok, 3 * C, generator=g)
    c = 0.125 * 1.4426950408889634
    qs = qkv.clone()
    qs[..., :C] *= c
    qd = qs.bfloat16().cuda()
    out = torch.empty(S, ntok, C, device="cuda", dtype=torch.bfloat16)
    p = L.AttnParams()
    p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym = qd.data_ptr(), out.data_ptr(), S, Bm, ntok, n_t, C, H, asym
    p.scale, p.impl = 1.0 / 1.4426950408889634, impl
    L.check(L.LIB.mmt_mam_attention(p, L.MMT_BF16, torch.cuda.current_stream().cuda_stream), "attn")
    torch.cuda.synchronize()
    qr = qs.bfloat16().float()
    qr[..., :C] /= c
    ref = _attn_ref(qr, S, Bm, ntok, n_t, C, H, asym)
    err = (out.float().cpu() - ref).abs().max().item()
    assert err <= 1.5e-2, err


@pytest.mark.parametrize("impl", [0, 4, 8, 17, 21, 22])
@pytest.mark.parametrize("asym", [0, 1])
def test_mam_attention_extreme_scores(impl, asym):
    """Scores far outside the fp32 exponent range of exp2 without a reference point: a key that
    overflows it for one query (key 500 = 60 x query 300) and a query whose every score is huge in
    magnitude (query 310 x 40: both signs).  The range-checked kernels (16, 17) must detect this in
    their epilogue and take the exact two-pass fallback; every kernel must match the fp64 softmax."""
    L = _lib()
    Bm, ntok, n_t, H = 2, 528, 128, 2
    S, C = 2 * Bm, 64 * H
    g = torch.Generator().manual_seed(5 + asym)
    qkv = torch.randn(S, ntok, 3 * C, generator=g) * 0.5
    qkv[:, 500, C:2 * C] = qkv[:, 300, :C] * 60
    qkv[:, 310, :C] *= 40
    qkv[:, 40, :C] *= 40  # a template query too
    qd = qkv.bfloat16().cuda()
    out = torch.empty(S, ntok, C, device="cuda", dtype=torch.bfloat16)
    p = L.AttnParams()
    p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym, p.scale = qd.data_ptr(), out.data_ptr(), S, Bm, ntok, n_t, C, H, asym, 0.125
    p.impl = impl
    L.check(L.LIB.mmt_mam_attention(p, L.MMT_BF16, torch.cuda.current_stream().cuda_stream), "attn")
    torch.cuda.synchronize()
    ref = _attn_ref(qkv.bfloat16().double(), S, Bm, ntok, n_t, C, H, asym).float()
    o = out.float().cpu()
    assert torch.isfinite(o).all()
    assert (o - ref).abs().max().item() < 2.5e-2 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("asym", [0, 1])
def test_mam_attention_pipelined_is_default_and_bitwise(asym):
    """impl 21 (impl 17 with the two blocks of each tile software-pipelined) and impl 22 (64
    queries per wave sharing the K / V fragments) compute the same MFMAs and exponentials per query
    in the same accumulation order, so their outputs are bit-identical to impl 17's; impl 0 launches
    impl 22 on this grid (B = 8: 960 workgroups of 128 queries)."""
    L = _lib()
    Bm, ntok, n_t, H = 8, 528, 128, 12
    S, C = 2 * Bm, 64 * H
    g = torch.Generator().manual_seed(123 + asym)
    qkv = torch.randn(S, ntok, 3 * C, generator=g) * 0.5
    qkv[..., :C] *= 0.125 * 1.4426950408889634  # the runtime's pre-scaled q
    qd = qkv.bfloat16().cuda()
    outs = {}
    for impl in (17, 21, 22, 0):
        out = torch.empty(S, ntok, C, device="cuda", dtype=torch.bfloat16)
        p = L.AttnParams()
        p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym = qd.data_ptr(), out.data_ptr(), S, Bm, ntok, n_t, C, H, asym
        p.scale, p.impl = 1.0 / 1.4426950408889634, impl
        L.check(L.LIB.mmt_mam_attention(p, L.MMT_BF16, torch.cuda.current_stream().cuda_stream), "attn")
        torch.cuda.synchronize()
        outs[impl] = out
    assert torch.equal(outs[17], outs[21])
    assert torch.equal(outs[17], outs[22])
    assert torch.equal(outs[22], outs[0])
    qr = qkv.bfloat16().float()
    qr[..., :C] /= 0.125 * 1.4426950408889634
    # every sequence (joint and cross-modal asymmetric key streams) against the fp32 reference at
    # this grid, i.e. the impl-22 default of BASELINE config 3's per-rank batch
    ref = _attn_ref(qr, S, Bm, ntok, n_t, C, H, asym)
    err = (outs[0].float().cpu() - ref).abs().max().item()
    assert err <= 1.5e-2, err


def _attn_run(L, qd, S, Bm, ntok, n_t, C, H, asym, impl, scale=1.0 / 1.4426950408889634, **kw):
    out = torch.full((S, kw.get("out_rows", ntok), C), float("nan"), device="cuda", dtype=torch.bfloat16)
    p = L.AttnParams()
    p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym = qd.data_ptr(), out.data_ptr(), S, Bm, ntok, n_t, C, H, asym
    p.scale, p.impl = scale, impl
    rc = L.LIB.mmt_mam_attention(p, L.MMT_BF16, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return rc, out


@pytest.mark.parametrize("asym", [0, 1])
@pytest.mark.parametrize("Bm", [1, 3, 8, 32])
def test_mam_attention_persistent_bitwise(asym, Bm):
    """impl 29 (persistent one-wave-per-SIMD workgroups walking (sequence, head) items over a continuous
    K / V tile stream) computes impl 22's MFMAs and exponentials in the same order per query: bitwise
    equal outputs at every grid size (B = 1: fewer items than CUs; B = 32: six items per workgroup),
    on the joint and the cross-modal key streams, every output row written."""
    L = _lib()
    ntok, n_t, H = 528, 128, 12
    S, C = 2 * Bm, 64 * H
    g = torch.Generator().manual_seed(400 + Bm + asym)
    qkv = torch.randn(S, ntok, 3 * C, generator=g) * 0.5
    qkv[..., :C] *= 0.125 * 1.4426950408889634  # the runtime's pre-scaled q
    qd = qkv.bfloat16().cuda()
    rc22, o22 = _attn_run(L, qd, S, Bm, ntok, n_t, C, H, asym, 22)
    rc29, o29 = _attn_run(L, qd, S, Bm, ntok, n_t, C, H, asym, 29)
    assert rc22 == 0 and rc29 == 0
    assert not torch.isnan(o29).any()
    assert torch.equal(o22, o29)
    if Bm <= 3:
        qr = qkv.bfloat16().float()
        qr[..., :C] /= 0.125 * 1.4426950408889634
        ref = _attn_ref(qr, S, Bm, ntok, n_t, C, H, asym)
        assert (o29.float().cpu() - ref).abs().max().item() <= 1.5e-2


@pytest.mark.parametrize("asym", [0, 1])
def test_mam_attention_persistent_natural_scale_and_fallback(asym):
    """impl 29 with q at its natural scale (the kernel pre-scales Q in registers) and with scores outside
    exp2's range without a reference point (the exact two-pass fallback, stored in place while the other
    query blocks go through the staged stores): bitwise equal to impl 22 and to the fp64 softmax."""
    L = _lib()
    Bm, ntok, n_t, H = 2, 528, 128, 4
    S, C = 2 * Bm, 64 * H
    g = torch.Generator().manual_seed(31 + asym)
    qkv = torch.randn(S, ntok, 3 * C, generator=g) * 0.5
    qkv[:, 500, C:2 * C] = qkv[:, 300, :C] * 60
    qkv[:, 310, :C] *= 40
    qkv[:, 40, :C] *= 40  # a template query (template wave of the mixed item)
    qkv[:, 520, :C] *= 40  # a query of the 16-query last block
    qd = qkv.bfloat16().cuda()
    rc22, o22 = _attn_run(L, qd, S, Bm, ntok, n_t, C, H, asym, 22, scale=0.125)
    rc29, o29 = _attn_run(L, qd, S, Bm, ntok, n_t, C, H, asym, 29, scale=0.125)
    assert rc22 == 0 and rc29 == 0
    assert torch.equal(o22, o29)
    ref = _attn_ref(qkv.bfloat16().double(), S, Bm, ntok, n_t, C, H, asym).float()
    o = o29.float().cpu()
    assert torch.isfinite(o).all()
    assert (o - ref).abs().max().item() < 2.5e-2 * max(1.0, ref.abs().max().item())


def test_mam_attention_persistent_rejects_other_shapes():
    """impl 29 takes the ViT-B 128/320 token layout only (n_t 128, 400 search tokens, all queries):
    other shapes and the template K/V cache's partial passes are refused, nothing launched."""
    L = _lib()
    qd = torch.zeros(2, 864, 3 * 128, device="cuda", dtype=torch.bfloat16)
    assert _attn_run(L, qd, 2, 1, 864, 288, 128, 2, 0, 29)[0] == -10000
    qd = torch.zeros(2, 528, 3 * 128, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(2, 528, 128, device="cuda", dtype=torch.bfloat16)
    p = L.AttnParams()
    p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym = qd.data_ptr(), out.data_ptr(), 2, 1, 528, 128, 128, 2, 0
    p.scale, p.impl, p.q_part = 1.0, 29, 2
    assert L.LIB.mmt_mam_attention(p, L.MMT_BF16, torch.cuda.current_stream().cuda_stream) == -10000


@pytest.mark.parametrize("dname", ["f32", "bf16", "fp16"])
@pytest.mark.parametrize("C", [256, 512, 768, 1024])
def test_layernorm_groups_and_add(dname, C):
    dt = DT[dname]
    L = _lib()
    rows, rpg = 50, 25
    g = torch.Generator().manual_seed(C)
    x = torch.randn(rows, C, generator=g) * 3 + 1
    add = torch.randn(rpg, C, generator=g)
    ga, ba, gb, bb = (torch.randn(C, generator=g) for _ in range(4))
    xd = x.cuda()
    of = torch.empty(rows, C, device="cuda")
    ot = torch.empty(rows, C, device="cuda", dtype=dt)
    gs = [t.cuda() for t in (ga, ba, gb, bb)]
    addd = add.cuda()
    L.check(L.LIB.mmt_layernorm(xd.data_ptr(), addd.data_ptr(), rpg, of.data_ptr(), ot.data_ptr(),
                                *[t.data_ptr() for t in gs], rows, rpg, C, 1e-5,
                                _code(dt),
                                torch.cuda.current_stream().cuda_stream), "ln")
    torch.cuda.synchronize()
    xa = x + torch.cat([add, add])
    ref = torch.cat([F.layer_norm(xa[:rpg], (C,), ga, ba, 1e-5), F.layer_norm(xa[rpg:], (C,), gb, bb, 1e-5)])
    assert (of.cpu() - ref).abs().max().item() < 2e-5
    assert (ot.float().cpu() - ref).abs().max().item() < (3e-2 if dt != torch.float32 else 2e-5)


def test_groupnorm():
    L = _lib()
    n, P, Ct, G = 4, 400, 768, 32
    g = torch.Generator().manual_seed(2)
    x = torch.randn(n, P, Ct, generator=g) * 2 + 0.5
    ga, ba, gb, bb = (torch.randn(Ct, generator=g) for _ in range(4))
    out = torch.empty(n, P, Ct, device="cuda")
    gs = [t.cuda() for t in (ga, ba, gb, bb)]
    xd = x.cuda()
    L.check(L.LIB.mmt_groupnorm(xd.data_ptr(), out.data_ptr(), None, *[t.data_ptr() for t in gs], n, 2, P, Ct, G,
                                1e-5, L.MMT_F32, torch.cuda.current_stream().cuda_stream), "gn")
    torch.cuda.synchronize()
    xin = x.permute(0, 2, 1)
    ref = torch.cat([F.group_norm(xin[:2], G, ga, ba, 1e-5), F.group_norm(xin[2:], G, gb, bb, 1e-5)]).permute(0, 2, 1)
    assert (out.cpu() - ref).abs().max().item() < 3e-5


def _msda_call(value, shapes, starts, loc, w, dtcode):
    L = _lib()
    N, S, M, D = value.shape
    _, Lq, _, Lv, Pn, _ = loc.shape
    out = torch.empty(N, Lq, M * D, device="cuda", dtype=value.dtype)
    sh = torch.as_tensor(shapes, dtype=torch.long).cuda()
    st = torch.as_tensor(starts, dtype=torch.long).cuda()
    L.check(L.LIB.mmt_ms_deform_attn_forward(value.data_ptr(), sh.data_ptr(), st.data_ptr(), loc.data_ptr(), w.data_ptr(),
                                             out.data_ptr(), N, S, M, D, Lq, Lv, Pn, dtcode,
                                             torch.cuda.current_stream().cuda_stream), "msda")
    torch.cuda.synchronize()
    return out.cpu()


@pytest.mark.parametrize("tag", ["double", "float"])
def test_msda_reference_op_test_vectors(tag):
    """ops/test.py:28-59 cases (golden vectors from the reference's own pytorch core)."""
    L = _lib()
    z = np.load(GOLDEN + "/op_msda.npz")
    dt = torch.float64 if tag == "double" else torch.float32
    v = torch.from_numpy(z["test_%s_value" % tag]).to(dt).cuda()
    loc = torch.from_numpy(z["test_%s_loc" % tag]).to(dt).cuda()
    w = torch.from_numpy(z["test_%s_w" % tag]).to(dt).cuda()
    out = _msda_call(v, [(6, 4), (3, 2)], [0, 24], loc, w, L.MMT_F64 if tag == "double" else L.MMT_F32)
    ref = torch.from_numpy(z["test_%s_out" % tag])
    if tag == "double":
        assert torch.allclose(out, ref.double())
    else:
        assert torch.allclose(out, ref, rtol=1e-2, atol=1e-3)
        assert (out - ref).abs().max().item() < 1e-7


@pytest.mark.parametrize("channels", [30, 32, 64, 71, 1025, 2048, 3096])
def test_msda_channels_sweep(channels):
    """Channel counts of ops/test.py:62-89 (forward parity vs the oracle restatement, fp64)."""
    from oracle.msda import ms_deform_attn
    L = _lib()
    torch.manual_seed(3)
    shapes = [(6, 4), (3, 2)]
    v = torch.rand(1, 30, 2, channels, dtype=torch.float64) * 0.01
    loc = torch.rand(1, 2, 2, 2, 2, 2, dtype=torch.float64)
    w = torch.rand(1, 2, 2, 2, 2, dtype=torch.float64) + 1e-5
    w /= w.sum(-1, keepdim=True).sum(-2, keepdim=True)
    out = _msda_call(v.cuda(), shapes, [0, 24], loc.cuda(), w.cuda(), L.MMT_F64)
    ref = ms_deform_attn(v, shapes, [0, 24], loc, w)
    assert torch.allclose(out, ref, rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("dname", ["f32", "bf16", "fp16"])
def test_msda_bimodal_vs_oracle(dname):
    from oracle.msda import ms_deform_attn
    dt = DT[dname]
    L = _lib()
    B, hw = 2, 20
    nq = hw * hw
    g = torch.Generator().manual_seed(11)
    value = torch.randn(2, B, nq, 512, generator=g)
    offw = torch.randn(B * nq, 192, generator=g)
    offw[:, :128] *= 3.0
    out = torch.empty(B * nq, 512, device="cuda", dtype=dt)
    offd, vald = offw.cuda(), value.to(dt).cuda()
    L.check(L.LIB.mmt_msda_bimodal(offd.data_ptr(), vald.data_ptr(), out.data_ptr(), B, hw,
                                   _code(dt),
                                   torch.cuda.current_stream().cuda_stream), "msda_bimodal")
    torch.cuda.synchronize()
    # reference formulation (ms_deform_attn_bimodal.py:97-128) on the v-half queries
    off = offw[:, :128].view(B, nq, 8, 2, 4, 2)
    aw = torch.softmax(offw[:, 128:].view(B, nq, 8, 8), -1).view(B, nq, 8, 2, 4)
    ry, rx = torch.meshgrid(torch.linspace(0.5, hw - 0.5, hw), torch.linspace(0.5, hw - 0.5, hw), indexing="ij")
    ref_pts = torch.stack([rx.reshape(-1) / hw, ry.reshape(-1) / hw], -1)
    loc = ref_pts[None, :, None, None, None, :] + off / torch.tensor([hw, hw])
    val = torch.cat([value[0], value[1]], 1).to(dt).float().view(B, 2 * nq, 8, 64)
    ref = ms_deform_attn(val, [(hw, hw), (hw, hw)], [0, nq], loc, aw).reshape(B * nq, 512)
    err = (out.float().cpu() - ref).abs().max().item()
    assert err <= (2e-2 if dt != torch.float32 else 2e-5) * max(1.0, ref.abs().max().item()), err


def test_prroi_known_answer():
    """test_prroi_pooling2d.py:21-35: integer RoIs at scale 0.5 equal avg_pool2d(k=2, s=1) slices."""
    from oracle.prroi import prroi_pool2d
    L = _lib()
    g = torch.Generator().manual_seed(4)
    feat = torch.rand(4, 16, 24, 32, generator=g)
    rois = torch.tensor([[0, 0, 0, 14, 14], [1, 14, 14, 28, 28]], dtype=torch.float32)
    out = torch.empty(2, 16, 7, 7, device="cuda")
    fd, rd = feat.cuda(), rois.cuda()
    L.check(L.LIB.mmt_prroi_pool_forward(fd.data_ptr(), rd.data_ptr(), out.data_ptr(), 2, 16, 24, 32,
                                         16 * 24 * 32, 24 * 32, 32, 1, 7, 7, 0.5, 16 * 49, 49, 1,
                                         torch.cuda.current_stream().cuda_stream), "prroi")
    torch.cuda.synchronize()
    gold = F.avg_pool2d(feat, kernel_size=2, stride=1)
    ref = torch.stack((gold[0, :, :7, :7], gold[1, :, 7:14, 7:14]), 0)
    assert torch.allclose(out.cpu(), ref, atol=1e-5)
    o2 = torch.from_numpy(prroi_pool2d(feat.numpy(), rois.numpy(), 7, 7, 0.5))
    assert torch.allclose(out.cpu(), o2, atol=1e-6)


def test_prroi_fractional_vs_oracle():
    from oracle.prroi import prroi_pool2d
    L = _lib()
    g = torch.Generator().manual_seed(5)
    feat = torch.randn(2, 8, 20, 20, generator=g)
    rois = torch.tensor([[0, 1.3, 2.7, 15.2, 9.9], [1, -2.0, 3.5, 7.25, 21.0], [0, 5.0, 5.0, 5.0, 9.0]])
    out = torch.empty(3, 8, 4, 4, device="cuda")
    fd, rd = feat.cuda(), rois.cuda()
    L.check(L.LIB.mmt_prroi_pool_forward(fd.data_ptr(), rd.data_ptr(), out.data_ptr(), 3, 8, 20, 20,
                                         8 * 400, 400, 20, 1, 4, 4, 1.0, 8 * 16, 16, 1,
                                         torch.cuda.current_stream().cuda_stream), "prroi")
    torch.cuda.synchronize()
    ref = torch.from_numpy(prroi_pool2d(feat.numpy(), rois.numpy(), 4, 4, 1.0))
    assert (out.cpu() - ref).abs().max().item() < 1e-5


@pytest.mark.parametrize("M,N,K,act", [(1, 768, 768, 0), (3, 1024, 1024, 2), (8, 1, 768, 0), (2, 100, 64, 1),
                                       (16, 1536, 768, 0)])
def test_gemv_small_m_fp32(M, N, K, act):
    """fp32 GEMMs with M <= 8 (the score head's single-token Linears) take the GEMV path: vs torch fp64."""
    g = torch.Generator().manual_seed(M * 7 + N)
    a, w, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.05, torch.randn(N, generator=g)
    ad, wd, bd = a.cuda(), w.cuda(), b.cuda()
    c = torch.empty(M, N, device="cuda")
    _gemm([ad.data_ptr()], [wd.data_ptr()], [c.data_ptr()], M, N, K, K, N, torch.float32, bias=[bd.data_ptr()], act=act,
          c_f32=1)
    torch.cuda.synchronize()
    ref = a.double() @ w.double().T + b.double()
    ref = F.gelu(ref) if act == 1 else (F.relu(ref) if act == 2 else ref)
    assert (c.cpu().double() - ref).abs().max().item() <= 1e-4 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("B,Lk,H", [(1, 16, 12), (2, 128, 12), (1, 288, 16), (3, 300, 2)])
def test_spm_attention(B, Lk, H):
    """ScoreDecoder single-query multi-head attention (score_decoder.py:55-61) vs torch fp64."""
    L = _lib()
    C = 64 * H
    g = torch.Generator().manual_seed(Lk + H)
    q, kv = torch.randn(B, C, generator=g), torch.randn(B, Lk, 2 * C, generator=g)
    out = torch.empty(B, C, device="cuda")
    scale = C ** -0.5
    qd, kvd = q.cuda(), kv.cuda()  # keep the device copies alive across the launch
    L.check(L.LIB.mmt_spm_attention(qd.data_ptr(), C, kvd.data_ptr(), out.data_ptr(), B, Lk, C, H, scale,
                                    torch.cuda.current_stream().cuda_stream), "spm_attention")
    torch.cuda.synchronize()
    qh = q.double().view(B, H, 1, 64)
    k = kv[:, :, :C].double().view(B, Lk, H, 64).transpose(1, 2)
    v = kv[:, :, C:].double().view(B, Lk, H, 64).transpose(1, 2)
    ref = (torch.softmax(qh @ k.transpose(-1, -2) * scale, -1) @ v).view(B, C)
    err = (out.cpu().double() - ref).abs().view(B, H, 64).amax(-1)
    print("spm per (b, h) err", err)
    assert err.max().item() <= 1e-5


@pytest.mark.parametrize("dname", ["f32", "bf16", "fp16"])
def test_conv3x3_c1_pair_matches_single(dname):
    """mmt_conv3x3_c1_pair (adjust3[2] beside adjust4[1] in one launch) writes exactly what two
    mmt_conv3x3_c1 launches write (20x20 and 40x40 maps, 48 channels, padded pixel stride)."""
    L = _lib()
    dt = DT[dname]
    G, B, cin = 2, 2, 48
    g = torch.Generator().manual_seed(3)
    st = torch.cuda.current_stream().cuda_stream
    ins, ws, bs, outs, refs = [], [], [], [], []
    for h, pad in ((20, 0), (40, 8)):
        ins.append(torch.randn(G, B, h, h, cin + pad, generator=g).to(dt).cuda())
        ws.append((torch.randn(G, 9, cin, generator=g) / math.sqrt(9 * cin)).to(dt).cuda())
        bs.append((torch.randn(G, generator=g) * 0.1).cuda())
        outs.append(torch.full((G, B, h * h), float("nan"), device="cuda"))
        refs.append(torch.full((G, B, h * h), float("nan"), device="cuda"))
        L.check(L.LIB.mmt_conv3x3_c1(ins[-1].data_ptr(), ws[-1].data_ptr(), bs[-1].data_ptr(), refs[-1].data_ptr(), G, B,
                                     h, cin, cin + pad, _code(dt), st), "conv3x3_c1")
    L.check(L.LIB.mmt_conv3x3_c1_pair(ins[0].data_ptr(), ws[0].data_ptr(), bs[0].data_ptr(), outs[0].data_ptr(), 20, cin,
                                      ins[1].data_ptr(), ws[1].data_ptr(), bs[1].data_ptr(), outs[1].data_ptr(), 40,
                                      cin + 8, G, B, cin, _code(dt), st), "conv3x3_c1_pair")
    torch.cuda.synchronize()
    for o, r in zip(outs, refs):
        assert torch.equal(o.cpu(), r.cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("dname", ["f32", "bf16", "fp16"])
@pytest.mark.parametrize("h,cin,pad", [(20, 48, 0), (40, 48, 16), (10, 16, 0), (16, 96, 8)])
def test_conv3x3_c1_vs_torch(dname, h, cin, pad):
    """mmt_conv3x3_c1 (adjust3 / adjust4 closing conv, head.py:115-120): Cout = 1 3x3/pad-1 conv +
    bias + ReLU on NHWC [G][B][h*h][cin] with pixel stride cin + pad, vs F.conv2d in fp32."""
    L = _lib()
    dt = DT[dname]
    G, B = 2, 2
    g = torch.Generator().manual_seed(h * 1000 + cin + pad)
    x = torch.randn(G, B, h, h, cin + pad, generator=g)
    w = torch.randn(G, 9, cin, generator=g) / math.sqrt(9 * cin)
    b = torch.randn(G, generator=g) * 0.1
    xd, wd, bd = x.to(dt).cuda(), w.to(dt).cuda(), b.cuda()
    out = torch.empty(G, B, h * h, device="cuda")
    L.check(L.LIB.mmt_conv3x3_c1(xd.data_ptr(), wd.data_ptr(), bd.data_ptr(), out.data_ptr(), G, B, h, cin, cin + pad,
                                 _code(dt),
                                 torch.cuda.current_stream().cuda_stream), "conv3x3_c1")
    torch.cuda.synchronize()
    xr = x.to(dt).float()[..., :cin]
    wr = w.to(dt).float()
    for gi in range(G):
        ref = F.relu(F.conv2d(xr[gi].permute(0, 3, 1, 2), wr[gi].t().reshape(1, cin, 3, 3), b[gi:gi + 1], padding=1))
        got = out[gi].cpu().reshape(B, 1, h, h)
        assert (got - ref).abs().max().item() <= 1e-4 * (1 + ref.abs().max().item())


def _fixture_sub(x, n=4096):
    """tests/golden/make_golden.py's `sub`: every step-th element of the flattened output (float64 sums)."""
    f = x.detach().reshape(-1).double()
    step = max(1, f.numel() // n)
    return f[::step][:n].float(), torch.tensor([f.sum().item(), f.abs().sum().item(), f.numel()], dtype=torch.float64)


@pytest.mark.parametrize("dname", ["f32", "bf16"])
@pytest.mark.parametrize("kind", ["mam", "mam_asym"])
def test_mam_module_matches_reference_fixture(kind, dname):
    """the whole MAM `Attention` module on the GPU -- qkv Linear (mmt_gemm, bias), the MAM
    kernel the dtype's default picks (mmt_mam_attention), proj Linear (mmt_gemm, bias) -- against the
    outputs the reference's OWN modules produced (tests/golden/op_attention.npz, make_golden.py
    attention_fixture: mixformer.py:52-78 `Attention` and asymmetric_shared.py:55-104 `Attention`, B = 1,
    528 tokens of N(0,1), seed-5 inputs, synthetic weights).  Bars: fp32 1e-4, bf16 1e-2, relative to the
    output's largest magnitude (and the float64 sum of |y| within the same fraction)."""
    from mmt_amd import synthetic
    dt = DT[dname]
    L = _lib()
    z = np.load(GOLDEN + "/op_attention.npz")
    g = torch.Generator().manual_seed(5)
    x = torch.randn(1, 528, 768, generator=g)
    xi = torch.randn(1, 528, 768, generator=g)
    shapes = [("attn.qkv.weight", [2304, 768]), ("attn.qkv.bias", [2304]), ("attn.proj.weight", [768, 768]),
              ("attn.proj.bias", [768])]
    sd = {k: torch.from_numpy(v) for k, v in synthetic.synth_state_dict(shapes).items()}
    asym = kind == "mam_asym"
    X = torch.cat([x, xi], 0) if asym else x  # modality-major sequences: s = m * Bm + b
    S, M = X.shape[0], X.shape[0] * 528
    Xd = X.reshape(M, 768).to(dt).cuda()
    Wq, bq = sd["attn.qkv.weight"].to(dt).cuda(), sd["attn.qkv.bias"].cuda()
    Wp, bp = sd["attn.proj.weight"].to(dt).cuda(), sd["attn.proj.bias"].cuda()
    qkv = torch.empty(M, 2304, device="cuda", dtype=dt)
    ao = torch.empty(M, 768, device="cuda", dtype=dt)
    y = torch.empty(M, 768, device="cuda")
    _gemm([Xd.data_ptr()], [Wq.data_ptr()], [qkv.data_ptr()], M, 2304, 768, 768, 2304, dt, bias=[bq.data_ptr()])
    p = L.AttnParams()
    p.qkv, p.out, p.S, p.Bm, p.ntok, p.n_t, p.C, p.H, p.asym, p.scale = (qkv.data_ptr(), ao.data_ptr(), S, 1, 528, 128,
                                                                       768, 12, int(asym), 0.125)
    L.check(L.LIB.mmt_mam_attention(p, _code(dt), torch.cuda.current_stream().cuda_stream), "attn")
    _gemm([ao.data_ptr()], [Wp.data_ptr()], [y.data_ptr()], M, 768, 768, 768, 768, dt, bias=[bp.data_ptr()], c_f32=1)
    torch.cuda.synchronize()
    y = y.cpu().view(S, 528, 768)
    bar = 1e-4 if dt == torch.float32 else 1e-2
    outs = [(y[0], "mam")] if not asym else [(y[0], "mam_asym_v"), (y[1], "mam_asym_i")]
    for out, key in outs:
        sub, sums = _fixture_sub(out)
        ref = torch.from_numpy(z[key + "_sub"])
        scale = ref.abs().max().item()
        err = (sub - ref).abs().max().item() / scale
        assert err <= bar, (key, dname, err)
        assert abs(sums[1].item() - z[key + "_sum"][1]) <= bar * z[key + "_sum"][1], (key, sums, z[key + "_sum"])
        assert int(sums[2].item()) == int(z[key + "_sum"][2])
