"""The C-ABI library loads (without a GPU) and exports every entry point include/mmt_hip.h declares."""
import ctypes
import os
import re

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mmt_hip.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(mmt_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ("mmt_gemm", "mmt_mam_attention", "mmt_ms_deform_attn_forward", "mmt_prroi_pool_forward",
              "mmt_layernorm", "mmt_groupnorm", "mmt_msda_bimodal", "mmt_corner_softargmax"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from mmt_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert set(declared_symbols()) == set(_lib.EXPORTED)
    assert _lib.LIB.mmt_version().startswith(b"libmmt_hip")


def test_struct_layouts_match_header(tmp_path):
    """ctypes mirrors of the param structs have the C sizes and field offsets (checked by gcc)."""
    import subprocess
    from mmt_amd import _lib
    fields = [f for f, _ in _lib.GemmParams._fields_]
    afields = [f for f, _ in _lib.AttnParams._fields_]
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "%s"' % HEADER, "int main(void){",
           'printf("%zu %zu\\n", sizeof(mmt_gemm_params), sizeof(mmt_attn_params));']
    src += ['printf("%%zu\\n", offsetof(mmt_gemm_params, %s));' % f for f in fields]
    src += ['printf("%%zu\\n", offsetof(mmt_attn_params, %s));' % f for f in afields]
    src += ["return 0;}"]
    c = tmp_path / "abi.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "abi"
    subprocess.check_call(["gcc", str(c), "-o", str(exe)])
    out = subprocess.check_output([str(exe)]).decode().split()
    assert int(out[0]) == ctypes.sizeof(_lib.GemmParams)
    assert int(out[1]) == ctypes.sizeof(_lib.AttnParams)
    offs = [int(x) for x in out[2:]]
    assert offs[:len(fields)] == [getattr(_lib.GemmParams, f).offset for f in fields]
    assert offs[len(fields):] == [getattr(_lib.AttnParams, f).offset for f in afields]


def test_bad_arguments_rejected_without_gpu_work():
    """Shape validation happens on the host before any launch (MMT_EBADARG)."""
    from mmt_amd import _lib
    p = _lib.GemmParams()
    p.M, p.N, p.K, p.groups = 0, 16, 16, 1
    assert _lib.LIB.mmt_gemm(ctypes.byref(p), _lib.MMT_BF16, None) == -10000
    a = _lib.AttnParams()
    a.C, a.H = 100, 2
    assert _lib.LIB.mmt_mam_attention(ctypes.byref(a), _lib.MMT_BF16, None) == -10000
    # multi-problem GEMM: problem count out of 1..4, or any problem failing mmt_gemm's checks
    arr = (_lib.GemmParams * 5)()
    for q in arr:
        q.M, q.N, q.K, q.groups = 16, 16, 16, 1
    assert _lib.LIB.mmt_gemm_multi(arr, 0, _lib.MMT_BF16, None) == -10000
    assert _lib.LIB.mmt_gemm_multi(arr, 5, _lib.MMT_BF16, None) == -10000
    assert _lib.LIB.mmt_gemm_multi(arr, 2, _lib.MMT_BF16, None) == -10000  # null operands
    # paired Cout=1 conv: null operands / channel count not a multiple of the 16-B vector
    fake = 1 << 20
    assert _lib.LIB.mmt_conv3x3_c1_pair(None, fake, fake, fake, 20, 48, fake, fake, fake, fake, 40, 48, 2, 1, 48,
                                        _lib.MMT_BF16, None) == -10000
    assert _lib.LIB.mmt_conv3x3_c1_pair(fake, fake, fake, fake, 20, 44, fake, fake, fake, fake, 40, 44, 2, 1, 44,
                                        _lib.MMT_BF16, None) == -10000


def test_attention_impl_and_lse_gate():
    """mmt_mam_attention takes impl 0 (library choice), 4, 8, 17, 21, 22 only (the round-2 A/B-only
    kernels 2, 9-12, 16, 18-20 are no longer in the library; 23-28 -- incl. round 4's one-wave-per-SIMD
    impl 24 / 25 and round 5's ping-pong impl 28 -- are in the A/B build only); impl 22 never writes the
    log-sum-exp
    the training backward consumes, so lse with them is rejected; fp16 takes the running-maximum kernels
    only.  Every case fails validation on the host, before a launch."""
    from mmt_amd import _lib
    fake = 1 << 20  # 16-B aligned, never dereferenced

    def attn(dt=_lib.MMT_BF16, **kw):
        a = _lib.AttnParams()
        a.qkv, a.out, a.S, a.Bm, a.ntok, a.n_t, a.H, a.C, a.scale = fake, fake, 2, 1, 528, 128, 12, 768, 0.125
        for k, v in kw.items():
            setattr(a, k, v)
        return _lib.LIB.mmt_mam_attention(ctypes.byref(a), dt, None)

    for impl in (2, 9, 10, 11, 12, 16, 18, 19, 20, 23, 24, 25, 26, 27, 28, 99):
        assert attn(impl=impl) == -10000, impl
    assert attn(impl=22, lse=fake) == -10000
    assert attn(impl=23, lse=fake) == -10000
    # compact out rows (template K/V cache passes): pitch must hold the part's rows; not with lse
    assert attn(q_part=2, out_pitch=399, out_q0=128) == -10000
    assert attn(q_part=2, out_pitch=400, out_q0=129) == -10000
    assert attn(q_part=1, out_pitch=127) == -10000
    assert attn(q_part=1, out_pitch=128, lse=fake) == -10000
    assert attn(out_pitch=-1) == -10000
    assert attn(dt=_lib.MMT_F16, impl=17) == -10000
    assert attn(dt=_lib.MMT_F16, lse=fake) == -10000


def test_adamw_table_layouts_match_header(tmp_path):
    """mmt_amd.optim's numpy mirrors of mmt_adamw_tensor / mmt_adamw_chunk have the C sizes and field
    offsets (checked by gcc), and mmt_adamw_chunk_elems answers without a GPU."""
    import subprocess
    import numpy as np
    from mmt_amd import _lib
    from mmt_amd.optim import TENSOR_DTYPE, CHUNK_DTYPE
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "%s"' % HEADER, "int main(void){",
           'printf("%zu %zu\\n", sizeof(mmt_adamw_tensor), sizeof(mmt_adamw_chunk));']
    src += ['printf("%%zu\\n", offsetof(mmt_adamw_tensor, %s));' % f for f in TENSOR_DTYPE.names]
    src += ['printf("%%zu\\n", offsetof(mmt_adamw_chunk, %s));' % f for f in CHUNK_DTYPE.names]
    src += ["return 0;}"]
    c = tmp_path / "adamw.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "adamw"
    subprocess.check_call(["gcc", str(c), "-o", str(exe)])
    out = [int(x) for x in subprocess.check_output([str(exe)]).decode().split()]
    assert out[0] == TENSOR_DTYPE.itemsize and out[1] == CHUNK_DTYPE.itemsize
    offs = [TENSOR_DTYPE.fields[f][1] for f in TENSOR_DTYPE.names] + [CHUNK_DTYPE.fields[f][1] for f in CHUNK_DTYPE.names]
    assert out[2:] == offs
    assert _lib.LIB.mmt_adamw_chunk_elems() == 1 << 16
    assert _lib.LIB.mmt_adamw_step(None, None, 0, None, None, None, None, 1, 0.9, 0.999, 1e-8, 0.1, 0, None) == -10000
    _ = np
