"""ctypes binding of libmmt_hip.so (include/mmt_hip.h).

The library is the product: there is no CPU or PyTorch fallback.  If it is missing or fails to
load, importing this module raises.  torch is imported first so that the library binds to the
HIP runtime torch already loaded (same SONAME), i.e. streams and device pointers are shared.
"""
import ctypes
import os

import torch  # noqa: F401  (loads the HIP runtime the kernels must share)

# MMT_HIP_LIB may name another build of the same library (A/B or ablation builds of tools/).
LIB_PATH = os.environ.get("MMT_HIP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib",
                                                         "libmmt_hip.so")

MMT_F32, MMT_BF16, MMT_F64, MMT_F16 = 0, 1, 2, 3
MAX_GROUPS = 2

vp = ctypes.c_void_p
i32 = ctypes.c_int32
i64 = ctypes.c_int64
f32 = ctypes.c_float


class GemmParams(ctypes.Structure):
    _fields_ = [
        ("a", vp * MAX_GROUPS), ("a1", vp * MAX_GROUPS), ("w", vp * MAX_GROUPS), ("bias", vp * MAX_GROUPS),
        ("r", vp * MAX_GROUPS), ("c", vp * MAX_GROUPS), ("c2", vp * MAX_GROUPS),
        ("lda", i64), ("ldr", i64), ("ldc", i64),
        ("a_seg_rows", i64), ("a_segs_a", i64), ("a_stride_a", i64), ("a_stride_b", i64),
        ("M", i32), ("N", i32), ("K", i32), ("k_split", i32),
        ("act", i32), ("c_f32", i32),
        ("r_mode", i32), ("r_p0", i32), ("r_p1", i32),
        ("conv_h", i32), ("conv_up", i32), ("conv_cin", i32), ("conv_k3", i32),
        ("groups", i32), ("r_t", i32), ("impl", i32),
        ("ln_fold", i32), ("ln_eps", f32), ("ln_colsum", vp * MAX_GROUPS), ("c2_copy", i32),
        ("splitk", i32), ("sk_ws", vp), ("sk_ws_floats", i64), ("sk_cnt", vp), ("sk_cnt_n", i64),
        ("c_seg_rows", i64), ("c_seg_pitch", i64),
        ("ln_stats_out", vp * MAX_GROUPS), ("ln_stats_in", vp * MAX_GROUPS),
        ("a_t", i32), ("w_t", i32), ("ldw", i64), ("row_scale", vp), ("row_scale_div", i32), ("pad_", i32),
    ]


class AttnParams(ctypes.Structure):
    _fields_ = [("qkv", vp), ("out", vp), ("S", i32), ("Bm", i32), ("ntok", i32), ("n_t", i32), ("C", i32),
                ("H", i32), ("asym", i32), ("scale", f32), ("impl", i32), ("lse", vp), ("q_part", i32),
                ("tok_pitch", i32), ("out_pitch", i32), ("out_q0", i32)]


class AttnBwdParams(ctypes.Structure):
    _fields_ = [("qkv", vp), ("out", vp), ("dout", vp), ("lse", vp), ("delta", vp), ("dqkv", vp),
                ("S", i32), ("Bm", i32), ("ntok", i32), ("n_t", i32), ("C", i32), ("H", i32), ("asym", i32),
                ("scale", f32)]


MAX_CROPS = 4
f64 = ctypes.c_double
u8p = ctypes.c_void_p


class CropParams(ctypes.Structure):
    _fields_ = [("image", vp), ("H", i32), ("W", i32), ("box", vp), ("factor", f64), ("out_sz", i32),
                ("lut", vp), ("mean", f32 * 3), ("std", f32 * 3), ("out", vp), ("patch", vp), ("crop", vp)]


class ConvWprep(ctypes.Structure):
    _fields_ = [("w", vp), ("b", vp), ("wf", vp), ("wb", vp), ("bp", vp), ("cout", i32), ("cp", i32), ("cin", i32),
                ("pad_", i32)]


WPREP_MAX = 24

_PROTOS = {
    "mmt_gemm": [ctypes.POINTER(GemmParams), i32, vp],
    "mmt_gemm_multi": [ctypes.POINTER(GemmParams), i32, i32, vp],
    "mmt_mam_attention": [ctypes.POINTER(AttnParams), i32, vp],
    "mmt_mam_attention_bwd": [ctypes.POINTER(AttnBwdParams), i32, vp],
    "mmt_transpose_bf16": [vp, vp, i32, i32, i64, i64, i32, i64, i64, i32, vp],
    "mmt_im2col3x3_bf16": [vp, vp, i32, i32, i32, i32, vp],
    "mmt_batchnorm_ws_floats": [i64, i32],
    "mmt_batchnorm_relu": [vp, vp, i64, i32, i32, vp, vp, vp, vp, f32, f32, i32, i32, vp, vp, i64, vp],
    "mmt_batchnorm_relu_bwd": [vp, vp, vp, i64, i32, i32, vp, vp, i32, i32, vp, vp, i64, vp],
    "mmt_layernorm": [vp, vp, i64, vp, vp, vp, vp, vp, vp, i64, i64, i32, f32, i32, vp],
    "mmt_layernorm_bwd": [vp, vp, i32, vp, vp, vp, vp, i32, vp, i64, i64, i64, i32, f32, vp],
    "mmt_layernorm_bwd_add": [vp, vp, i32, vp, vp, vp, vp, vp, i32, vp, i64, i64, i64, i32, f32, vp],
    "mmt_groupnorm": [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, f32, i32, vp],
    "mmt_groupnorm_bwd": [vp, vp, vp, vp, vp, i32, vp, i64, i32, i32, i32, i32, f32, vp],
    "mmt_add_cast": [vp, vp, i64, vp, vp, i64, i32, vp],
    "mmt_scale_rows_cast": [vp, vp, i64, vp, i64, i64, i32, vp],
    "mmt_patch_im2col": [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp],
    "mmt_ms_deform_attn_forward": [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp],
    "mmt_ms_deform_attn_backward": [vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp],
    "mmt_ms_deform_attn_backward_impl": [vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32,
                                         i32, i32, vp],
    "mmt_msda_bimodal": [vp, vp, vp, i32, i32, i32, vp],
    "mmt_msda_bimodal_train_fwd": [vp, vp, i32, vp, i32, vp, vp, i32, i32, vp],
    "mmt_msda_bimodal_train_bwd": [vp, vp, i32, vp, i32, vp, vp, vp, vp, vp, i32, i32, vp],
    "mmt_ft_query_prep": [vp, vp, vp, vp, i32, i32, i32, vp],
    "mmt_ft_rows_cast": [vp, vp, i32, i32, i32, i32, i32, vp],
    "mmt_ft_rows_cast_bwd": [vp, vp, i32, i32, i32, i32, i32, vp],
    "mmt_corner_boxes": [vp, vp, vp, vp, i32, i32, f32, f32, vp],
    "mmt_corner_boxes_bwd": [vp, vp, vp, vp, vp, vp, i32, i32, f32, f32, vp],
    "mmt_box_loss": [vp, vp, vp, i32, f32, f32, vp],
    "mmt_box_loss_bwd": [vp, vp, vp, vp, i32, f32, f32, vp],
    "mmt_ft_query_prep_bwd": [vp, vp, vp, vp, vp, i32, i32, i32, vp],
    "mmt_ft_drop_residual": [vp, vp, vp, vp, i32, f32, i32, i32, i32, i32, vp],
    "mmt_ft_drop_residual_bwd": [vp, vp, vp, i32, f32, i32, i32, i32, i32, vp],
    "mmt_ft_relu_drop": [vp, vp, vp, i32, f32, i64, vp],
    "mmt_ft_relu_drop_bwd": [vp, vp, vp, vp, i32, f32, i64, vp],
    "mmt_conv3x3_c1": [vp, vp, vp, vp, i32, i32, i32, i32, i64, i32, vp],
    "mmt_conv3x3_c1_pair": [vp, vp, vp, vp, i32, i64, vp, vp, vp, vp, i32, i64, i32, i32, i32, i32, vp],
    "mmt_corner_softargmax": [vp, vp, vp, vp, vp, vp, vp, vp, vp, f32, i32, i32, i32, i32, i32, vp],
    "mmt_corner_score_train": [vp, vp, vp, vp, i64, vp, i64, vp, i32, i32, i32, vp],
    "mmt_im2col3x3_up_bf16": [vp, vp, i32, i32, i32, i32, i32, vp],
    "mmt_upsample_sum_bf16": [vp, vp, i32, i32, i32, i32, i32, vp],
    "mmt_add_up_bf16": [vp, vp, vp, i32, i32, i32, i32, i32, vp],
    "mmt_im2col3x3_cm_bf16": [vp, vp, i32, i32, i32, i32, i32, vp],
    "mmt_conv3x3_wprep": [ctypes.POINTER(ConvWprep), i32, vp],
    "mmt_corner_score_train_ws_floats": [i32, i32, i32],
    "mmt_corner_score_train_bwd": [vp, vp, vp, vp, vp, i32, vp, i32, vp, vp, vp, i32, i32, i32, vp],
    "mmt_prroi_pool_forward": [vp, vp, vp, i32, i32, i32, i32, i64, i64, i64, i64, i32, i32, f32, i64, i64, i64, vp],
    "mmt_prroi_pool_backward": [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, f32, vp],
    "mmt_prroi_pool_coor_backward": [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, f32, vp],
    "mmt_spm_attention": [vp, i64, vp, vp, i32, i32, i32, i32, f32, vp],
    "mmt_ce_t2s_attention": [vp, vp, i32, i32, i32, i32, i32, i32, f32, i32, vp],
    "mmt_ce_t2s_attention_masked": [vp, vp, vp, i32, i32, i32, i32, i32, i32, f32, i32, vp],
    "mmt_ce_select": [vp, i32, i32, i32, i32, i32, vp, vp, vp, vp, f32, vp],
    "mmt_ce_gather": [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, vp],
    "mmt_ce_recover": [vp, vp, i32, vp, i32, i32, i32, i32, i32, i32, vp],
    "mmt_sample_target": [ctypes.POINTER(CropParams), i32, vp],
    "mmt_track_update": [vp, vp, vp, i32, i32, i32, i32, f64, vp],
    "mmt_adamw_chunk_elems": [],
    "mmt_adamw_step": [vp, vp, i32, vp, vp, vp, vp, i32, f64, f64, f64, f32, i32, vp],
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "libmmt_hip.so not found at %s: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(or `make -C multi-modal-tracking_amd/csrc`). There is no CPU fallback." % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, args in _PROTOS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    lib.mmt_batchnorm_ws_floats.restype = ctypes.c_int64
    lib.mmt_corner_score_train_ws_floats.restype = ctypes.c_int64
    lib.mmt_version.argtypes = []
    lib.mmt_version.restype = ctypes.c_char_p
    return lib


LIB = _load()
EXPORTED = tuple(_PROTOS) + ("mmt_version",)


class MMTError(RuntimeError):
    pass


def check(status, name):
    if status != 0:
        if status == -10000:
            raise MMTError("%s: rejected arguments (MMT_EBADARG)" % name)
        raise MMTError("%s: HIP error %d" % (name, -status))
