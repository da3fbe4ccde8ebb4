"""ctypes binding of the C-ABI library ``libvaeunet_hip.so`` (include/vaeunet.h).

This is the only place the product path touches native code.  There is no
CPU or PyTorch fallback: if the library is missing or a launch fails the call
raises, loudly (the oracle under ``oracle/`` is test infrastructure only).
"""
import ctypes as C
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libvaeunet_hip.so")
# A/B timing of two builds of the same sources (tools/*_bench.py): an
# alternative library file; the product never sets it
if os.environ.get("VU_LIB_PATH"):
    LIB_PATH = os.environ["VU_LIB_PATH"]

F32, BF16 = 0, 1

_p = C.c_void_p
_i = C.c_int
_l = C.c_int64
_f = C.c_float


class VuGather(C.Structure):
    _fields_ = [("src", _p * 3), ("stride", _l * 3), ("cend", C.c_int32 * 3),
                ("nsrc", C.c_int32), ("C", C.c_int32),
                ("N", C.c_int32), ("H", C.c_int32), ("W", C.c_int32),
                ("Hs", C.c_int32), ("Ws", C.c_int32), ("R", C.c_int32), ("S", C.c_int32),
                ("sy", C.c_int32), ("sx", C.c_int32), ("dy", C.c_int32), ("dx", C.c_int32),
                ("oy", C.c_int32), ("ox", C.c_int32)]


class VuGemmFwd(C.Structure):
    _fields_ = [("a", VuGather), ("b", _p), ("ldb", _l), ("ncol", C.c_int32),
                ("out_mode", C.c_int32), ("out", _p), ("out_stride", _l),
                ("out_coff", C.c_int32), ("oH", C.c_int32), ("oW", C.c_int32),
                ("opy", C.c_int32), ("opx", C.c_int32), ("cout", C.c_int32),
                ("bias", _p), ("stat_sum", _p), ("stat_m2", _p), ("accumulate", C.c_int32),
                ("ksplit", C.c_int32), ("workspace", _p),
                ("bnb_x", _p), ("bnb_xstride", _l), ("bnb_scale", _p), ("bnb_shift", _p),
                ("bnb_mean", _p), ("bnb_invstd", _p), ("bnb_part", _p), ("bnb_relu", C.c_int32),
                ("relu", C.c_int32), ("zbias", _p)]


class VuGemmWgrad(C.Structure):
    _fields_ = [("p", VuGather), ("q", VuGather), ("ni", C.c_int32), ("nj", C.c_int32),
                ("splits", C.c_int32), ("m_per_split", _l), ("out", _p)]


class VuConvFp8(C.Structure):
    _fields_ = [("a", VuGather), ("w", _p), ("ldw", _l), ("ncol", C.c_int32), ("out_coff", C.c_int32),
                ("x_scale", _p), ("w_scale", _p), ("bias", _p), ("out", _p), ("out_stride", _l),
                ("stat_sum", _p), ("stat_m2", _p), ("workspace", _p), ("stat_min", _p), ("stat_max", _p)]


class VuPermJob(C.Structure):
    _fields_ = [("inp", _p), ("base", _l), ("s0", _l), ("s1", _l), ("s2", _l), ("s3", _l),
                ("d0", C.c_int32), ("d1", C.c_int32), ("d2", C.c_int32), ("d3", C.c_int32),
                ("d3v", C.c_int32), ("dtype", C.c_int32), ("out", _p), ("chunk0", _l),
                ("q", C.c_int32), ("pad_", C.c_int32)]


class VuMtEntry(C.Structure):
    _fields_ = [("param", _p), ("grad", _p), ("exp_avg", _p), ("exp_avg_sq", _p),
                ("numel", _l), ("chunk0", _l), ("step_size", _f), ("bc2_sqrt", _f)]


class VuLatentJob(C.Structure):
    _fields_ = [("w", _p), ("bias", _p), ("gamma", _p), ("beta", _p), ("running_mean", _p),
                ("running_var", _p), ("num_batches_tracked", _p), ("momentum", _f), ("eps", _f),
                ("train", C.c_int32), ("co", C.c_int32), ("cpad", C.c_int32), ("HW", C.c_int32),
                ("out", _p), ("out_stride", _l), ("y", _p), ("coef", _p), ("block0", _l),
                ("cgroups", C.c_int32), ("grad_acc", C.c_int32), ("dmap", _p), ("dmap_stride", _l),
                ("part", _p), ("sblock0", _l), ("dw", _p), ("dbias", _p), ("dgamma", _p), ("dbeta", _p),
                ("act", _p)]


class VuZbJob(C.Structure):
    _fields_ = [("w", _p), ("ws_co", _l), ("ws_ci", _l), ("ws_ky", _l), ("ws_kx", _l), ("cz0", C.c_int32),
                ("L", C.c_int32), ("co", C.c_int32), ("H", C.c_int32), ("W", C.c_int32), ("act", _p),
                ("row_scale", _p), ("table", _p), ("dy", _p), ("dy_stride", _l), ("rs", _p), ("part", _p),
                ("dw", _p), ("grad_acc", C.c_int32), ("rs_ready", C.c_int32), ("block0", _l)]


class VuLatentHeads(C.Structure):
    _fields_ = [("z", _p), ("eps", _p), ("logvar", _p), ("dmu_in", _p), ("dlv_in", _p), ("dz_in", _p), ("pooled", _p),
                ("w_mu", _p), ("w_lv", _p), ("dw_mu", _p), ("db_mu", _p), ("dw_lv", _p), ("db_lv", _p),
                ("dpooled", _p), ("C", C.c_int32), ("grad_acc", C.c_int32)]


# name -> (restype, argtypes)
_SIGS = {
    "vu_gemm_fwd": (_i, [C.POINTER(VuGemmFwd), _i, _p]),
    "vu_gemm_fwd_row_tile": (_l, [C.POINTER(VuGemmFwd), _i]),
    "vu_gemm_fwd_workspace_bytes": (_l, [C.POINTER(VuGemmFwd), _i]),
    "vu_gemm_fwd_bnb_tile": (_l, [C.POINTER(VuGemmFwd), _i]),
    "vu_gemm_fwd_kernel": (_i, [C.POINTER(VuGemmFwd), _i]),
    "vu_abi_struct_sizes": (None, [_p]),
    "vu_bn_bwd_finish": (_i, [_p, _i, _l, _i, _p, _p, _i, _p, _p, _i, _p, _p, _p]),
    "vu_bn_bwd_finish_workspace_bytes": (_l, [_i, _i]),
    "vu_gemm_wgrad": (_i, [C.POINTER(VuGemmWgrad), _i, _p]),
    "vu_gemm_wgrad_tile": (_i, [C.POINTER(VuGemmWgrad), _i, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "vu_gemm_set_tuning": (_i, [_i, _i]),
    "vu_gemm_experiment_modes": (_i, []),
    "vu_slab_reduce": (_i, [_p, _i, _i, _i, _i, _i, _l, _l, _l, _p, _i, _p]),
    "vu_amax": (_i, [_p, _l, _l, _i, _p, _i, _i, _p]),
    "vu_quant_fp8": (_i, [_p, _l, _l, _i, _p, _p, _l, _p, _i, _p]),
    "vu_quant_rows_fp8": (_i, [_p, _i, _l, _p, _l, _p, _p]),
    "vu_bn_apply_fp8": (_i, [_p, _l, _p, _l, _l, _i, _p, _p, _i, _p, _i, _i, _p, _i, _p]),
    "vu_conv3x3_fp8_row_tile": (_l, [C.POINTER(VuConvFp8)]),
    "vu_conv3x3_fp8": (_i, [C.POINTER(VuConvFp8), _p]),
    "vu_conv3x3_fp8_workspace_bytes": (_l, [C.POINTER(VuConvFp8)]),
    "vu_conv3x3_fp8_minmax_ok": (_i, [C.POINTER(VuConvFp8)]),
    "vu_fp8_relu_amax": (_i, [_p, _p, _l, _i, _p, _p, _i, _p, _p]),
    "vu_permute4_chunk": (_l, []),
    "vu_permute4_tile": (_l, []),
    "vu_permute4_batch": (_i, [_p, _i, _l, _p]),
    "vu_permute4_batch2": (_i, [_p, _i, _i, _l, _l, _p]),
    "vu_permute4": (_i, [_p, _l, _l, _l, _l, _l, _i, _i, _i, _i, _i, _p, _i, _p]),
    "vu_bn_finalize": (_i, [_p, _p, _i, _l, _l, _i, _p, _p, _p, _p, _f, _f, _p, _p, _p, _p,
                            _p, _p, _p]),
    "vu_bn_finalize_workspace_bytes": (_l, [_i, _i]),
    "vu_bn_eval_coeffs": (_i, [_p, _p, _p, _p, _f, _i, _p, _p, _p, _p, _p]),
    "vu_bn_apply": (_i, [_p, _l, _p, _l, _l, _i, _p, _p, _i, _i, _p]),
    "vu_bn_fwd_fused_supported": (_i, [_i, _i, _l, _l, _l]),
    "vu_bn_bwd_fused_supported": (_i, [_l, _i, _l, _l, _l]),
    "vu_bn_bwd_fused": (_i, [_p, _l, _p, _l, _l, _i, _p, _p, _p, _p, _p, _i, _i, _p, _p, _i, _p, _l, _p, _i,
                             _p]),
    "vu_bn_fwd_fused": (_i, [_p, _p, _i, _l, _l, _i, _p, _p, _p, _p, _p, _f, _f, _p, _p, _l, _p, _l, _p, _p,
                             _p, _l, _i, _i, _p]),
    "vu_bn_bwd_pool_supported": (_i, [_i, _i, _i, _l, _l, _l, _l]),
    "vu_bn_bwd_pool": (_i, [_p, _l, _p, _l, _p, _l, _i, _i, _i, _i, _p, _p, _p, _p, _p, _i, _i, _p, _p, _i, _p, _p,
                            _p, _l, _i, _p]),
    "vu_bn_bwd_reduce": (_i, [_p, _l, _p, _l, _l, _i, _p, _p, _p, _p, _p, _i, _i, _p, _p, _i,
                              _p, _p, _i, _p]),
    "vu_bn_bwd_apply": (_i, [_p, _l, _p, _l, _l, _i, _p, _p, _p, _p, _i, _p, _l, _i, _p]),
    "vu_bn_bwd_apply2_ok": (_i, [_i, _l, _l, _l, _l, _l]),
    "vu_bn_bwd_apply2": (_i, [_p, _l, _p, _l, _p, _l, _l, _i, _p, _p, _p, _p, _p, _l, _p, _l, _i, _p]),
    "vu_reduce_workspace_bytes": (_l, [_l, _i]),
    "vu_chan_sum": (_i, [_p, _l, _i, _i, _i, _i, _i, _i, _i, _i, _p, _i, _p, _i, _p]),
    "vu_copy": (_i, [_p, _l, _i, _p, _l, _i, _l, _i, _i, _p]),
    "vu_zero": (_i, [_p, _l, _l, _i, _i, _p]),
    "vu_gpu_delay": (_i, [_i, _p]),
    "vu_zero_insert2": (_i, [_p, _l, _i, _i, _i, _i, _p, _l, _i, _i, _i, _p]),
    "vu_input_pack": (_i, [_p, _l, _l, _l, _l, _i, _i, _i, _i, _i, _p, _i, _p]),
    "vu_maxpool2_fwd": (_i, [_p, _l, _i, _i, _i, _i, _p, _l, _i, _p]),
    "vu_maxpool2_bwd": (_i, [_p, _l, _p, _l, _i, _i, _i, _i, _p, _l, _p, _l, _i, _p]),
    "vu_bn_apply_maxpool2": (_i, [_p, _l, _p, _l, _p, _l, _i, _i, _i, _i, _p, _p, _i, _i, _p]),
    "vu_upsample_fwd": (_i, [_p, _l, _i, _i, _i, _i, _p, _l, _i, _i, _i, _i, _i, _i, _i, _p]),
    "vu_upsample_bwd": (_i, [_p, _l, _i, _i, _i, _i, _p, _l, _i, _i, _i, _i, _i, _i, _i, _i,
                             _p]),
    "vu_attn_tile_rows": (_l, []),
    "vu_attn_psi_fwd": (_i, [_p, _p, _l, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _l, _i, _p]),
    "vu_attn_gate_fwd": (_i, [_p, _p, _p, _l, _l, _i, _p, _p, _l, _i, _p]),
    "vu_attn_gate_bwd": (_i, [_p, _l, _p, _l, _p, _l, _i, _p, _l, _p, _i, _p]),
    "vu_attn_psi_bwd_workspace_bytes": (_l, [_l, _i]),
    "vu_attn_psi_bwd_blocks": (_l, [_l]),
    "vu_attn_psi_bwd_bnb_ok": (_i, [_i]),
    "vu_attn_psi_bwd_bnb": (_i, [_p, _p, _l, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _p, _p, _p, _p, _p, _p, _p,
                                 _i, _p]),
    "vu_attn_psi_bwd": (_i, [_p, _p, _l, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _p, _i,
                             _p]),
    "vu_pointwise_fwd": (_i, [_p, _l, _l, _i, _i, _p, _p, _p, _l, _i, _p]),
    "vu_pointwise_bwd_workspace_bytes": (_l, [_l, _i, _i]),
    "vu_pointwise_bn_fwd": (_i, [_p, _l, _l, _i, _i, _p, _p, _p, _p, _p, _l, _i, _p]),
    "vu_pointwise_bn_bwd_blocks": (_l, [_l]),
    "vu_pointwise_bn_bwd": (_i, [_p, _l, _p, _l, _p, _l, _l, _i, _i, _p, _p, _l, _p, _p, _i, _p, _p, _i, _p]),
    "vu_pointwise_bwd": (_i, [_p, _l, _p, _l, _l, _i, _i, _p, _p, _l, _p, _p, _i, _p, _i, _p]),
    "vu_loss_workspace_bytes": (_l, []),
    "vu_bce_dice_fwd2": (_i, [_p, _p, _l, _p, _f, _f, _f, _p, _p, _p, _p]),
    "vu_bce_dice_bwd": (_i, [_p, _p, _l, _p, _f, _f, _f, _p, _p, _p]),
    "vu_kl_free_bits2": (_i, [_p, _p, _i, _i, _f, _p, _p, _p, _p, _p]),
    "vu_sumsq": (_i, [_p, _l, _p, _p, _p]),
    "vu_dice_score": (_i, [_p, _p, _l, _f, _p, _p, _p, _p]),
    "vu_mt_chunk_elems": (_l, []),
    "vu_mt_grad_norm": (_i, [_p, _i, _l, _f, _p, _p, _p, _p]),
    "vu_mt_scale_grads": (_i, [_p, _i, _l, _p, _p]),
    "vu_mt_adamw": (_i, [_p, _i, _l, _f, _f, _f, _f, _f, _p, _p]),
    "vu_mt_adamw_dev": (_i, [_p, _i, _l, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double, _p, _i,
                             _p]),
    "vu_mt_adamw_dev_scaled": (_i, [_p, _i, _l, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double, _p,
                                    _i, _p, _p]),
    "vu_maxpool3s2_fwd": (_i, [_p, _l, _i, _i, _i, _i, _p, _l, _p, _i, _p]),
    "vu_maxpool3s2_bwd": (_i, [_p, _l, _p, _i, _i, _i, _i, _p, _l, _i, _i, _p]),
    "vu_bn_add_relu": (_i, [_p, _l, _p, _p, _p, _l, _p, _p, _l, _i, _p, _l, _i, _p]),
    "vu_relu_mask": (_i, [_p, _l, _p, _l, _l, _i, _p, _l, _i, _p]),
    "vu_sample_sum": (_i, [_p, _l, _i, _i, _i, _f, _p, _i, _p, _i, _p]),
    "vu_sample_sum_workspace_bytes": (_l, [_i, _i]),
    "vu_sample_broadcast": (_i, [_p, _i, _i, _i, _f, _p, _l, _i, _i, _p]),
    "vu_linear_small_fwd": (_i, [_p, _i, _i, _p, _p, _i, _p, _p]),
    "vu_linear_small_bwd": (_i, [_p, _i, _i, _p, _i, _p, _p, _i, _p, _p, _i, _p]),
    "vu_reparam_fwd": (_i, [_p, _p, _p, _i, _p, _p]),
    "vu_reparam_bwd": (_i, [_p, _p, _p, _i, _p, _p, _i, _p]),
    "vu_vae_heads_fwd": (_i, [_p, _l, _i, _i, _i, _p, _p, _p, _p, _i, _p, _p, _p, _p, _p, _i, _p]),
    "vu_latent_fwd_blocks": (_l, [_i, _i, _i]),
    "vu_latent_fwd": (_i, [_p, _i, _p, _i, _i, _i, _p]),
    "vu_latent_part_floats": (_l, [_i, _i]),
    "vu_latent_bwd_supported": (_i, [_i, _i, _l, _i]),
    "vu_latent_bwd_sums": (_i, [_p, _i, _i, _i, _p]),
    "vu_latent_bwd_workspace_bytes": (_l, [_i, _i, _l]),
    "vu_latent_bwd": (_i, [_p, _i, C.POINTER(VuLatentHeads), _i, _i, _p, _p]),
    "vu_latent_check_job": (_i, [_i, _i, _l, _i]),
    "vu_zbias_supported": (_i, [_i, _i, _i]),
    "vu_zbias_rs_floats": (_l, [_i, _i, _i, _i]),
    "vu_zbias_fwd": (_i, [_p, _i, _i, _p]),
    "vu_zbias_bwd": (_i, [_p, _i, _i, _i, _p]),
    "vu_bn_bwd_apply_zrs_ok": (_i, [_i, _i, _i, _l, _l, _l]),
    "vu_bn_bwd_apply_zrs": (_i, [_p, _l, _p, _l, _i, _i, _i, _i, _p, _p, _p, _p, _i, _p, _l, _p, _i, _p]),
    "vu_mean_groups": (_i, [_p, _i, _l, _p, _p]),
    "vu_sigmoid": (_i, [_p, _l, _p, _p]),
    "vu_patch_blend": (_i, [_p, _l, _i, _i, _i, _p, _p, _i, _i, _i, _i, _p, _i, _i, _i, _i, _i, _p]),
    "vu_blend_finish": (_i, [_p, _p, _l, _p]),
    "vu_uncertainty": (_i, [_p, _i, _l, _p, _p, _p, _p, _p, _p]),
    "vu_gather_affine": (_i, [_p, _i, _i, _i, _i, _p, _p, _i, _i, _i, _p]),
    "vu_patch_stats": (_i, [_p, _i, _i, _i, _p, _i, _i, _i, _i, _p, _p, _p]),
}

_lib = None


def lib():
    """Load the library once; raise if it is absent (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"vaeunet_amd: HIP library {LIB_PATH} is missing; run "
                "`python -c 'import __graft_entry__ as g; g.build()'` (or `make`)")
        h = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _lib = h
    return _lib


def exported_symbols():
    return sorted(_SIGS)


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"vaeunet_amd: {name} failed with hipError {rc}")
    return rc


def query(name, *args):
    return getattr(lib(), name)(*args)


def stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())
