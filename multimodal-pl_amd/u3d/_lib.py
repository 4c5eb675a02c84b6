"""ctypes binding of libu3d.so (include/u3d.h). No fallback: if the library is missing or the tensors are
not on a ROCm device, calls raise."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("U3D_LIB") or os.path.join(_HERE, "libu3d.so")  # U3D_LIB: A/B builds (tools/ab_lib)

F32, BF16 = 0, 1

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_longlong
F = ctypes.c_float

# name -> argtypes (restype int unless noted)
_SIGS = {
    "u3d_abi_version": [],
    "u3d_set_option": [ctypes.c_char_p, I],
    "u3d_get_option": [ctypes.c_char_p, P],
    "u3d_wstd_fwd": [I, P, I, I, I, I, P, P, P, P],
    "u3d_wstd_bwd": [P, I, P, P, I, I, I, I, P, I, P],
    "u3d_wstd_fwd_batch": [I, P, I, P],
    "u3d_wstd_bwd_batch": [P, I, P, P],
    "u3d_wgrad_sum_slabs": [P, I, I, I, I, P],
    "u3d_wstd_bwd_scratch_bytes": [P, I],
    "u3d_conv_fwd": [I, P, I, I, I, I, I, P, I, I, I, P, P, P, I, P, P, P, I, P, L, P],
    "u3d_conv_dgrad": [I, P, I, I, P, I, I, I, I, I, I, P, P, L, P],
    "u3d_conv_wgrad_splits": [I, I, I, I, I, I, I, I],
    "u3d_conv_wgrad": [I, P, P, I, I, I, I, I, I, I, I, P, P, P, I, P, I, P],
    "u3d_head_fwd": [P, I, L, I, P, I, P, P, P, P, I, P, P],
    "u3d_head_bwd_blocks": [L],
    "u3d_head_loss_bwd_gn_bps": [I, L, I],
    "u3d_head_bwd": [P, L, I, P, I, P, P, P, P],
    "u3d_head_loss_bwd": [P, P, L, I, P, P, P, P, I, P, P, P, P],
    "u3d_head_loss_bwd_gn": [P, P, I, L, I, P, P, P, P, I, P, P, P, P, P, P, P, I, P, P, P, P],
    "u3d_partial_target": [P, I, L, P, I, I, I, I, P, P],
    "u3d_window_accumulate": [P, I, I, I, I, I, P, P, P, F, F, P, P, I, I, I, I, I, I, I, I, P],
    "u3d_window_normalize": [P, P, I, I, L, P],
    "u3d_sgd_step": [P, I, P, F, F, F, I, I, I, P],
    "u3d_conv_dgrad_s2": [P, I, I, P, I, I, I, I, P, P],
    "u3d_conv1x1": [P, I, I, I, I, I, P, I, I, I, P, P, P, I, P, P],
    "u3d_conv_small": [I, P, I, I, I, I, I, P, I, P, P, P, I, P, P, P, L, P],
    "u3d_conv_small_cnt_bytes": [I, I, I, I, I],
    "u3d_conv_small_spart_floats": [I, I, I, I],
    "u3d_conv_small2": [I, P, I, I, I, I, I, P, I, P, P, P, I, P, P, P, L, P, P, P, P, P],
    "u3d_conv_small_gb_parts_floats": [I, I, I, I, I],
    "u3d_conv_small_dgrad_gn": [P, I, I, I, I, I, P, I, P, P, P, P, I, P, P, L, P, P, P, P, P, P, P],
    "u3d_gn_bwd_apply_coef": [P, P, I, I, L, I, P, P, I, P],
    "u3d_conv_s2_ring_ok": [I, I, I, I, I, I],
    "u3d_conv32_ring_dgrad_gn_fused": [P, I, I, I, I, P, P, P, P, P, I, P, P, P, P, P, P, P],
    "u3d_conv_s2_ring_ws_floats": [I, I, I, I],
    "u3d_conv_s2_ring": [P, I, I, I, I, P, P, P, P, I, P, P, P, P, P],
    "u3d_conv32_brick": [I, P, I, I, I, I, P, P, P, P, I, P, P, P],
    "u3d_conv32_ring": [I, P, I, I, I, I, P, P, P, P, I, P, P, P],
    "u3d_conv32_ring_stats_ws_floats": [I],
    "u3d_conv32_ring_stats": [P, I, I, I, I, P, P, P, P, I, P, P, P, P],
    "u3d_conv32_ring_stats_xn": [P, I, I, I, I, P, P, P, P, I, P, P, P, P, P],
    "u3d_conv32_ring_stats_fused": [P, I, I, I, I, P, P, P, P, I, P, P, P, P, P, P],
    "u3d_conv32_ring_wps": [I, I, I, I],
    "u3d_conv32_ring_dgrad_gn": [P, I, I, I, I, P, P, P, P, P, I, P, P, P],
    "u3d_conv32_ring_stats_finalize": [P, I, I, I, I, P, P],
    "u3d_conv32_ring_q_stats_ws_floats": [I, I, I, I],
    "u3d_conv32_ring_q_queue_bytes": [I, I, I, I],
    "u3d_diag_occupy": [I, L, P, P],
    "u3d_conv32_ring_q": [I, P, I, I, I, I, P, P, P, P, I, P, P, P, P, P],
    "u3d_conv32_ring_q_stats_finalize": [P, I, I, I, I, P, P],
    "u3d_conv_wgrad_ring_splits": [I, I, I, I, I, I],
    "u3d_conv_wgrad_ring_splits_target": [I, I, I, I, I, I, I],
    "u3d_conv_wgrad_ring": [P, P, I, I, I, I, I, I, P, P, P, I, P, I, P],
    "u3d_convg_brick": [I, P, I, I, I, I, I, P, I, P, P, P, I, P, P, P],
    "u3d_convg_brick_stats_ws_floats": [I, I, I, I, I],
    "u3d_convg_brick_stats": [P, I, I, I, I, I, P, I, P, P, P, I, P, P, P, L, P, P],
    "u3d_convg_brick_stats_fused": [P, I, I, I, I, I, P, I, P, P, P, I, P, P, P, L, P, P, P],
    "u3d_convg_brick_gn_nparts": [I, I, I, I, I, I],
    "u3d_convg_brick_dgrad_gn": [P, I, I, I, I, I, P, I, P, P, P, P, I, P, P, I, P],
    "u3d_conv_wgrad_brick_splits": [I, I, I, I, I, I, I],
    "u3d_conv_wgrad_brick": [P, P, I, I, I, I, I, I, I, P, P, P, I, P, I, P],
    "u3d_conv_wgrad1_splits": [I, I, I, I, I, I, I],
    "u3d_conv_wgrad1": [P, P, I, I, I, I, I, I, I, P, P, P, I, P, I, P],
    "u3d_stem_fwd": [I, P, I, I, I, I, I, P, I, I, P, P, P],
    "u3d_stem_fwd_ws_bytes": [],
    "u3d_stem1_stats_ws_floats": [I, I, I, I],
    "u3d_upsample2x_stats_ws_floats": [I, I, I, I, I],
    "u3d_upsample2x_add_stats": [P, I, I, I, I, I, P, P, P, P, P],
    "u3d_stem1_fwd_stats": [P, I, I, I, I, P, P, P, P, P, P],
    "u3d_stem_wgrad_splits": [I, I, I, I, I],
    "u3d_stem_wgrad_splits2": [I, I, I, I, I, I, I, I],
    "u3d_stem_wgrad": [I, P, P, I, I, I, I, I, I, I, P, I, P],
    "u3d_gn_workspace_bytes": [I, I, L],
    "u3d_gn_stats": [I, P, I, I, L, I, P, P, P],
    "u3d_gn_apply": [I, P, I, I, L, I, P, P, P, P, P],
    "u3d_gn_bwd": [I, P, P, I, I, L, I, P, P, P, P, I, P, P, I, P, P],
    "u3d_gn_bwd_parts": [P, P, I, I, L, I, P, P, P, P, I, P, I, P, P, I, P, P],
    "u3d_gn_bwd2": [I, P, P, P, I, I, L, I, P, P, P, P, P, P, I, P, P, P, P, I, P, P],
    "u3d_gn_bwd2_s2": [I, P, P, P, I, I, I, I, I, I, P, P, P, P, P, P, I, P, P, P, P, I, P, P],
    "u3d_upsample2x_add": [I, P, I, I, I, I, I, P, P, P],
    "u3d_upsample2x_bwd": [I, P, I, I, I, I, I, P, I, P],
    "u3d_add_inplace": [I, P, P, L, P],
    "u3d_channel_sum": [I, P, L, I, P, I, P, P],
    "u3d_channel_sum_workspace_bytes": [L, I],
    "u3d_cast": [I, P, I, P, L, I, I, P],
    "u3d_loss_workspace_bytes": [I, L, I],
    "u3d_partial_loss_fwd": [P, P, I, L, I, I, P, I, P, P, P, P],
    "u3d_partial_loss_bwd": [I, P, P, I, L, I, I, P, I, P, P, P, P],
    "u3d_dice_metric": [P, P, I, L, I, I, P, P, P, P],
    "u3d_dice_metric_binary": [P, I, L, L, L, L, P, P, P, P, P],
    "u3d_gn_relu_mean": [I, P, I, I, L, I, P, P, P, P, P],
    "u3d_dyn_controller": [P, I, I, P, I, P, P, I, P, P],
    "u3d_dynhead_fwd": [P, P, I, L, P, P],
    "u3d_dynhead_bwd_blocks": [L],
    "u3d_dynhead_bwd": [P, P, P, I, L, P, P, P, P],
    "u3d_dyn_controller_bwd": [I, P, I, I, P, I, P, P, I, P, P, I, L, P, P],
    "u3d_eam_prep": [P, I, I, P, P, P, P, F, P, P, P, P],
    "u3d_eam_attn_fwd": [I, P, I, L, I, P, P, P, I, P, P],
    "u3d_eam_attn_bwd_blocks": [I, L],
    "u3d_eam_attn_bwd_part_floats": [I, L, I, I],
    "u3d_eam_attn_bwd": [I, P, I, L, I, P, P, P, I, P, P, I, P, P, P, P, I, P],
    "u3d_eam_param_bwd": [P, I, I, P, P, P, P, P, P, F, P, P, P, P, P, P, I, P],
    "u3d_upsample_trilinear": [P, L, I, I, I, I, P, P],
    "u3d_upsample_trilinear_bwd_ws_floats": [L, I, I, I, I],
    "u3d_upsample_trilinear_bwd": [P, L, I, I, I, I, P, I, P, P],
    "u3d_renew_token_ws_bytes": [I, I, I, I, I, I],
    "u3d_renew_token": [I, P, L, L, I, I, I, I, I, P, I, I, I, I, I, F, P, P, P],
    "u3d_consistency_ws_bytes": [I],
    "u3d_consistency_fwd": [P, P, P, I, L, L, P, L, L, I, P, L, L, L, P, I, L, F, F, P, P, P, P, P],
    "u3d_consistency_bwd": [P, P, P, I, L, L, P, L, L, I, P, L, L, L, P, I, L, F, P, P, P, P, P, P, P],
    "u3d_edice_full2_fwd": [P, P, P, L, I, I, P, P, P, P],
    "u3d_edice_full2_bwd": [P, P, P, L, I, P, P, P, P],
    "u3d_volume_stats_ws_bytes": [],
    "u3d_volume_stats": [P, L, L, P, P, P],
    "u3d_crop_transpose": [P, I, I, I, I, I, I, I, I, I, I, I, P, P, P],
    "u3d_aug_noise": [P, L, F, ctypes.c_ulonglong, P],
    "u3d_aug_blur_axis": [P, P, L, I, L, P, I, P],
    "u3d_aug_affine": [P, L, F, F, P],
    "u3d_aug_contrast": [P, L, F, P, I, P],
}
_RESTYPE = {"u3d_stem_fwd_ws_bytes": L, "u3d_stem1_stats_ws_floats": L, "u3d_conv_small_cnt_bytes": L, "u3d_conv_small_spart_floats": L, "u3d_conv_small_gb_parts_floats": L, "u3d_conv_s2_ring_ws_floats": L, "u3d_upsample2x_stats_ws_floats": L, "u3d_wstd_bwd_scratch_bytes": L, "u3d_gn_workspace_bytes": L, "u3d_channel_sum_workspace_bytes": L, "u3d_loss_workspace_bytes": L,
            "u3d_eam_attn_bwd_part_floats": L, "u3d_upsample_trilinear_bwd_ws_floats": L, "u3d_renew_token_ws_bytes": L,
            "u3d_consistency_ws_bytes": L, "u3d_volume_stats_ws_bytes": L, "u3d_convg_brick_stats_ws_floats": L}

_lib = None


class WstdDesc(ctypes.Structure):
    """u3d_wstd_desc (include/u3d.h)."""
    _fields_ = [("w", P), ("wpk_fwd", P), ("wpk_dgrad", P), ("wstats", P), ("part", P), ("dw", P),
                ("cout", I), ("cin", I), ("ksize", I), ("standardize", I), ("nsplit", I), ("accumulate", I)]


WSTD_BATCH_MAX = 48


class SgdDesc(ctypes.Structure):
    """u3d_sgd_desc (include/u3d.h)."""
    _fields_ = [("p", P), ("g", P), ("buf", P), ("n", L)]


SGD_BATCH_MAX = 48


class U3DError(RuntimeError):
    pass


def lib():
    """Load libu3d.so once. Raises U3DError if it is absent (build with __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise U3DError(f"libu3d.so not found at {LIB_PATH}: build it (python -c 'import __graft_entry__ as g; "
                           "g.build()'); the HIP path has no fallback")
        h = ctypes.CDLL(LIB_PATH)
        ab = bool(os.environ.get("U3D_LIB"))  # an A/B build of an older tree may lack entry points added since
        for name, args in _SIGS.items():
            if ab and not hasattr(h, name):
                continue
            f = getattr(h, name)
            f.argtypes = args
            f.restype = _RESTYPE.get(name, I)
        h.u3d_last_error.argtypes = []
        h.u3d_last_error.restype = ctypes.c_char_p
        _lib = h
    return _lib


def exported_symbols():
    return list(_SIGS) + ["u3d_last_error"]


def call(name, *args):
    f = getattr(lib(), name)
    rc = f(*args)
    if rc != 0:
        msg = lib().u3d_last_error().decode(errors="replace")
        raise U3DError(f"{name} failed (rc={rc}): {msg}")
    return rc


def query(name, *args):
    return getattr(lib(), name)(*args)
