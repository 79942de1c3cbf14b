"""ctypes binding of libvisionseg_hip.so (the C ABI declared in include/visionseg.h).

The library is built in-tree by `make -C vision-instance-seg_amd` (or
`__graft_entry__.build()`).  There is no fallback: if the library is missing or a
tensor is not on a HIP device, the ops raise — the product path never silently runs
something else.
"""
from __future__ import annotations

import ctypes
import os

import torch  # load torch (and its HIP runtime) before the kernels library

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libvisionseg_hip.so")
# torch.ops.visionseg.* (csrc/torch_ops.cpp, TORCH_LIBRARY over this C ABI): the §8(b)
# operator surface; the remaining helper kernels are called through ctypes below
TORCH_LIB_PATH = os.path.join(_HERE, "libvisionseg_torch.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "visionseg.h")

VS_F32, VS_BF16 = 0, 1

_c_int, _c_void_p, _c_float = ctypes.c_int, ctypes.c_void_p, ctypes.c_float
_P = _c_void_p

# name -> argtypes (restype int unless noted); keep in sync with include/visionseg.h
SIGNATURES = {
    "vs_abi_version": [],
    "vs_last_error": [],
    "vs_msda_forward": [_c_int, _P, _P, _P, _P, _P, _P] + [_c_int] * 7 + [_P],
    "vs_msda_backward": [_c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P] + [_c_int] * 7 + [_P],
    "vs_msda_backward_workspace_bytes": [_c_int] * 5,
    "vs_msda_backward_ex": [_c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P] + [_c_int] * 7 + [_P],
    "vs_msda_backward_tiled_workspace_bytes": [_c_int] * 5 + [_P],
    "vs_msda_backward_tiled": [_c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P] + [_c_int] * 7 + [_P],
    "vs_msda_prep_forward": [_c_int, _P, ctypes.c_longlong, _P, ctypes.c_longlong, _P, ctypes.c_longlong, _P, _P,
                             _P] + [_c_int] * 5 + [_P],
    "vs_msda_prep_backward": [_c_int, _P, _P, _P, _P, _P, ctypes.c_longlong, _P, ctypes.c_longlong] + [_c_int] * 5
                             + [_P],
    "vs_window_partition": [_P, _P] + [_c_int] * 7 + [_P],
    "vs_window_reverse": [_P, _P] + [_c_int] * 7 + [_P],
    "vs_window_attn_forward": [_c_int, _P, _P, _P, _P] + [_c_int] * 6 + [_c_float, _P],
    "vs_window_attn_backward": [_c_int, _P, _P, _P, _P, _P, _P, _P] + [_c_int] * 6 + [_c_float, _P],
    "vs_window_attn_forward_fp8": [_P, _P, _P, _P] + [_c_int] * 6 + [_c_float, _P],
    "vs_window_attn_backward_fp8": [_P, _P, _P, _P, _P, _P, _P] + [_c_int] * 6 + [_c_float, _P],
    "vs_window_attn_forward_image": [_c_int, _c_int, _P, _P, _P, _P] + [_c_int] * 8 + [_c_float, _P],
    "vs_window_attn_backward_image": [_c_int, _c_int, _P, _P, _P, _P, _P, _P, _P] + [_c_int] * 8 + [_c_float, _P],
    "vs_token_gemm": [_c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P, _c_int, _c_int, _c_int, _P],
    "vs_mx_quantize": [_P, _P, _P, _c_int, _c_int, _P],
    "vs_row_quantize_fp8": [_P, _P, _P, _c_int, _c_int, _P],
    "vs_gelu_row_quantize_fp8": [_P, _P, _P, _P, _c_int, _c_int, _P],
    "vs_layer_norm_forward_rows_q": [_P] * 8 + [_c_int, _c_int, _c_float, _P, _P],
    "vs_add_layer_norm_forward_q": [_P] * 10 + [_c_int, _c_int, _c_float, _P, _P],
    "vs_layer_norm_forward_qr": [_P] * 8 + [_c_int, _c_int, _c_float, _P, _P],
    "vs_add_layer_norm_forward_qr": [_P] * 10 + [_c_int, _c_int, _c_float, _P, _P],
    "vs_mask_head_forward": [_c_int, _P, _P, _P] + [_c_int] * 5 + [_P],
    "vs_mask_head_backward_workspace_bytes": [_c_int] * 3,
    "vs_mask_head_backward": [_c_int] + [_P] * 6 + [_c_int] * 5 + [_P],
    "vs_mask_head_backward_ex": [_c_int] + [_P] * 6 + [_c_int] * 6 + [_P],
    "vs_attn_bitmask": [_P, _P] + [_c_int] * 5 + [_P],
    "vs_mask_head_forward_grouped": [_P, _P, _P] + [_c_int] * 6 + [_P],
    "vs_point_scatter": [_P, _P, _P] + [_c_int] * 6 + [_P],
    "vs_point_sample_rows": [_P, _P, _P, _P] + [_c_int] * 5 + [_P],
    "vs_point_sample_masks": [_P, _P, _P, _P] + [_c_int] * 7 + [_P],
    "vs_topk_rows": [_P, _P] + [_c_int] * 3 + [_P],
    "vs_masked_attn_workspace_bytes": [_c_int] * 4,
    "vs_masked_attn_forward": [_c_int, _P, _P, _P, _P, _P, _P, _P] + [_c_int] * 4 + [_c_float, _P],
    "vs_masked_attn_backward": [_c_int] + [_P] * 11 + [_c_int] * 4 + [_c_float, _P],
    "vs_self_attn_forward": [_c_int, _P, _P, _P, _P, ctypes.c_longlong, _P, _P, _P] + [_c_int] * 4 + [_c_float, _P],
    "vs_self_attn_backward": [_c_int, _P, _P, _P, _P, ctypes.c_longlong] + [_P] * 6 + [_c_int] * 4 + [_c_float, _P],
    "vs_layer_norm_forward": [_c_int] + [_P] * 6 + [_c_int] * 2 + [_c_float, _P],
    "vs_layer_norm_backward_workspace_bytes": [_c_int] * 2,
    "vs_layer_norm_backward": [_c_int] + [_P] * 9 + [_c_int] * 2 + [_P],
    "vs_add_layer_norm_forward": [_c_int] + [_P] * 8 + [_c_int] * 2 + [_c_float, _P],
    "vs_layer_norm_backward_add": [_c_int] + [_P] * 10 + [_c_int] * 2 + [_P],
    "vs_layer_norm_backward_ex": [_c_int] + [_P] * 11 + [_c_int] * 2 + [_P],
    "vs_layer_norm_forward_rows": [_c_int] + [_P] * 6 + [_c_int] * 2 + [_c_float, _P, _P],
    "vs_add_layer_norm_forward_rows": [_c_int] + [_P] * 8 + [_c_int] * 2 + [_c_float, _P, _P],
    "vs_layer_norm_backward_rows": [_c_int] + [_P] * 11 + [_c_int] * 2 + [_P, _P],
    "vs_column_sum_workspace_bytes": [_c_int] * 2,
    "vs_column_sum": [_c_int] + [_P] * 3 + [_c_int] * 2 + [_P],
    "vs_column_sum_segments_workspace_bytes": [_c_int] * 3,
    "vs_rel_table_grad_workspace_bytes": [_c_int] * 3,
    "vs_rel_table_grad": [_c_int, _P, _P, _P, _c_int, _c_int, _c_int, _P],
    "vs_column_sum_segments": [_c_int] + [_P] * 3 + [_c_int] * 3 + [_P, _c_int, _P],
    "vs_act_backward_colsum": [_c_int, _c_int] + [_P] * 5 + [_c_int] * 2 + [_P],
    "vs_flat_step_workspace_bytes": [_c_int],
    "vs_flat_step": [_c_int, _P, _P, _c_float, _P, _P, _P, _P, _P, _P, _c_int, _c_int, _c_int] + [_c_float] * 6
                    + [_P, _P, _P, _P, _P],
    "vs_event_create": [ctypes.POINTER(_c_void_p)],
    "vs_event_destroy": [_P],
    "vs_event_record_external": [_P, _P],
    "vs_stream_wait_event": [_P, _P],
    "vs_lsa_max_targets": [_c_int],
    "vs_lsa_batch": [_P, _P] + [_c_int] * 4 + [_P, _P],
    "vs_lsa_batch_device_counts": [_P, _P] + [_c_int] * 4 + [_P, _P],
    "vs_match_cost": [_P, _c_int, _P, _c_int, _P, _P, _P, _P] + [_c_int] * 6 + [_c_float] * 3 + [_P],
    "vs_feature_resize_hilo": [_P, _P] + [_c_int] * 6 + [_P],
    "vs_level_bitmask_hilo": [_P, _P, _P] + [_c_int] * 5 + [_P],
    "vs_feature_sample_hilo": [_P, _P, _P] + [_c_int] * 5 + [_P],
    "vs_match_cost_factors_workspace_bytes": [_c_int] * 5,
    "vs_match_cost_factors": [_P, _P, _c_int, _P, _c_int, _P, _P, _P, _P] + [_c_int] * 5 + [_c_float] * 3 + [_P],
    "vs_group_norm_workspace_bytes": [_c_int] * 4,
    "vs_group_norm_forward": [_c_int] + [_P] * 7 + [_c_int] * 4 + [_c_float, _c_int, _P],
    "vs_group_norm_backward": [_c_int] + [_P] * 10 + [_c_int] * 5 + [_P],
    "vs_splitk_sum": [_c_int, _P, _c_int, ctypes.c_longlong, _P, _P, _P],
    "vs_group_norm_nchw_workspace_bytes": [_c_int] * 3,
    "vs_small_linear_wgrad": [_c_int, _P, _P, _P, _P, _c_int, _c_int, _c_int, _P],
    "vs_small_linear_forward": [_c_int, _P, _P, _c_int, _P, _P, _c_int, _P, _c_int, _c_int, _c_int, _P],
    "vs_small_linear_backward": [_c_int, _P, _P, _P, _c_int, _P, _P, _P, _P, _P, _c_int, _P, _P, _c_int, _c_int,
                                 _c_int, _P],
    "vs_self_attn_in_proj_forward": [_c_int, _P, _P, _c_int, _P, _P, _P, _c_int, _c_int, _P],
    "vs_self_attn_in_proj_backward": [_c_int, _P, _P, _c_int, _P, _P, _P, _P, _P, _c_int, _P, _P, _c_int, _c_int,
                                      _P],
    "vs_group_norm_nchw_forward": [_c_int] + [_P] * 7 + [_c_int] * 4 + [_c_float, _c_int, _P],
    "vs_group_norm_nchw_backward": [_c_int] + [_P] * 10 + [_c_int] * 5 + [_P],
    "vs_upsample_add_forward": [_c_int, _P, _P, _P] + [_c_int] * 6 + [ctypes.c_longlong, _P],
    "vs_upsample_backward": [_c_int, _P, _P] + [_c_int] * 6 + [_P],
    "vs_upsample_add_forward_nhwc": [_c_int, _P, _P, _P] + [_c_int] * 6 + [ctypes.c_longlong, _P],
    "vs_upsample_backward_nhwc": [_c_int, _P, _P] + [_c_int] * 6 + [_P],
    "vs_token_wgrad_workspace_bytes": [ctypes.c_longlong, _c_int, _c_int],
    "vs_token_wgrad_grouped_workspace_bytes": [_P, _c_int],
    "vs_token_wgrad_grouped": [_c_int, _P, _c_int, _P, _P],
    "vs_transpose_batched": [_c_int, _P, _c_int, _P],
    "vs_token_wgrad": [_c_int, _P, ctypes.c_longlong, _P, ctypes.c_longlong, _P, _P, _P, ctypes.c_longlong, _c_int,
                       _c_int, _P],
    "vs_conv3x3_forward": [_P, _P, _P, _P] + [_c_int] * 5 + [_P],
    "vs_conv3x3_weight_layouts": [_P, _P, _P, _c_int, _c_int, _P],
    "vs_conv3x3_wgrad_workspace_bytes": [_c_int] * 5,
    "vs_conv3x3_wgrad": [_c_int, _P, _P, _P, _P] + [_c_int] * 5 + [_P],
}
RESTYPES = {"vs_last_error": ctypes.c_char_p, "vs_masked_attn_workspace_bytes": ctypes.c_longlong,
            "vs_mask_head_backward_workspace_bytes": ctypes.c_longlong,
            "vs_layer_norm_backward_workspace_bytes": ctypes.c_longlong,
            "vs_column_sum_workspace_bytes": ctypes.c_longlong,
            "vs_column_sum_segments_workspace_bytes": ctypes.c_longlong,
            "vs_rel_table_grad_workspace_bytes": ctypes.c_longlong,
            "vs_flat_step_workspace_bytes": ctypes.c_longlong,
            "vs_group_norm_workspace_bytes": ctypes.c_longlong,
            "vs_group_norm_nchw_workspace_bytes": ctypes.c_longlong,
            "vs_msda_backward_tiled_workspace_bytes": ctypes.c_longlong,
            "vs_msda_backward_workspace_bytes": ctypes.c_longlong,
            "vs_match_cost_factors_workspace_bytes": ctypes.c_longlong,
            "vs_conv3x3_wgrad_workspace_bytes": ctypes.c_longlong,
            "vs_token_wgrad_workspace_bytes": ctypes.c_longlong,
            "vs_token_wgrad_grouped_workspace_bytes": ctypes.c_longlong}

_lib = None
_tops = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is not built: run `make -C vision-instance-seg_amd` or "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, args in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = RESTYPES.get(name, _c_int)
        _lib = L
    return _lib


def tops():
    """torch.ops.visionseg, loaded from the in-tree libvisionseg_torch.so (no fallback)."""
    global _tops
    if _tops is None:
        lib()
        if not os.path.exists(TORCH_LIB_PATH):
            raise RuntimeError(f"{TORCH_LIB_PATH} is not built: run `make -C vision-instance-seg_amd`")
        torch.ops.load_library(TORCH_LIB_PATH)
        _tops = torch.ops.visionseg
    return _tops


_level_tensors = {}


def level_tensors(shapes):
    """CPU int64 (spatial_shapes [L,2], level_start_index [L]) for msda_fwd/bwd, cached per
    shape list (host tensors: the op reads them without a device sync)."""
    key = tuple(shapes)
    t = _level_tensors.get(key)
    if t is None:
        starts, s = [], 0
        for h, w in shapes:
            starts.append(s)
            s += h * w
        t = (torch.tensor(shapes, dtype=torch.int64).reshape(-1, 2), torch.tensor(starts, dtype=torch.int64))
        _level_tensors[key] = t
    return t


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().vs_last_error().decode(errors="replace")
        raise RuntimeError(f"visionseg {what} failed (status {rc}): {msg}")


def dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return VS_F32
    if t.dtype == torch.bfloat16:
        return VS_BF16
    raise TypeError(f"visionseg kernels take float32 or bfloat16 activations, got {t.dtype}")


def require_hip(*ts: torch.Tensor):
    for t in ts:
        if not t.is_cuda:
            raise RuntimeError("visionseg ops run only on a HIP device (no CPU fallback); "
                               f"got a tensor on {t.device}")


def ptr(t: torch.Tensor):
    return ctypes.c_void_p(t.data_ptr())


def stream(t: torch.Tensor | None = None):
    dev = t.device if t is not None else None
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
