"""ctypes binding of libhlmc.so (include/hlmc.h).

The product path has no fallback: if the HIP library is missing or cannot be loaded, every entry
point raises.  Tensors cross the boundary as raw device pointers of torch tensors; the stream is
torch's current HIP stream.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HLMC_LIB") or os.path.join(_HERE, "libhlmc.so")  # HLMC_LIB: A/B builds

c_int, c_i64, c_f32, c_f64, c_vp, c_char_p = C.c_int, C.c_int64, C.c_float, C.c_double, C.c_void_p, C.c_char_p
P_vp = C.POINTER(c_vp)
P_i64 = C.POINTER(c_i64)

HLMC_F32, HLMC_BF16 = 0, 1
NET_HYBRID, NET_CVAE, NET_SIMPLE = 0, 1, 2

_SIGS = {
    "hlmc_version": (c_int, []),
    "hlmc_last_error": (c_char_p, []),
    "hlmc_device_status": (c_int, [c_int]),
    "hlmc_test_bn_fused": (c_int, [c_i64, c_int]),
    "hlmc_mel_plan_create": (c_int, [c_int, c_int, c_int, c_int, c_f64, c_f64, P_vp]),
    "hlmc_mel_plan_destroy": (c_int, [c_vp]),
    "hlmc_mel_filterbank": (c_int, [c_vp, c_vp]),
    "hlmc_mel_frames": (c_i64, [c_vp, c_i64]),
    "hlmc_mel_workspace": (c_i64, [c_vp, c_i64, c_i64]),
    "hlmc_melspectrogram": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "hlmc_mel_db": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_f32, c_f32, c_vp, c_vp]),
    "hlmc_mel_db_zscore": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_f32, c_f32, c_vp, c_vp, c_int, c_vp,
                                   c_vp]),
    "hlmc_power_to_db": (c_int, [c_vp, c_vp, c_i64, c_i64, c_int, c_f32, c_f32, c_f32, c_vp, c_vp]),
    "hlmc_mfcc": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_int, c_vp, c_vp]),
    "hlmc_spectral_shape": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_f64, c_vp]),
    "hlmc_zcr_rms": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "hlmc_chroma_workspace": (c_i64, [c_vp, c_i64, c_i64]),
    "hlmc_chroma_stft": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "hlmc_row_mean_std": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "hlmc_colstats_workspace": (c_i64, [c_i64, c_i64]),
    "hlmc_colstats_sum": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "hlmc_colstats_centered": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "hlmc_zscore_apply": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_int, c_vp]),
    "hlmc_net_create": (c_int, [c_int, P_i64, c_int, c_int, P_vp]),
    "hlmc_net_destroy": (c_int, [c_vp]),
    "hlmc_net_num_params": (c_int, [c_vp]),
    "hlmc_net_param_info": (c_int, [c_vp, c_int, c_char_p, c_int, C.POINTER(c_int), P_i64]),
    "hlmc_net_num_bn": (c_int, [c_vp]),
    "hlmc_net_state_bytes": (c_i64, [c_vp]),
    "hlmc_net_workspace_bytes": (c_i64, [c_vp, c_i64]),
    "hlmc_net_bind": (c_int, [c_vp, P_vp, P_vp, P_vp, P_vp, c_vp]),
    "hlmc_net_forward": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                 c_vp, c_vp]),
    "hlmc_net_encode": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "hlmc_net_decode": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "hlmc_net_backward": (c_int, [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "hlmc_net_adam_step": (c_int, [c_vp, c_vp, P_vp, P_vp, c_f32, c_f32, c_f32, c_f32, c_f32, c_int]),
    "hlmc_net_set_trust_packs": (c_int, [c_vp, c_int]),
    "hlmc_net_adam_step_dev": (c_int, [c_vp, c_vp, P_vp, P_vp, c_vp]),
    "hlmc_adam_coef": (c_int, [c_f32, c_f32, c_f32, c_f32, c_f32, c_int, c_vp]),
    "hlmc_net_set_overlap_adam": (c_int, [c_vp, c_int]),
    "hlmc_net_set_rng": (c_int, [c_vp, C.c_uint64, C.c_uint64]),
    "hlmc_net_get_rng": (c_int, [c_vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "hlmc_randn": (c_int, [c_vp, c_vp, c_i64, C.c_uint64, C.c_uint64]),
    "hlmc_net_settle": (c_int, [c_vp, c_vp]),
    "hlmc_net_grad_buckets": (c_int, [c_vp, C.POINTER(c_int), c_int]),
    "hlmc_net_set_bucket_sync": (c_int, [c_vp, c_int]),
    "hlmc_net_bucket_wait": (c_int, [c_vp, c_int, c_vp]),
    "hlmc_probe_arm": (c_int, [c_int, c_int]),
    "hlmc_probe_read": (c_int, [C.POINTER(c_int), C.POINTER(c_f64), C.POINTER(c_f64), C.POINTER(c_f64),
                                C.POINTER(c_f32), c_int]),
    "hlmc_loss_workspace": (c_i64, [c_i64, c_i64, c_i64]),
    "hlmc_loss_sums": (c_int, [c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "hlmc_loss_backward": (c_int, [c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64,
                                   c_vp, c_vp, c_vp]),
    "hlmc_loss_sums_backward": (c_int, [c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64,
                                        c_vp, c_vp, c_vp, c_vp, c_vp]),
    "hlmc_adam_scratch_bytes": (c_i64, [c_int]),
    "hlmc_adam_step": (c_int, [c_vp, c_int, P_vp, P_vp, P_vp, P_vp, P_i64, c_f32, c_f32, c_f32, c_f32, c_f32,
                               c_int, c_vp]),
    "hlmc_km_center": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp]),
    "hlmc_km_sqdist_rows": (c_int, [c_vp, c_vp, c_i64, c_int, P_i64, c_int, c_vp]),
    "hlmc_km_assign": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_int, c_vp, c_vp, c_vp]),
    "hlmc_km_sums": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_int, c_vp, c_vp]),
    "hlmc_km_sums_workspace": (c_i64, [c_i64, c_int]),
    "hlmc_km_sums_part": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_i64]),
    "hlmc_km_rowdist": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp]),
    "hlmc_km_inertia": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp, c_vp]),
    "hlmc_op_bn_bwd_workspace": (c_i64, [c_int]),
    "hlmc_op_bn_bwd": (c_int, [c_vp, c_int, c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                               c_i64]),
    "hlmc_km_assign_batch": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_int, c_int, C.c_uint64, c_vp, c_vp, c_vp]),
    "hlmc_km_sums_batch": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_int, c_int, C.c_uint64, c_vp, c_vp, c_vp, c_i64]),
    "hlmc_km_update_batch": (c_int, [c_vp, c_int, c_int, c_int, C.c_uint64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "hlmc_km_pp_search": (c_int, [c_vp, c_i64, c_int, c_int, c_vp, c_int, C.POINTER(C.c_int32), C.POINTER(c_f64), c_vp,
                                  c_vp]),
    "hlmc_km_pp_dist": (c_int, [c_vp, c_vp, c_i64, c_int, c_int, c_int, c_vp, c_vp, c_int, C.POINTER(C.c_int32), c_vp]),
    "hlmc_km_inertia_batch": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_int, c_vp, c_int, c_vp, c_vp]),
    "hlmc_silhouette_workspace": (c_i64, [c_i64, c_int]),
    "hlmc_silhouette": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_i64]),
    "hlmc_cluster_scores_workspace": (c_i64, [c_int, c_int]),
    "hlmc_cluster_scores": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp, c_int, c_vp, c_vp, c_i64]),
    "hlmc_op_conv_s2": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_i64]),
    "hlmc_op_subpixel": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_i64]),
    "hlmc_op_wgrad_s2": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_i64]),
    "hlmc_op_linear": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp, c_int, c_vp, c_int, c_int,
                               c_int, c_int, c_vp, c_i64, c_vp]),
    "hlmc_op_linear_wgrad": (c_int, [c_vp, c_int, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp,
                                     c_i64]),
    "hlmc_op_conv_c1_s2": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_int, c_vp]),
    "hlmc_op_convT_c1": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp]),
    "hlmc_op_wgrad_c1": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_i64]),
    "hlmc_op_halo_workspace": (c_i64, [c_int, c_int]),
    "hlmc_op_halo_fwd": (c_int, [c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_vp,
                                 c_vp, c_vp, c_vp, c_vp, c_f32, c_f32, c_vp, c_vp, c_vp, c_vp, c_i64]),
}

_lib = None


def lib():
    """Load libhlmc.so once; raise (never fall back) when it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libhlmc.so not built at {LIB_PATH}: run `python -c 'import __graft_entry__ as g; g.build()'`")
        handle = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def exported_symbols():
    return list(_SIGS)


class HLMCError(RuntimeError):
    pass


def check(status: int, what: str = "") -> None:
    if status != 0:
        msg = lib().hlmc_last_error().decode(errors="replace")
        raise HLMCError(f"{what or 'libhlmc'} failed (status {status}): {msg}")


def check_device(what: str = "") -> None:
    """Raise when a kernel raised a fault bit in the library's device status word (include/hlmc.h
    hlmc_device_status: e.g. a one-launch BatchNorm backward whose grid-wide count timed out, outputs NaN).  Reads
    pinned host memory, no synchronisation; a launch's bit is visible once the launch has completed."""
    st = lib().hlmc_device_status(0)
    if st:
        raise HLMCError(f"{what or 'libhlmc'}: device status {st} (bit 0: BatchNorm backward grid-wide count timed "
                        f"out; its outputs are NaN) -- clear with hlmc_device_status(1)")


def ptr(t) -> int | None:
    """Device pointer of a tensor (None passes NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def require_cuda(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise HLMCError("libhlmc operates on GPU tensors; got a CPU tensor")
        if t is not None and not t.is_contiguous():
            raise HLMCError("libhlmc needs contiguous tensors")


def vp_array(values):
    arr = (c_vp * len(values))()
    for i, v in enumerate(values):
        arr[i] = v
    return arr


def i64_array(values):
    arr = (c_i64 * len(values))()
    for i, v in enumerate(values):
        arr[i] = int(v)
    return arr
