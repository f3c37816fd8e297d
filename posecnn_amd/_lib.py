"""Loader and thin ctypes binding of libposecnn_hip.so (include/posecnn_hip.h).

The HIP library is the only compute path: if it is missing, or no GPU is
visible, every op raises — there is no CPU fallback.  torch is imported first
so that the library binds to the same HIP runtime instance as torch's streams
and allocations (both resolve the soname libamdhip64.so.7).
"""
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("POSECNN_HIP_LIB") or os.path.join(_HERE, "libposecnn_hip.so")  # override: experiments

_lib = None
_lock = threading.Lock()

c_int = ctypes.c_int
c_float = ctypes.c_float
c_size_t = ctypes.c_size_t
c_void_p = ctypes.c_void_p

# name -> (restype, argtypes); v = c_void_p (device/host pointer or stream)
_SIGS = {
    "pcnn_abi_version": (c_int, []),
    "pcnn_strerror": (ctypes.c_char_p, [c_int]),
    "pcnn_set_completion_event": (c_int, [c_void_p]),
    "pcnn_completion_event_pending": (c_int, []),
    "pcnn_hough_voting_workspace_size": (c_size_t, [c_int, c_int, c_int, c_int, c_int, c_float]),
    "pcnn_hough_voting": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int,
                                  c_int, c_int, c_int, c_int, c_int, c_float, c_int, c_float, c_float, c_int,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                  c_void_p, c_size_t, c_void_p]),
    "pcnn_hough_voting_prob": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int,
                                       c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_int, c_float,
                                       c_float, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pcnn_hough_voting_compact": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int,
                                          c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_int, c_float, c_float,
                                          c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                          c_void_p, c_void_p, c_size_t, c_void_p]),
    "pcnn_hough_voting_grad": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "pcnn_hough_voting_diag": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_float, c_void_p, c_void_p]),
    "pcnn_roi_pool_fwd": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int,
                                  c_void_p, c_float, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "pcnn_roi_pool_fwd_accumulate": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int,
                                             c_int, c_void_p, c_float, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "pcnn_roi_pool_fwd_pair": (c_int, [c_void_p, c_int, c_int, c_float, c_void_p, c_int, c_int, c_float, c_int, c_int,
                                       c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                       c_void_p, c_void_p]),
    "pcnn_roi_pool_fwd_pair_px": (c_int, [c_void_p, c_int, c_int, c_float, c_void_p, c_int, c_int, c_float, c_int,
                                          c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                                          c_void_p, c_void_p, c_void_p]),
    "pcnn_roi_pool_bwd_workspace_size": (c_size_t, [c_int, c_int]),
    "pcnn_roi_pool_bwd_px": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int,
                                     c_void_p, c_float, c_int, c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pcnn_roi_pool_bwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int,
                                  c_int, c_void_p, c_float, c_int, c_int, c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pcnn_add_loss_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "pcnn_add_loss_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int,
                                  c_float, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pcnn_add_loss_fwd_prepared": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int,
                                  c_float, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pcnn_add_loss_prep": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_size_t, c_void_p]),
    "pcnn_add_loss_ws_offset": (ctypes.c_long, [c_int, c_int, c_int, c_int]),
    "pcnn_add_loss_prep_points": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p,
                                          c_size_t, c_void_p]),
    "pcnn_add_loss_fwd_head_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int,
                                           c_int, c_float, c_int, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p,
                                           c_void_p, c_void_p, c_void_p]),
    "pcnn_add_loss_total": (c_int, [c_int, c_void_p, c_int, c_int, c_void_p, c_size_t, c_void_p, c_void_p]),
    "pcnn_add_loss_bwd": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p]),
    "pcnn_div_rn_check": (c_int, [c_void_p, c_float, c_int, c_int, c_void_p, c_void_p]),
    "pcnn_backproject_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int,
                                     c_int, c_int, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pcnn_backproject_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                     c_void_p, c_void_p]),
    "pcnn_gemm_workspace_size": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "pcnn_gemm": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                          c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_size_t,
                          c_void_p]),
    "pcnn_gemm_drop": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_int,
                               c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_float, c_void_p,
                               c_void_p, c_int, c_void_p, c_size_t, c_void_p]),
    "pcnn_gemm_drop_gen": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_int,
                                   c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_float, ctypes.c_uint64,
                                   c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_size_t, c_void_p]),
    "pcnn_dropout_mask": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, ctypes.c_uint64, c_void_p, c_int, c_float,
                                  c_void_p]),
    "pcnn_philox_check": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "pcnn_pose2d_workspace_size": (c_size_t, [c_int, c_int, c_int, c_int]),
    "pcnn_pose2d": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_float, c_float, c_float,
                            ctypes.c_uint64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_size_t, c_void_p]),
    "pcnn_pose3d_workspace_size": (c_size_t, [c_int, c_int, c_int, c_int]),
    "pcnn_pose3d": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_float, c_float,
                            c_float, c_float, ctypes.c_uint64, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pcnn_tp_bytes": (c_size_t, [c_int, c_int]),
    "pcnn_split_tp": (c_int, [c_void_p, ctypes.c_long, ctypes.c_long, c_int, c_void_p, c_int, c_void_p, c_void_p,
                              c_size_t, c_void_p]),
    "pcnn_gemm_tp": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p,
                             c_int, c_void_p, c_int, c_float, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pcnn_colsum": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "pcnn_box_nms": (c_int, [c_void_p, c_int, c_int, c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                             c_void_p, c_void_p, c_void_p]),
    "pcnn_argmax_2d": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "pcnn_hard_label_fwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_void_p, c_void_p]),
    "pcnn_hard_label_bwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "pcnn_vertex_pred_compact": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                         c_void_p, c_void_p]),
    "pcnn_pose_head_fwd": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "pcnn_pose_head_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p,
                                   c_void_p]),
    "pcnn_icp_live_vertices": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_float, c_float, c_float,
                                       c_float, c_float, c_void_p, c_void_p]),
    "pcnn_icp_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "pcnn_icp": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_float, c_float,
                         c_float, c_float, c_float, c_float, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_size_t, c_void_p]),
    "pcnn_icp_reduce_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "pcnn_icp_center": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pcnn_icp_score_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "pcnn_icp_score": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_float, c_void_p,
                               c_void_p, c_void_p, c_size_t, c_void_p]),
    "pcnn_energy_records_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "pcnn_energy_records": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_float, c_float, c_int,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "pcnn_energy_rec": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_float, c_float, c_void_p,
                                c_void_p]),
    "pcnn_nelder_mead_energy": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                        c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pcnn_nelder_mead_energy_workspace_size": (c_size_t, [c_int]),
    "pcnn_nelder_mead_energy_coop": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                             c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                             c_void_p]),
    "pcnn_nelder_mead_energy_coop_path": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                                  c_int, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                                                  c_size_t, c_int, c_void_p, c_void_p]),
    "pcnn_pose_energy_batch": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_float,
                                       c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                       c_void_p]),
    "pcnn_pose_energy": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_float, c_float, c_void_p, c_int,
                                 c_void_p, c_void_p, c_size_t, c_void_p]),
}


class PcnnError(RuntimeError):
    pass


def load():
    """Load libposecnn_hip.so (raises if absent: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise PcnnError(f"{LIB_PATH} not built; run __graft_entry__.build() "
                                "(hipcc --offload-arch=gfx950). No CPU fallback exists.")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in _SIGS.items():
                if name.endswith("_check") and not hasattr(lib, name):
                    continue  # self-check entry points (tests only); absent from older A/B builds
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def exported_symbols():
    return list(_SIGS.keys())


def check(rc, what):
    if rc != 0:
        msg = load().pcnn_strerror(rc).decode()
        if rc == 1:
            raise ValueError(f"{what}: {msg}")
        raise PcnnError(f"{what}: {msg} (code {rc})")


def require_gpu(*tensors):
    if not torch.cuda.is_available():
        raise PcnnError("posecnn_amd ops run only on an AMD GPU (HIP); none is visible")
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise ValueError("posecnn_amd ops take device tensors (got a CPU tensor)")


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


_ws = {}


def workspace(nbytes, device, tag="default", stream=None):
    """Per-(device, tag, stream) grow-only byte workspace (no allocation on
    the hot path once sized).  `stream` is the stream the op launches on
    (default: the current stream): ops on different streams never share
    scratch, so concurrent calls stay reentrant."""
    s = stream if stream is not None else torch.cuda.current_stream(device)
    key = (str(device), tag, s.cuda_stream)
    buf = _ws.get(key)
    if buf is None or buf.numel() < nbytes:
        # allocated under the launch stream: when a grown buffer replaces the
        # old one, the caching allocator hands the old block out again only in
        # order with that stream, whose kernels are the old block's users
        with torch.cuda.stream(s):
            buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
        _ws[key] = buf
    return buf
