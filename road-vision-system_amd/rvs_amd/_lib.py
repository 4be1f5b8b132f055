"""ctypes binding of librvhip.so (the C ABI declared in include/rvhip.h).

The product path has exactly one implementation: the gfx950 HIP kernels in
this library.  If the library is missing or cannot be loaded, every op raises
immediately -- there is deliberately no CPU fallback (the reference's
``ops_cuda`` soft-fallback, src/preprocess/ops_cuda/cuda_clahe_dehaze.py:22-39,
is replaced by a loud failure so a silent slow path can never be measured).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_char_p, c_double, c_float, c_int, c_size_t, c_void_p, POINTER

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "librvhip.so")
# A/B runs of two builds on one box (tools/ab_env.sh): RV_LIB_VARIANT=x loads
# librvhip_x.so from this directory instead ("default" or unset: librvhip.so).
_variant = os.environ.get("RV_LIB_VARIANT", "default")
if _variant != "default":
    LIB_PATH = os.path.join(_HERE, "librvhip_%s.so" % _variant)

_lib = None


class RVError(RuntimeError):
    """A non-zero status returned through the C ABI."""


# name -> (restype, argtypes)
_SIGS = {
    "rv_abi_version": (c_int, []),
    "rv_last_error": (ctypes.c_char_p, []),
    "rv_clahe_ws_bytes": (c_size_t, [c_int, c_int]),
    "rv_clahe_ycrcb_u8": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                  c_double, c_void_p, c_size_t, c_void_p]),
    "rv_clahe_lab_u8": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                c_double, c_void_p, c_size_t, c_void_p]),
    "rv_lab_init": (c_int, []),
    "rv_lab_tables_host": (c_int, [c_void_p, c_size_t]),
    "rv_median_u8c3": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "rv_clahe_median_u8": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                   c_double, c_int, c_void_p, c_size_t, c_void_p]),
    "rv_clahe_median_fits": (c_int, [c_int, c_int, c_int, c_int]),
    "rv_clahe_median_letterbox_u8": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                             c_int, c_double, c_int, c_void_p, c_size_t,
                                             c_void_p, POINTER(c_int), c_void_p]),
    "rv_clahe_median_letterbox_fits": (c_int, [c_int, c_int, c_int, c_int, POINTER(c_int)]),
    "rv_gray_span_u8": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                c_void_p]),
    # result hand-back
    "rv_results_bytes": (c_size_t, [c_int, c_int]),
    "rv_results_handback": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                    c_void_p, c_size_t, c_void_p, c_void_p]),
    # standalone tracker / geometry pieces
    "rv_iou_matrix_batched": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                      c_int, c_int, c_void_p]),
    "rv_greedy_assign_batched": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                         c_double, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p]),
    "rv_homography_project_f64": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_double,
                                          c_void_p, c_void_p, c_void_p]),
    "rv_untracked_metrics": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                     c_double, c_void_p, c_void_p, c_void_p, c_void_p]),
    # ingest
    "rv_nv12_to_bgr_u8": (c_int, [c_void_p, c_void_p, c_int, c_int, c_size_t, c_size_t, c_void_p,
                                  c_int, c_int, c_int, c_int, c_void_p]),
    # augment
    "rv_fog_ws_bytes": (c_size_t, [c_int]),
    "rv_fog_rain_u8": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int,
                               c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_size_t,
                               c_void_p]),
    # capture front end
    "rv_capture_open": (c_int, [c_char_p, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "rv_capture_info": (c_int, [c_void_p, c_void_p]),
    "rv_capture_next": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rv_capture_release": (c_int, [c_void_p, c_int]),
    "rv_capture_upload_batch": (c_int, [c_void_p, c_int, c_void_p, c_size_t, c_void_p, c_void_p,
                                        c_void_p]),
    "rv_capture_close": (c_int, [c_void_p]),
    "rv_fog_full_ws_bytes": (c_size_t, [c_int, c_int, c_int]),
    "rv_fog_full_u8": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int,
                               c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_size_t,
                               c_void_p]),
    "rv_letterbox_geometry": (c_int, [c_int, c_int, c_int, c_int, POINTER(c_int)]),
    "rv_letterbox_u8": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                POINTER(c_int), c_void_p]),
    # detect
    "rv_yolo_num_convs": (c_int, [c_int]),
    "rv_yolo_conv_info": (c_int, [c_int, c_int, POINTER(c_int), ctypes.c_char_p, c_int]),
    "rv_yolo_flat_floats": (c_size_t, [c_int]),
    "rv_yolo_packed_bytes": (c_size_t, [c_int]),
    "rv_yolo_pack": (c_int, [c_int, c_void_p, c_size_t, c_void_p, c_size_t]),
    "rv_yolo_create": (c_int, [c_int, c_void_p, c_int, c_int, c_int, POINTER(c_void_p)]),
    "rv_yolo_destroy": (c_int, [c_void_p]),
    "rv_yolo_set_option": (c_int, [c_void_p, c_int, c_int]),
    "rv_conv_bf16": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                             c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p,
                             c_void_p]),
    "rv_yolo_packed_bytes2": (c_size_t, [c_int, c_int]),
    "rv_yolo_pack2": (c_int, [c_int, c_int, c_void_p, c_size_t, c_void_p, c_size_t]),
    "rv_yolo_create2": (c_int, [c_int, c_int, c_void_p, c_int, c_int, c_int, POINTER(c_void_p)]),
    "rv_yolo_set_act_scales": (c_int, [c_void_p, c_void_p, c_int]),
    "rv_yolo_buffer_esize": (c_int, [c_void_p, c_int]),
    "rv_yolo_buffer_name": (c_int, [c_void_p, c_int, ctypes.c_char_p, c_int]),
    "rv_fp8_scale": (c_float, [c_double]),
    "rv_yolo_ws_bytes": (c_size_t, [c_void_p, c_int]),
    "rv_yolo_num_anchors": (c_int, [c_void_p]),
    "rv_yolo_forward": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_size_t, c_void_p, c_float,
                                c_void_p, c_int, c_void_p, c_void_p]),
    "rv_yolo_forward_part": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_size_t, c_void_p,
                                     c_float, c_void_p, c_int, c_void_p, c_void_p, c_int]),
    "rv_yolo_num_buffers": (c_int, [c_void_p]),
    "rv_yolo_buffer_info": (c_int, [c_void_p, c_int, c_int, POINTER(c_int), POINTER(c_size_t)]),
    "rv_yolo_trace": (c_int, [c_void_p, c_void_p, c_int]),
    "rv_yolo_profile": (c_int, [c_void_p, c_int]),
    "rv_yolo_profile_reps": (c_int, [c_void_p, c_int, c_int]),
    "rv_yolo_profile_read": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int]),
    "rv_yolo_profile_bytes": (c_int, [c_void_p, c_void_p, c_int]),
    "rv_yolo_profile_times": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int]),
    "rv_yolo_autotune": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_size_t, c_int, c_int,
                                 POINTER(c_int), c_void_p]),
    "rv_yolo_tuned_config": (c_int, [c_void_p, c_int, POINTER(c_int)]),
    "rv_yolo_set_tuned": (c_int, [c_void_p, c_int, c_int, POINTER(c_int)]),
    "rv_yolo_conv_candidates": (c_int, [c_void_p, c_int, c_void_p, c_int]),
    "rv_trace_marker": (c_int, [c_int, c_void_p]),
    "rv_install_crash_handler": (c_int, []),
    # native launch schedule
    "rv_sched_create": (c_int, [c_void_p]),
    "rv_sched_destroy": (c_int, [c_void_p]),
    "rv_sched_add_op": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p,
                                c_size_t, c_void_p]),
    "rv_sched_add_record": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "rv_sched_event_sync": (c_int, [c_void_p, c_int]),
    "rv_sched_event_query": (c_int, [c_void_p, c_int]),
    "rv_sched_event_elapsed": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "rv_sched_add_wait": (c_int, [c_void_p, c_void_p, c_int]),
    "rv_sched_num_nodes": (c_int, [c_void_p]),
    "rv_sched_run": (c_int, [c_void_p, c_void_p]),
    "rv_nms_smem_bytes": (c_size_t, []),
    "rv_nms_postprocess": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_int,
                                   c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_size_t, c_void_p]),
    "rv_nms_ws_bytes": (c_size_t, [c_int]),
    "rv_cand_segments": (c_int, [c_int]),
    "rv_yolo_cand_segments": (c_int, [c_void_p]),
    "rv_candidates_from_raw": (c_int, [c_void_p, c_int, c_int, c_int, c_float, c_void_p, c_int,
                                       c_void_p, c_void_p]),
    # track
    "rv_sort_state_bytes": (c_size_t, [c_int, c_int]),
    "rv_sort_ws_bytes": (c_size_t, [c_int, c_int, c_int]),
    "rv_sort_init": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "rv_sort_update": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int,
                               c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                               c_void_p, c_void_p, c_void_p, c_void_p]),
    "rv_sort_stats": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rv_sort_export": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
}


def load():
    """Load librvhip.so once; raise if it is missing (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RVError(
            f"{LIB_PATH} not found: build it with `make -C road-vision-system_amd/csrc` "
            "or __graft_entry__.build(); the HIP path has no CPU fallback")
    import torch  # noqa: F401 -- bind librvhip to torch's HIP runtime (libamdhip64.so.7),
    # never to a second copy from /opt/rocm: two runtimes in one process do not share devices
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        if not hasattr(lib, name) and _variant != "default":
            continue  # an older A/B build (RV_LIB_VARIANT) without this entry
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def register(name, restype, argtypes):
    """Declare an additional ABI entry (used by modules as they grow)."""
    _SIGS[name] = (restype, argtypes)
    if _lib is not None:
        fn = getattr(_lib, name)
        fn.restype = restype
        fn.argtypes = argtypes


def check(status: int, what: str = "") -> None:
    if status != 0:
        msg = load().rv_last_error().decode(errors="replace")
        raise RVError(f"{what or 'rvhip'} failed with status {status}: {msg}")


# stream-ordered calls a launch schedule can record (rvs_amd.schedule._OPS)
_RECORDABLE = {"rv_clahe_median_letterbox_u8", "rv_clahe_median_u8", "rv_letterbox_u8",
               "rv_yolo_forward_part", "rv_nms_postprocess", "rv_sort_update",
               "rv_results_handback", "rv_untracked_metrics"}

_NOCHECK = {"rv_sched_num_nodes", "rv_sched_event_query", "rv_abi_version", "rv_cand_segments", "rv_yolo_cand_segments", "rv_clahe_median_fits", "rv_clahe_median_letterbox_fits", "rv_yolo_num_convs", "rv_yolo_num_anchors",
            "rv_yolo_num_buffers", "rv_yolo_trace", "rv_yolo_profile_read", "rv_yolo_tuned_config",
            "rv_yolo_profile_bytes", "rv_yolo_profile_times", "rv_yolo_buffer_esize", "rv_yolo_conv_candidates"}


_recorder = None  # a schedule.Schedule while one is being recorded


class recording:
    """Inside this context, recordable calls (schedule._OPS) are appended to
    `sched` as launch-list nodes instead of running (rvs_amd.schedule)."""

    def __init__(self, sched):
        self.sched = sched

    def __enter__(self):
        global _recorder
        if _recorder is not None:
            raise RuntimeError("a schedule is already being recorded")
        _recorder = self.sched
        return self.sched

    def __exit__(self, *exc):
        global _recorder
        _recorder = None
        return False


def call(name: str, *args) -> int:
    if _recorder is not None and name in _RECORDABLE:
        _recorder.add(name, args)
        return 0
    fn = getattr(load(), name)
    st = fn(*args)
    if fn.restype is c_int and name not in _NOCHECK:
        check(st, name)
    return st


def stream_ptr(stream=None) -> int:
    """hipStream_t of a torch stream (default: current stream) as an int."""
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def ptr(t) -> int:
    """Device pointer of a torch tensor (None -> 0).  While a schedule is
    being recorded, the schedule keeps the tensor alive: a recorded node
    holds the raw pointer, so a temporary made for the call (a .contiguous()
    copy, a freshly grown workspace) must outlive every later run()."""
    if t is None:
        return 0
    if _recorder is not None:
        _recorder.keep(t)
    return int(t.data_ptr())


def int_array(vals):
    arr = (c_int * len(vals))(*[int(v) for v in vals])
    return arr


__all__ = ["load", "check", "call", "stream_ptr", "ptr", "int_array", "register", "RVError",
           "LIB_PATH", "c_int", "c_float", "c_double", "c_size_t", "c_void_p", "POINTER"]
