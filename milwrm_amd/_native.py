"""ctypes binding of the milwrm_amd C ABI (include/milwrm_amd.h).

``torch`` is imported first so that ``libmilwrm_amd.so`` binds to the HIP
runtime already loaded by PyTorch (same soname ``libamdhip64.so.7``): device
pointers and streams are then shared between the two.  There is no fallback:
if the library is missing or a call fails, an exception is raised.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch  # noqa: F401  (must precede the library load: one HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MW_LIB") or os.path.join(_HERE, "libmilwrm_amd.so")  # MW_LIB: tools only

MW_U8, MW_U16, MW_F32 = 0, 1, 2
_EINVAL, _EHIP, _EUNSUP = -1, -2, -3

_lib = None
_lock = threading.Lock()

c_i64, c_i32, c_u32, c_u64 = C.c_int64, C.c_int, C.c_uint32, C.c_uint64
c_f32, c_sz, c_vp = C.c_float, C.c_size_t, C.c_void_p
c_dp = C.POINTER(C.c_double)

# name -> (restype, argtypes)
_PROTOS = {
    "mw_version": (c_i32, []),
    "mw_host_labels_f64": (c_i32, [c_vp, c_i64, c_vp, c_i32]),
    "mw_host_f32_to_f64": (c_i32, [c_vp, c_i64, c_vp, c_i32]),
    "mw_last_error": (C.c_char_p, []),
    "mw_stream_blocks": (c_i32, [c_i64]),
    "mw_nz_stats_ws_bytes": (c_sz, [c_i64, c_i32]),
    "mw_nz_stats": (c_i32, [c_vp, c_i32, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp]),
    "mw_lognorm": (c_i32, [c_vp, c_i32, c_i64, c_i32, c_vp, c_f32, c_vp, c_vp]),
    "mw_blur_ws_bytes": (c_sz, [c_i32, c_i32, c_i32, c_i32]),
    "mw_blur": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_f32, c_vp, c_i32, c_vp, c_vp, c_vp]),
    "mw_block_mean": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp]),
    "mw_mask_rank_ws_bytes": (c_sz, [c_i64]),
    "mw_mask_rank": (c_i32, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "mw_gather_ws_bytes": (c_sz, [c_i64, c_i32]),
    "mw_gather_rows": (c_i32, [c_vp, c_i32, c_vp, c_i32, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "mw_col_stats_finalize": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_i32, c_vp]),
    "mw_legacy_randint_host": (c_i32, [c_u32, c_i64, c_i64, c_vp]),
    "mw_mt_jump_tables": (c_i32, [c_i64, c_i32, c_vp]),
    "mw_mt_jump_host": (c_i32, [c_vp, c_vp, c_vp]),
    "mw_mt_seed_state": (c_i32, [c_u32, c_vp]),
    "mw_legacy_randint_ws_bytes": (c_sz, [c_i64, c_i64, c_i64]),
    "mw_legacy_randint_device": (c_i32, [c_u32, c_i64, c_i64, c_vp, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "mw_legacy_randint_segments": (c_i64, [c_i64, c_i64, c_i64]),
    "mw_mt_segment_states": (c_i32, [c_u32, c_i64, c_vp, c_i32, c_vp, c_vp]),
    "mw_legacy_randint_gen_ws_bytes": (c_sz, [c_i64, c_i64, c_i64]),
    "mw_legacy_randint_from_states": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "mw_kpp_ws_bytes": (c_sz, [c_i64, c_i32]),
    "mw_kpp_init": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp]),
    "mw_kpp_step": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_i32, c_vp, c_i32, c_vp, c_vp]),
    "mw_kpp_indices": (c_i32, [c_vp, c_i64, c_i32, c_i32, c_vp, c_vp]),
    "mw_kpp_step_fold": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_i32, c_vp, c_i32, c_vp, c_i64, c_vp, c_vp,
                                 c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mw_kpp_fold_rec_bytes": (c_sz, [c_i64, c_i32, c_i32]),
    "mw_kpp_fold_supported": (c_i32, [c_i32, c_i32, c_i32]),
    "mw_kmeans_fit_history": (c_i32, [c_vp, c_i32]),
    "mw_kpp_best_ptr": (c_vp, [c_vp, c_i64, c_i32]),
    "mw_kpp_pots": (c_i32, [c_vp, c_i64, c_i32, c_i32, c_vp, c_vp]),
    "mw_kpp_search": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp]),
    "mw_kpp_trial": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_i32, c_i32, c_vp, c_i32, c_vp, c_vp]),
    "mw_lloyd_ws_bytes": (c_sz, [c_i64, c_i32, c_i32]),
    "mw_lloyd_ws_bytes_kinds": (c_sz, [c_i64, c_i32, c_i32, c_i32]),
    "mw_lloyd_list_moved": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp]),
    "mw_lloyd_rec_len": (c_i32, [c_i32, c_i32]),
    "mw_lloyd_pass": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_i32, c_vp, c_i32, c_i32, c_vp]),
    "mw_col_absmax": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp]),
    "mw_col_absmax_acc": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp]),
    "mw_kmeans_fit_ws_bytes": (c_sz, [c_i64, c_i32, c_i32]),
    "mw_kmeans_fit": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_u32, c_i32,
                              C.c_double, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "mw_kmeans_fit_async": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_u32, c_i32,
                                    C.c_double, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp, c_vp, c_vp]),
    "mw_lloyd_fits": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                              c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, C.c_double,
                              c_i32, c_i32, C.c_double, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp,
                              c_vp, c_vp]),
    "mw_lloyd_fits_msg_len": (c_i64, [c_i64, c_i32, c_i32]),
    "mw_lloyd_fits_sharded": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                      c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, C.c_double,
                                      c_i32, c_i32, C.c_double, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i32,
                                      c_vp, c_vp, c_vp, c_vp]),
    "mw_farthest_ws_bytes": (c_sz, [c_i64]),
    "mw_farthest": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp]),
    "mw_assign_ws_bytes": (c_sz, [c_i64, c_i32]),
    "mw_assign_conf": (c_i32, [c_vp, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "mw_assign_reduce": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp]),
    "mw_domain_sse_ws_bytes": (c_sz, [c_i64, c_i32, c_i32]),
    "mw_domain_sse_out_len": (c_i32, [c_i32, c_i32]),
    "mw_domain_sse": (c_i32, [c_vp, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_vp,
                              c_i64, c_vp, c_i32, c_vp, c_vp]),
    "mw_domain_sse_f64": (c_i32, [c_vp, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_vp,
                                  c_i64, c_vp, c_i32, c_vp, c_vp]),
    "mw_neighbor_mean": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_i32, c_vp, c_vp]),
    "mw_col_stats_rows": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp]),
    "mw_col_stats_absmax": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_i32, c_vp]),
    "mw_sample_slot_elems": (c_sz, [c_i64]),
    "mw_sample_map": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "mw_blur_sample": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_f32, c_vp, c_i32, c_vp, c_i64, c_vp, c_i32, c_vp, c_vp]),
    "mw_sample_overflow": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp]),
    "mw_blur_assign_conf": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_f32, c_vp, c_i32, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp]),
    "mw_domain_records": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp]),
    "mw_synth_slide": (c_i32, [c_i32, c_i32, c_i32, c_vp, c_i32, c_vp, c_i32, c_i32, c_i32, c_u64, c_vp, c_vp, c_vp]),
    "mw_synth_rows": (c_i32, [c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_i32, c_vp, c_i32, c_i32, c_i32, c_u64,
                              c_vp, c_vp, c_vp]),
    "mw_blur_sample_rows": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_i32, c_i64, c_i32, c_i32, c_vp, c_f32, c_vp,
                                    c_i32, c_vp, c_i64, c_vp, c_i32, c_vp, c_vp]),
    "mw_rank_index_bytes": (c_sz, [c_i64]),
    "mw_mask_rank_index": (c_i32, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "mw_gather_rows_ri": (c_i32, [c_vp, c_i32, c_vp, c_i32, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "mw_rank_to_pixel_ri": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_i64, c_vp]),
    "mw_gather_rows_px": (c_i32, [c_vp, c_i32, c_vp, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "mw_sample_map_ri": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "mw_sample_overflow_ri": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp]),
    "mw_slot_gather": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_vp, c_i64, c_vp, c_i32, c_vp, c_vp]),
    "mw_blur_assign_rows": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_i32, c_i64, c_i32, c_i32, c_vp, c_f32, c_vp,
                                    c_i32, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp]),
}

EXPORTED = tuple(_PROTOS)


class LloydFit(C.Structure):
    """``mw_lloyd_fit`` (include/milwrm_amd.h)."""
    _fields_ = [("centers", c_vp), ("drift", c_vp), ("half_sep", c_vp), ("labels", c_vp),
                ("ub", c_vp), ("lb", c_vp), ("ws", c_vp), ("out", c_vp), ("k", c_i32),
                ("drift_max", c_f32), ("inertia_exp", c_i32)]


# mw_fit_comm's collectives (include/milwrm_amd.h): all_reduce_sum(ctx, off, n,
# stream), all_gather(ctx, in_off, n, out_off, stream)
ALL_REDUCE_SUM_FN = C.CFUNCTYPE(c_i32, c_vp, c_i64, c_i64, c_vp)
ALL_GATHER_FN = C.CFUNCTYPE(c_i32, c_vp, c_i64, c_i64, c_i64, c_vp)


class FitComm(C.Structure):
    """``mw_fit_comm`` (include/milwrm_amd.h)."""
    _fields_ = [("ctx", c_vp), ("world", c_i32), ("rank", c_i32), ("rows_total", c_i64),
                ("row_offset", c_i64), ("d_msg", c_vp), ("msg_len", c_i64),
                ("all_reduce_sum", ALL_REDUCE_SUM_FN), ("all_gather", ALL_GATHER_FN)]


class NativeError(RuntimeError):
    pass


def load():
    """Load (once) and return the library; raises if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"milwrm_amd HIP library not found at {LIB_PATH}; build it with "
                "`python -m milwrm_amd.build` (hipcc --offload-arch=gfx950)")
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in _PROTOS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def last_error() -> str:
    return load().mw_last_error().decode(errors="replace")


def check(status: int, what: str):
    if status == 0:
        return
    msg = last_error()
    if status == _EINVAL:
        raise ValueError(f"{what}: {msg}")
    if status == _EUNSUP:
        raise NotImplementedError(f"{what}: {msg}")
    raise NativeError(f"{what}: {msg} (status {status})")


def call(name: str, *args):
    """Invoke ``name`` and raise on a non-zero status."""
    fn = getattr(load(), name)
    check(fn(*args), name)


def try_call(name: str, *args) -> bool:
    """Invoke ``name``; False when it reports MW_EUNSUPPORTED (nothing was
    launched: the caller takes its materialising path), raise on any other
    non-zero status."""
    st = getattr(load(), name)(*args)
    if st == _EUNSUP:
        return False
    check(st, name)
    return True


def query(name: str, *args) -> int:
    return int(getattr(load(), name)(*args))
