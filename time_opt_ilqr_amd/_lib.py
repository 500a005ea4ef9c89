"""ctypes binding of libhop_amd.so (include/hop.h).

The shared library is plain HIP (no torch types cross the boundary): callers
hand over device pointers (``tensor.data_ptr()``) and the raw HIP stream
(``torch.cuda.current_stream().cuda_stream``).  There is deliberately no CPU
fallback: without the built library or a GPU every entry point raises.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HOP_LIB", os.path.join(HERE, "libhop_amd.so"))

ST_JITTER = 1
ST_LU = 2
ST_NONFINITE = 4
ST_FAIL = 8
MAX_DIM = 16

_P = C.c_void_p
_I32 = C.c_int32
_I64 = C.c_int64
_U32 = C.c_uint32

# (name, restype, argtypes) -- must match include/hop.h exactly
_LFT = [_P, _P, _P, _P, _I64, _I64, _I32, _P, _P, _I64, _I64, _I32, _I32, _I32, _I32, _I32,
        _I32, _I32, _P, _P, _P, _P, _P, _P, _P]
# tile64 sweep: A B Q R r_bs r_inv QT z0 z_bs batch n_alloc n_use s m tries t_min t_max J st ts js stream
_LFT_T64 = [_P, _P, _P, _P, _I64, _I32, _P, _P, _I64, _I64, _I32, _I32, _I32, _I32, _I32, _I32,
            _I32, _P, _P, _P, _P, _P]
_SEL = [_P, _I64, _I32, _I32, _I32, _P, _P, _P]
_RIC64 = [_P, _P, _P, _P, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _P, _P, _P, _P,
          C.c_double, _U32, _I32, _I32, _I64, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _P]
_RIC32 = list(_RIC64)
_RIC32[19] = C.c_float
# J-curve form: the 17 Riccati inputs, lm w wrap batch n_alloc n m t_max J status stream
_JC64 = _RIC64[:17] + [C.c_double, C.c_double, _U32, _I64, _I32, _I32, _I32, _I32, _P, _P, _P]
_JC32 = _RIC64[:17] + [C.c_float, C.c_float, _U32, _I64, _I32, _I32, _I32, _I32, _P, _P, _P]
# the legacy twin's passes: A Bm X U, (xg u_ref Q R Qf) with batch strides, then
# horizon lm w wrap mode batch n_alloc n m K k Vxx Vx V0 status stream / the J-curve tail
_LEG_IN = [_P, _P, _P, _P] + [_P, _I64] * 5
_RICLEG = _LEG_IN + [_P, _P, C.c_double, _U32, _I32, _I64, _I32, _I32, _I32, _P, _P, _P, _P, _P,
                     _P, _P]
_JCLEG = _LEG_IN + [C.c_double, C.c_double, _U32, _I64, _I32, _I32, _I32, _I32, _P, _P, _P]
# trajectory-form inputs shared by hop_augment_* and hop_lft_sweep_traj_*:
# A Bm a_res X U xg xg_bs u_ref ur_bs Q q_bs P p_bs w w_bs qxx qx c wrap q_reg rho_reg
_TRJ64 = [_P, _P, _P, _P, _P, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _P, _P, _U32,
          C.c_double, C.c_double]
_TRJ32 = _TRJ64[:19] + [C.c_float, C.c_float]
_AUG_TAIL = [_I64, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P]
_TRAJ_TAIL = [_P, _I64, _I64, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _I64,
              _P]
# tile64 trajectory select tail: R_inv r_bs batch n_alloc n_use n m tries t_min t_max J st ts js stream
_T64TAIL = [_P, _I64, _I64, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P]
# tile64 linearisation: system dt X U batch n_alloc n_use central epsx epsu relx relu A B a Xt Ut stream
_LIN64 = [_I32, C.c_double, _P, _P, _I64, _I32, _I32, _I32, C.c_double, C.c_double, C.c_double,
          C.c_double, _P, _P, _P, _P, _P, _P]
# cost parameters of the forward-pass entries: xg bs u_ref bs Q bs R bs Qf bs w bs obs n_obs wrap
_COST = [_P, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _I32, _U32]

SIGNATURES = {
    "hop_abi_version": (C.c_int, []),
    "hop_last_error": (C.c_char_p, []),
    "hop_set_options": (C.c_int, [_U32, _I32]),
    "hop_get_options": (C.c_int, [_P, _P]),
    "hop_build_flags": (C.c_int, []),
    "hop_cu_fallbacks": (C.c_int, []),
    "hop_lft_sweep_f64": (C.c_int, _LFT),
    "hop_lft_sweep_f32": (C.c_int, _LFT),
    "hop_lft_sweep_tile64_f64": (C.c_int, _LFT_T64),
    "hop_lft_sweep_tile64_f32": (C.c_int, _LFT_T64),
    "hop_tile64_elems": (C.c_int64, [_I64, _I32, _I32]),
    "hop_tile64_f64": (C.c_int, [_P, _P, _I64, _I32, _I32, _I32, _P]),
    "hop_tile64_f32": (C.c_int, [_P, _P, _I64, _I32, _I32, _I32, _P]),
    "hop_select_horizon_f64": (C.c_int, _SEL),
    "hop_select_horizon_f32": (C.c_int, _SEL),
    "hop_augment_f64": (C.c_int, _TRJ64 + _AUG_TAIL),
    "hop_augment_f32": (C.c_int, _TRJ32 + _AUG_TAIL),
    "hop_lft_sweep_traj_workspace_bytes": (C.c_int64, [_I64, _I32, _I32, _I32, _I32, _I32]),
    "hop_lft_sweep_traj_f64": (C.c_int, _TRJ64 + _TRAJ_TAIL),
    "hop_lft_sweep_traj_f32": (C.c_int, _TRJ32 + _TRAJ_TAIL),
    "hop_riccati_f64": (C.c_int, _RIC64),
    "hop_riccati_f32": (C.c_int, _RIC32),
    "hop_bruteforce_jcurve_f64": (C.c_int, _JC64),
    "hop_bruteforce_jcurve_f32": (C.c_int, _JC32),
    "hop_riccati_legacy_f64": (C.c_int, _RICLEG),
    "hop_bruteforce_jcurve_legacy_f64": (C.c_int, _JCLEG),
    "hop_lft_sweep_traj_tile64_f64": (C.c_int, _TRJ64[:15] + [_U32, C.c_double, C.c_double] +
                                      _T64TAIL),
    "hop_lft_sweep_traj_tile64_f32": (C.c_int, _TRJ64[:15] + [_U32, C.c_float, C.c_float] +
                                      _T64TAIL),
    "hop_linearize_tile64_f64": (C.c_int, _LIN64),
    "hop_linearize_tile64_f32": (C.c_int, _LIN64),
    "hop_system_dims": (C.c_int, [_I32, _P, _P]),
    "hop_linearize_f64": (C.c_int, [_I32, C.c_double, _P, _P, _I64, _I32, _I32, _I32,
                                    C.c_double, C.c_double, C.c_double, C.c_double, _P, _P, _P,
                                    _P, _P]),
    "hop_dynamics_f64": (C.c_int, [_I32, C.c_double, _P, _I64, _P, _I64, _I64, _P, _I64, _P]),
    "hop_rollout_f64": (C.c_int, [_I32, C.c_double, _P, _I64, _P, _I64, _I32, C.c_double, _P,
                                  _P]),
    "hop_cost_true_f64": (C.c_int, [_I32, _P, _P, _P] + _COST + [_I64, _I32, _P, _P]),
    "hop_forward_workspace_bytes": (C.c_size_t, [_I32, _I64, _I32, _I32]),
    "hop_forward_linesearch_f64": (C.c_int, [_I32, C.c_double, _P, _P] + _COST +
                                   [_P, _P, _P, _P, _P, _I32, _I64, _I32, _P, C.c_size_t, _P, _P,
                                    _P, _P, _P, _P]),
    "hop_obstacle_cost_f64": (C.c_int, [_P, _I64, _I64, _I32, _P, _I32, _P, _P, _P, _P]),
    "hop_ilqr_accept_f64": (C.c_int, [_I64, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _I32, _P,
                                      _P]),
    "hop_ilqr_select_mask": (C.c_int, [_I64, _P, _P, _P, _P, _P, _P]),
}

_lock = threading.Lock()
_lib = None


class HopError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load (once) and return the ctypes handle; raises if the .so is missing."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise HopError(f"{p} not built: run `python -m time_opt_ilqr_amd.build` "
                           "(the HIP engine has no CPU fallback)")
        # torch's HIP runtime must be the process's one: the library resolves
        # libamdhip64.so.7 against what is already loaded, and loaded first it would
        # pull in /opt/rocm's copy beside torch's bundled one -- two runtimes, and
        # the library's launches then see no device (measured: HIP error 100)
        import torch  # noqa: F401
        lib = C.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            if path is not None and not hasattr(lib, name):
                continue  # an older build loaded for an A/B (tools/ab_libs.py)
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.hop_abi_version() != 1:
            raise HopError("libhop_amd.so ABI mismatch")
        if path is None:
            _lib = lib
        return lib


# test / diagnostic controls (include/hop.h HOP_OPT_*); never needed by a caller
OPT_FORCE_GENERIC = 1
OPT_FORCE_HANDOVER = 2
OPT_REFERENCE_ASSOC = 4
OPT_TRAJ_UNFUSED = 8
OPT_STAMPS = 16
OPT_NO_RERUN = 32
OPT_SMALL_LANE = 64
OPT_RERUN_LANE = 128
ST_HANDOVER = 16  # status bit left by the conditioned kernels under OPT_NO_RERUN
# the hand-over word (include/hop.h): ST_HANDOVER | first flagged horizon << HANDOVER_SHIFT
HANDOVER_SHIFT = 13


def handover_horizon(status):
    """The first flagged horizon of hand-over words (HOP_HANDOVER_HORIZON); works on
    ints and integer arrays."""
    return status >> HANDOVER_SHIFT


def dev_build() -> bool:
    """True when libhop_amd.so is a developer build (A/B schedules, stamps)."""
    return bool(load().hop_build_flags() & 1)


@contextlib.contextmanager
def options(*, force_generic=None, force_handover=None, reference_assoc=None,
            traj_unfused=None, stamps=None, no_rerun=None, small_lane=None,
            rerun_lane=None, variant=None):
    """Set hop_set_options for the duration of a `with` block (tests, tools).
    Arguments left at None keep the enclosing block's setting; the previous
    controls are restored afterwards.  The library keeps them per host thread
    and reads them at launch, so the block affects only this thread's calls."""
    lib = load()
    f0, v0 = C.c_uint32(), C.c_int32()
    check(lib.hop_get_options(C.byref(f0), C.byref(v0)))
    prev = (f0.value, v0.value)
    flags, var = prev
    for on, bit in ((force_generic, OPT_FORCE_GENERIC), (force_handover, OPT_FORCE_HANDOVER),
                    (reference_assoc, OPT_REFERENCE_ASSOC), (traj_unfused, OPT_TRAJ_UNFUSED),
                    (stamps, OPT_STAMPS), (no_rerun, OPT_NO_RERUN), (small_lane, OPT_SMALL_LANE),
                    (rerun_lane, OPT_RERUN_LANE)):
        if on is not None:
            flags = (flags | bit) if on else (flags & ~bit)
    if variant is not None:
        var = int(variant)
    check(lib.hop_set_options(flags, var))
    try:
        yield
    finally:
        lib.hop_set_options(*prev)


def get_options() -> tuple:
    """(flags, variant) of the calling host thread."""
    f, v = C.c_uint32(), C.c_int32()
    check(load().hop_get_options(C.byref(f), C.byref(v)))
    return f.value, v.value


def check(rc: int):
    if rc != 0:
        msg = load().hop_last_error()
        raise HopError(f"hop call failed ({rc}): {msg.decode() if msg else ''}")


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    return None if t is None else C.c_void_p(t.data_ptr())


def stream_handle(device=None):
    import torch
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)
