"""MI355X-native batched LFT / Riccati horizon-selection engine.

Drop-in for the hot path of dmmsjtu-umich/time-opt-ilqr:

  engine.propagate / engine.select_horizon / engine.riccati   batched device API
  engine.propagate_traj / engine.augment                       trajectory form (augmented.py
                                                               builders on the device)
  engine.linearize / engine.dynamics                           batched FD linearisation and
                                                               dynamics of the benchmark systems
  systems.make_* / linearization.*                             reference-shaped drop-ins
  horizon_selection.propagator_all_Jt_aug, ...                 reference-shaped drop-ins

All arithmetic runs in libhop_amd.so (hand-written gfx950 HIP, C ABI in
include/hop.h).  There is no CPU fallback: without the library or a GPU the
calls raise.
"""
from . import _lib
from ._lib import HopError, ST_FAIL, ST_JITTER, ST_LU, ST_NONFINITE
from . import linearization, systems
from .engine import (augment, dynamics, linearize, propagate, propagate_traj, riccati,
                     select_horizon)
from .horizon_selection import (backward_pass_truncated, bruteforce_all_Jt_backward_expansion,
                                propagator_all_Jt_aug, select_from_trajectory,
                                value_expansions_and_gains_prefix)

__all__ = [
    "propagate", "select_horizon", "riccati", "propagate_traj", "augment", "linearize",
    "dynamics", "systems", "linearization",
    "propagator_all_Jt_aug", "backward_pass_truncated", "value_expansions_and_gains_prefix",
    "bruteforce_all_Jt_backward_expansion", "select_from_trajectory",
    "HopError", "ST_JITTER", "ST_LU", "ST_NONFINITE", "ST_FAIL",
]


def library():
    """Load libhop_amd.so (raises HopError if it has not been built)."""
    return _lib.load()
