"""Per-step comparison of Riccati outputs (test infrastructure).

The north star's parity claim is per gain: K_k / k_k / V_k to 1e-6 relative.  A
whole-array max-norm (max |got - ref| / max |ref|) lets a step whose gains are
small next to the largest step be badly wrong and still pass, so the Riccati tests
compare every step on its own:

    rel_k = ||got_k - ref_k||_F / ||ref_k||_F

and report the worst k.  A step whose reference is exactly zero is compared
absolutely (rel_k = ||got_k||_F); none of the fixtures has one.
"""
from __future__ import annotations

import numpy as np


def per_step_rel(got, ref):
    """max over steps k (axis 0) of ||got_k - ref_k|| / ||ref_k|| (Frobenius over the
    remaining axes), and that k."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    if got.shape != ref.shape:
        raise ValueError(f"shape {got.shape} != reference {ref.shape}")
    if ref.ndim == 1:
        got, ref = got[:, None], ref[:, None]
    d = np.sqrt(np.sum((got - ref) ** 2, axis=tuple(range(1, ref.ndim))))
    r = np.sqrt(np.sum(ref ** 2, axis=tuple(range(1, ref.ndim))))
    rel = np.where(r > 0, d / np.where(r > 0, r, 1.0), d)
    if not np.all(np.isfinite(rel)):
        return float("inf"), int(np.nonzero(~np.isfinite(rel))[0][0])
    k = int(np.argmax(rel))
    return float(rel[k]), k


def assert_per_step(got, ref, tol, what):
    rel, k = per_step_rel(got, ref)
    assert rel <= tol, f"{what}: step {k} relative error {rel:.3e} > {tol:.0e}"
    return rel
