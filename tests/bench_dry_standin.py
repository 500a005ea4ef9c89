"""CPU stand-in for one rank's shard in `bench.py --dry-run` (test infrastructure).

bench.py's rank / shard / gather / max-over-ranks path is rehearsed on gloo with
no GPU: each rank computes its contiguous shard [lo, hi) of small synthetic LFT
problems with the oracle (problem i uses seed DRY_SEED + i in every path), so a
test can compare the gathered (T*, J*) with a single-process oracle run.
Nothing in time_opt_ilqr_amd imports this file.
"""
import types

import torch

DRY_SEED, DRY_S, DRY_M, DRY_N, DRY_TMIN = 500, 4, 1, 12, 3


def select_for(index):
    """(T*, J*, J curve) of global problem `index` from the oracle."""
    from oracle import hop_oracle as orc
    A, B, Q, R, Ri, z0, QT = orc.synth_lft_problem(DRY_SEED + index, DRY_S, DRY_M, DRY_N)
    o = orc.lft_sweep(A, B, Q, Ri, z0, QT)
    t, j = orc.select_horizon(o["J"], DRY_TMIN, DRY_N)
    return int(t), float(j), o["J"]


def workload(args, world, lo, hi, dev):
    def launch():
        n = hi - lo
        t_star = torch.zeros(n, dtype=torch.int32)
        j_star = torch.zeros(n, dtype=torch.float64)
        J = torch.zeros((n, DRY_N), dtype=torch.float64)
        for i in range(n):
            t, j, curve = select_for(lo + i)
            t_star[i], j_star[i] = t, j
            J[i] = torch.as_tensor(curve)
        return types.SimpleNamespace(t_star=t_star, j_star=j_star, J=J,
                                     status=torch.zeros(n, dtype=torch.int32))

    info = dict(kernel="oracle stand-in (dry run)", bound="fp64", flops=0, bytes=0, executed=None,
                t_min=DRY_TMIN, t_max=DRY_N, s=DRY_S, m=DRY_M, N=DRY_N, host=None)
    return launch, info
