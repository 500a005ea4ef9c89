"""Which handed-over problems of tests/test_gpu_rerun.py's several-per-workgroup case
differ between the pipelined rerun and the reference-association kernel, and where."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    import torch
    from oracle import hop_oracle as orc
    from time_opt_ilqr_amd import _lib, engine
    dev = torch.device("cuda", 0)
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float64, device=dev)  # noqa: E731

    def esc_(Q, b, k, target=5e-7):
        Q = Q.copy()
        lo = np.linalg.eigvalsh(orc.sym(Q[b, k])).min()
        Q[b, k] = Q[b, k] - np.eye(Q.shape[-1]) * (lo + target)
        return Q
    Bn, s, m, N = 96, 13, 4, 30
    A, Bm, Q, R, Ri, z0, QT = orc.synth_lft_batch(4700, Bn, s, m, N)
    for variant in ("all", "one_per_wg", "k_nonzero"):
        Qv = Q.copy()
        esc = [0, 16, 17, 32, 33, 34, 35, 48, 49, 50, 51, 52, 64, 65]
        if variant == "one_per_wg":
            esc = [0, 16, 32, 48, 64]
        for b in esc:
            k = (3 * b) % N
            if variant == "k_nonzero" and k == 0:
                k = 1
            Qv = esc_(Qv, b, k)
        args = [t(x) for x in (A, Bm, Qv, Ri, z0, QT)]
        kw = dict(t_min=5, t_max=N)
        res = engine.propagate(*args, **kw)
        with _lib.options(reference_assoc=True):
            ref = engine.propagate(*args, **kw)
        with _lib.options(no_rerun=True):
            ho = engine.propagate(*args, **kw).status.cpu().numpy()
        torch.cuda.synchronize()
        J, Jr = res.J.cpu().numpy(), ref.J.cpu().numpy()
        st, sr = res.status.cpu().numpy(), ref.status.cpu().numpy()
        print("==", variant, "handed over:", np.nonzero(ho & _lib.ST_HANDOVER)[0].tolist(), flush=True)
        for b in range(Bn):
            d = np.abs(J[b] - Jr[b])
            if not np.array_equal(J[b], Jr[b]) or st[b] != sr[b]:
                bad = np.nonzero(J[b] != Jr[b])[0]
                print(f"b={b} st={st[b]} ref_st={sr[b]} first_diff_t={bad[0] + 1 if len(bad) else None} "
                      f"n_diff={len(bad)} max_abs={np.nanmax(d):.3e} rel={np.nanmax(d / np.abs(Jr[b])):.3e}",
                      flush=True)


if __name__ == "__main__":
    main()
