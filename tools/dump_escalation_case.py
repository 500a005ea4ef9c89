"""Dump the escalated config-2 problem of tests/test_gpu_rerun.py (inputs, the product's
J, the reference-association kernel's J, status) for a 50-digit check on the host.

    python tools/dump_escalation_case.py <out.npz> [target]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    import torch
    from oracle import hop_oracle as orc
    from time_opt_ilqr_amd import _lib, engine, synth
    dev = torch.device("cuda", 0)
    target = float(sys.argv[2]) if len(sys.argv) > 2 else 5e-7
    Bn, s, m, N, b, k = 4096, 13, 4, 100, 1234, 37
    A, Bm, Q, Ri, z0, QT = synth.device_batch(Bn, s, m, N, seed=21, device=dev)
    q = Q[b, k].cpu().numpy()
    lo = np.linalg.eigvalsh(orc.sym(q)).min()
    Q[b, k] = torch.as_tensor(q - np.eye(s) * (lo + target), device=dev)
    res = engine.propagate(A, Bm, Q, Ri, z0, QT, t_min=40, t_max=N)
    with _lib.options(reference_assoc=True):
        ref = engine.propagate(A, Bm, Q, Ri, z0, QT, t_min=40, t_max=N)
    torch.cuda.synchronize()
    h = lambda x: x[b].cpu().numpy()  # noqa: E731
    np.savez(sys.argv[1], A=h(A), B=h(Bm), Q=h(Q), Ri=h(Ri), z0=z0.cpu().numpy(), QT=h(QT),
             J=h(res.J), J_ref=h(ref.J), status=h(res.status), status_ref=h(ref.status), k=k)
    print("saved", int(res.status[b]), int(ref.status[b]))


if __name__ == "__main__":
    main()
