"""Where the pipelined rerun's beats go: per wave, the clocks spent working and the
clocks spent waiting at the beat barrier (developer build with -DHOP_PIPE_STAMP,
e.g. `python tools/exp_build.py pstamp=-DHOP_PIPE_STAMP`), on tools/bench_rerun.py's
escalated config-2 batch (one problem rerun).  s_memtime clocks summed over the
workgroups that ran the pipeline.

    python tools/pipe_stamps.py tools/exp/libhop_pstamp.so [more.so ...]
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ROLE = ["Gbar chain", "Ebar/Fbar chain", "stage blocks", "queries"]


def main():
    import numpy as np
    import torch
    from time_opt_ilqr_amd import _lib, engine, synth
    dev = torch.device("cuda", 0)
    Bn, s, m, N, b, k = 4096, 13, 4, 100, 1234, 37
    A, Bm, Q, Ri, z0, QT = synth.device_batch(Bn, s, m, N, seed=21, device=dev)
    q = Q[b, k].cpu().numpy()
    lo = np.linalg.eigvalsh(0.5 * (q + q.T)).min()
    Q[b, k] = torch.as_tensor(q - np.eye(s) * (lo + 5e-9), device=dev)
    for path in sys.argv[1:]:
        lib = _lib.load(path)
        _lib._lib = lib
        lib.hop_debug_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
        buf = (C.c_ulonglong * 16)()
        engine.propagate(A, Bm, Q, Ri, z0, QT, t_min=40, t_max=N)
        torch.cuda.synchronize()
        lib.hop_debug_stamps(buf, 1)
        engine.propagate(A, Bm, Q, Ri, z0, QT, t_min=40, t_max=N)
        torch.cuda.synchronize()
        lib.hop_debug_stamps(buf, 1)
        nw = max(buf[15], 1)
        out = {"lib": os.path.basename(path), "waves": int(buf[15])}
        for w in range(4):
            out[ROLE[w]] = {"busy": round(buf[w] * 4 / nw), "wait": round(buf[4 + w] * 4 / nw)}
        out["Gbar step sections"] = {nm: round(buf[8 + j] * 4 / nw) for j, nm in enumerate(
            ["ring reads + E+Gbar into the tiles", "inverse", "products + exchange"])}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
