"""Per-section cycle breakdown of the small-s row-group kernel (lft_cond_kernel<SchedCondSmall>)
from a diagnostic build with HOP_SMALL_STAMP=1 (tools/exp_build.py stamp=-DHOP_SMALL_STAMP=1;
load it with HOP_LIB=...).  fp64 s = 5, m = 1, N = 200 synthetic blocks, B = 4,096.

    HOP_LIB=tools/exp/libhop_stamp.so python tools/stamps_small.py

Prints shader-clock cycles per wave per step for each section; the stamps themselves
perturb the schedule (each s_memtime is a scalar memory op): a breakdown, not a speed.
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
NAMES = ["top wait (DMA of step k)", "J store + diag offsets", "Q/QT image reads (sym)", "E/Xt sweeps",
         "A/B reads + symmetrisation + DMA issue", "update (CondLdl)", "predict products",
         "query (ElimQ)"]


def main():
    import torch
    from time_opt_ilqr_amd import _lib, engine, synth
    lib = _lib.load()
    lib.hop_debug_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    dev = torch.device("cuda", 0)
    Bn, N = 4096, 200
    blk = synth.device_batch(Bn, 5, 1, N, seed=6, device=dev)
    buf = (C.c_ulonglong * 16)()
    for _ in range(3):
        engine.propagate(*blk, t_min=40, t_max=N)
    torch.cuda.synchronize()
    lib.hop_debug_stamps(buf, 1)
    reps = 5
    for _ in range(reps):
        engine.propagate(*blk, t_min=40, t_max=N)
    torch.cuda.synchronize()
    lib.hop_debug_stamps(buf, 1)
    waves = buf[15]
    out = {"waves": int(waves), "per_wave_step": {}}
    tot = 0.0
    for j, nm in enumerate(NAMES):
        v = buf[j] / max(waves, 1) / N
        out["per_wave_step"][nm] = round(v, 1)
        tot += v
    out["total"] = round(tot, 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
