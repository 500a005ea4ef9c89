"""The config-5 s = 13 fp32-block bucket on the conditioned kernel with its predict on
the f32 matrix cores (developer variant 56, SchedCondMfma) and on the default DPP
predict (variant 0), one process, for a rocprofv3 --pmc pass that reports
SQ_VALU_MFMA_BUSY_CYCLES per dispatch (BASELINE north_star: "MFMA utilisation shown
in rocprof"):

    HOP_LIB=time_opt_ilqr_amd/libhop_amd_dev.so rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES \
        SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- python3 tools/mfma_pmc.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from time_opt_ilqr_amd import _lib, engine, synth
    dev = torch.device("cuda", 0)
    A, Bm, Q, Ri, z0, QT = synth.device_batch(5461, 13, 4, 128, seed=77, device=dev,
                                              dtype=torch.float32)
    for v in (56, 0, 56, 0):
        with _lib.options(variant=v):
            r = engine.propagate(A, Bm, Q, Ri, z0, QT, t_min=40, t_max=128)
        torch.cuda.synchronize()
        print(f"variant {v}: J[0, -1] = {float(r.J[0, -1]):.6e}", flush=True)


if __name__ == "__main__":
    main()
