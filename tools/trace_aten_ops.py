"""The aten ops (device kernels other than the library's) issued by one step of a bench
workload: TorchDispatchMode logging around one launch() after a warm-up.  The kernel
trace of select_gains shows two fill kernels and a copy kernel per step besides the
library's launches (tools/launch_gaps.py); this names their call sites.

    python tools/trace_aten_ops.py [--workload select_gains]
"""
import argparse
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="select_gains")
    a = ap.parse_args()
    import torch
    from torch.utils._python_dispatch import TorchDispatchMode
    import bench
    dev = torch.device("cuda", 0)
    args = argparse.Namespace(s=13, m=4, N=100, dtype="f64", t_min=40, layout="auto",
                              no_alt=True, rho_reg=1e-12)
    launch, _ = bench.WORKLOADS[a.workload](args, 1, 0, 4096, dev)
    launch()
    torch.cuda.synchronize()

    class Log(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = str(func)
            if not any(s in name for s in ("empty", "view", "expand", "reshape", "_to_copy.default@noop",
                                              "detach", "alias", "is_same_size")):
                st = [f for f in traceback.extract_stack() if "time_opt_ilqr_amd" in f.filename
                      or "bench.py" in f.filename]
                where = "; ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in st[-3:])
                print(f"{name}  <- {where}", flush=True)
            return func(*args, **(kwargs or {}))

    with Log():
        launch()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
