"""Build experimental variants of libhop_amd.so with extra -D flags for
same-box A/B runs (HOP_LIB=<path> selects one at run time).

    python tools/exp_build.py NAME=-DFOO=1 [NAME2=-DBAR=2 ...]

Writes tools/exp/libhop_<NAME>.so (git-ignored; travels with gpurun).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from time_opt_ilqr_amd import build
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "exp")
    os.makedirs(out, exist_ok=True)
    base_flags = list(build.FLAGS)
    for spec in sys.argv[1:]:
        name, _, flags = spec.partition("=")
        build.FLAGS = base_flags + flags.split()
        build.LIB = os.path.join(out, f"libhop_{name}.so")
        build.build(force=True, verbose=False)
        print("built", build.LIB)
    build.FLAGS = base_flags


if __name__ == "__main__":
    main()
