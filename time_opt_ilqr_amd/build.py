"""Build libhop_amd.so (gfx950) in-tree with hipcc; no torch extension machinery.

    python -m time_opt_ilqr_amd.build        # or __graft_entry__.build()

The .so is git-ignored but travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
REPO = os.path.dirname(HERE)
LIB = os.path.join(HERE, "libhop_amd.so")
SOURCES = ["capi.hip", "augment.hip", "lft_sweep.hip", "lft_sweep_v2.hip", "lft_small.hip",
           "riccati.hip", "riccati_fast.hip", "linearize.hip", "forward.hip"]
# developer builds (HOP_DEV_BUILD=1 or --dev): the A/B schedules and stamped
# instantiations, selected at run time by hop_set_options' variant number;
# product builds compile none of them
DEV = os.environ.get("HOP_DEV_BUILD", "0") not in ("", "0") or "--dev" in sys.argv
DEV_SOURCES = []
if DEV:  # a separate library (load it with HOP_LIB=<path>): the product .so stays product
    LIB = os.path.join(HERE, "libhop_amd_dev.so")
EXTRA = {}
HEADERS = ["hop_device.hpp", "hop_kernels.hpp", "dpp_blocks.inc", "small_math.hpp", "wrap.hpp", "dynamics.hpp"]
ARCH = os.environ.get("HOP_OFFLOAD_ARCH", "gfx950")
# device code from its assembly, minus the DPP hazard pads the compiled code does not
# need (tools/nop_elide.py); HOP_NO_ELIDE=1 compiles the plain way (hipcc -c)
LLVM_BIN = os.environ.get("HOP_LLVM_BIN", "/opt/rocm/lib/llvm/bin")
ELIDE = (os.environ.get("HOP_NO_ELIDE", "0") in ("", "0")
         and os.path.exists(os.path.join(REPO, "tools", "nop_elide.py"))
         and all(os.path.exists(os.path.join(LLVM_BIN, t))
                 for t in ("clang", "lld", "clang-offload-bundler")))
FLAGS = ["-O3", "-std=c++20", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-variable", "-Wno-pass-failed",
         "-Wno-unused-but-set-variable"] + (["-DHOP_DEV=1"] if DEV else [])


def _sources():
    return SOURCES + (DEV_SOURCES if DEV else [])


def _hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.sep not in cand or os.path.exists(cand)):
            return cand
    raise RuntimeError("hipcc not found")


def _digest():
    h = hashlib.sha256()
    for name in SOURCES + DEV_SOURCES + HEADERS:
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(f.read())
    with open(os.path.join(REPO, "include", "hop.h"), "rb") as f:
        h.update(f.read())
    if ELIDE:  # the device code is what tools/nop_elide.py leaves of the compiler's
        for t in ("nop_elide.py", "check_dpp_hazards.py"):  # the pads it drops follow the checker's rules
            with open(os.path.join(REPO, "tools", t), "rb") as f:
                h.update(f.read())
    h.update(b"elide" if ELIDE else b"plain")
    h.update(" ".join(FLAGS).encode())
    h.update(repr(sorted(EXTRA.items())).encode())
    return h.hexdigest()


def _stamp_path():
    return LIB + ".sha256"


def up_to_date():
    if not os.path.exists(LIB) or not os.path.exists(_stamp_path()):
        return False
    with open(_stamp_path()) as f:
        return f.read().strip() == _digest()


def check_hazards(objdir, verbose=True):
    """Fail the build if any inline-asm DPP source can be read inside its VALU
    write hazard window, or any other modelled gfx950 hazard is met
    (tools/check_dpp_hazards.py; hipcc does not pad asm).  Returns the number of
    hazards only listed (developer builds under HOP_HAZARD_REPORT); build() writes no
    up-to-date stamp for such a library, so nothing reuses it as a checked build."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import check_dpp_hazards as chk
    # developer A/B builds only: list, don't fail (product builds always fail)
    report = os.environ.get("HOP_HAZARD_REPORT") if DEV else None
    listed = 0
    for src in _sources():
        s = os.path.join(objdir, src.replace(".hip", "") + f"-hip-amdgcn-amd-amdhsa-{ARCH}.s")
        n, bad = chk.check(s)
        if verbose:
            print(f"[hop] {os.path.basename(s)}: {n} DPP instructions, {len(bad)} hazards")
        if bad and report:
            listed += len(bad)
            with open(report, "a") as f:
                for fn, text, why in bad:
                    f.write(f"{src}\t{fn}\t{text}\t{why}\n")
        elif bad:
            raise RuntimeError(f"hazard in {src}: {bad[:3]}")
    return listed


def _run_all(cmds, verbose):
    procs = []
    for cmd in cmds:
        if verbose:
            print("[hop]", " ".join(cmd))
        procs.append(subprocess.Popen(cmd))
    for cmd, p in zip(cmds, procs):
        if p.wait() != 0:
            raise RuntimeError(f"build step failed: {' '.join(cmd[:3])} ...")


def _compile_elided(hipcc, objdir, objs, verbose):
    """Each source: the device assembly (hipcc --cuda-device-only -S), the hazard pads
    it does not need dropped (tools/nop_elide.py), the hazard check on the result,
    assembled and linked into the code object, bundled, and the host side compiled
    around that fat binary (-fcuda-include-gpubinary: hipcc's own -c does the same
    steps with the assembly unchanged)."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import check_dpp_hazards as chk
    import nop_elide
    base = {src: os.path.join(objdir, src.replace(".hip", "")) for src in _sources()}
    _run_all([[hipcc, *FLAGS, *EXTRA.get(src, []), "--cuda-device-only", "-S",
               os.path.join(CSRC, src), "-o", base[src] + "-device-raw.s"]
              for src in _sources()], verbose)
    for src in _sources():
        b = base[src]
        checked = b + f"-hip-amdgcn-amd-amdhsa-{ARCH}.s"  # the name check_hazards reads
        with open(b + "-device-raw.s") as f:
            lines = f.read().split("\n")
        out, dropped, kept = nop_elide.elide(lines, chk)
        with open(checked, "w") as f:
            f.write("\n".join(out))
        if verbose:
            print(f"[hop] {src}: {dropped} hazard-pad pairs dropped, {kept} kept")
    listed = check_hazards(objdir, verbose)
    for src in _sources():
        b = base[src]
        checked = b + f"-hip-amdgcn-amd-amdhsa-{ARCH}.s"
        for cmd in ([os.path.join(LLVM_BIN, "clang"), "-x", "assembler", "--target=amdgcn-amd-amdhsa",
                     f"-mcpu={ARCH}", "-c", checked, "-o", b + "-device.o"],
                    [os.path.join(LLVM_BIN, "lld"), "-flavor", "gnu", "-m", "elf64_amdgpu",
                     "--no-undefined", "-shared", "-o", b + "-device.out", b + "-device.o"],
                    [os.path.join(LLVM_BIN, "clang-offload-bundler"), "-type=o", "-bundle-align=4096",
                     f"-targets=host-x86_64-unknown-linux-gnu,hipv4-amdgcn-amd-amdhsa--{ARCH}",
                     "-input=/dev/null", "-input=" + b + "-device.out", "-output=" + b + ".hipfb"]):
            subprocess.check_call(cmd)
    _run_all([[hipcc, *FLAGS, *EXTRA.get(src, []), "--cuda-host-only", "-Xclang",
               "-fcuda-include-gpubinary", "-Xclang", base[src] + ".hipfb", "-c",
               os.path.join(CSRC, src), "-o", obj]
              for src, obj in zip(_sources(), objs)], verbose)
    return listed


def build(force=False, jobs=None, verbose=True):
    """Compile every .hip source for gfx950 and link libhop_amd.so."""
    gen = os.path.join(REPO, "tools", "gen_dpp.py")
    inc = os.path.join(CSRC, "dpp_blocks.inc")
    if not os.path.exists(inc) and os.path.exists(gen):
        subprocess.check_call([sys.executable, gen])
    if not force and up_to_date():
        if verbose:
            print("[hop] libhop_amd.so up to date")
        return LIB
    # the digest of the sources as compiled: taken before compiling, so a source edited
    # while the build runs leaves a stale stamp (the next build recompiles) instead of
    # a stamp that claims the edit is in the library
    digest = _digest()
    hipcc = _hipcc()
    objdir = os.path.join(HERE, "_obj_dev" if DEV else "_obj")
    os.makedirs(objdir, exist_ok=True)
    objs = [os.path.join(objdir, src.replace(".hip", ".o")) for src in _sources()]
    if ELIDE:
        listed = _compile_elided(hipcc, objdir, objs, verbose)
    else:
        procs = []
        for src, obj in zip(_sources(), objs):
            # -save-temps=obj keeps the device assembly for the DPP hazard check
            cmd = [hipcc, *FLAGS, *EXTRA.get(src, []), "-save-temps=obj", "-c",
                   os.path.join(CSRC, src), "-o", obj]
            if verbose:
                print("[hop]", " ".join(cmd))
            procs.append(subprocess.Popen(cmd))
        for p in procs:
            if p.wait() != 0:
                raise RuntimeError("hipcc failed")
        listed = check_hazards(objdir, verbose)
    tmp = LIB + ".tmp"
    cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp]
    if verbose:
        print("[hop]", " ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    if listed:  # hazards listed, not failed: no stamp (up_to_date() stays False)
        if os.path.exists(_stamp_path()):
            os.remove(_stamp_path())
        print(f"[hop] {listed} hazards listed in $HOP_HAZARD_REPORT: no build stamp written")
        return LIB
    with open(_stamp_path(), "w") as f:
        f.write(digest)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
