"""VGPR / AGPR / scratch / LDS of the kernels in a device assembly file (build
-save-temps output), filtered by a name substring:

    python tools/kernel_regs.py time_opt_ilqr_amd/_obj/lft_sweep_v2-hip-amdgcn-amd-amdhsa-gfx950.s cond
"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", s, re.S):
    name, body = m.group(1), m.group(2)
    if pat not in name:
        continue
    g = lambda k: re.search(rf"\.amdhsa_{k} (\d+)", body).group(1)  # noqa: E731
    print(f"scratch {g('private_segment_fixed_size'):>5} vgpr {g('next_free_vgpr'):>4} "
          f"accum_offset {g('accum_offset'):>4} sgpr {g('next_free_sgpr'):>4} {name[:120]}")
