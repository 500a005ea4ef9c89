"""Tiny CPU emulator for the generated DPP asm blocks (one 16-lane row, fp64).

Executes the instruction strings of a dpp_blocks.inc asm statement with the
operand map of its C++ wrapper, so the hand-scheduled blocks (SweepQ, ElimQ)
can be checked against numpy on the CPU.  Supported: v_mov_b64,
v_fmac_f64_dpp (row_newbcast), v_fma_f64, v_mul_f64, v_min_f64, v_rcp_f64,
s_nop.  Hazards are not modelled (tools/check_dpp_hazards.py covers them).
"""
import re

import numpy as np

LANES = 16


def _val(tok, regs):
    neg = tok.startswith("-")
    t = tok[1:] if neg else tok
    if t.startswith("%"):
        v = regs[int(t[1:])].copy()
    else:
        v = np.full(LANES, float(t))
    return -v if neg else v


def run(asm_lines, regs, lds=None):
    """regs: dict operand index -> np.array(16) (modified in place).  lds: optional
    float64 array addressed in bytes / 8; ds_read_b64 %d, %a offset:o then reads
    lds[(a + o) / 8] per lane (without it, LDS reads are skipped: checked on the GPU)."""
    for line in asm_lines:
        line = line.split(" row_mask")[0].strip()
        if line.startswith("ds_read_b64") and lds is not None:
            m = re.match(r"ds_read_b64 %(\d+), %(\d+)(?: offset:(\d+))?", line)
            addr = regs[int(m.group(2))].astype(np.int64) + int(m.group(3) or 0)
            regs[int(m.group(1))] = lds[addr // 8].astype(float)
            continue
        if not line or line.startswith(("s_nop", "s_waitcnt", "ds_read", ".")):
            continue  # LDS reads riding in a block are checked on the GPU; directives
        op, rest = line.split(None, 1)
        if op.endswith("_e64"):  # the 8-byte VOP3 encoding of a VOP1 op (code placement)
            op = op[:-4]
        bc = None
        m = re.search(r"row_newbcast:(\d+)", rest)
        if m:
            bc = int(m.group(1))
            rest = rest[:m.start()].strip()
        args = [a.strip() for a in rest.split(",")]
        dst = int(args[0][1:])
        if op == "v_mov_b64":
            regs[dst] = _val(args[1], regs)
        elif op == "v_mov_b64_dpp":
            x = _val(args[1], regs)
            regs[dst] = np.full(LANES, x[bc]) if bc is not None else x
        elif op == "v_fmac_f64_dpp":
            x = _val(args[1], regs)
            if bc is not None:
                x = np.full(LANES, x[bc])
            regs[dst] = regs[dst] + x * _val(args[2], regs)
        elif op == "v_fma_f64":
            regs[dst] = _val(args[1], regs) * _val(args[2], regs) + _val(args[3], regs)
        elif op == "v_mul_f64":
            regs[dst] = _val(args[1], regs) * _val(args[2], regs)
        elif op == "v_min_f64":
            regs[dst] = np.fmin(_val(args[1], regs), _val(args[2], regs))
        elif op == "v_rcp_f64":
            regs[dst] = 1.0 / _val(args[1], regs)
        else:
            raise ValueError(f"unsupported: {line}")
    return regs


def extract(inc_text, struct, n):
    """Instruction strings of `struct<n>`'s asm statement in dpp_blocks.inc."""
    i = inc_text.index(f"template <> struct {struct}<{n}> {{")
    j = inc_text.index("    : ", i)
    body = inc_text[inc_text.index("asm volatile(", i):j]
    return [s.replace("\\n", "") for s in re.findall(r'^"(.*)"$', body, flags=re.M)]
