"""Static check of the gfx950 DPP read-after-VALU-write hazard in generated device assembly.

gfx9 needs two wait states between a VALU instruction that writes a VGPR and a
DPP instruction that reads that VGPR as its (broadcast) source, and five after
a VALU write of EXEC.  hipcc pads only the instructions it generated itself,
not those inside inline asm, so the engine's DPP blocks rely on their own
placement.  This script walks every instruction of a device `.s` file and
fails if any DPP source could have been written inside the hazard window:

    python tools/check_dpp_hazards.py file.s [file.s ...]

It also flags a v_fmac_f64_dpp whose multiplier operand shares VGPRs with its
accumulator: the signature of LLVM coalescing an asm input with a value-equal
"+v" output (the generated blocks use "+&v" to prevent it).

Wait states: each instruction counts 1, `s_nop N` counts N + 1.  A label
inside the window (another control path may enter there) counts as a
violation unless two wait states follow it (the compiler writes EXEC only
with SALU instructions, so the 5-state VALU-EXEC case cannot cross a label).
"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(op):
    out = set()
    for m in REG.finditer(op):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def parse(path):
    """Yield (kind, text) with kind in {'label', 'ins', 'func'}."""
    for raw in open(path):
        line = raw.split(";")[0].rstrip()
        if not line.strip():
            continue
        s = line.strip()
        if s.endswith(":") and not s.startswith("."):
            yield ("func" if not s.startswith(".L") else "label"), s[:-1]
        elif s.startswith(".LBB") and s.endswith(":"):
            yield "label", s[:-1]
        elif s.startswith("."):
            continue
        else:
            yield "ins", s


def vgpr_writes(ins):
    op = ins.split()[0]
    if not op.startswith("v_"):
        return set(), False
    if op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")) or op.startswith("v_cmpx"):
        return set(), op.startswith("v_cmpx")
    args = ins[len(op):].split(",")
    if not args:
        return set(), False
    dst = args[0].strip()
    if dst == "exec":
        return set(), True
    if op.startswith(("v_permlane16_swap", "v_permlane32_swap", "v_swap_b")) and len(args) > 1:
        return regs(dst) | regs(args[1].strip()), False  # both operands are written
    return regs(dst), False


def dpp_source(ins):
    if "row_newbcast" not in ins and "_dpp" not in ins.split()[0]:
        return None
    args = [a.strip() for a in ins[len(ins.split()[0]):].split(",")]
    return regs(args[1]) if len(args) > 1 else None


def wait_states(ins):
    op = ins.split()[0]
    if op == "s_nop":
        return int(ins.split()[1], 0) + 1
    return 1


def check(path, verbose=False):
    bad = []
    hist = []  # (wait_states_of_this_entry, written_vgprs, writes_exec, is_label, text)
    func = "?"
    n_dpp = 0
    for kind, text in parse(path):
        if kind == "func":
            func = text
            hist = []
            continue
        if kind == "label":
            hist.append((0, set(), False, True, text))
            continue
        src = dpp_source(text)
        if src is not None and text.startswith("v_fmac_f64_dpp"):
            # the multiplier operand never legitimately shares the accumulator's VGPRs:
            # that is an input operand coalesced with a value-equal "+v" output
            args = [a.strip() for a in text[len("v_fmac_f64_dpp"):].split(" row_")[0].split(",")]
            if len(args) >= 3 and regs(args[0]) & regs(args[2].lstrip("-")):
                bad.append((func, text, "src1 aliases the accumulator (asm operand coalescing)"))
        if src is not None:
            n_dpp += 1
            ws = 0
            for w, written, wexec, is_label, t in reversed(hist):
                if is_label:
                    if ws < 2:
                        bad.append((func, text, f"label {t} within {ws} wait states"))
                    break
                if written & src and ws < 2:
                    bad.append((func, text, f"source written by '{t}' {ws} wait states before"))
                    break
                if wexec and ws < 5:
                    bad.append((func, text, f"EXEC written by '{t}' {ws} wait states before"))
                    break
                ws += w
                if ws >= 5:
                    break
        written, wexec = vgpr_writes(text)
        hist.append((wait_states(text), written, wexec, False, text))
        if len(hist) > 16:
            hist = hist[-16:]
    return n_dpp, bad


def main(argv):
    rc = 0
    for p in argv:
        n, bad = check(p)
        print(f"{p}: {n} DPP instructions, {len(bad)} hazards")
        for f, t, why in bad[:20]:
            print(f"  {f}: {t}  <- {why}")
        rc |= bool(bad)
    return rc


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
