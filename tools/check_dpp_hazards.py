"""Static check of gfx950's software-managed hazards in generated device assembly.

hipcc pads only the instruction pairs it generated itself: inside an inline-asm
statement nothing is padded, and across the statement's boundary only a fixed
one-state pad is added (cdna_hip_programming.md §5.7 item 2).  The engine's DPP
blocks and LDS-DMA statements therefore rely on their own placement, and the build
drops the pads the compiled code makes unnecessary (tools/nop_elide.py).  This
script walks every instruction of a device `.s` file and fails if any consumer
below can read a register inside its producer's window:

    python tools/check_dpp_hazards.py file.s [file.s ...]

Rules (wait states the consumer needs after the producer; the gfx9/CDNA "required
software-inserted wait states" table of the ISA reference, which LLVM's
GCNHazardRecognizer implements for the compiler's own pairs; the guide rows cited are
those of /opt/skills/guides/cdna_hip_programming.md that restate them):

  dpp     VALU writes VGPR     -> DPP op reads it (src0)                      2
  dppexec VALU writes EXEC     -> DPP op                                      5
  trans   transcendental VALU (v_rcp/rsq/sqrt/exp/log/sin/cos) writes VGPR
                               -> a non-transcendental VALU reads it          1
          (gfx940+ trans forwarding; GCNHazardRecognizer TransDefWaitstates)
  vmemsgpr VALU writes SGPR (v_readfirstlane, v_readlane, v_cmp, carry-out)
                               -> VMEM (buffer/global/flat/scratch) reads it  5
          (guide §5.7 item 2: "an 's' operand fresh from readfirstlane -> a
          buffer_*/global_* reading it as descriptor, soffset or base: s_nop 4")
  rwlane  VALU writes SGPR     -> v_readlane/v_writelane lane select          4
  divfmas VALU writes VCC      -> v_div_fmas                                  4
  readlane VALU writes VGPR    -> v_readfirstlane/v_readlane reads it (src0)  1
          (guide §5.7 item 2: "a VGPR write -> v_readfirstlane (s_nop 0)")
  permlane VALU writes VGPR    -> v_permlane16/32_swap reads it               2
          (guide T21: "VALU write vdst -> v_permlane read")
  m0lds   SALU writes M0       -> LDS-DMA (buffer_/global_load ... lds)       1
          (guide §5.7 operands: "the s_nop 0 is ... row 16")

Wait states: each instruction counts 1, `s_nop N` counts N + 1.  The walk follows
control flow backwards: at a label it continues on every `s_branch`/`s_cbranch_*`
that targets the label and on the fall-through path (unless the instruction before
the label is an unconditional jump).  The two DPP rules keep the original, stricter
label rule: a label inside their window is a violation unless two wait states follow
it (the hand-written blocks never need one there).

It also flags a v_fmac_f64_dpp whose multiplier operand shares VGPRs with its
accumulator: the signature of LLVM coalescing an asm input with a value-equal
"+v" output (the generated blocks use "+&v" to prevent it).
"""
import functools
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b|\b(vcc|vcc_lo|vcc_hi|m0|exec|exec_lo|exec_hi)\b")
SPECIAL = {"vcc": (106, 107), "vcc_lo": (106,), "vcc_hi": (107,), "m0": (124,),
           "exec": (126, 127), "exec_lo": (126,), "exec_hi": (127,)}
VCC = {106, 107}
M0 = 124
TRANS = ("v_rcp_", "v_rsq_", "v_sqrt_", "v_exp_", "v_log_", "v_sin_", "v_cos_", "v_rcp_iflag")
VMEM = ("buffer_", "global_", "flat_", "scratch_", "tbuffer_")
# VOP3b: the second operand is an SGPR (carry / VCC) destination
VOP3B = ("v_add_co_", "v_addc_co_", "v_sub_co_", "v_subb_co_", "v_subrev_co_", "v_subbrev_co_",
         "v_div_scale_", "v_mad_u64_u32", "v_mad_i64_i32")
JUMPS = ("s_branch", "s_endpgm", "s_setpc_b64", "s_trap")
BRANCH = re.compile(r"^s_(c?branch)\w*\s+(\.L\w+)")


def regs(op):
    out = set()
    for m in REG.finditer(op):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def sregs(op):
    out = set()
    for m in SREG.finditer(op):
        if m.group(4) is not None:
            out.update(SPECIAL[m.group(4)])
        elif m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def _opargs(ins):
    op = ins.split()[0]
    return op, [a.strip() for a in ins[len(op):].split(",")] if ins[len(op):].strip() else []


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


@functools.lru_cache(maxsize=1 << 16)
def salu_writes_m0(ins):
    op, args = _opargs(ins)
    return op.startswith("s_") and bool(args) and M0 in sregs(args[0])


@functools.lru_cache(maxsize=1 << 16)
def vgpr_writes(ins):
    """(VGPRs written, writes EXEC) of a VALU instruction."""
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


@functools.lru_cache(maxsize=1 << 16)
def sgpr_writes(ins):
    """SGPRs (VCC as 106/107, EXEC as 126/127) written by a VALU instruction."""
    op, args = _opargs(ins)
    if not op.startswith("v_") or not args:
        return set()
    out = set()
    if op.startswith(("v_readfirstlane", "v_readlane", "v_cmp")):
        out |= sregs(args[0])
    if op.startswith(VOP3B) and len(args) > 1:
        out |= sregs(args[1])
    elif "_e32" in op and op.startswith(("v_add_co", "v_sub_co", "v_subrev_co", "v_addc_co",
                                        "v_subb_co", "v_subbrev_co")):
        out |= VCC
    return out


def vgpr_reads(ins):
    """VGPRs a VALU instruction reads (sources; the accumulator of fmac / mac too)."""
    op, args = _opargs(ins)
    if not op.startswith("v_") or not args:
        return set()
    src = ",".join(args[1:]).split(" row_")[0]
    out = regs(src)
    if "fmac" in op or "_mac_" in op or op.startswith(("v_permlane16_swap", "v_permlane32_swap",
                                                      "v_swap_b", "v_writelane")):
        out |= regs(args[0])
    return out


def is_trans(ins):
    return ins.split()[0].startswith(TRANS)


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


class Need:
    """A consumer's requirement: no producer matching `pred` within `ws` wait states."""
    __slots__ = ("ws", "pred", "why", "strict_label")

    def __init__(self, ws, pred, why, strict_label=False):
        self.ws, self.pred, self.why, self.strict_label = ws, pred, why, strict_label


@functools.lru_cache(maxsize=1 << 16)
def needs_of(ins):
    """The hazard windows instruction `ins` opens backwards (see the module docstring)."""
    op, args = _opargs(ins)
    out = []
    src = dpp_source(ins)
    if src is not None:
        out.append(Need(2, lambda t, s=src: bool(vgpr_writes(t)[0] & s), "dpp: source written",
                        True))
        out.append(Need(5, lambda t: vgpr_writes(t)[1], "dppexec: EXEC written", True))
    if op.startswith("v_") and not op.startswith(TRANS):
        rd = vgpr_reads(ins)
        if rd:
            out.append(Need(1, lambda t, r=rd: is_trans(t) and bool(vgpr_writes(t)[0] & r),
                            "trans: transcendental result read"))
    if op.startswith(VMEM):
        sr = sregs(",".join(args)) - {M0}
        if sr:
            out.append(Need(5, lambda t, r=sr: bool(sgpr_writes(t) & r),
                            "vmemsgpr: SGPR written by VALU"))
        if re.search(r"\blds\b", ins) or op.startswith("global_load_lds"):
            out.append(Need(1, salu_writes_m0, "m0lds: M0 written"))
    if op.startswith(("v_readlane", "v_writelane")) and len(args) > 2:
        sel = sregs(args[2])
        if sel:
            out.append(Need(4, lambda t, r=sel: bool(sgpr_writes(t) & r),
                            "rwlane: lane select written by VALU"))
    if op.startswith("v_div_fmas"):
        out.append(Need(4, lambda t: bool(sgpr_writes(t) & VCC), "divfmas: VCC written by VALU"))
    if op.startswith(("v_readfirstlane", "v_readlane")) and len(args) > 1:
        s0 = regs(args[1])
        out.append(Need(1, lambda t, r=s0: bool(vgpr_writes(t)[0] & r),
                        "readlane: source VGPR written"))
    if op.startswith(("v_permlane16_swap", "v_permlane32_swap")):
        both = regs(",".join(args[:2]))
        out.append(Need(2, lambda t, r=both: bool(vgpr_writes(t)[0] & r),
                        "permlane: operand written"))
    return out


class Cfg:
    """A function's entries (kind, text) with label / branch maps for the backward walk.
    `alive(i)` lets the elider hide entries it tentatively removed."""

    def __init__(self, entries):
        self.e = entries
        self.label_at = {}
        self.branches_to = {}
        for i, (k, t) in enumerate(entries):
            if k == "label":
                self.label_at[t] = i
            elif k == "ins":
                m = BRANCH.match(t)
                if m:
                    self.branches_to.setdefault(m.group(2), []).append(i)

    def violations(self, k, alive=lambda i: True, needs=None):
        kind, text = self.e[k]
        if kind != "ins":
            return []
        needs = needs_of(text) if needs is None else needs
        if not needs:
            return []
        bad = []
        seen = set()
        # (index to examine, wait states so far, came via a label, needs still active)
        stack = [(k - 1, 0, False, tuple(needs))]
        while stack:
            j, ws, via_label, act = stack.pop()
            while j >= 0 and act and ws < max(n.ws for n in act):
                if not alive(j):
                    j -= 1
                    continue
                if (j, ws, len(act)) in seen:
                    break
                seen.add((j, ws, len(act)))
                kind, t = self.e[j]
                if kind == "func":
                    break
                if kind == "label":
                    # the DPP rules' label rule: two wait states after any label, and no
                    # further (the compiler writes EXEC only with SALU instructions, so
                    # the 5-state VALU-EXEC window cannot cross a label)
                    for n in act:
                        if n.strict_label and ws < 2:
                            bad.append((n.why, f"label {t} within {ws} wait states"))
                    act = tuple(n for n in act if not n.strict_label)
                    for b in self.branches_to.get(t, ()):
                        stack.append((b, ws, False, act))
                    via_label = True
                    j -= 1
                    continue
                if via_label and t.split()[0] in JUMPS:
                    break  # no fall-through into the label
                via_label = False
                for n in act:
                    if ws < n.ws and n.pred(t):
                        bad.append((n.why, f"'{t}' {ws} wait states before"))
                ws += wait_states(t)
                j -= 1
        return bad


def functions(entries):
    """Split (kind, text) entries into per-function lists."""
    cur = []
    for kind, text in entries:
        if kind == "func":
            if cur:
                yield cur
            cur = [(kind, text)]
        else:
            cur.append((kind, text))
    if cur:
        yield cur


def check(path, verbose=False):
    """(DPP instruction count, [(function, instruction, why)]) of a device .s file."""
    bad = []
    n_dpp = 0
    for fn in functions(list(parse(path))):
        cfg = Cfg(fn)
        name = fn[0][1] if fn[0][0] == "func" else "?"
        for k, (kind, text) in enumerate(fn):
            if kind != "ins":
                continue
            src = dpp_source(text)
            if src is not None:
                n_dpp += 1
                if text.startswith("v_fmac_f64_dpp"):
                    # the multiplier never legitimately shares the accumulator's VGPRs: an
                    # input operand coalesced with a value-equal "+v" output
                    args = [a.strip() for a in text[len("v_fmac_f64_dpp"):].split(" row_")[0].split(",")]
                    if len(args) >= 3 and regs(args[0]) & regs(args[2].lstrip("-")):
                        bad.append((name, text, "src1 aliases the accumulator (asm operand coalescing)"))
            for why, where in cfg.violations(k):
                bad.append((name, text, f"{why}: {where}"))
    bad += split_load_violations(path)
    return n_dpp, bad


LDISSUE, LDWAIT = "hop_ldissue", "hop_ldwait"


def split_load_violations(path):
    """The split asm loads (an asm statement of ds_read_* marked hop_ldissue, its
    s_waitcnt in a later statement marked hop_ldwait): every instruction textually
    between the two must leave the loads' destination VGPRs alone (the compiler
    believes them written at the first statement's end, so a copy, spill or reuse of
    one would read or clobber a register whose data has not landed).  Textual order
    covers every path from the issue to the wait when the wait follows the issue in
    the layout; a function that ends, or issues again, before its wait is reported."""
    bad = []
    func, pending, dst = "?", None, set()
    in_blk, blk_dst, blk_issue = False, set(), False
    for raw in open(path):
        code = raw.split(";")[0].strip()
        if code.endswith(":") and not code.startswith("."):
            if pending is not None:
                bad.append((func, pending, "split load: no hop_ldwait before the function ends"))
            func, pending, dst = code[:-1], None, set()
            continue
        if ";;#ASMSTART" in raw:
            in_blk, blk_dst, blk_issue = True, set(), False
            continue
        if ";;#ASMEND" in raw:
            if blk_issue:
                if pending is not None:
                    bad.append((func, pending, "split load: issued again before its hop_ldwait"))
                pending, dst = "the hop_ldissue reads", blk_dst
            in_blk = False
            continue
        if LDWAIT in raw:
            pending, dst = None, set()
            continue
        if not code or code.startswith("."):
            continue
        if in_blk and code.startswith("ds_read"):
            blk_dst |= regs(code.split(",")[0])
        if LDISSUE in raw:
            blk_issue = True
            continue
        if pending is not None and not (in_blk and code.startswith("ds_read") and blk_issue):
            if regs(code) & dst:
                bad.append((func, code, f"split load: touches a destination of {pending} "
                            "before their hop_ldwait"))
    return bad


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
