"""Drop the hazard pads that the compiled code makes unnecessary.

The generated DPP blocks (dpp_blocks.inc) open with two wait states of padding,
"s_nop 0 ; hnop" twice, because the block cannot know how recently the compiler
wrote its first broadcast source; the generated sweeps pad their own internal
read-after-write distances the same way.  The LDS-DMA statements open with
"s_nop 2 ; vmnop" (HOP_VMNOP, hop_device.hpp) for the VALU-SGPR-write -> VMEM window.
In the compiled device assembly the distances are known.  This pass walks every
function of a device `.s` file and removes

  * each consecutive PAIR of "hnop" pads (no directive or label between them in the
    raw lines: a `.p2align` between two pads would make the pair's removal shift the
    instructions after the directive off their 8-byte alignment), and
  * each single "vmnop" pad (it sits before its statement's `.p2align`, so the
    alignment of the statement does not depend on it),

whose removal leaves every modelled hazard window intact: every rule of
tools/check_dpp_hazards.py (DPP source and EXEC, transcendental forwarding,
VALU SGPR -> VMEM, lane select, VCC -> v_div_fmas, readlane, permlane, M0 -> LDS-DMA),
checked on the instructions that follow the pad, and on those after the target of
any branch within five wait states of it (a pad whose removal could shorten a window
on a path the re-check cannot follow is kept).  Pairs only for
"hnop": the blocks keep their 8-byte instructions at 0 mod 8 (an unpaired removal
would shift them; the alignment pads, unmarked, are never touched).  The build
assembles the result and runs the full hazard check on it.

    python tools/nop_elide.py in.s out.s
"""
import re
import sys

HNOP = re.compile(r"^\s*s_nop\s+0\s*;\s*hnop\s*$")
VMNOP = re.compile(r"^\s*s_nop\s+\d+\s*;\s*vmnop\s*$")
LOOKAHEAD = 12  # instructions after a removed pad whose hazard windows are re-checked
BRANCH_WINDOW = 5  # wait states after a pad within which a branch target is re-checked too


def _classify(lines):
    """Per line: ('ins', text) | ('label', name) | ('func', name) | None (directive,
    comment or blank)."""
    out = []
    for raw in lines:
        line = raw.split(";")[0].rstrip()
        s = line.strip()
        if not s:
            out.append(None)
        elif s.endswith(":") and not s.startswith("."):
            out.append(("func", s[:-1]))
        elif s.startswith(".LBB") and s.endswith(":"):
            out.append(("label", s[:-1]))
        elif s.startswith("."):
            out.append(("dir", s))
        else:
            out.append(("ins", s))
    return out


def elide(lines, chk):
    """Returns (new_lines, pads_removed, pads_kept); a removed / kept "hnop" pair counts
    once, as does a single "vmnop" pad."""
    kinds = _classify(lines)
    n = len(lines)
    alive = [k is not None and k[0] != "dir" for k in kinds]
    entries = [k if k is not None else ("dir", "") for k in kinds]
    cfg = chk.Cfg(entries)
    is_alive = alive.__getitem__

    def next_live(i):
        j = i + 1
        while j < n and not alive[j]:
            j += 1
        return j

    def window_ok(j, depth):
        """No hazard window violated in the LOOKAHEAD live instructions from entry j on,
        nor (depth permitting) after the target of a branch met within BRANCH_WINDOW
        wait states."""
        seen, ws = 0, 0
        while j < n and seen < LOOKAHEAD:
            kind, t = entries[j]
            if kind == "func":
                break
            if kind == "ins":
                seen += 1
                if cfg.violations(j, is_alive):
                    return False
                m = chk.BRANCH.match(t)
                if m and ws < BRANCH_WINDOW:
                    tgt = cfg.label_at.get(m.group(2))
                    if tgt is None or depth == 0 or not window_ok(tgt + 1, depth - 1):
                        return False
                    if t.startswith("s_branch"):
                        break  # no fall-through
                ws += chk.wait_states(t)
            j = next_live(j)
        return True

    def safe_without(pads):
        """With `pads` removed, no hazard window is violated in the instructions that
        follow them (window_ok)."""
        for p in pads:
            alive[p] = False
        ok = window_ok(next_live(max(pads)), 2)
        if not ok:
            for p in pads:
                alive[p] = True
        return ok

    removed = kept = 0
    i = 0
    while i < n:
        if alive[i] and VMNOP.match(lines[i]):
            if safe_without([i]):
                removed += 1
            else:
                kept += 1
            i += 1
            continue
        if alive[i] and HNOP.match(lines[i]):
            # its partner: the next line that is not blank / a pure comment
            j = i + 1
            while j < n and kinds[j] is None:
                j += 1
            if j < n and alive[j] and HNOP.match(lines[j]):
                if safe_without([i, j]):
                    removed += 1
                else:
                    kept += 1
                i = j + 1
                continue
        i += 1
    return [l for i, l in enumerate(lines) if alive[i] or kinds[i] is None or kinds[i][0] == "dir"], \
        removed, kept


def main(argv):
    import os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import check_dpp_hazards as chk
    src, dst = argv[1], argv[2]
    lines = open(src).read().split("\n")
    out, removed, kept = elide(lines, chk)
    open(dst, "w").write("\n".join(out))
    print(f"{os.path.basename(src)}: {removed} hazard pads dropped, {kept} kept")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
