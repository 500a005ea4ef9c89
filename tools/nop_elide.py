"""Drop the DPP hazard pads that the compiled code makes unnecessary.

The generated DPP blocks (dpp_blocks.inc) open with two wait states of padding,
"s_nop 0 ; hnop" twice, because the block cannot know how recently the compiler
wrote its first broadcast source; the generated sweeps pad their own internal
read-after-write distances the same way.  In the compiled device assembly the
distance is known.  This pass walks every function of a device `.s` file and
removes each consecutive PAIR of marked pads whose removal leaves no DPP source
read inside its hazard window (the rules of tools/check_dpp_hazards.py: two wait
states after a VALU write of the source, five after a VALU write of EXEC, a label
inside the window counts as a violation).  Pairs only: the blocks keep their
8-byte instructions at 0 mod 8 (an unpaired removal would shift them; the
alignment pads, unmarked, are never touched).  The build assembles the result and
runs the full hazard check on it.

    python tools/nop_elide.py in.s out.s
"""
import re
import sys

HNOP = re.compile(r"^\s*s_nop\s+0\s*;\s*hnop\s*$")
LOOKAHEAD = 12  # instructions after a removed pair whose DPP reads are re-checked


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
            out.append(None)
        else:
            out.append(("ins", s))
    return out


def elide(lines, chk):
    """Returns (new_lines, pairs_removed, pairs_kept)."""
    kinds = _classify(lines)
    n = len(lines)
    alive = [True] * n
    # instruction indices per function, in order
    seq = [i for i in range(n) if kinds[i] is not None]

    def hazard_at(pos_list, k):
        """Is the DPP instruction at pos_list[k] inside a hazard window, looking back
        over the live entries of pos_list?"""
        kind, text = kinds[pos_list[k]]
        if kind != "ins":
            return False
        src = chk.dpp_source(text)
        if src is None:
            return False
        ws = 0
        j = k - 1
        seen = 0
        while j >= 0 and seen < 16:
            i = pos_list[j]
            j -= 1
            if not alive[i]:
                continue
            kk, t = kinds[i]
            seen += 1
            if kk == "func":
                return False
            if kk == "label":
                return ws < 2
            written, wexec = chk.vgpr_writes(t)
            if written & src and ws < 2:
                return True
            if wexec and ws < 5:
                return True
            ws += chk.wait_states(t)
            if ws >= 5:
                return False
        return False

    removed = kept = 0
    k = 0
    while k + 1 < len(seq):
        a, b = seq[k], seq[k + 1]
        if HNOP.match(lines[a]) and HNOP.match(lines[b]) and alive[a] and alive[b]:
            alive[a] = alive[b] = False
            # re-check the DPP reads that follow (their windows may have shrunk)
            bad = False
            m, seen = k + 2, 0
            while m < len(seq) and seen < LOOKAHEAD:
                if alive[seq[m]]:
                    seen += 1
                    if kinds[seq[m]][0] == "func":
                        break
                    if hazard_at(seq, m):
                        bad = True
                        break
                m += 1
            if bad:
                alive[a] = alive[b] = True
                kept += 1
            else:
                removed += 1
            k += 2
            continue
        k += 1
    return [l for i, l in enumerate(lines) if alive[i]], removed, kept


def main(argv):
    import os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import check_dpp_hazards as chk
    src, dst = argv[1], argv[2]
    lines = open(src).read().split("\n")
    out, removed, kept = elide(lines, chk)
    open(dst, "w").write("\n".join(out))
    print(f"{os.path.basename(src)}: {removed} hazard-pad pairs dropped, {kept} kept")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
