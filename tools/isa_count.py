"""Static instruction mix of a kernel's main loop from the build's device assembly.

    python tools/isa_count.py <asm.s> <kernel-symbol-substring> [--steps 2]

Finds the kernel's function body, takes its largest depth-1 loop (header to the
back-edge branch), drops nested (depth-2) loops, and prints the per-step counts
(the loop body divided by --steps, the unroll factor of the step loop) by opcode,
plus the VGPR / AGPR counts the assembler reports.
"""
import argparse
import collections
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--whole", action="store_true", help="count the whole function body")
    args = ap.parse_args()
    lines = open(args.asm).read().split("\n")
    start = next(i for i, l in enumerate(lines)
                 if re.match(r"^[A-Za-z_]\w*:", l) and args.kernel in l.split(":")[0])
    name = lines[start].split(":")[0]
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end")
               and i > start)
    body = lines[start:end]
    # depth-1 loop headers and their back edges (the last branch to the header)
    best = None
    for i, l in enumerate(body):
        if "Loop Header: Depth=1" in l:
            lab = l.split(":")[0].strip()
            last = max((j for j, x in enumerate(body) if re.search(r"s_(c)?branch\w*\s+" +
                                                                   re.escape(lab) + r"$", x.strip())),
                       default=None)
            if last is not None and (best is None or last - i > best[1] - best[0]):
                best = (i, last)
    if args.whole or (best is not None and best[1] < best[0]):
        best = (0, len(body) - 1)
    if best is None:
        raise SystemExit("no loop found")
    loop = body[best[0]:best[1] + 1]
    # drop nested loops: from a depth-2 header to its back edge
    keep, i = [], 0
    while i < len(loop):
        l = loop[i]
        if "Loop Header: Depth=2" in l:
            lab = l.split(":")[0].strip()
            if not lab.startswith("."):
                lab = loop[i - 1].split(":")[0].strip()
            j = max((k for k in range(i, len(loop)) if re.search(re.escape(lab) + r"$", loop[k].strip())
                     and "branch" in loop[k]), default=i)
            i = j + 1
            continue
        keep.append(l)
        i += 1
    cnt = collections.Counter()
    for l in keep:
        s = l.strip()
        if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
            continue
        op = s.split()[0]
        cnt[op] += 1
    valu = sum(v for k, v in cnt.items() if k.startswith("v_"))
    print(f"{name}: loop lines {best[0]}..{best[1]}, per step (/{args.steps}):")
    print(f"  VALU {valu / args.steps:.0f}  DPP FMA {cnt['v_fmac_f64_dpp'] / args.steps:.0f}  "
          f"s_nop {cnt['s_nop'] / args.steps:.0f}")
    for k, v in cnt.most_common(args.top):
        print(f"  {k:28s} {v / args.steps:7.1f}")
    txt = "\n".join(lines)
    for key in ("num_vgpr", "num_agpr"):
        m = re.search(re.escape(name) + r"\." + key + r", (\d+)", txt)
        if m:
            print(f"  {key} {m.group(1)}")


if __name__ == "__main__":
    main()
