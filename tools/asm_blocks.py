#!/usr/bin/env python3
"""Basic blocks of one kernel in a gfx950 .s file: instruction counts per
class for blocks with a barrier or more than N instructions.

    python tools/asm_blocks.py kernel.s MANGLED_PREFIX [N]
"""
import collections
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    pre = sys.argv[2]
    nmin = int(sys.argv[3]) if len(sys.argv) > 3 else 120
    m = re.search(r"^(" + re.escape(pre) + r"[^:\s]*):", s, re.M)
    i = m.start()
    j = s.index(".Lfunc_end", i)
    blocks, cur = [], ["entry", []]
    blocks.append(cur)
    for line in s[i:j].splitlines()[1:]:
        mm = re.match(r"^(\.LBB\S+):", line)
        if mm:
            cur = [mm.group(1), []]
            blocks.append(cur)
            continue
        t = line.strip()
        if not t or t.startswith((";", ".")):
            continue
        cur[1].append(t.split()[0])
    for name, ins in blocks:
        c = collections.Counter()
        for op in ins:
            if op.startswith("s_waitcnt"):
                k = "wait"
            elif op.startswith("v_readlane") or op.startswith("v_writelane"):
                k = "lane"
            elif op.startswith("v_"):
                k = "valu"
            elif op.startswith("s_"):
                k = "salu"
            elif op.startswith("ds_"):
                k = "lds"
            elif op.startswith(("buffer", "global", "scratch")):
                k = "vmem"
            else:
                k = "other"
            c[k] += 1
        if "s_barrier" in ins or len(ins) > nmin:
            print(name, len(ins), dict(c), "BARRIER" if "s_barrier" in ins else "", ins[-1])


if __name__ == "__main__":
    main()
