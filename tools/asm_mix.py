#!/usr/bin/env python3
"""Instruction mix of kernels in a gfx950 .s file (hipcc -S --cuda-device-only):
counts per class for the whole kernel and for its largest basic-block loop.

    python tools/asm_mix.py kernel.s NAME_SUBSTRING [...]
"""
import collections
import re
import sys


def classify(op):
    if op.startswith("v_pk_"):
        return "valu_pk"
    if op.startswith(("v_cndmask", "v_cmp")):
        return "valu_sel"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_load", "global_load")):
        return "vmem_ld"
    if op.startswith(("buffer_store", "global_store")):
        return "vmem_st"
    return "other"


def main():
    text = open(sys.argv[1]).read()
    parts = re.split(r"\n(_Z\S+):[^\n]*\n", text)
    for name, body in zip(parts[1::2], parts[2::2]):
        if not any(k in name for k in sys.argv[2:]):
            continue
        body = body.split(".Lfunc_end")[0]
        blocks, cur, label = {}, [], "entry"
        for line in body.splitlines():
            t = line.strip()
            if re.match(r"^\.LBB\S+:", t):
                blocks[label] = cur
                label, cur = t.split(":")[0], []
                continue
            tok = t.split()
            if not tok or tok[0].startswith((".", ";")):
                continue
            cur.append(tok[0])
        blocks[label] = cur
        tot = collections.Counter(classify(o) for b in blocks.values() for o in b)
        big = max(blocks, key=lambda k: len(blocks[k]))
        loop = collections.Counter(classify(o) for o in blocks[big])
        print(name[:70])
        print("  kernel:", dict(sorted(tot.items())))
        print("  largest block %s (%d instrs):" % (big, len(blocks[big])), dict(sorted(loop.items())))


if __name__ == "__main__":
    main()
