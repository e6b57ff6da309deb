"""Instruction classes of the MFMA basic blocks of one kernel in a hipcc -S listing (diagnostic).

usage: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --cuda-device-only -S knn.hip -o knn.s
       python tools/isa_count.py knn.s knn2_i8_kernel

Splits the kernel's body at its labels and, for every basic block holding MFMAs, counts MFMA, VALU (v_*
other than MFMA), SALU (s_* other than branches, waitcnt, nop, barrier), branches, waitcnt, s_nop, LDS
(ds_*), LDS-DMA / global, and the VGPR moves (v_mov / v_accvgpr) among the VALU: the hot loop's issue
mix per 8 MFMAs.
"""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_mov") or op.startswith("v_accvgpr"):
        return "valu_move"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("global_") or op.startswith("buffer_"):
        return "vmem"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "branch"
    if op == "s_waitcnt":
        return "waitcnt"
    if op == "s_nop":
        return "nop"
    if op == "s_barrier":
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, kname = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(rf"^_Z\S*{kname}\S*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur, name = [], [], "entry"
    for l in lines[start + 1:end]:
        if re.match(r"^\.LBB\S+:", l) or l.startswith("; %bb."):
            blocks.append((name, cur))
            name, cur = l.split(":")[0].split()[-1], []
            continue
        t = l.strip()
        if not t or t.startswith(";") or t.startswith("."):
            continue
        cur.append(t.split()[0])
    blocks.append((name, cur))
    print(f"{kname}: {len(blocks)} basic blocks; blocks with MFMAs (counts per block, and per 8 MFMAs):")
    for name, ops in blocks:
        c = Counter(classify(o) for o in ops)
        if c["mfma"] == 0:
            continue
        per = 8.0 / c["mfma"]
        keys = ["mfma", "valu", "valu_move", "salu", "branch", "lds", "vmem", "waitcnt", "nop", "barrier"]
        print(f"  {name:12s} " + "  ".join(f"{k} {c[k]}" for k in keys)
              + "   | per 8 MFMA: " + "  ".join(f"{k} {c[k] * per:.1f}" for k in keys[1:6]))


if __name__ == "__main__":
    main()
