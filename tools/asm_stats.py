#!/usr/bin/env python3
"""Instruction statistics of one kernel in a hipcc device assembly dump (hipcc --cuda-device-only -S).

  tools/asm_stats.py evam_pp.s SYMBOL_SUBSTRING

Prints the kernel's resource metadata lines and, for every basic block that ends in a backward branch
(a loop latch) plus the blocks it spans, the instruction count by class (VALU, SALU, LDS, VMEM, waitcnt).
"""
import re
import sys


def classify(op):
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("ds_", "buffer_load_lds", "global_load_lds")):
        return "lds" if op.startswith("ds_") else "vmem"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main(path, sym):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(sym), l))
    name = lines[start].split(":")[0]
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.size") or lines[i].startswith(".Lfunc_end"))
    body = lines[start + 1:end]
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB[^:\s]+):", l)
        if m:
            labels[m.group(1)] = i
    total = {}
    for l in body:
        t = l.strip()
        if not t or t.startswith((";", ".")) or re.match(r"^\S+:", t):
            continue
        c = classify(t.split()[0])
        total[c] = total.get(c, 0) + 1
    print(name)
    print("  whole kernel:", total)
    for i, l in enumerate(body):
        t = l.strip()
        m = re.match(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", t)
        if not m:
            continue
        tgt = m.group(1) or m.group(2)
        j = labels.get(tgt)
        if j is None or j > i:
            continue
        cnt = {}
        for k in range(j, i + 1):
            u = body[k].strip()
            if not u or u.startswith((";", ".")) or re.match(r"^\S+:", u):
                continue
            c = classify(u.split()[0])
            cnt[c] = cnt.get(c, 0) + 1
        print(f"  loop {tgt} .. line {i}: {cnt}")
    meta = [l for l in lines[end:end + 400] if re.search(r"\.(sgpr_count|vgpr_count|group_segment_fixed_size|agpr_count):", l)]
    print("  " + " ".join(x.strip() for x in meta[:4]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
