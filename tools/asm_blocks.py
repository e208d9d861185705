#!/usr/bin/env python3
"""Per-basic-block instruction mix of a gfx950 .s file (measurement tool).
usage: asm_blocks.py file.s [min_ds_reads]"""
import re
import sys
from collections import Counter

path = sys.argv[1]
thr = int(sys.argv[2]) if len(sys.argv) > 2 else 8
blocks, cur, name = [], [], "entry"
for line in open(path):
    t = line.strip()
    if re.match(r"^\.LBB\d+_\d+:", t) or t.startswith("_Z") and t.endswith(":"):
        blocks.append((name, cur))
        name, cur = t.split(":")[0] + " " + (t.split(";")[1].strip() if ";" in t else ""), []
        continue
    if not t or t.startswith((".", ";")):
        continue
    cur.append(t.split()[0])
blocks.append((name, cur))
for name, ins in blocks:
    c = Counter()
    for op in ins:
        if op.startswith("ds_read") or op.startswith("ds_load"):
            c["ds_read"] += 1
        elif op.startswith("ds_"):
            c["ds_other"] += 1
        elif op.startswith(("global_load", "buffer_load")):
            c["vmem_ld"] += 1
        elif op.startswith(("global_store", "buffer_store")):
            c["vmem_st"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("s_waitcnt"):
            c["waitcnt"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    if c["ds_read"] >= thr:
        print(f"{name[:60]:60s} n={len(ins):4d} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
