#!/usr/bin/env python3
"""Instruction counts per marked section of a kernel's assembly (FS_MARKS diagnostic builds;
measurement tool). usage: asm_sections.py file.s kernel-substring"""
import re
import sys
from collections import Counter, defaultdict

s = open(sys.argv[1]).read()
sub = sys.argv[2]
m = [x for x in re.finditer(r"^(_Z\S+):\s*(;.*)?$", s, re.M) if sub in x.group(1)][0]
body = s[m.end(): s.find(".Lfunc_end", m.end())]
sec = "prologue"
cnt = defaultdict(Counter)
inst = defaultdict(Counter)  # per instance: (name, ordinal)
seen = Counter()
cur = ("prologue", 0)
for line in body.splitlines():
    t = line.strip()
    mm = re.match(r";\s*@@(\w+)", t)
    if mm:
        sec = mm.group(1)
        seen[sec] += 1
        cur = (sec, seen[sec])
        continue
    if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
        continue
    op = t.split()[0]
    kind = "valu" if op.startswith("v_") else "salu" if op.startswith("s_") and not op.startswith("s_waitcnt") else \
        "lds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_", "flat_", "scratch_")) else "other"
    cnt[sec][kind] += 1
    inst[cur][kind] += 1
for k, c in cnt.items():
    print(f"{k:16s} valu {c['valu']:5d} salu {c['salu']:5d} lds {c['lds']:4d} vmem {c['vmem']:3d}")
if len(sys.argv) > 3:  # per-instance listing of the named sections
    for (k, i), c in inst.items():
        if k in sys.argv[3].split(","):
            print(f"  {k}#{i:<3d} valu {c['valu']:5d} salu {c['salu']:5d} lds {c['lds']:4d} vmem {c['vmem']:3d}")
