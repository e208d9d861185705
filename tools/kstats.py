#!/usr/bin/env python3
"""Per-kernel register / spill / call / full-drain counts of a gfx950 .s file (measurement tool).
usage: kstats.py file.s [name-substring]"""
import re
import sys

s = open(sys.argv[1]).read()
sub = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"^(_Z\S+):\s*(;.*)?$", s, re.M):
    name = m.group(1)
    if sub not in name or "Lfunc" in name:
        continue
    end = s.find(".Lfunc_end", m.end())
    body = s[m.end():end]
    tail = s[end:end + 1500]
    def meta(k):
        mm = re.search(r"; " + k + r": (\S+)", tail)
        return mm.group(1) if mm else "?"
    nv0 = len(re.findall(r"vmcnt\(0\)", body))
    print(f"{name[:60]:60s} vgpr {meta('NumVgprs'):>4} sgpr {meta('NumSgprs'):>4} scratch {meta('ScratchSize'):>4} "
          f"calls {body.count('s_swappc')} vmcnt0 {nv0} "
          f"writelane {body.count('v_writelane')} readlane {body.count('v_readlane')} lines {body.count(chr(10))}")
