"""Per-wave phase timeline from an FS_STAMPS diagnostic build (measurement tool).
Usage: FRAMESUM_LIB=seqs_amd/lib/diag/libframesum_st4.so python tools/stamps.py [--config c2]"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from seqs_amd import Engine, synth  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--config", default="c2")
p.add_argument("--frames", type=int, default=65536)
p.add_argument("--kernel", type=int, default=0)
p.add_argument("--op", choices=["digest", "fill"], default="digest",
               help="fill: fs_fill_batch (FS_FILL_CSUM|FS_FCS_APPEND) on C2 frames with 4 spare bytes each")
a = p.parse_args()
dev = torch.device("cuda:0")
bs = []
for b in range(4):
    buf, off, ln = (synth.uniform_batch(a.frames, 1500, seed=1 + b) if a.config == "c2"
                    else synth.mixed_batch(a.frames, seed=2 + b))
    if a.op == "fill":  # 4 spare bytes after every frame (the FCS), 4-byte aligned (as tools/prof_driver.py)
        step = (ln.astype(np.int64) + 4 + 3) // 4 * 4
        noff = np.zeros_like(off)
        noff[1:] = np.cumsum(step[:-1])
        nbuf = np.zeros(int(noff[-1] + step[-1]) + 16, np.uint8)
        for i in range(0, len(ln), 4096):  # (block copies: frames are contiguous in both layouts)
            j = min(len(ln), i + 4096)
            for k in range(i, j):
                nbuf[noff[k]:noff[k] + ln[k]] = buf[off[k]:off[k] + ln[k]]
        buf, off = nbuf, noff
    bs.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)))
e = Engine(0)
e.set_kernel(a.kernel)
out = torch.empty((a.frames, 2), dtype=torch.int32, device=dev)
st = torch.empty((a.frames,), dtype=torch.uint8, device=dev)
for i in range(8 if a.kernel else 40):  # (variant 0: past the automatic choice's initial window)
    if a.op == "fill":
        e.fill_device(*bs[i % 4], flags=3, out=out, status=st)
    else:
        e.digest_device(*bs[i % 4], out=out, status=st)
torch.cuda.synchronize()
arr = np.zeros(8192 * 16, dtype=np.uint64)
rc = e.lib.fs_debug_read_stamps(arr.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(arr.nbytes))
assert rc == 0, rc
nw = min(8192, (a.frames + 15) // 16)
s = arr.reshape(8192, 16)[:nw].astype(np.int64)
names = ["fill+desc->sync", "main loop", "combine", "finalize"]
print(f"waves={nw}  (cycles, s_memtime ticks)")
for k, nm in enumerate(names):
    d = s[:, k + 1] - s[:, k]
    print(f"  {nm:18s} median {int(np.median(d)):8d}  p10 {int(np.percentile(d, 10)):8d}  p90 {int(np.percentile(d, 90)):8d}")
tot = s[:, 4] - s[:, 0]
blk = np.arange(nw) // 16
ml = s[:, 2] - s[:, 1]
print("  main loop median by blockIdx % 8 (XCD group):",
      [int(np.median(ml[(blk % 8) == x])) for x in range(8)])
print("  main loop median by wave-in-block:", [int(np.median(ml[(np.arange(nw) % 16) == w])) for w in range(16)])
st = s[:, 0] - s[:, 0].min()
print("  start skew (ticks) p50/p90/max:", int(np.median(st)), int(np.percentile(st, 90)), int(st.max()))
print(f"  {'wave total':18s} median {int(np.median(tot)):8d}  p10 {int(np.percentile(tot, 10)):8d}  p90 {int(np.percentile(tot, 90)):8d}")
# s_memrealtime (100 MHz, chip-wide) timeline: launch ramp and tail, in microseconds
rs, re_ = s[:, 5], s[:, 6]
t0 = rs.min()
us = lambda x: x * 0.01  # noqa: E731
print(f"  realtime: span {us(re_.max() - t0):.2f} us; wave start offset p50/p90/max "
      f"{us(np.median(rs - t0)):.2f}/{us(np.percentile(rs - t0, 90)):.2f}/{us((rs - t0).max()):.2f} us; "
      f"wave end p10/p50/p90/max {us(np.percentile(re_ - t0, 10)):.2f}/{us(np.median(re_ - t0)):.2f}/"
      f"{us(np.percentile(re_ - t0, 90)):.2f}/{us((re_ - t0).max()):.2f} us")
print(f"  memtime ticks per us (median over waves): {np.median((s[:, 4] - s[:, 0]) / np.maximum(1, us(re_ - rs))):.0f}")
if s[:, 9].any():
    for nm, a_, b_ in (("start->regionA", 0, 7), ("regionA->desc", 7, 8), ("start->desc (fine)", 0, 8), ("desc->geom+issue", 8, 9), ("start->geom+issue", 0, 9),
                       ("issue->waitcnt", 9, 10), ("waitcnt->barrier", 10, 1),
                       ("desc->geometry", 8, 11), ("geometry->report", 11, 12), ("report->header", 12, 13),
                       ("header->rows issued", 13, 9)):
        if s[:, b_].any() and s[:, a_].any():
            d = s[:, b_] - s[:, a_]
            print(f"  {nm:18s} median {int(np.median(d)):8d}  p10 {int(np.percentile(d, 10)):8d}  p90 {int(np.percentile(d, 90)):8d}")
wib = np.arange(nw) % 16
for nm, a_, b_ in (("start->desc", 0, 8), ("start->issue", 0, 9), ("barrier wait", 10, 1)):
    if s[:, b_].any():
        d = s[:, b_] - s[:, a_]
        print(f"  {nm} median by wave-in-block:", [int(np.median(d[wib == w])) for w in range(16)])
# active-wave profile over the launch (realtime, 1-us bins) and the phase boundaries' spread
span = us(re_.max() - t0)
bins = np.arange(0, span + 1.0, 1.0)
act = [int(((us(rs - t0) <= b + 0.5) & (us(re_ - t0) > b + 0.5)).sum()) for b in bins]
print("  active waves per 1-us bin:", act)
ends = np.sort(us(re_ - t0))
print("  wave end quantiles (us) 1/5/25/50/75/95/99/100%:",
      [round(float(np.percentile(ends, q)), 2) for q in (1, 5, 25, 50, 75, 95, 99, 100)])
