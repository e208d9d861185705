#!/usr/bin/env python3
"""End-to-end rate of the host-staged TX fill (fs_fill_batch_host, checksums + FCS append in
place) on a C2-shaped batch with 4 spare bytes per frame, pinned and pageable (measurement tool;
FRAMESUM_LIB picks the library)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from seqs_amd import FCS_APPEND, FILL_CSUM, Engine, synth  # noqa: E402

n, flen, room = 65536, 1500, 4
src, soff, _ = synth.uniform_batch(n, flen, seed=1)
off = np.arange(n, dtype=np.int64) * (flen + room)
pageable = np.zeros(int(off[-1] + flen + room + 64), dtype=np.uint8)
pageable[off[:, None] + np.arange(flen)[None, :]] = src[soff[:, None] + np.arange(flen)[None, :]]
ln = np.full(n, flen, dtype=np.int32)
pinned = torch.empty(pageable.size, dtype=torch.uint8).pin_memory().numpy()
pinned[:] = pageable
eng = Engine(0)
for name, buf in (("pinned", pinned), ("pageable", pageable)):
    for _ in range(5):
        eng.fill_host(buf, off, ln, 0, FILL_CSUM | FCS_APPEND)
    t0 = time.perf_counter()
    reps = 20
    for _ in range(reps):
        eng.fill_host(buf, off, ln, 0, FILL_CSUM | FCS_APPEND)
    el = (time.perf_counter() - t0) / reps
    print(json.dumps({"case": f"TX fill + FCS append, C2 65536 x 1500 B, host-staged ({name})",
                      "GiB_s": round(n * flen / el / 2**30, 2), "ms_per_batch": round(el * 1e3, 3)}))
