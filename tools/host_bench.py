#!/usr/bin/env python3
"""End-to-end (PCIe-inclusive) rate of the host-staged path, fs_digest_batch_host: frames in
host memory -> chunked H2D / kernel / D2H pipeline -> digests + verdicts in host memory.
Reported in DESIGN.md; never the bench `value` (which is device-resident)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from seqs_amd import Engine, digest_host_multi, synth  # noqa: E402


def rate(fn, nbytes, reps):
    for _ in range(10):  # warm: the first host-staged batches of a process run slower
        fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    el = time.perf_counter() - t0
    return nbytes * reps / el / 2**30, el / reps * 1e3


def main():
    eng = Engine(0)
    cases = [("C2 65536 x 1500-B TCP", synth.uniform_batch(65536, 1500, seed=1)),
             ("C5 16384 x 9000-B jumbo", synth.uniform_batch(16384, 9000, seed=2))]
    # raw H2D copy rate for reference (torch pinned tensor -> device)
    x = torch.empty(98304000, dtype=torch.uint8).pin_memory()
    d = torch.empty_like(x, device="cuda:0")

    def h2d():
        d.copy_(x, non_blocking=True)
        torch.cuda.synchronize()

    g, ms = rate(h2d, x.numel(), 20)
    print(json.dumps({"case": "raw pinned H2D copy 98.3 MB", "GiB_s": round(g, 2), "ms": round(ms, 3)}), flush=True)
    for name, (buf, off, ln) in cases:
        nbytes = int(ln.astype(np.int64).sum())
        off64, ln32 = off.astype(np.uint64), ln.astype(np.uint32)
        out = eng.host_empty(len(ln), dtype=np.dtype([("crc32", "<u4"), ("ip_csum", "<u2"), ("l4_csum", "<u2")]))
        st = eng.host_empty(len(ln), dtype=np.uint8)
        pin = eng.host_empty(buf.shape)
        pin[:] = buf
        for kind, b in (("pinned", pin), ("pageable", buf)):
            g, ms = rate(lambda: eng.digest_host(b, off64, ln32, out=out, status=st), nbytes, 20)
            assert int(st.max()) == 0, "synthetic frames must verify"
            print(json.dumps({"case": f"{name}, host-staged ({kind})", "GiB_s": round(g, 2), "ms_per_batch": round(ms, 3),
                              "bytes": nbytes}), flush=True)
    # fs_digest_batch_multi: one context per visible GPU (C5's 8-GPU streaming form), and on a
    # one-GPU box 2 contexts sharing it (the threading and block split; one PCIe link either way)
    ndev = torch.cuda.device_count()
    buf, off, ln = cases[1][1]
    nbytes = int(ln.astype(np.int64).sum())
    pin = eng.host_empty(buf.shape)
    pin[:] = buf
    layouts = [[0] * 2] if ndev == 1 else [list(range(ndev))]
    for devs in layouts:
        engs = [eng] + [Engine(d) for d in devs[1:]]
        g, ms = rate(lambda: digest_host_multi(engs, pin, off.astype(np.uint64), ln.astype(np.uint32)), nbytes, 20)
        print(json.dumps({"case": f"{cases[1][0]}, fs_digest_batch_multi over devices {devs} (pinned)",
                          "GiB_s": round(g, 2), "ms_per_batch": round(ms, 3), "bytes": nbytes}), flush=True)
        for e in engs[1:]:
            e.close()
    eng.close()


if __name__ == "__main__":
    main()
