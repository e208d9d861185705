"""Bring-up check of the 16-lane kernel (variant 6; measurement/diagnostic tool): bit-exact
against the C oracle on C2, C3, the edge batch and random lengths, then the C2 kernel time beside
the one-pass kernel's (HIP events around K back-to-back launches, alternated)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
from oracle import coracle  # noqa: E402
from seqs_amd import Engine, pack_frames, split_digests, synth  # noqa: E402

dev = torch.device("cuda:0")
VARIANT = int(os.environ.get("W2_VARIANT", "6"))


def check(name, buf, off, ln, mtu=0, variants=(VARIANT,)):
    dig, est = coracle.digest_batch(buf, off, ln, mtu=mtu, nthreads=16)
    tb, to, tl = (torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (buf, off.astype(np.int64), ln.astype(np.int32)))
    ok = True
    for v in variants:
        e = Engine(0)
        e.set_kernel(v)
        out, st = e.digest_device(tb, to, tl, mtu=mtu)
        torch.cuda.synchronize()
        crc, ipc, l4c = split_digests(out.cpu().numpy())
        st = st.cpu().numpy()
        bad = np.nonzero((crc != dig["crc32"]) | (ipc != dig["ip_csum"]) | (l4c != dig["l4_csum"]) | (st != est))[0]
        msg = "OK" if bad.size == 0 else f"{bad.size} BAD, first {int(bad[0])} len {int(ln[bad[0]])} crc {crc[bad[0]]:08x}/{dig['crc32'][bad[0]]:08x} l4 {l4c[bad[0]]:04x}/{dig['l4_csum'][bad[0]]:04x} st {st[bad[0]]}/{est[bad[0]]}"
        print(f"{name:28s} variant {v}: {len(ln)} frames {msg}", flush=True)
        ok &= bad.size == 0
        e.close()
    return ok


def timing(n=65536, L=1500, K=400, reps=3):
    bs = []
    for b in range(4):
        buf, off, ln = synth.uniform_batch(n, L, seed=1 + b)
        bs.append(tuple(torch.from_numpy(x).to(dev) for x in (buf, off, ln)))
    engs = {}
    for v in (4, VARIANT):
        e = Engine(0)
        e.set_kernel(v)
        engs[v] = e
    out = torch.empty((n, 2), dtype=torch.int32, device=dev)
    st = torch.empty((n,), dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)
    res = {v: [] for v in engs}
    for _ in range(reps):
        for v, e in engs.items():
            for i in range(200):
                e.digest_device(*bs[i % 4], out=out, status=st, stream=s)
            k0, k1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            k0.record(s)
            for i in range(K):
                e.digest_device(*bs[i % 4], out=out, status=st, stream=s)
            k1.record(s)
            torch.cuda.synchronize()
            res[v].append(k0.elapsed_time(k1) / K * 1e3)
    for v, t in res.items():
        print(f"C2 kernel variant {v}: " + " ".join(f"{x:.2f}" for x in t) + " us per launch (single stream)", flush=True)


if __name__ == "__main__":
    ok = True
    buf, off, ln = synth.uniform_batch(65536, 1500, seed=3)
    ok &= check("C2 65536x1500", buf, off, ln)
    buf, off, ln = synth.uniform_batch(4099, 1500, seed=4)
    ok &= check("C2-like 4099 (partial quad)", buf, off, ln)
    buf, off, ln = synth.mixed_batch(65536, seed=5)
    ok &= check("C3 mixed", buf, off, ln)
    import framegen
    frames = framegen.edge_batch(9, n_random=3000)
    for al in (1, 4):
        b, o, l = pack_frames(frames, align=al)
        ok &= check(f"edge align {al}", b, o, l, mtu=0)
        ok &= check(f"edge align {al} mtu1514", b, o, l, mtu=1514)
    rng = np.random.default_rng(11)
    lens = rng.integers(0, 3000, 20000)
    fr = [framegen.valid_frame(__import__("random").Random(int(x)), 6, payload=max(0, int(x) - 54))[: int(x)] for x in lens]
    b, o, l = pack_frames(fr, align=1)
    ok &= check("random lengths 0-3000", b, o, l)
    b, o, l = synth.hello_batch(65536)
    ok &= check("hello 47-B", b, o, l)
    # TX fill and FCS verify through the variant
    from seqs_amd import Engine as _E
    b, o, l = pack_frames(frames, align=4)
    import bench
    b2, o2, l2 = bench.with_room(b, o.astype(np.int64), l.astype(np.int32))
    exp = b2.copy()
    edig, est = coracle.fill_batch(exp, o2, l2, 0, 3)
    e = _E(0)
    e.set_kernel(VARIANT)
    tb = torch.from_numpy(b2.copy()).to(dev)
    out, st = e.fill_device(tb, torch.from_numpy(o2).to(dev), torch.from_numpy(l2).to(dev), flags=3)
    torch.cuda.synchronize()
    got = tb.cpu().numpy()
    fok = np.array_equal(got, exp) and np.array_equal(st.cpu().numpy(), est)
    print(f"TX fill + FCS append variant {VARIANT}: {'OK' if fok else 'FAIL'}", flush=True)
    l3 = torch.from_numpy(l2 + 4).to(dev)
    out, st = e.digest_fcs_device(tb, torch.from_numpy(o2).to(dev), l3)
    torch.cuda.synchronize()
    vok = bool((st.cpu().numpy()[est == 0] == 0).all())
    print(f"FCS verify of the filled frames variant {VARIANT}: {'OK' if vok else 'FAIL'}", flush=True)
    ok &= fok and vok
    e.close()
    print("PARITY", "OK" if ok else "FAIL", flush=True)
    if ok and "--time" in sys.argv:
        timing()
    sys.exit(0 if ok else 1)
