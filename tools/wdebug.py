"""Bring-up probe for the 16-lane kernel (fs_ctx_set_kernel 3): digest assorted batches and
report mismatches against the oracle with their super-tile coordinates."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from oracle import coracle  # noqa: E402
from seqs_amd import Engine, pack_frames, split_digests, synth  # noqa: E402

e = Engine(0)
e.set_kernel(int(os.environ.get("KV", "3")))
dev = torch.device("cuda:0")


def run(name, buf, off, ln, mtu=0):
    tb, to, tl = (torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in
                  (buf, off.astype(np.int64), ln.astype(np.int32)))
    out, st = e.digest_device(tb, to, tl, mtu=mtu)
    torch.cuda.synchronize()
    crc, ipc, l4c = split_digests(out.cpu().numpy())
    st = st.cpu().numpy()
    dig, est = coracle.digest_batch(buf, off, ln, mtu=mtu, nthreads=8)
    bad = np.nonzero((crc != dig["crc32"]) | (ipc != dig["ip_csum"]) | (l4c != dig["l4_csum"]) | (st != est))[0]
    n = len(ln)
    print(f"{name}: n={n} bad={bad.size}", flush=True)
    for i in bad[:12]:
        i = int(i)
        what = []
        if crc[i] != dig["crc32"][i]: what.append("crc")
        if ipc[i] != dig["ip_csum"][i]: what.append("ip")
        if l4c[i] != dig["l4_csum"][i]: what.append("l4")
        if st[i] != est[i]: what.append(f"st {st[i]}!={est[i]}")
        print(f"   i={i} st={i // 16} slot={i % 16} len={int(ln[i])} off={int(off[i])} {' '.join(what)}")


for n in (1, 5, 16, 17, 64, 100, 1000, 4097, 65536):
    b, o, l = synth.uniform_batch(n, 1500, seed=n)
    run(f"uniform1500 n={n}", b, o, l)
b, o, l = synth.mixed_batch(9000, seed=21)
run("mixed 9000", b, o, l)
for n in (64, 4500, 9000, 65536):
    b, o, l = synth.mixed_batch(n, seed=3)
    run(f"mixed n={n}", b, o, l)
rng = np.random.default_rng(4)
for n in (100, 5000):
    lens = rng.integers(60, 3000, n)
    frames = [bytes(rng.integers(0, 256, L, dtype=np.uint8)) for L in lens]
    b, o, l = pack_frames(frames, align=1)
    run(f"random n={n}", b, o, l)
import framegen  # noqa: E402

fr = framegen.edge_batch(5, n_random=3000)
b, o, l = pack_frames(fr, align=1)
run("edge align1", b, o, l)
run("edge align1 mtu", b, o, l, mtu=1514)
