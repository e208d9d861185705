"""Randomized parity stress through the C ABI: seeded random batches that mix frame lengths (short,
MTU, jumbo, odd sizes), protocols, corrupted checksums, malformed frames, unaligned offsets with
gaps and MTU settings, run through every kernel variant (the parity columns of tests/engines.py) on
the device path and through the host-staged path, each launch compared bit for bit with the C oracle.

FS_STRESS_BATCHES sets the number of batches (default 8, a few seconds; the round-end stress run in
profiles/ used more). Results never depend on the kernel choice, so every column must agree."""
import os
import random
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import engines  # noqa: E402
import framegen  # noqa: E402
from oracle import coracle  # noqa: E402
from seqs_amd import FCS_APPEND, FILL_CSUM, split_digests, synth  # noqa: E402

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N_BATCHES = int(os.environ.get("FS_STRESS_BATCHES", "8"))


def random_batch(seed: int, room: int = 0):
    """(buf, offsets, lengths, mtu): 1 to ~6,000 frames of one of four shapes; `room` spare bytes at
    least after every frame (a TX fill appends its FCS there)."""
    rnd = random.Random(seed)
    rng = np.random.default_rng(seed)
    kind = seed % 4
    frames: list[bytes] = []
    if kind == 0:  # many lengths, valid and corrupted
        for _ in range(rnd.randrange(1, 12)):
            length = rnd.choice((54, 60, 64, 127, 128, 129, 576, 1499, 1500, 1514, 3001, 9000, 9018))
            length = max(length + rnd.randrange(-3, 4), 54)
            f = synth.make_frames(rnd.randrange(1, 400), length, rnd.choice((6, 17)), rng)
            frames += [bytes(r) for r in f]
    elif kind == 1:  # the reference's short frames with a few long ones between them
        hb, ho, hl = synth.hello_batch(rnd.randrange(1, 5000), seed=seed)
        frames += [bytes(hb[int(o):int(o) + int(l)]) for o, l in zip(ho, hl)]
        frames += [bytes(r) for r in synth.make_frames(rnd.randrange(0, 6), rnd.choice((1500, 9000)), 6, rng)]
    elif kind == 2:  # the edge batch: option headers, paddings, zero sums, malformed frames
        frames += framegen.edge_batch(seed, n_random=rnd.randrange(50, 600))
    else:  # random bytes of random lengths (mostly rejected by the gates: verdict parity)
        frames += [rnd.randbytes(rnd.choice((rnd.randrange(0, 64), rnd.randrange(0, 3000)))) for _ in range(rnd.randrange(1, 800))]
    # corrupt a few frames anywhere (checksum mismatches, or broken headers)
    for _ in range(len(frames) // 10):
        i = rnd.randrange(len(frames))
        if frames[i]:
            f = bytearray(frames[i])
            f[rnd.randrange(len(f))] ^= 1 << rnd.randrange(8)
            frames[i] = bytes(f)
    rnd.shuffle(frames)
    # pack at a random alignment with random gaps between frames
    align = rnd.choice((1, 2, 4, 8))
    offsets = np.zeros(len(frames), np.int64)
    pos = rnd.randrange(0, 64)
    for i, f in enumerate(frames):
        pos = (pos + align - 1) // align * align
        offsets[i] = pos
        pos += len(f) + max(room, rnd.choice((0, 0, 0, 1, 4, 13, 64)))
    buf = np.zeros(pos + 64, np.uint8)
    for o, f in zip(offsets, frames):
        buf[int(o):int(o) + len(f)] = np.frombuffer(f, np.uint8)
    lengths = np.fromiter((len(f) for f in frames), np.int32, count=len(frames))
    mtu = rnd.choice((0, 0, 1514, 1518, 2048, 9014))
    return buf, offsets, lengths, mtu


@pytest.mark.parametrize("variant", engines.VARIANTS, ids=engines.IDS)
def test_random_batches_every_variant(variant):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    dev = torch.device("cuda:0")
    e = engines.engine_for(variant)
    try:
        for seed in range(N_BATCHES):
            buf, off, ln, mtu = random_batch(1000 + seed)
            dig, est = coracle.digest_batch(buf, off, ln, mtu=mtu, nthreads=8)
            # the device path, the frames at a base 4 bytes past a 16-B boundary on odd seeds
            shift = 4 * (seed & 1)
            tb = torch.zeros(len(buf) + 16, dtype=torch.uint8, device=dev)
            tb[shift:shift + len(buf)] = torch.from_numpy(buf).to(dev)
            out, st = e.digest_device(tb[shift:], torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev), mtu=mtu)
            torch.cuda.synchronize()
            crc, ipc, l4c = split_digests(out.cpu().numpy())
            stn = st.cpu().numpy()
            bad = np.nonzero((crc != dig["crc32"]) | (ipc != dig["ip_csum"]) | (l4c != dig["l4_csum"]) | (stn != est))[0]
            assert bad.size == 0, f"seed {1000 + seed}, device: {bad.size} of {len(ln)} differ, first {int(bad[0])} (len {int(ln[bad[0]])})"
            # the host-staged path on the same batch
            hout, hst = e.digest_host(buf, off.astype(np.uint64), ln.astype(np.uint32), mtu=mtu)
            assert np.array_equal(hout["crc32"], dig["crc32"]) and np.array_equal(hout["ip_csum"], dig["ip_csum"])
            assert np.array_equal(hout["l4_csum"], dig["l4_csum"]) and np.array_equal(hst, est), f"seed {1000 + seed}, host"
    finally:
        e.close()


@pytest.mark.parametrize("variant", engines.VARIANTS, ids=engines.IDS)
def test_random_fill_then_fcs_verify(variant):
    """TX fill in place (fs_fill_batch, every flag combination) on the random batches, byte for byte
    and digest for digest against the oracle's fill; then the FCS verify (fs_digest_batch_fcs) of
    the wire frames it wrote, against the oracle's."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    dev = torch.device("cuda:0")
    e = engines.engine_for(variant)
    try:
        for seed in range(N_BATCHES):
            buf, off, ln, mtu = random_batch(2000 + seed, room=4)
            flags = (FILL_CSUM, FCS_APPEND, FILL_CSUM | FCS_APPEND, 0)[seed % 4]
            tb = torch.from_numpy(buf.copy()).to(dev)
            to, tl = torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)
            out, st = e.fill_device(tb, to, tl, mtu=mtu, flags=flags)
            torch.cuda.synchronize()
            ebuf = buf.copy()
            edig, est = coracle.fill_batch(ebuf, off, ln, mtu, flags)
            gbuf = tb.cpu().numpy()
            diff = np.nonzero(gbuf != ebuf)[0]
            assert diff.size == 0, f"seed {2000 + seed} flags {flags}: {diff.size} bytes differ, first at {int(diff[0])}"
            crc, ipc, l4c = split_digests(out.cpu().numpy())
            stn = st.cpu().numpy()
            bad = np.nonzero((crc != edig["crc32"]) | (ipc != edig["ip_csum"]) | (l4c != edig["l4_csum"]) | (stn != est))[0]
            assert bad.size == 0, f"seed {2000 + seed} flags {flags}: {bad.size} fill digests differ, first {int(bad[0])}"
            if flags & FCS_APPEND:
                wl = (ln + 4).astype(np.int32)
                fout, fst = e.digest_fcs_device(tb, to, torch.from_numpy(wl).to(dev), mtu=mtu)
                torch.cuda.synchronize()
                fdig, fest = coracle.digest_fcs_batch(ebuf, off, wl, mtu)
                crc, ipc, l4c = split_digests(fout.cpu().numpy())
                fstn = fst.cpu().numpy()
                bad = np.nonzero((crc != fdig["crc32"]) | (ipc != fdig["ip_csum"]) | (l4c != fdig["l4_csum"]) | (fstn != fest))[0]
                assert bad.size == 0, f"seed {2000 + seed}: {bad.size} FCS verifies differ, first {int(bad[0])}"
    finally:
        e.close()
