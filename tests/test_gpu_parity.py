"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle, bit-exact.

Sizes: golden fixtures and seeded edge batches at oracle-friendly sizes; the
full BASELINE configs (65,536 x 1500 B; 65,536 mixed 64/576/1500/9000) are
checked element-wise against the C oracle too (it finishes them in ~1 s).
"""
import json
import os
import zlib

import numpy as np
import pytest

import engines  # noqa: E402

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from oracle import coracle  # noqa: E402
from seqs_amd import Engine, pack_frames, split_digests, synth  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", params=engines.VARIANTS, ids=engines.IDS)
def engine(request):
    # every case through every kernel variant (and the automatic choice)
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    e = engines.engine_for(request.param)
    yield e
    e.close()


def run_device(engine, buf, off, ln, mtu=0):
    dev = torch.device("cuda:0")
    tb = torch.from_numpy(np.ascontiguousarray(buf)).to(dev)
    to = torch.from_numpy(np.ascontiguousarray(off).astype(np.int64)).to(dev)
    tl = torch.from_numpy(np.ascontiguousarray(ln).astype(np.int32)).to(dev)
    out, st = engine.digest_device(tb, to, tl, mtu=mtu)
    torch.cuda.synchronize()
    crc, ipc, l4c = split_digests(out.cpu().numpy())
    return crc, ipc, l4c, st.cpu().numpy()


def check(engine, buf, off, ln, mtu=0, label=""):
    crc, ipc, l4c, st = run_device(engine, buf, off, ln, mtu)
    dig, est = coracle.digest_batch(buf, off, ln, mtu=mtu, nthreads=8)
    bad = np.nonzero((crc != dig["crc32"]) | (ipc != dig["ip_csum"]) | (l4c != dig["l4_csum"]) | (st != est))[0]
    if bad.size:
        i = int(bad[0])
        raise AssertionError(
            f"{label}: {bad.size}/{len(ln)} mismatches; first i={i} len={int(ln[i])} off={int(off[i])} "
            f"gpu=({crc[i]:#010x},{ipc[i]:#06x},{l4c[i]:#06x},{st[i]}) "
            f"oracle=({int(dig['crc32'][i]):#010x},{int(dig['ip_csum'][i]):#06x},{int(dig['l4_csum'][i]):#06x},{est[i]})")
    return crc, ipc, l4c, st


def test_kat_frames(engine):
    kats = json.load(open(os.path.join(GOLDEN, "kats.json")))
    frames = [bytes.fromhex(t["hex"]) for t in kats["frames"]]
    digs = engine.digest_batch(frames, mtu=2048)
    for t, d, f in zip(kats["frames"], digs, frames):
        assert (d.verdict, d.ip_csum, d.l4_csum) == (t["verdict"], t["ip_csum"], t["l4_csum"])
        assert d.crc32 == zlib.crc32(f)
    d = engine.digest_batch([b"123456789"])[0]
    assert d.crc32 == kats["crc32_check"]["expected"]


def test_golden_batch(engine):
    g = json.load(open(os.path.join(GOLDEN, "batch.json")))
    frames = [bytes.fromhex(e["hex"]) for e in g["frames"]]
    for align in (4, 1):  # 1 = every possible start alignment
        buf, off, ln = pack_frames(frames, align=align)
        crc, ipc, l4c, st = run_device(engine, buf, off, ln)
        for i, e in enumerate(g["frames"]):
            assert (int(crc[i]), int(ipc[i]), int(l4c[i]), int(st[i])) == (e["crc32"], e["ip_csum"], e["l4_csum"], e["verdict"]), i
    buf, off, ln = pack_frames(frames, align=4)
    crc, ipc, l4c, st = run_device(engine, buf, off, ln, mtu=600)
    for e in g["mtu600"]:
        i = e["index"]
        assert (int(ipc[i]), int(l4c[i]), int(st[i])) == (e["ip_csum"], e["l4_csum"], e["verdict"])


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_edge_batches_unaligned(engine, seed):
    import framegen

    frames = framegen.edge_batch(seed, n_random=400)
    for align in (1, 2, 4, 16):
        buf, off, ln = pack_frames(frames, align=align)
        check(engine, buf, off, ln, label=f"seed{seed}/align{align}")
        check(engine, buf, off, ln, mtu=1514, label=f"seed{seed}/align{align}/mtu")


def test_frames_at_buffer_start_and_tiny(engine):
    # a frame at offset 0 of the allocation with odd starts right after it, and sub-4-byte frames
    rng = np.random.default_rng(4)
    buf = rng.integers(0, 256, 4096, dtype=np.uint8)
    off = np.array([0, 1, 2, 3, 5, 6, 7, 100, 101, 0, 0, 3], dtype=np.int64)
    ln = np.array([40, 3, 2, 1, 0, 4, 5, 1500, 64, 0, 1, 9], dtype=np.int32)
    check(engine, buf, off, ln, label="start")


@pytest.mark.parametrize("base", [4, 8, 12])
def test_frames_base_not_16_aligned(engine, base):
    """The frames pointer only has to be 4-byte aligned: a base at 16k + 4/8/12 (a view into a larger
    device buffer) gives the same results, and the small-frame kernel reads 16-B chunks at absolute
    16-B boundaries. Short frames, MTU frames and jumbo frames at every start."""
    import framegen

    frames = framegen.edge_batch(31, n_random=300)
    buf, off, ln = pack_frames(frames, align=1)
    dig, est = coracle.digest_batch(buf, off, ln, mtu=1514, nthreads=8)
    dev = torch.device("cuda:0")
    big = torch.zeros(len(buf) + 64, dtype=torch.uint8, device=dev)
    assert big.data_ptr() % 16 == 0
    big[base:base + len(buf)] = torch.from_numpy(buf).to(dev)
    view = big[base:base + len(buf)]
    assert view.data_ptr() % 16 == base
    out, st = engine.digest_device(view, torch.from_numpy(off.astype(np.int64)).to(dev),
                                   torch.from_numpy(ln.astype(np.int32)).to(dev), mtu=1514)
    torch.cuda.synchronize()
    crc, ipc, l4c = split_digests(out.cpu().numpy())
    st = st.cpu().numpy()
    bad = np.nonzero((crc != dig["crc32"]) | (ipc != dig["ip_csum"]) | (l4c != dig["l4_csum"]) | (st != est))[0]
    assert bad.size == 0, f"base +{base}: {bad.size} mismatches, first at {int(bad[0])}"


@pytest.mark.parametrize("n", [1, 15, 16, 17, 255, 4097])
def test_partial_tiles(engine, n):
    buf, off, ln = synth.uniform_batch(n, 1500, seed=n)
    crc, ipc, l4c, st = check(engine, buf, off, ln, label=f"n={n}")
    assert (st == 0).all()


def test_c2_full_config(engine):
    # BASELINE configs[1]: 65,536 x 1500-B frames, bit-exact vs the oracle
    buf, off, ln = synth.uniform_batch(65536, 1500, seed=1)
    crc, ipc, l4c, st = check(engine, buf, off, ln, label="C2")
    assert (st == 0).all()


def test_c3_mixed_config(engine):
    # BASELINE configs[2]: 65,536 frames cycling 64/576/1500/9000, TCP/UDP 50/50
    buf, off, ln = synth.mixed_batch(65536, seed=2)
    crc, ipc, l4c, st = check(engine, buf, off, ln, label="C3")
    assert (st == 0).all()


def test_random_lengths_large(engine):
    rng = np.random.default_rng(7)
    n = 20000
    ln = rng.integers(0, 9100, n).astype(np.int32)
    gaps = rng.integers(0, 7, n)
    off = np.zeros(n, np.int64)
    off[1:] = np.cumsum(ln[:-1].astype(np.int64) + gaps[:-1])
    buf = rng.integers(0, 256, int(off[-1] + ln[-1] + 16), dtype=np.uint8)
    # make ~half the frames well-formed TCP/UDP so the checksum path is exercised at all lengths
    for i in range(0, n, 2):
        L = int(ln[i])
        p = 6 if (i // 2) % 2 == 0 else 17
        if L >= 54:
            f = synth.make_frames(1, L, p, rng)[0]
            buf[off[i] : off[i] + L] = f
    check(engine, buf, off, ln, label="random")


def test_giant_padded_frame(engine):
    # A >= 512 KiB frame whose IP datagram is short: RecvEth still checksums [off, end) and the
    # rest is Ethernet padding (the kernel's exact-from-memory fallback for huge frames).
    import random
    import framegen

    rnd = random.Random(8)
    frames = []
    for L, pad in ((1000, 600000), (1400, 700001), (200, 3)):
        f = framegen.valid_frame(rnd, 6 if L != 200 else 17, payload=L, pad=pad)
        frames.append(f)
    frames.append(bytes(rnd.randbytes(530000)))  # giant non-IP frame: CRC only
    buf, off, ln = pack_frames(frames, align=1)
    check(engine, buf, off, ln, label="giant")


def test_corruption_detected(engine):
    buf, off, ln = synth.uniform_batch(4096, 1500, seed=9)
    rng = np.random.default_rng(1)
    hit = rng.choice(4096, 300, replace=False)
    for i in hit:
        pos = int(off[i]) + int(rng.integers(34, 1500))
        buf[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
    crc, ipc, l4c, st = check(engine, buf, off, ln, label="corrupt")
    assert (st[hit] == 13).sum() >= 290  # a single-bit flip in the L4 range always fails the checksum
    assert (st[np.setdiff1d(np.arange(4096), hit)] == 0).all()


def test_host_staged_path(engine):
    buf, off, ln = synth.mixed_batch(4096, seed=5)
    dig, st = engine.digest_host(buf, off.astype(np.uint64), ln.astype(np.uint32))
    edig, est = coracle.digest_batch(buf, off, ln)
    assert np.array_equal(dig, edig) and np.array_equal(st, est)


def test_empty_batch(engine):
    out, st = engine.digest_host(np.zeros(16, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32))
    assert out.size == 0


def test_host_staged_multichunk_unordered(engine):
    # > 16 MiB of frames in shuffled buffer order: several pipeline chunks, non-monotonic
    # offsets (chunk byte spans computed from min/max), pinned and pageable inputs
    buf, off0, ln0 = synth.mixed_batch(12000, seed=9)
    perm = np.random.default_rng(3).permutation(len(ln0))
    for order in (np.arange(len(ln0)), perm):
        off, ln = off0[order].astype(np.uint64), ln0[order].astype(np.uint32)
        edig, est = coracle.digest_batch(buf, off.astype(np.int64), ln.astype(np.int32))
        dig, st = engine.digest_host(buf, off, ln)
        assert np.array_equal(dig, edig) and np.array_equal(st, est)
    pin = engine.host_empty(buf.shape)
    pin[:] = buf
    dig2, st2 = engine.digest_host(pin, off, ln)
    assert np.array_equal(dig2, edig) and np.array_equal(st2, est)


def test_piece_boundaries_and_mixed_tiles(engine):
    # Mixed tiles (mode B): a jumbo frame beside short ones at every start alignment, lengths
    # around the 768-byte piece boundaries (stream dwords = 192 k + {0, 1, 2, 3}), frames whose
    # Ethernet padding lies in their last piece or past the header slot, tiles whose full pieces
    # do not fill the last pass, and a tile with more full pieces than the passes allow.
    import random

    import framegen

    rnd = random.Random(11)
    frames = []
    for k in range(1, 13):
        for d in (-5, -4, -3, -2, -1, 0, 1, 2, 3, 4, 5):
            L = 768 * k + d
            frames.append(framegen.valid_frame(rnd, 6 if (k + d) % 2 else 17, payload=max(0, L - 54)))
            frames.append(bytes(rnd.randbytes(max(1, 60 + d))))
    for pad in (1, 46, 300, 2000):
        frames.append(framegen.valid_frame(rnd, 6, payload=3000, pad=pad))
        frames.append(framegen.valid_frame(rnd, 17, payload=20, pad=pad))
    frames += [framegen.valid_frame(rnd, 6, payload=9000 - 54) for _ in range(3)] + [b"\x01" * 64] * 13
    frames += [bytes(rnd.randbytes(100000))] + [b"\x02" * 60] * 15  # too many full pieces: one pass
    for align in (1, 4):
        buf, off, ln = pack_frames(frames, align=align)
        check(engine, buf, off, ln, label=f"pieces/align{align}")
        check(engine, buf, off, ln, mtu=1514, label=f"pieces/align{align}/mtu")


def test_host_multi_contexts(engine):
    # fs_digest_batch_multi: byte-balanced contiguous blocks over 1, 2, 3 and 5 contexts (all on
    # this one GPU here; one per GPU in production), mixed lengths in shuffled buffer order,
    # more contexts than frames, MTU gates; digests and verdicts land in batch order
    from seqs_amd import Engine, digest_host_multi

    extra = [Engine(0) for _ in range(4)]
    try:
        buf, off0, ln0 = synth.mixed_batch(9000, seed=21)
        perm = np.random.default_rng(5).permutation(len(ln0))
        for order in (np.arange(len(ln0)), perm):
            off, ln = off0[order].astype(np.uint64), ln0[order].astype(np.uint32)
            for mtu in (0, 1514):
                edig, est = coracle.digest_batch(buf, off.astype(np.int64), ln.astype(np.int32), mtu)
                for k in (1, 2, 3, 5):
                    dig, st = digest_host_multi([engine] + extra[: k - 1], buf, off, ln, mtu)
                    assert np.array_equal(dig, edig) and np.array_equal(st, est), (k, mtu)
        few_off, few_ln = off0[:3].astype(np.uint64), ln0[:3].astype(np.uint32)
        edig, est = coracle.digest_batch(buf, few_off.astype(np.int64), few_ln.astype(np.int32))
        dig, st = digest_host_multi([engine] + extra, buf, few_off, few_ln)
        assert np.array_equal(dig, edig) and np.array_equal(st, est)
        dig, st = digest_host_multi([engine] + extra, buf, np.zeros(0, np.uint64), np.zeros(0, np.uint32))
        assert dig.size == 0
        with pytest.raises(Exception):  # a frame past the buffer fails its block's call
            digest_host_multi([engine, extra[0]], np.zeros(100, np.uint8), np.array([0, 90], np.uint64),
                              np.array([20, 20], np.uint32))
    finally:
        for e in extra:
            e.close()


def test_host_staged_rejects_out_of_range(engine):
    buf = np.zeros(100, np.uint8)
    with pytest.raises(Exception):
        engine.digest_host(buf, np.array([90], np.uint64), np.array([20], np.uint32))


def test_random_batch_stress(engine):
    # many independent random batches: sizes from 1 frame to several tiles per wave, lengths
    # from 0 to jumbo (some batches uniform, some mixed), random gaps and start alignments,
    # valid / corrupted / random frames, random MTU; every digest and verdict bit-exact
    rng = np.random.default_rng(2024)
    for it in range(24):
        n = int(rng.choice([1, 7, 16, 300, 4096, 20000, 70000]))
        kind = it % 3
        if kind == 0:  # uniform length
            ln = np.full(n, int(rng.choice([60, 64, 128, 577, 1500, 4000, 9000])), np.int64)
        elif kind == 1:  # mixed
            ln = rng.choice([0, 3, 34, 54, 64, 200, 576, 1500, 9000], size=n).astype(np.int64)
        else:  # anything up to jumbo
            ln = rng.integers(0, 9200, n).astype(np.int64)
        gaps = rng.integers(0, 9, n) if it % 2 else np.zeros(n, np.int64)
        off = np.zeros(n, np.int64)
        off[1:] = np.cumsum(ln[:-1] + gaps[:-1])
        off += int(rng.integers(0, 4))
        buf = rng.integers(0, 256, int(off[-1] + ln[-1] + 16), dtype=np.uint8)
        # about half the frames well-formed TCP/UDP (some then corrupted)
        sel = np.nonzero((ln >= 54) & (rng.random(n) < 0.5))[0]
        for i in sel[:3000]:
            f = synth.make_frames(1, int(ln[i]), 6 if i % 2 else 17, rng)[0]
            if rng.random() < 0.1:
                f[int(rng.integers(14, len(f)))] ^= 0x40
            buf[off[i] : off[i] + ln[i]] = f
        mtu = int(rng.choice([0, 0, 1514, 9018]))
        check(engine, buf, off, ln.astype(np.int32), mtu=mtu, label=f"stress{it}/n={n}/kind={kind}")


def test_too_many_frames_rejected(engine):
    import ctypes

    dev = torch.device("cuda:0")
    t = torch.zeros(64, dtype=torch.uint8, device=dev)
    p = ctypes.c_void_p(t.data_ptr())
    st = engine.lib.fs_digest_batch(engine._ctx, p, p, p, (1 << 31) + 1, 0, p, p, None)
    assert st == -1 and b"too large" in engine.lib.fs_last_error(engine._ctx)


@pytest.mark.parametrize("n,flen", [(40000, 1500), (16384, 9000), (2000, 9000), (3000, 64)])
def test_frames_per_tile_adaptation(engine, n, flen):
    # batches too small to give every wave a 16-frame tile run the one-pass kernel with 8 or
    # 4 frames per tile (40,000 frames: 8; 16,384 jumbo frames: 4), the empty groups idle
    buf, off, ln = synth.uniform_batch(n, flen, seed=n)
    crc, ipc, l4c, st = check(engine, buf, off, ln, label=f"fpt n={n} len={flen}")
    assert (st == 0).all()


@pytest.mark.parametrize("n,flen", [(300000, 0), (1 << 20, 64), (200000, 1500)])
def test_many_tiles_per_wave(engine, n, flen):
    # several tiles per wave: the one-pass kernel's tile loop carries its descriptor, header
    # and row prefetch across tiles (flen 0: random lengths up to 2 KB)
    if flen:
        buf, off, ln = synth.uniform_batch(n, flen, seed=n)
    else:
        rng = np.random.default_rng(n)
        ln = rng.integers(0, 2048, n).astype(np.int64)
        off = np.zeros(n, np.int64)
        off[1:] = np.cumsum(ln[:-1] + 3)
        buf = rng.integers(0, 256, int(off[-1] + ln[-1] + 16), dtype=np.uint8)
        ln = ln.astype(np.int32)
    check(engine, buf, off, ln, label=f"many tiles n={n} len={flen}")


def _tile_mix_batch(ntiles: int, seed: int):
    """Tiles of 16 frames, each tile one random length class, so a wave streaming several tiles
    meets every transition of the one-pass kernel's tile loop: tiles of frames under 4
    bytes (no rows), one-block tiles (<= 5 blocks), two-block tiles, MTU and jumbo tiles, tiles of
    widely mixed lengths (header slots loaded, not captured) and a partial last tile."""
    rng = np.random.default_rng(seed)
    classes = [(0, 3), (20, 300), (301, 620), (1400, 1514), (8000, 9000), (0, 3000)]
    lens = []
    for _ in range(ntiles):
        lo, hi = classes[rng.integers(0, len(classes))]
        lens.extend(rng.integers(lo, hi + 1, 16).tolist())
    lens = lens[: 16 * ntiles - 5]
    import random

    import framegen
    r = random.Random(seed)
    frames = [framegen.valid_frame(r, 6 if i % 2 else 17, payload=max(0, L - 54))[:L] for i, L in enumerate(lens)]
    return pack_frames(frames, align=1)


@pytest.mark.parametrize("workgroups", [1, 7, 64])
def test_few_workgroups(engine, workgroups):
    """fs_ctx_set_workgroups: a capped grid gives each wave many tiles, streamed back to back (every
    transition between tile classes: no rows, one- and two-block tiles, MTU, jumbo, mixed)."""
    engine.set_workgroups(workgroups)
    try:
        buf, off, ln = synth.uniform_batch(20000, 1500, seed=workgroups)
        check(engine, buf, off, ln, label=f"uniform wg={workgroups}")
        buf, off, ln = _tile_mix_batch(600, seed=workgroups)
        check(engine, buf, off, ln, label=f"tile mix wg={workgroups}")
        check(engine, buf, off, ln, mtu=1514, label=f"tile mix mtu wg={workgroups}")
    finally:
        engine.set_workgroups(0)


def test_prepared_calls_match(engine):
    """Engine.prepare_digest (checked and marshalled once, the bench's path) gives what
    digest_device gives, call after call, for the RX digest and the FCS verify."""
    import framegen

    dev = torch.device("cuda:0")
    frames = framegen.edge_batch(21, n_random=500)
    buf, off, ln = pack_frames(frames, align=4)
    tb, to, tl = (torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (buf, off.astype(np.int64),
                                                                             ln.astype(np.int32)))
    ref_out, ref_st = engine.digest_device(tb, to, tl, mtu=1514)
    out = torch.empty_like(ref_out)
    st = torch.empty_like(ref_st)
    s = torch.cuda.Stream(dev)
    call = engine.prepare_digest(tb, to, tl, mtu=1514, out=out, status=st, stream=s)
    for _ in range(3):
        out.fill_(0)
        st.fill_(0xFF)
        o, v = call()
        assert o is out and v is st
        torch.cuda.synchronize()
        assert torch.equal(out, ref_out) and torch.equal(st, ref_st)
    dig, est = coracle.digest_batch(buf, off, ln, mtu=1514)
    crc, ipc, l4c = split_digests(out.cpu().numpy())
    assert np.array_equal(crc, dig["crc32"]) and np.array_equal(st.cpu().numpy(), est)


def test_host_path_picks_small_kernel():
    """fs_digest_batch_host sees the lengths on the host: with the automatic choice a batch whose
    frames are all <= 128 B runs the small-frame kernel (variant 8), any longer frame keeps the
    4-lane kernels; results match the oracle either way."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    e = Engine(0)
    try:
        buf, off, ln = synth.hello_batch(5000, seed=9)
        dig, st = e.digest_host(buf, off, ln)
        assert e.last_kernel() == 8
        edig, est = coracle.digest_batch(buf, off, ln)
        assert np.array_equal(dig["crc32"], edig["crc32"]) and np.array_equal(st, est)
        assert np.array_equal(dig["l4_csum"], edig["l4_csum"]) and (st == 0).all()
        import framegen
        frames = framegen.edge_batch(33, n_random=300)
        b2, o2, l2 = pack_frames(frames, align=4)
        assert int(l2.max()) > 128
        dig2, st2 = e.digest_host(b2, o2, l2, mtu=1514)
        assert e.last_kernel() in (2, 4)
        edig2, est2 = coracle.digest_batch(b2, o2, l2, mtu=1514)
        assert np.array_equal(dig2["crc32"], edig2["crc32"]) and np.array_equal(st2, est2)
        e.set_kernel(4)  # a forced choice wins
        e.digest_host(buf, off, ln)
        assert e.last_kernel() == 4
    finally:
        e.close()


def test_set_workgroups_rejects_negative():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from seqs_amd import FramesumError

    e = Engine(0)
    try:
        e.set_workgroups(0)
        e.set_workgroups(3)
        with pytest.raises(FramesumError, match="workgroups"):
            e.set_workgroups(-1)
    finally:
        e.close()


def test_auto_choice_first_launches():
    """Variant 0 (automatic): a fresh context's first launches run the mixed-length kernel, so a
    mixed batch is fast from its first call (the one-pass kernel's report would reach the host
    launches late); it stays chosen while its own batches have mode-B tiles, and uniform traffic
    moves to the block-aligned one-pass kernel once the initial window (16 launches) ends.
    Results are the same either way (checked against the oracle after each switch)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    e = Engine(0)
    try:
        assert e.last_kernel() == 0
        buf, off, ln = synth.mixed_batch(4096, seed=5)
        check(e, buf, off, ln, label="first mixed launch")
        assert e.last_kernel() == Engine.KERNEL_MIXED
        for _ in range(40):
            run_device(e, buf, off, ln)
        assert e.last_kernel() == Engine.KERNEL_MIXED  # sticky through its own reports
        check(e, buf, off, ln, label="mixed traffic")
    finally:
        e.close()
    e = Engine(0)
    try:
        buf, off, ln = synth.uniform_batch(4096, 1500, seed=6)
        kinds = []
        for _ in range(24):
            run_device(e, buf, off, ln)
            kinds.append(e.last_kernel())
        assert kinds[:16] == [Engine.KERNEL_MIXED] * 16 and kinds[16:] == [Engine.KERNEL_ONE_PASS] * 8, kinds
        check(e, buf, off, ln, label="uniform traffic after the window")
        assert e.last_kernel() == Engine.KERNEL_ONE_PASS
    finally:
        e.close()


@pytest.mark.parametrize("seed", [81, 82])
def test_random_giant_mix(engine, seed):
    """Tiles mixing frames beyond mode B's reach (60 KB .. 400 KB: valid TCP/UDP frames up to IP's
    64-KB TotalLength, random bytes past it) with short and MTU frames, at every byte alignment:
    whatever kernel the column runs (the segment kernel's chunks cut them into up to 16 segments,
    the piece kernel falls back to one group per frame), bit-exact against the oracle."""
    import random

    import framegen
    rnd = random.Random(seed)
    frames = []
    for _ in range(48):  # 48 tiles of 16 frames
        tile = []
        for _ in range(rnd.choice([1, 1, 2, 3])):
            if rnd.random() < 0.5:
                tile.append(framegen.valid_frame(rnd, proto=rnd.choice([6, 17]), payload=rnd.randrange(60000, 65400)))
            else:
                tile.append(rnd.randbytes(rnd.randrange(65536, 400000)))
        while len(tile) < 16:
            r = rnd.random()
            tile.append(framegen.valid_frame(rnd, proto=rnd.choice([6, 17]),
                                             payload=rnd.randrange(0, 40) if r < 0.5 else rnd.randrange(400, 1446)))
        rnd.shuffle(tile)
        frames.extend(tile)
    buf, off, ln = pack_frames(frames, align=1)
    check(engine, buf, off, ln, label=f"random giant mix {seed}")


def test_auto_choice_giant_frames():
    """Tiles that mix a 128-KB frame with 64-B frames: more pieces than the mixed-length kernel's mode B
    covers (6 passes of 16), so it would stream the long frame with one group (~15x slower); the
    kernels report such tiles (kReportMixedGiant) and the automatic choice moves to the segment kernel
    (variant 3), which cuts any frame into equal chunks. Bit-exact before and after the switch; C3-like
    traffic keeps the mixed-length kernel (test_auto_choice_first_launches)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rng = np.random.default_rng(71)
    ln = np.tile(np.array([131072] + [64] * 15, dtype=np.int32), 256)
    off = np.zeros(len(ln), np.int64)
    off[1:] = np.cumsum(ln[:-1].astype(np.int64))
    buf = rng.integers(0, 256, int(off[-1] + ln[-1] + 64), dtype=np.uint8)
    e = Engine(0)
    try:
        check(e, buf, off, ln, label="giant mix, first launch")
        kinds = []
        for _ in range(40):
            run_device(e, buf, off, ln)
            kinds.append(e.last_kernel())
        assert kinds[-1] == Engine.KERNEL_SEGMENTS, kinds
        check(e, buf, off, ln, label="giant mix, segment kernel")
        assert e.last_kernel() == Engine.KERNEL_SEGMENTS
    finally:
        e.close()


def test_host_first_call_kernel_choice():
    """a fresh context's FIRST host-staged call (what a short-lived Go
    RecvEthBatch context makes) runs the one-pass kernel when the batch's lengths lie within 256 B of
    each other (no tile can be mixed), and the mixed-length kernel when they do not; bit-exact
    against the oracle either way. (Device-resident batches keep the initial mixed window: their
    lengths are in device memory.)"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    for label, (b, o, l), expect in (
            ("uniform 1500 B", synth.uniform_batch(2048, 1500, seed=61), Engine.KERNEL_ONE_PASS),
            ("uniform 576..800 B", (None, None, None), Engine.KERNEL_ONE_PASS),
            ("mixed C3", synth.mixed_batch(2048, seed=62), Engine.KERNEL_MIXED)):
        if b is None:  # valid TCP frames of 576..800 B at every start alignment
            import random

            import framegen
            rnd = random.Random(63)
            frames = [framegen.valid_frame(rnd, payload=rnd.randrange(522, 747)) for _ in range(1500)]
            b, o, l = pack_frames(frames, align=1)
            assert 576 <= int(l.min()) and int(l.max()) <= 800
        e = Engine(0)
        try:
            dig, st = e.digest_host(b, o, l)
            assert e.last_kernel() == expect, (label, e.last_kernel())
            edig, est = coracle.digest_batch(b, o, l, nthreads=8)
            for f in ("crc32", "ip_csum", "l4_csum"):
                assert np.array_equal(dig[f], edig[f]), (label, f)
            assert np.array_equal(st, est), label
        finally:
            e.close()


def test_set_kernel_accepts_shipped_variants_only():
    """fs_ctx_set_kernel: 0 (automatic), 2 (mixed-length: pieces), 3 (the segment kernel), 4 (one-pass)
    and 8 (small-frame) only (the losing variants
    were removed from the library)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from seqs_amd import FramesumError

    e = Engine(0)
    try:
        for v in (0, 2, 3, 4, 8):
            e.set_kernel(v)
        for v in (-1, 1, 5, 6, 7, 9):
            with pytest.raises(FramesumError, match="variant"):
                e.set_kernel(v)
    finally:
        e.close()


def test_host_fill_after_failed_digest():
    """a host-staged digest that fails half-way (the test library's
    fs_test_set_fault injects FS_E_NOMEM at chunk 1, after chunk 0's kernel and chunk 1's copy are
    queued on the copy streams; the product library has no such hook) must not
    leave copies in flight that corrupt the next host-staged call's staging: a TX fill right after
    it is byte-exact against the oracle, and so is a digest on a fresh context."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from seqs_amd import FramesumError
    from seqs_amd.framesum import TEST_LIB_PATH

    e = Engine(0, lib_path=TEST_LIB_PATH)
    assert e.lib.fs_test_set_fault(e._ctx, 1) == 0
    try:
        big, boff, bln = synth.uniform_batch(30000, 1500, seed=31)  # 45 MB: three 16-MiB chunks
        with pytest.raises(FramesumError, match="injected"):
            e.digest_host(big, boff.astype(np.uint64), bln.astype(np.uint32))
        assert e.lib.fs_test_set_fault(e._ctx, -1) == 0
        buf, off, ln = synth.mixed_batch(3000, seed=32)
        exp = buf.copy()
        edig, est = coracle.fill_batch(exp, off, ln, 0, 1)
        got = buf.copy()
        dig, st = e.fill_host(got, off, ln, 0, 1)
        assert np.array_equal(got, exp) and np.array_equal(dig, edig) and np.array_equal(st, est)
    finally:
        e.close()


def _dev_batch(buf, off, ln):
    dev = torch.device("cuda:0")
    return (torch.from_numpy(np.ascontiguousarray(buf)).to(dev),
            torch.from_numpy(np.ascontiguousarray(off).astype(np.int64)).to(dev),
            torch.from_numpy(np.ascontiguousarray(ln).astype(np.int32)).to(dev))


def _exact(out, st, buf, off, ln, label, mtu=0):
    crc, ipc, l4c = split_digests(out.cpu().numpy())
    st = st.cpu().numpy()
    dig, est = coracle.digest_batch(buf, off, ln, mtu=mtu, nthreads=8)
    bad = np.nonzero((crc != dig["crc32"]) | (ipc != dig["ip_csum"]) | (l4c != dig["l4_csum"]) | (st != est))[0]
    assert bad.size == 0, f"{label}: {bad.size} mismatches, first at {int(bad[0])}"


def test_auto_choice_short_frames_device():
    """variant 0 on device-resident batches moves to the small-frame kernel
    after kShortLaunchesAuto launches it has seen run with no frame over 128 B, leaves it on the
    first long report, and comes back when short traffic resumes. Short (47-B) and jumbo (9000-B)
    batches alternate; every launch's results are bit-exact against the oracle whichever kernel ran."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    e = Engine(0)
    try:
        sb, so, sl = synth.hello_batch(8192, seed=21)
        jb, jo, jl = synth.uniform_batch(1024, 9000, seed=22)
        ts, tj = _dev_batch(sb, so, sl), _dev_batch(jb, jo, jl)
        seen = []

        def run(t, host, label, k=1):
            for _ in range(k):
                out, st = e.digest_device(*t)
                torch.cuda.synchronize()  # the launch's reports are in before the next launch chooses
                seen.append(e.last_kernel())
                _exact(out, st, *host, label)

        run(ts, (sb, so, sl), "short warm-up", 40)
        assert seen[-1] == Engine.KERNEL_SMALL, seen
        assert Engine.KERNEL_SMALL not in seen[:16], seen  # not before the initial window and the count
        run(tj, (jb, jo, jl), "jumbo after short", 4)
        assert seen[-1] in (Engine.KERNEL_MIXED, Engine.KERNEL_ONE_PASS), seen[-6:]
        run(ts, (sb, so, sl), "short again", 24)
        assert seen[-1] == Engine.KERNEL_SMALL, seen[-26:]
        for r in range(3):  # alternating batch by batch: always exact
            run(tj, (jb, jo, jl), f"alternate jumbo {r}")
            run(ts, (sb, so, sl), f"alternate short {r}")
    finally:
        e.close()


def test_auto_choice_holds_under_sampled_reports():
    """The kernels' report posts are sampled on steady traffic (ran on every 4th launch under variant
    0, the mixed-length kernel's own mixed posts on every 32nd): 300 launches of mixed traffic keep
    the mixed-length kernel from the first launch on, and 300 launches of uniform 1500-B traffic run
    the 4-lane kernels and never the small-frame kernel (every sampled "ran" carries the long flag,
    so no launch is counted short). Bit-exact at the end of each run."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    for label, (b, o, l), expect in (("mixed", synth.mixed_batch(4096, seed=31), {Engine.KERNEL_MIXED}),
                                     ("uniform", synth.uniform_batch(4096, 1500, seed=32),
                                      {Engine.KERNEL_MIXED, Engine.KERNEL_ONE_PASS})):
        e = Engine(0)
        try:
            t = _dev_batch(b, o, l)
            seen = []
            for i in range(300):
                out, st = e.digest_device(*t)
                seen.append(e.last_kernel())
                if i == 0 or i % 25 == 24:
                    torch.cuda.synchronize()  # let reports land now and then, as a paced caller would
            torch.cuda.synchronize()
            assert set(seen) <= expect, (label, sorted(set(seen)))
            if label == "uniform":
                assert seen[-1] == Engine.KERNEL_ONE_PASS, seen[-5:]
            _exact(out, st, b, o, l, f"sampled reports, {label}")
        finally:
            e.close()


def test_variant8_leaves_small_kernel_on_jumbo_frames():
    """with variant 8 a batch of jumbo frames runs the small-frame kernel only
    until its long report arrives; the launches after it run the 4-lane kernels, within 2x of the
    automatic choice, and short traffic brings the small-frame kernel back. Bit-exact throughout."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    jb, jo, jl = synth.uniform_batch(8192, 9000, seed=23)
    sb, so, sl = synth.hello_batch(4096, seed=24)
    tj, ts = _dev_batch(jb, jo, jl), _dev_batch(sb, so, sl)

    def timed(e, k=10):
        out, st = e.digest_device(*tj)
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(k):
            out, st = e.digest_device(*tj)
        t1.record()
        torch.cuda.synchronize()
        return t0.elapsed_time(t1) / k, out, st

    e8, e0 = Engine(0), Engine(0)
    try:
        e8.set_kernel(8)
        out, st = e8.digest_device(*tj)  # the first launch: the small-frame kernel (no report yet)
        torch.cuda.synchronize()
        assert e8.last_kernel() == Engine.KERNEL_SMALL
        _exact(out, st, jb, jo, jl, "variant 8, first jumbo launch")
        ms8, out, st = timed(e8)
        assert e8.last_kernel() in (Engine.KERNEL_MIXED, Engine.KERNEL_ONE_PASS)
        _exact(out, st, jb, jo, jl, "variant 8 after the long report")
        for _ in range(20):
            timed(e0, 1)  # past variant 0's initial window
        ms0, _, _ = timed(e0)
        assert ms8 <= 2.0 * ms0, (ms8, ms0)
        for _ in range(4):
            out, st = e8.digest_device(*ts)
            torch.cuda.synchronize()
        assert e8.last_kernel() == Engine.KERNEL_SMALL
        _exact(out, st, sb, so, sl, "variant 8, short again")
    finally:
        e8.close()
        e0.close()


@pytest.mark.parametrize("pinned_results", [False, True])
def test_host_small_batch_read_in_place(pinned_results):
    """fs_digest_batch_host with frames, offsets and lengths all in pinned host memory and every
    frame <= 128 B: the small-frame kernel reads them in place over PCIe (no staging copies) and
    writes the results to host memory (into the caller's arrays when they are pinned). Bit-exact
    against the oracle, including frames at odd offsets and a frames base at 16k + 4."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from seqs_amd.framesum import DIGEST_DTYPE

    from seqs_amd.framesum import TEST_LIB_PATH

    e = Engine(0, lib_path=TEST_LIB_PATH)
    try:
        import framegen
        frames = [f for f in framegen.edge_batch(41, n_random=3000) if len(f) <= 128]
        hb, ho, hl = synth.hello_batch(3000, seed=42)
        frames += [bytes(hb[int(o):int(o) + int(l)]) for o, l in zip(ho, hl)]
        buf, off, ln = pack_frames(frames, align=1)
        assert int(ln.max()) <= 128 and len(ln) > 3000
        n = len(ln)
        pin = e.host_empty((len(buf) + 4,), np.uint8)
        view = pin[4:]  # a base at 16k + 4
        view[:] = buf
        desc = e.host_empty((12 * n,), np.uint8)
        poff, plen = desc[: 8 * n].view(np.uint64), desc[8 * n:].view(np.uint32)
        poff[:] = off
        plen[:] = ln
        if pinned_results:
            out, st = e.host_empty((n,), DIGEST_DTYPE), e.host_empty((n,), np.uint8)
        else:
            out, st = np.zeros(n, DIGEST_DTYPE), np.zeros(n, np.uint8)
        # in place: every array pinned; staged (path 1): the same frames from pageable memory
        for frames_arg, path in ((view, 2), (buf, 1)):
            for mtu in (0, 1514):
                out[:] = np.zeros(1, DIGEST_DTYPE)
                st[:] = 0xFF
                e.digest_host(frames_arg, poff, plen, mtu=mtu, out=out, status=st)
                assert e.last_kernel() == Engine.KERNEL_SMALL
                assert e.lib.fs_test_last_host_path(e._ctx) == path
                dig, est = coracle.digest_batch(buf, off, ln, mtu=mtu, nthreads=8)
                assert np.array_equal(out["crc32"], dig["crc32"]) and np.array_equal(out["ip_csum"], dig["ip_csum"])
                assert np.array_equal(out["l4_csum"], dig["l4_csum"]) and np.array_equal(st, est)
    finally:
        e.close()


@pytest.mark.parametrize("pinned_results", [False, True])
def test_host_inplace_refilled_buffer(pinned_results):
    """ONE fs_host_alloc frames buffer and ONE descriptor buffer, refilled by the host
    with new random contents before each of 200 in-place calls (path 2, as the Go binding reuses its
    staging buffer): every call reads the new bytes, never lines cached from an earlier launch.
    Lengths, offsets and contents change per call; pinned and pageable result arrays."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from seqs_amd.framesum import DIGEST_DTYPE, TEST_LIB_PATH

    e = Engine(0, lib_path=TEST_LIB_PATH)
    try:
        n, cap = 2048, 2048 * 132 + 64
        pin = e.host_empty((cap,), np.uint8)
        desc = e.host_empty((12 * n,), np.uint8)
        poff, plen = desc[: 8 * n].view(np.uint64), desc[8 * n:].view(np.uint32)
        if pinned_results:
            out, st = e.host_empty((n,), DIGEST_DTYPE), e.host_empty((n,), np.uint8)
        else:
            out, st = np.zeros(n, DIGEST_DTYPE), np.zeros(n, np.uint8)
        for it in range(200):
            rng = np.random.default_rng(1000 + it)
            hb, ho, hl = synth.hello_batch(n, seed=it)
            ln = rng.integers(0, 129, size=n).astype(np.uint32)
            valid = rng.random(n) < 0.5  # half the frames: valid UDP frames (47 B), checksums verified
            ln[valid] = hl[valid]
            gaps = rng.integers(0, 4, size=n).astype(np.uint64)
            off = np.zeros(n, np.uint64)
            off[1:] = np.cumsum(ln[:-1].astype(np.uint64) + gaps[:-1])
            off += np.uint64(rng.integers(0, 4))
            assert int(off[-1]) + int(ln[-1]) <= cap
            buf = rng.integers(0, 256, size=cap, dtype=np.uint8)
            for i in np.nonzero(valid)[0]:
                o = int(off[i])
                buf[o:o + int(ln[i])] = hb[int(ho[i]):int(ho[i]) + int(hl[i])]
            pin[:] = buf
            poff[:] = off
            plen[:] = ln
            out[:] = np.zeros(1, DIGEST_DTYPE)
            st[:] = 0xFF
            e.digest_host(pin, poff, plen, out=out, status=st)
            assert e.lib.fs_test_last_host_path(e._ctx) == 2
            dig, est = coracle.digest_batch(buf, off.astype(np.int64), ln.astype(np.int32), nthreads=8)
            bad = np.nonzero((out["crc32"] != dig["crc32"]) | (out["ip_csum"] != dig["ip_csum"]) |
                             (out["l4_csum"] != dig["l4_csum"]) | (st != est))[0]
            assert bad.size == 0, (it, bad[:5])
    finally:
        e.close()
