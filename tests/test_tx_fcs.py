"""TX checksum fill (fs_fill_batch) and wire frames with an FCS (fs_digest_batch_fcs).

SURVEY.md §8f rank 2 (TX fill: stacks/port_tcp.go:178/:193, dhcp_client.go:479/:486) and
rank 4 (FCS append / verify; not in the reference). The C oracle (oracle_fill_batch,
oracle_digest_fcs_batch) is checked against the independent Python restatement
(oracle/pyref.fill_frame / frame_digest_fcs) on CPU; the GPU path is compared with the C
oracle byte for byte (the frames as written, digests and verdicts), and round trips
(fill + append -> FCS verify; fill -> RX digest) are checked at the BASELINE sizes.
"""
import random

import numpy as np
import pytest

import engines  # noqa: E402

from oracle import coracle, pyref
from seqs_amd import FCS_APPEND, FILL_CSUM, FS_ERR_FCS, synth

import framegen


def pack_with_room(frames, align=1, room=4, seed=0):
    """Pack frames with `room` spare bytes after each (filled with noise); lengths exclude them."""
    rng = np.random.default_rng(seed)
    lens = np.array([len(f) for f in frames], dtype=np.int64)
    step = (lens + room + align - 1) // align * align
    off = np.zeros(len(frames), dtype=np.int64)
    off[1:] = np.cumsum(step[:-1])
    buf = rng.integers(0, 256, int(off[-1] + step[-1] + 16), dtype=np.uint8)
    for f, o in zip(frames, off):
        buf[o : o + len(f)] = np.frombuffer(f, dtype=np.uint8)
    return buf, off, lens.astype(np.int32)


def stale(frames, seed):
    """The same frames with random bytes in both checksum fields (what a TX path starts from)."""
    rnd = random.Random(seed)
    out = []
    for f in frames:
        b = bytearray(f)
        if len(b) >= 26:
            b[24:26] = rnd.randbytes(2)
        if len(b) >= 34 and b[12:14] == b"\x08\x00":
            off = 14 + (b[14] & 0xF) * 4
            pos = off + (16 if b[23] == 6 else 6)
            if pos + 2 <= len(b):
                b[pos : pos + 2] = rnd.randbytes(2)
        out.append(bytes(b))
    return out


def tx_frames(seed, n_random=300):
    return stale(framegen.edge_batch(seed, n_random=n_random), seed)


# ---------------------------------------------------------------- CPU: oracle vs pyref


@pytest.mark.parametrize("flags", [FILL_CSUM, FCS_APPEND, FILL_CSUM | FCS_APPEND])
def test_oracle_fill_matches_pyref(flags):
    frames = tx_frames(1)
    buf, off, ln = pack_with_room(frames, align=1)
    out, st = coracle.fill_batch(buf, off, ln, 0, flags)
    extra = 4 if flags & FCS_APPEND else 0
    for i, f in enumerate(frames):
        nf, d = pyref.fill_frame(f, 0, flags)
        assert bytes(buf[off[i] : off[i] + ln[i] + extra]) == nf, i
        assert (int(out[i]["crc32"]), int(out[i]["ip_csum"]), int(out[i]["l4_csum"]), int(st[i])) == d, i


def test_oracle_fill_then_recv_accepts():
    frames = tx_frames(2)
    buf, off, ln = pack_with_room(frames)
    before = coracle.digest_batch(buf, off, ln)[1]
    out, st = coracle.fill_batch(buf, off, ln, 0, FILL_CSUM)
    after_dig, after = coracle.digest_batch(buf, off, ln)
    reach = np.isin(before, [0, 13])
    assert reach.sum() > 200 and (before[reach] == 13).any()
    assert (after[reach] == 0).all() and (st[reach] == 0).all()
    assert np.array_equal(after[~reach], before[~reach])
    assert np.array_equal(after_dig, out) and np.array_equal(after, st)


def test_oracle_fcs_verify_matches_pyref():
    frames = framegen.edge_batch(3, n_random=200)
    rnd = random.Random(3)
    wires = []
    for k, f in enumerate(frames):
        fcs = pyref.crc32_ieee(f).to_bytes(4, "little")
        if k % 5 == 1:
            fcs = bytes([fcs[0] ^ 0x10]) + fcs[1:]
        wires.append(f + fcs)
    wires += [b"", b"\x01", b"\x01\x02\x03", b"\x00\x00\x00\x00", rnd.randbytes(4)]
    buf, off, ln = pack_with_room(wires, room=0)
    out, st = coracle.digest_fcs_batch(buf, off, ln)
    for i, w in enumerate(wires):
        assert pyref.frame_digest_fcs(w) == (int(out[i]["crc32"]), int(out[i]["ip_csum"]),
                                             int(out[i]["l4_csum"]), int(st[i])), i
    assert (st == FS_ERR_FCS).sum() >= len(frames) // 5


# ---------------------------------------------------------------- GPU parity


def _dev(x, torch):
    return torch.from_numpy(np.ascontiguousarray(x)).to("cuda:0")


@pytest.fixture(scope="module", params=engines.VARIANTS, ids=engines.IDS)
def engine(request):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    e = engines.engine_for(request.param)
    yield e
    e.close()


def gpu_fill(engine, buf, off, ln, mtu, flags):
    import torch

    tb, to, tl = _dev(buf, torch), _dev(off.astype(np.int64), torch), _dev(ln.astype(np.int32), torch)
    out, st = engine.fill_device(tb, to, tl, mtu=mtu, flags=flags)
    torch.cuda.synchronize()
    w = out.cpu().numpy().view(np.uint32).reshape(-1, 2)
    return tb.cpu().numpy(), w, st.cpu().numpy()


def gpu_fcs(engine, buf, off, ln, mtu=0):
    import torch

    tb, to, tl = _dev(buf, torch), _dev(off.astype(np.int64), torch), _dev(ln.astype(np.int32), torch)
    out, st = engine.digest_fcs_device(tb, to, tl, mtu=mtu)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32).reshape(-1, 2), st.cpu().numpy()


def words(dig):
    return np.stack([dig["crc32"].astype(np.uint32),
                     dig["ip_csum"].astype(np.uint32) | (dig["l4_csum"].astype(np.uint32) << 16)], axis=1)


def check_fill(engine, frames_or_batch, mtu, flags, label, align=1):
    if isinstance(frames_or_batch, tuple):
        buf, off, ln = frames_or_batch
    else:
        buf, off, ln = pack_with_room(frames_or_batch, align=align)
    gbuf, gw, gst = gpu_fill(engine, buf, off, ln, mtu, flags)
    ebuf = buf.copy()
    edig, est = coracle.fill_batch(ebuf, off, ln, mtu, flags)
    diff = np.nonzero(gbuf != ebuf)[0]
    assert diff.size == 0, f"{label}: {diff.size} bytes differ, first at {int(diff[0])}"
    bad = np.nonzero((gw != words(edig)).any(axis=1) | (gst != est))[0]
    assert bad.size == 0, f"{label}: {bad.size} digests differ, first {int(bad[0])} len={int(ln[bad[0]])}"
    return gbuf, gw, gst


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [FILL_CSUM, FCS_APPEND, FILL_CSUM | FCS_APPEND, 0])
def test_gpu_fill_edge(engine, flags):
    for seed in (1, 2):
        frames = tx_frames(seed)
        for align in (1, 4):
            check_fill(engine, frames, 0, flags, f"seed{seed}/align{align}/flags{flags}", align=align)
        check_fill(engine, frames, 1514, flags, f"seed{seed}/mtu/flags{flags}")


@pytest.mark.gpu
def test_gpu_fill_long_and_mixed(engine):
    # jumbo and giant frames beside short ones (mode B tiles), fields at every IHL / TCP offset
    rnd = random.Random(5)
    frames = []
    for L in (60, 64, 100, 576, 769, 1500, 1537, 4000, 9000, 9018, 20000):
        for proto in (6, 17):
            frames.append(framegen.valid_frame(rnd, proto, payload=max(0, L - 54)))
    frames.append(framegen.valid_frame(rnd, 6, payload=1000, pad=600000))
    frames += [rnd.randbytes(rnd.randint(0, 80)) for _ in range(20)]
    check_fill(engine, stale(frames, 5), 0, FILL_CSUM | FCS_APPEND, "long")


@pytest.mark.gpu
def test_gpu_fill_c2_round_trip(engine):
    # BASELINE configs[1] shape with 4 spare bytes per frame: fill + append on the GPU equals
    # the oracle byte for byte; the FCS verify of the written wire frames passes everywhere
    import torch

    n, L = 65536, 1500
    rng = np.random.default_rng(21)
    f = synth.make_frames(n, L, 6, rng)
    f[:, 24:26] = rng.integers(0, 256, (n, 2), dtype=np.uint8)  # stale checksums
    f[:, 50:52] = rng.integers(0, 256, (n, 2), dtype=np.uint8)
    stride = L + 4
    buf = np.zeros(n * stride + 16, np.uint8)
    buf[: n * stride].reshape(n, stride)[:, :L] = f
    off = np.arange(n, dtype=np.int64) * stride
    ln = np.full(n, L, np.int32)
    gbuf, gw, gst = check_fill(engine, (buf, off, ln), 0, FILL_CSUM | FCS_APPEND, "C2 fill")
    assert (gst == 0).all()
    w2, st2 = gpu_fcs(engine, gbuf, off, ln + 4)
    assert (st2 == 0).all() and np.array_equal(w2, gw)


@pytest.mark.gpu
def test_gpu_fcs_verify(engine):
    frames = framegen.edge_batch(4, n_random=300)
    rng = np.random.default_rng(4)
    wires = []
    for k, fr in enumerate(frames):
        fcs = bytearray(pyref.crc32_ieee(fr).to_bytes(4, "little"))
        if k % 7 == 3:
            fcs[int(rng.integers(0, 4))] ^= 1 << int(rng.integers(0, 8))
        wires.append(fr + bytes(fcs))
    wires += [b"", b"\x01", b"\x01\x02\x03", b"\x00\x00\x00\x00", b"\x01\x02\x03\x04"]
    for align in (1, 4):
        buf, off, ln = pack_with_room(wires, align=align, room=0)
        for mtu in (0, 1514):
            gw, gst = gpu_fcs(engine, buf, off, ln, mtu)
            edig, est = coracle.digest_fcs_batch(buf, off, ln, mtu)
            bad = np.nonzero((gw != words(edig)).any(axis=1) | (gst != est))[0]
            assert bad.size == 0, f"align{align}/mtu{mtu}: first {int(bad[0])} len={int(ln[bad[0]])}"
    assert (est == FS_ERR_FCS).sum() > len(frames) // 7


@pytest.mark.gpu
def test_gpu_fcs_c3_round_trip(engine):
    # BASELINE configs[2] frames as wire frames (FCS appended on the host by zlib)
    import zlib

    buf0, off0, ln0 = synth.mixed_batch(8192, seed=6)
    wires = []
    for o, l in zip(off0, ln0):
        fr = bytes(buf0[o : o + l])
        wires.append(fr + (zlib.crc32(fr) & 0xFFFFFFFF).to_bytes(4, "little"))
    buf, off, ln = pack_with_room(wires, align=4, room=0)
    gw, gst = gpu_fcs(engine, buf, off, ln)
    edig, est = coracle.digest_fcs_batch(buf, off, ln)
    assert (gst == 0).all() and np.array_equal(gst, est) and np.array_equal(gw, words(edig))


@pytest.mark.gpu
def test_gpu_fill_host_and_calculate_headers(engine):
    # host-staged fill (fs_fill_batch_host) and the reference-shaped list surface, against the
    # Python restatement of the TX header calculation
    frames = tx_frames(7, n_random=200)
    buf, off, ln = pack_with_room(frames, align=1)
    ebuf = buf.copy()
    edig, est = coracle.fill_batch(ebuf, off, ln, 0, FILL_CSUM | FCS_APPEND)
    dig, st = engine.fill_host(buf, off, ln, 0, FILL_CSUM | FCS_APPEND)
    assert np.array_equal(buf, ebuf) and np.array_equal(dig, edig) and np.array_equal(st, est)
    got = engine.calculate_headers_batch(frames, append_fcs=True)
    for f, g in zip(frames, got):
        assert g == pyref.fill_frame(f, 0, FILL_CSUM | FCS_APPEND)[0]
    with pytest.raises(Exception):
        engine.fill_host(np.zeros(100, np.uint8), np.array([90], np.uint64), np.array([8], np.uint32), 0, FCS_APPEND)


@pytest.mark.gpu
def test_gpu_fill_host_large(engine):
    # the host-staged fill of a batch spanning several 16-MiB chunks, from pinned and pageable
    # memory: byte-for-byte equal to the oracle's fill, stale checksum fields and the noise
    # between frames included
    from seqs_amd import synth

    n, flen, room = 28000, 1500, 4
    src, soff, _ = synth.uniform_batch(n, flen, seed=11)
    rng = np.random.default_rng(12)
    off = np.arange(n, dtype=np.int64) * (flen + room + 2)  # 2-B phase steps: every alignment
    buf = rng.integers(0, 256, int(off[-1] + flen + room + 64), dtype=np.uint8)
    idx = off[:, None] + np.arange(flen)[None, :]
    buf[idx] = src[soff[:, None] + np.arange(flen)[None, :]]
    buf[off[:, None] + np.array([24, 25, 50, 51])[None, :]] = rng.integers(0, 256, (n, 4), dtype=np.uint8)
    ln = np.full(n, flen, dtype=np.int32)
    assert int(off[-1]) > 2 * (16 << 20)
    ebuf = buf.copy()
    edig, est = coracle.fill_batch(ebuf, off, ln, 0, FILL_CSUM | FCS_APPEND)
    torch = pytest.importorskip("torch")
    for pinned in (True, False):
        host = torch.empty(buf.size, dtype=torch.uint8).pin_memory().numpy() if pinned else np.empty_like(buf)
        host[:] = buf
        dig, st = engine.fill_host(host, off, ln, 0, FILL_CSUM | FCS_APPEND)
        assert np.array_equal(dig, edig) and np.array_equal(st, est), pinned
        assert (st == 0).all()
        assert np.array_equal(host, ebuf), pinned
