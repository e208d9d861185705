"""Synthetic frame batches for the benchmark configurations (BASELINE.json `configs`).

Frames are what stacks.PortStack.RecvEth receives (no FCS): Ethernet 14 B +
IPv4 20 B (IHL 5) + TCP 20 B (offset 5) or UDP 8 B + random payload, with
valid IPv4 and L4 checksums (so RecvEth would accept them), random MACs,
addresses, ports and sequence numbers. Checksums are filled with vectorised
numpy one's-complement arithmetic following the reference's formulas
(eth/headers.go:333-340, :382-393, :510-527); tests/test_synth.py checks every
generated frame against the CPU oracle.

Batch layout: frames packed back to back in one uint8 buffer, frame i at
offsets[i] (int64) with lengths[i] (int32) — the fs_digest_batch descriptor.
"""
from __future__ import annotations

import numpy as np

ETH, IP, TCP, UDP = 14, 20, 20, 8


def _fold_not(s: np.ndarray) -> np.ndarray:
    s = s.astype(np.uint64)
    while True:
        hi = s >> np.uint64(16)
        if not hi.any():
            break
        s = (s & np.uint64(0xFFFF)) + hi
    return (~s.astype(np.uint32)) & np.uint32(0xFFFF)


def _be_word_sum(a: np.ndarray) -> np.ndarray:
    """Sum of big-endian 16-bit words of each row (odd tail padded with a zero low byte)."""
    odd = a.shape[1] % 2
    even = np.ascontiguousarray(a[:, : a.shape[1] - odd])
    s = even.view(">u2").sum(axis=1, dtype=np.uint64)
    if odd:
        s = s + a[:, -1].astype(np.uint64) * np.uint64(256)
    return s


def _put16(a: np.ndarray, col: int, v: np.ndarray) -> None:
    a[:, col] = (v >> 8) & 0xFF
    a[:, col + 1] = v & 0xFF


def make_frames(n: int, frame_len: int, proto: int, rng: np.random.Generator) -> np.ndarray:
    """n valid frames of one length and protocol (6 = TCP, 17 = UDP) as an (n, frame_len) array."""
    l4h = TCP if proto == 6 else UDP
    if frame_len < ETH + IP + l4h:
        raise ValueError("frame too short for its headers")
    f = rng.integers(0, 256, size=(n, frame_len), dtype=np.uint8)
    tl = frame_len - ETH
    # Ethernet: random unicast dst/src MACs, EtherType IPv4.
    f[:, 0] &= 0xFE
    f[:, 12], f[:, 13] = 0x08, 0x00
    # IPv4 header.
    f[:, 14] = 0x45
    f[:, 15] = 0
    _put16(f, 16, np.full(n, tl, np.uint32))
    f[:, 20], f[:, 21] = 0x40, 0x00  # DF
    f[:, 22] = 64
    f[:, 23] = proto
    f[:, 24] = f[:, 25] = 0
    ipc = _fold_not(_be_word_sum(f[:, 14:34]))
    _put16(f, 24, ipc)
    seg = f[:, 34:]
    # ports never zero (RecvEth rejects zero ports, portstack.go:231, :292)
    seg[:, 0] |= 0x01
    seg[:, 2] |= 0x01
    pseudo = _be_word_sum(f[:, 26:34]) + np.uint64(proto)
    if proto == 6:
        seg[:, 12] = 0x50  # data offset 5
        seg[:, 13] = 0x18  # PSH|ACK
        seg[:, 16] = seg[:, 17] = 0
        seg[:, 18] = seg[:, 19] = 0  # urgent pointer (not summed by the reference anyway)
        pseudo = pseudo + np.uint64(tl - IP)
    else:
        ulen = tl - IP
        _put16(seg, 4, np.full(n, ulen, np.uint32))
        seg[:, 6] = seg[:, 7] = 0
        pseudo = pseudo + np.uint64(ulen)
    l4c = _fold_not(_be_word_sum(seg) + pseudo)
    _put16(seg, 16 if proto == 6 else 6, l4c)
    return f


def uniform_batch(n: int, frame_len: int = 1500, seed: int = 1, proto: int = 6):
    """C1/C2 workload: n frames of frame_len bytes (TCP), packed back to back."""
    rng = np.random.default_rng(seed)
    f = make_frames(n, frame_len, proto, rng)
    buf = np.concatenate([f.reshape(-1), np.zeros(16, np.uint8)])
    offsets = np.arange(n, dtype=np.int64) * frame_len
    lengths = np.full(n, frame_len, dtype=np.int32)
    return buf, offsets, lengths


MIXED_LENGTHS = (64, 576, 1500, 9000)


def mixed_batch(n: int, seed: int = 2):
    """C3 workload: lengths cycling 64/576/1500/9000, TCP and UDP alternating (50/50)."""
    rng = np.random.default_rng(seed)
    lens = np.array(MIXED_LENGTHS, dtype=np.int64)[np.arange(n) % 4]
    protos = np.where((np.arange(n) // 4) % 2 == 0, 6, 17)
    lengths = lens.astype(np.int32)
    offsets = np.zeros(n, dtype=np.int64)
    if n > 1:
        offsets[1:] = np.cumsum(lens[:-1])
    total = int(lens.sum())
    buf = np.zeros(total + 16, dtype=np.uint8)
    for L in MIXED_LENGTHS:
        for p in (6, 17):
            idx = np.nonzero((lens == L) & (protos == p))[0]
            if idx.size == 0:
                continue
            f = make_frames(idx.size, L, p, rng)
            pos = offsets[idx][:, None] + np.arange(L, dtype=np.int64)[None, :]
            buf[pos.reshape(-1)] = f.reshape(-1)
    return buf, offsets, lengths


HELLO_LEN = ETH + IP + UDP + 5  # 47 B


def hello_batch(n: int, seed: int = 0, stride: int = 48):
    """The reference's own benchmark shape (stacks/benchmark_test.go:12-46, 67-98): UDP frames
    carrying the 5-byte payload "hello" (47 B), built as NoisyUDPSource.WritePacket builds them:
    Ethernet dst 01:00:00:00:00:00, EtherType IPv4; IPv4 VersionAndIHL 5 (Put writes 0x45,
    eth/headers.go:289-301), TTL 64, protocol 17, destination 192.168.1.1, total length 33; UDP
    destination port 67, length 13; valid IPv4 and UDP checksums. randomizeSource's fields come
    from one 63-bit value per frame (Ethernet source = its 6 low bytes, IPv4 source = its 4 low
    bytes, UDP source port = bits 32..47, IP ID = low16 ^ bits 16..31), drawn here from numpy's
    PRNG, not Go's math/rand (seed 0). Frames sit `stride` bytes apart (48: dword-aligned slots)."""
    if stride < HELLO_LEN:
        raise ValueError("stride below the frame length")
    rng = np.random.default_rng(seed)
    v = rng.integers(0, 1 << 63, size=n, dtype=np.int64).astype(np.uint64)
    b = lambda k: ((v >> np.uint64(8 * k)) & np.uint64(0xFF)).astype(np.uint8)  # noqa: E731
    f = np.zeros((n, HELLO_LEN), np.uint8)
    f[:, 0] = 0x01
    for k in range(6):
        f[:, 6 + k] = b(k)
    f[:, 12], f[:, 13] = 0x08, 0x00
    f[:, 14] = 0x45
    _put16(f, 16, np.full(n, IP + UDP + 5, np.uint32))
    ipid = ((v & np.uint64(0xFFFF)) ^ ((v >> np.uint64(16)) & np.uint64(0xFFFF))).astype(np.uint32)
    _put16(f, 18, ipid)
    f[:, 22] = 64
    f[:, 23] = 17
    for k in range(4):
        f[:, 26 + k] = b(k)
    f[:, 30:34] = (192, 168, 1, 1)
    _put16(f, 24, _fold_not(_be_word_sum(f[:, 14:34])))
    sport = ((v >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.uint32)
    _put16(f, 34, sport)
    _put16(f, 36, np.full(n, 67, np.uint32))
    _put16(f, 38, np.full(n, UDP + 5, np.uint32))
    f[:, 42:47] = np.frombuffer(b"hello", np.uint8)
    pseudo = _be_word_sum(f[:, 26:34]) + np.uint64(17) + np.uint64(UDP + 5)
    _put16(f, 40, _fold_not(_be_word_sum(f[:, 34:]) + pseudo))
    buf = np.zeros(n * stride + 16, np.uint8)
    buf[: n * stride].reshape(n, stride)[:, :HELLO_LEN] = f
    offsets = np.arange(n, dtype=np.int64) * stride
    lengths = np.full(n, HELLO_LEN, dtype=np.int32)
    return buf, offsets, lengths
