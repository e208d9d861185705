"""Edge-case frame generator for parity tests (test infrastructure).

Produces the cases the reference's own tests and RecvEth's gates exercise
(stacks/portstack.go:163-308, eth/headers_test.go, stacks/fuzz_test.go):
valid TCP/UDP frames with and without IP/TCP options, odd lengths, trailing
Ethernet padding, corrupted checksums, computed-checksum 0x0000 (sum folds to
0xFFFF), all-zero segments, every RecvEth rejection class (short frames,
non-IPv4, ARP, bad version/IHL/TotalLength incl. uint16 wrap, unknown proto,
short L4, zero ports, bad UDP length, bad TCP offset) and sub-4-byte frames.
Checksums of "valid" frames are filled with the pure-Python restatement.
"""
from __future__ import annotations

import random
import struct
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import pyref  # noqa: E402


def _ip_header(total_length: int, proto: int, ihl: int, rnd: random.Random, version: int = 4) -> bytearray:
    h = bytearray(rnd.randbytes(ihl * 4))
    h[0] = (version << 4) | ihl
    struct.pack_into(">H", h, 2, total_length & 0xFFFF)
    h[9] = proto
    h[10:12] = b"\0\0"
    ihdr, _ = pyref.decode_ipv4_header(bytes(h[:20]))
    struct.pack_into(">H", h, 10, ihdr.calculate_checksum())
    return h


def _fill_l4(frame: bytearray, corrupt: bool, rnd: random.Random) -> None:
    v, ipc, got = pyref.recv_eth(bytes(frame))
    if v not in (pyref.FS_OK, pyref.FS_ERR_CHECKSUM):
        return
    ihl = frame[14] & 0xF
    off = 14 + ihl * 4
    pos = off + (16 if frame[23] == 6 else 6)
    struct.pack_into(">H", frame, pos, 0)
    _, _, got = pyref.recv_eth(bytes(frame))
    if corrupt:
        got ^= 1 << rnd.randrange(16)
    struct.pack_into(">H", frame, pos, got)


def valid_frame(rnd: random.Random, proto: int = 6, payload: int | None = None, ip_opts: int = 0,
                tcp_opts: int = 0, pad: int = 0, corrupt: bool = False) -> bytes:
    if payload is None:
        payload = rnd.randrange(0, 1500)
    ihl = 5 + ip_opts
    l4h = (20 + 4 * tcp_opts) if proto == 6 else 8
    tl = ihl * 4 + l4h + payload
    eth = bytearray(rnd.randbytes(12)) + b"\x08\x00"
    ip = _ip_header(tl, proto, ihl, rnd)
    l4 = bytearray(rnd.randbytes(l4h + payload))
    struct.pack_into(">HH", l4, 0, rnd.randrange(1, 65536), rnd.randrange(1, 65536))
    if proto == 6:
        l4[12] = ((5 + tcp_opts) << 4) | (l4[12] & 0x0F)
    else:
        struct.pack_into(">H", l4, 4, 8 + payload)
    frame = eth + ip + l4 + bytearray(rnd.randbytes(pad))
    _fill_l4(frame, corrupt, rnd)
    return bytes(frame)


def zero_sum_frame(rnd: random.Random, proto: int = 6) -> bytes:
    """A valid frame whose computed L4 checksum is 0x0000 (the fold hits 0xFFFF)."""
    for _ in range(200):
        f = bytearray(valid_frame(rnd, proto, payload=rnd.randrange(2, 400) & ~1))
        ihl = f[14] & 0xF
        off = 14 + ihl * 4
        pos = off + (16 if proto == 6 else 6)
        struct.pack_into(">H", f, pos, 0)
        # pick a payload word w so that the one's-complement sum becomes 0xFFFF
        wpos = len(f) - 2
        struct.pack_into(">H", f, wpos, 0)
        _, _, got = pyref.recv_eth(bytes(f))
        partial = (~got) & 0xFFFF  # folded sum without w (got = ~fold)
        w = (0xFFFF - partial) % 0xFFFF or 0xFFFF
        struct.pack_into(">H", f, wpos, w)
        _, _, got = pyref.recv_eth(bytes(f))
        if got == 0:
            struct.pack_into(">H", f, pos, 0)
            return bytes(f)
    raise RuntimeError("could not build a zero-checksum frame")


def malformed_frames(rnd: random.Random) -> list[bytes]:
    out = []
    base = bytearray(valid_frame(rnd, 6, payload=100))
    out.append(bytes(base[: rnd.randrange(0, 34)]))  # errPacketSmol
    out += [bytes(rnd.randbytes(k)) for k in range(0, 5)]  # tiny frames incl. len < 4
    f = bytearray(base); f[12:14] = b"\x86\xdd"; out.append(bytes(f))  # IPv6 ethertype -> ignored
    f = bytearray(base); f[12:14] = b"\x08\x06"; out.append(bytes(f))  # ARP
    f = bytearray(base[:40]); f[12:14] = b"\x08\x06"; out.append(bytes(f))  # short ARP
    f = bytearray(base); f[14] = 0x65; out.append(bytes(f))  # version 6
    f = bytearray(base); f[14] = 0x44; out.append(bytes(f))  # IHL 4
    f = bytearray(base); struct.pack_into(">H", f, 16, len(f)); out.append(bytes(f))  # TL > len-14
    f = bytearray(base); struct.pack_into(">H", f, 16, 10); out.append(bytes(f))  # TL < IHL*4
    f = bytearray(base); struct.pack_into(">H", f, 16, 65530); out.append(bytes(f))  # 14+TL wraps
    f = bytearray(base); f[23] = 1; out.append(bytes(f))  # ICMP -> unknown proto
    f = bytearray(base); struct.pack_into(">H", f, 16, 20 + 10); out.append(bytes(f))  # TCP too short
    u = bytearray(valid_frame(rnd, 17, payload=50))
    f = bytearray(u); struct.pack_into(">H", f, 16, 20 + 5); out.append(bytes(f))  # UDP too short
    f = bytearray(base); struct.pack_into(">H", f, 34, 0); out.append(bytes(f))  # zero sport
    f = bytearray(u); struct.pack_into(">H", f, 36, 0); out.append(bytes(f))  # zero dport
    f = bytearray(u); struct.pack_into(">H", f, 38, 7); out.append(bytes(f))  # UDP length < 8
    f = bytearray(base); f[46] = 0x40 | (f[46] & 0xF); out.append(bytes(f))  # TCP offset 4
    f = bytearray(base); f[46] = 0xF0 | (f[46] & 0xF); struct.pack_into(">H", f, 16, 20 + 40); out.append(bytes(f))  # offset > l4len
    f = bytearray(u); struct.pack_into(">H", f, 40, 0); out.append(bytes(f))  # UDP csum 0 (not special-cased)
    z = bytearray(base); z[34:] = bytes(len(z) - 34); z[35] = 1; z[37] = 1; out.append(bytes(z))
    return out


def edge_batch(seed: int, n_random: int = 200) -> list[bytes]:
    rnd = random.Random(seed)
    frames: list[bytes] = []
    for p in (6, 17):
        for payload in (0, 1, 2, 3, 4, 5, 6, 7, 9, 10, 63, 64, 65, 255, 1446 if p == 6 else 1472):
            frames.append(valid_frame(rnd, p, payload=payload))
    frames.append(valid_frame(rnd, 6, payload=300, ip_opts=10, tcp_opts=10))
    frames.append(valid_frame(rnd, 17, payload=301, ip_opts=3))
    frames.append(valid_frame(rnd, 6, payload=8986 - 40))  # 9000-B jumbo
    frames.append(valid_frame(rnd, 6, payload=10, pad=6))  # min-size frame with Ethernet padding
    frames.append(valid_frame(rnd, 17, payload=3, pad=17))
    frames.append(zero_sum_frame(rnd, 6))
    frames.append(zero_sum_frame(rnd, 17))
    frames += malformed_frames(rnd)
    for _ in range(n_random):
        p = rnd.choice((6, 17))
        frames.append(valid_frame(rnd, p, payload=rnd.randrange(0, 1600), ip_opts=rnd.choice((0, 0, 0, 1, 5, 10)),
                                  tcp_opts=rnd.choice((0, 0, 3, 10)), pad=rnd.choice((0, 0, 0, 1, 2, 3, 17)),
                                  corrupt=rnd.random() < 0.2))
    rnd.shuffle(frames)
    return frames
