"""Pure-Python model of the framesum kernel's arithmetic decomposition (test infrastructure).

It mirrors seqs_amd/csrc/framesum_kernel.hip step by step — end-anchored
64-byte rows, 4 lanes x 4 dword streams per frame with A <- Z64(A) ^ w,
the intra-lane Z4 Horner, the Z32/Z16 lane tree, the final Z_(4-t) step that
also removes the <=3 zero bytes of the dword rounding, the 4-byte init trick,
and the native-domain (little-endian dword) one's-complement sum streamed from
frame dword 10 with exact head/padding corrections — so the algebra can be
checked on CPU against zlib / the oracle before and independently of the GPU.
Small inputs only.
"""
from __future__ import annotations

import struct

POLY = 0xEDB88320


def _t1():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ POLY if c & 1 else c >> 1
        t.append(c)
    return t


T1 = _t1()
INV = [0] * 256
for _j, _v in enumerate(T1):
    INV[_v >> 24] = _j


def zero_shift(r: int, nbytes: int) -> int:
    for _ in range(nbytes):
        r = (r >> 8) ^ T1[r & 0xFF]
    return r


def op_table(nbytes: int):
    return [[zero_shift(v << (8 * b), nbytes) for v in range(256)] for b in range(4)]


Z64, Z4, Z32, Z16 = op_table(64), op_table(4), op_table(32), op_table(16)
ZFIN = [op_table(4 - t) for t in range(4)]  # final step Z_(4-t)


def apply(tab, a: int) -> int:
    return tab[0][a & 0xFF] ^ tab[1][(a >> 8) & 0xFF] ^ tab[2][(a >> 16) & 0xFF] ^ tab[3][a >> 24]


def crc32_model(buf: bytes, S: int, length: int) -> int:
    """CRC-32 of buf[S:S+length] computed the way the kernel does (dword grid of `buf`)."""
    E = S + length
    if length < 4:
        c = 0xFFFFFFFF
        for b in buf[S:E]:
            c = T1[(c ^ b) & 0xFF] ^ (c >> 8)
        return c ^ 0xFFFFFFFF
    sdw = S >> 2
    fp = (E + 3) >> 2
    nd = fp - sdw
    sa = S & 3
    te = (E & 3) or 4
    head_mask = (0xFFFFFFFF << (8 * sa)) & 0xFFFFFFFF
    init0 = head_mask
    init1 = (1 << (8 * sa)) - 1
    tail_mask = 0xFFFFFFFF if te == 4 else (1 << (8 * te)) - 1
    padded = bytes(buf) + b"\0" * 8

    def dword(rel):
        i = 4 * (sdw + rel)
        return struct.unpack_from("<I", padded, i)[0]

    R = (nd + 15) // 16
    A = [[0] * 4 for _ in range(4)]  # [lane][stream]
    for r in range(R):
        for lane in range(4):
            rel = nd - 16 * R + 16 * r + 4 * lane
            for j in range(4):
                rj = rel + j
                if rj < 0:
                    dc = 0
                else:
                    d = dword(rj)
                    mk, x = 0xFFFFFFFF, 0
                    if rj == 0:
                        mk &= head_mask
                        x ^= init0
                    if rj == 1:
                        x ^= init1
                    if rj == nd - 1:
                        mk &= tail_mask
                    dc = (d & mk) ^ x
                A[lane][j] = apply(Z64, A[lane][j]) ^ dc
    U = []
    for lane in range(4):
        u = apply(Z4, A[lane][0]) ^ A[lane][1]
        u = apply(Z4, u) ^ A[lane][2]
        u = apply(Z4, u) ^ A[lane][3]
        U.append(u)
    V = [apply(Z32, U[l]) ^ U[l ^ 2] for l in range(4)]
    W = apply(Z16, V[0]) ^ V[1]
    t = (4 - (E & 3)) & 3  # zero bytes appended by the dword rounding, removed by Z_(4-t)
    c = apply(ZFIN[t], W)
    return c ^ 0xFFFFFFFF


CSUM_REL0 = 10  # the kernel streams the checksum from frame dword 10


def native_sum(buf: bytes, S: int, p0: int, p1: int) -> int:
    """Exact native-domain sum of frame bytes [p0, p1): byte at absolute address a weighs 256^(a mod 4)."""
    return sum(buf[S + p] << (8 * ((S + p) & 3)) for p in range(p0, p1))


def l4_native_sum(buf: bytes, S: int, length: int, l4s: int, l4e: int) -> tuple[int, int]:
    """The kernel's split of the L4 sum: streamed dwords rel >= 10 (tail-masked at the frame end)
    plus the head correction [l4s, P10) or minus [P10, l4s), minus the Ethernet padding [l4e, len).
    Returns (native sum over [l4s, l4e), parity of the absolute L4 start)."""
    sa = S & 3
    sdw = S >> 2
    E = S + length
    nd = ((E + 3) >> 2) - sdw
    padded = bytes(buf) + b"\0" * 8
    total = 0
    for rel in range(CSUM_REL0, nd):
        w = struct.unpack_from("<I", padded, 4 * (sdw + rel))[0]
        if rel == nd - 1 and (E & 3):
            w &= (1 << (8 * (E & 3))) - 1
        total += w
    p10 = 4 * CSUM_REL0 - sa
    if l4s < p10:
        total += native_sum(buf, S, l4s, p10)
    else:
        total -= native_sum(buf, S, p10, l4s)
    total -= native_sum(buf, S, l4e, length)
    return total, (sa + l4s) & 1


def fold_native_to_be(total: int, parity: int) -> int:
    x = total
    while x >> 16:
        x = (x & 0xFFFF) + (x >> 16)
    r = (~x) & 0xFFFF
    if not parity:
        r = ((r & 0xFF) << 8) | (r >> 8)
    return r


def crc32_model_al(buf: bytes, S: int, length: int, base_phase: int = 0) -> int:
    """digest_kernel_a (the one-pass kernel): BLOCK-ALIGNED 64-byte rows (the last row ends on the 64-B
    block after the frame end; base_phase = absolute dword phase of buf[0] within a block),
    the stream dwords past the frame end leave their stream untouched, and the combine shifts
    stream (lane, j) by 4 * ((q - 4 lane - j) mod 16) bytes, q = the frame's last dword's
    position in the last row."""
    E = S + length
    if length < 4:
        return crc32_model(buf, S, length)
    sdw = S >> 2
    nd = ((E + 3) >> 2) - sdw
    sa = S & 3
    te = (E & 3) or 4
    head_mask = (0xFFFFFFFF << (8 * sa)) & 0xFFFFFFFF
    tail_mask = 0xFFFFFFFF if te == 4 else (1 << (8 * te)) - 1
    padded = b"\0" * 64 + bytes(buf) + b"\0" * 72
    ph = (base_phase + sdw) & 15
    e = (16 - ((ph + nd) & 15)) & 15
    ndb = nd + e
    R = (ph + ndb) // 16

    def dword(rel):
        return struct.unpack_from("<I", padded, 64 + 4 * (sdw + rel))[0]

    A = [[0] * 4 for _ in range(4)]
    for r in range(R):
        for lane in range(4):
            rel = ndb - 16 * R + 16 * r + 4 * lane
            for j in range(4):
                x = rel + j
                d = dword(x) if x >= 0 else 0
                c = 0
                if x == 0:
                    d &= head_mask
                    c = head_mask
                if x == 1:
                    c = ~head_mask & 0xFFFFFFFF
                if x == nd - 1:
                    d &= tail_mask
                if x < nd:
                    A[lane][j] = apply(Z64, A[lane][j]) ^ d ^ c
    # combine: stream j of a lane needs Z_4s, s = (K - j) mod 16, K = q - 4 lane = 4 a + C. Streams
    # j <= C have (a, s & 3) = (a, C - j), the others ((a - 1) & 3, 4 + C - j). Sorted by s & 3
    # (B_c = A_((C - c) & 3)), one round of Z4/Z8/Z12 and one of Z_16a per class.
    q = 15 - e
    Y = 0
    for lane in range(4):
        K = (q - 4 * lane) & 15
        a, C = K >> 2, K & 3
        B = [A[lane][(C - c) & 3] for c in range(4)]
        T = [B[0]] + [apply(op_table(4 * c), B[c]) for c in (1, 2, 3)]
        V1 = V2 = 0
        for c in range(4):
            if c <= C:
                V1 ^= T[c]
            else:
                V2 ^= T[c]
        a2 = (a - 1) & 3
        Y ^= (apply(op_table(16 * a), V1) if a else V1) ^ (apply(op_table(16 * a2), V2) if a2 else V2)
    t = (4 - (E & 3)) & 3
    return apply(ZFIN[t], Y) ^ 0xFFFFFFFF


Z8 = op_table(8)


def crc32_model_lane(buf: bytes, S: int, length: int, chains: int = 1) -> int:
    """The small-frame kernel (digest_kernel_s, one lane per frame): the pending-register Horner
    P <- Z4(P) ^ d over the frame's dwords (head/tail bytes masked, the init XOR-ed into frame
    bytes 0..3), or with chains=2 two Horner chains over the even and the odd dwords
    (E, O <- Z8(.) ^ d) joined at the last dword L: Z4(E) ^ O when L is odd, E ^ Z4(O) when even;
    then the final Z_(4-t)."""
    E_ = S + length
    if length < 4:
        return crc32_model(buf, S, length)
    sa = S & 3
    nd = (sa + length + 3) >> 2
    te = (E_ & 3) or 4
    head = (0xFFFFFFFF << (8 * sa)) & 0xFFFFFFFF
    tail = 0xFFFFFFFF if te == 4 else (1 << (8 * te)) - 1
    padded = bytes(buf) + b"\0" * 8
    ds = []
    for x in range(nd):
        d = struct.unpack_from("<I", padded, 4 * ((S >> 2) + x))[0]
        if x == 0:
            d &= head
        if x == nd - 1:
            d &= tail
        ds.append(d ^ (head if x == 0 else (~head & 0xFFFFFFFF) if x == 1 else 0))
    if chains == 1:
        P = 0
        for d in ds:
            P = apply(Z4, P) ^ d
    else:
        Ev = Od = 0
        for x, d in enumerate(ds):
            if x & 1:
                Od = apply(Z8, Od) ^ d
            else:
                Ev = apply(Z8, Ev) ^ d
        P = (apply(Z4, Ev) ^ Od) if (nd - 1) & 1 else (Ev ^ apply(Z4, Od))
    t = (4 - (E_ & 3)) & 3
    return apply(ZFIN[t], P) ^ 0xFFFFFFFF
