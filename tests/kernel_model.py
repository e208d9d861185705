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


def crc32_tile_segments(buf: bytes, frames: list[tuple[int, int]], base_phase: int = 0, groups: int = 16,
                        model_tail_select: bool = True) -> list[int]:
    """The segment kernel (digest_kernel_g): a tile's frames as BLOCK-ALIGNED 64-B
    rows (the one-pass kernel's rows), concatenated in frame order (frames of no stream dword left
    out) and cut into `groups` equal chunks of L = ceil(T / groups) rows; group g streams its chunk
    [gL, min(gL + L, T)) through one set of 16 streams, crossing frame boundaries:
      * a frame's head rows (its first block; the second too when dword 1 lies there) get the head
        mask and the CRC init (the streams are zero there: the previous segment was parked);
      * a frame's last block keeps the streams past its last dword untouched (the one-pass tail row);
      * the row that ends a segment (the frame's last block, or the chunk's last row) PARKS the
        streams as segment (rank k, group g) = slot k + g and restarts them from zero.
    After the rows every parked segment is combined like a one-pass frame (q = the frame's last
    dword's block position for its tail segment, 15 for a segment cut by its chunk's end) and
    shifted by its distance to the frame end (64 dblk - 4 ealign bytes); a frame's register is the
    XOR of its segments'. Returns the CRC-32 of every frame (zlib's value)."""
    padded = b"\0" * 64 + bytes(buf) + b"\0" * 136

    def dword(i):
        return struct.unpack_from("<I", padded, 64 + 4 * i)[0]

    info = []
    for S, ln in frames:
        sdw, sa = S >> 2, S & 3
        nd = ((S + ln + 3) >> 2) - sdw if ln >= 4 else 0
        ph = (base_phase + sdw) & 15
        ealign = (16 - ((ph + nd) & 15)) & 15
        nb = (ph + nd + ealign) >> 4 if nd > 0 else 0
        te = ((S + ln) & 3) or 4
        info.append(dict(S=S, ln=ln, sdw=sdw, sa=sa, nd=nd, ph=ph, ealign=ealign, nb=nb, te=te))
    ranked = [i for i, f in enumerate(info) if f["nb"] > 0]
    vs, T = [], 0
    for i in ranked:
        vs.append(T)
        T += info[i]["nb"]
    L = -(-T // groups) if T else 0
    slots = {}
    for g in range(groups):
        v0, v1 = g * L, min(g * L + L, T)
        A = [[0] * 4 for _ in range(4)]
        k = 0
        for v in range(v0, v1):
            while vs[k] + info[ranked[k]]["nb"] <= v:
                k += 1
            f = info[ranked[k]]
            hm = (0xFFFFFFFF << (8 * f["sa"])) & 0xFFFFFFFF
            tm = 0xFFFFFFFF if f["te"] == 4 else (1 << (8 * f["te"])) - 1
            rowdw0 = f["sdw"] - f["ph"] + 16 * (v - vs[k])  # absolute dword of the block's position 0
            for lane in range(4):
                for j in range(4):
                    x = 16 * (v - vs[k]) + 4 * lane + j - f["ph"]  # frame dword
                    d = dword(rowdw0 + 4 * lane + j)
                    c = 0
                    if x < 0:
                        d = 0
                    if x == 0:
                        d &= hm
                        c = hm
                    if x == 1:
                        c = ~hm & 0xFFFFFFFF
                    if x == f["nd"] - 1:
                        d &= tm
                    if x < f["nd"] or not model_tail_select:
                        A[lane][j] = apply(Z64, A[lane][j]) ^ d ^ c
            vend = vs[k] + f["nb"]
            if v == min(vend, v1) - 1:
                assert k + g not in slots
                slots[k + g] = (k, [a[:] for a in A], vend - 1 - v)
                A = [[0] * 4 for _ in range(4)]
    assert len(slots) <= len(ranked) + groups - 1 and all(s < len(ranked) + groups - 1 for s in slots)
    Yk = [0] * len(ranked)
    for s, (k, A, dblk) in slots.items():
        f = info[ranked[k]]
        q = 15 - f["ealign"] if dblk == 0 else 15
        y = 0
        for lane in range(4):
            for j in range(4):
                p = 4 * lane + j
                y ^= zero_shift(A[lane][j], 4 * ((q - p) % 16))
        if dblk:
            y = zero_shift(y, 64 * dblk - 4 * f["ealign"])
        Yk[k] ^= y
    out = []
    for i, f in enumerate(info):
        if f["nb"] == 0:
            out.append(crc32_model(buf, f["S"], f["ln"]))
            continue
        Y = Yk[ranked.index(i)]
        t = (4 - ((f["S"] + f["ln"]) & 3)) & 3
        out.append(apply(ZFIN[t], Y) ^ 0xFFFFFFFF)
    return out
