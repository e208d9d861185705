"""CPU check of the kernel's arithmetic decomposition (tests/kernel_model.py mirrors
seqs_amd/csrc/framesum_kernel.hip): stream/lane-tree CRC-32 vs zlib, and the
native-domain one's-complement split vs the reference restatement."""
import random
import zlib

import kernel_model as km
import framegen
from oracle import pyref


def test_crc_decomposition_vs_zlib():
    rnd = random.Random(11)
    for _ in range(400):
        L = rnd.choice([0, 1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 63, 64, 65, 255, 256, 257, 1500, rnd.randrange(0, 4000)])
        pre = rnd.randrange(0, 13)
        buf = rnd.randbytes(pre + L + 8)
        assert km.crc32_model(buf, pre, L) == zlib.crc32(buf[pre : pre + L])


def test_final_step_equals_unshift():
    rnd = random.Random(4)
    for _ in range(200):
        w = rnd.getrandbits(32)
        for t in range(4):
            c = km.apply(km.ZFIN[t], w)
            # Z_(4-t)(W) shifted forward by t bytes is Z_4(W)
            assert km.zero_shift(c, t) == km.apply(km.Z4, w)


def test_tables_properties():
    # Z_a o Z_b = Z_(a+b) on random registers; the one-byte inverse undoes Z_1.
    rnd = random.Random(2)
    for _ in range(200):
        r = rnd.getrandbits(32)
        assert km.apply(km.Z4, km.apply(km.Z4, r)) == km.zero_shift(r, 8)
        assert km.apply(km.Z32, r) == km.apply(km.Z16, km.apply(km.Z16, r))
        assert km.apply(km.Z64, r) == km.zero_shift(r, 64)
        c = km.zero_shift(r, 1)
        j = km.INV[c >> 24]
        assert ((((c ^ km.T1[j]) << 8) & 0xFFFFFFFF) | j) == r
    assert sorted(km.INV) == list(range(256))


def test_l4_native_split_matches_reference():
    # For every frame the reference checksums, the kernel's split (streamed inside dwords +
    # partial bytes + exact pseudo/excluded-word corrections, folded in the native domain)
    # reproduces RecvEth's gotsum bit-exactly, including unaligned frame starts.
    import struct

    frames = framegen.edge_batch(7, n_random=120)
    rnd = random.Random(9)
    checked = 0
    for f in frames:
        v, ipc, got = pyref.recv_eth(f)
        if v not in (pyref.FS_OK, pyref.FS_ERR_CHECKSUM):
            continue
        pre = rnd.randrange(0, 8)
        buf = bytes(rnd.randbytes(pre)) + f + bytes(8)
        ihl = f[14] & 0xF
        l4s, l4e = 14 + 4 * ihl, 14 + struct.unpack(">H", f[16:18])[0]
        total, parity = km.l4_native_sum(buf, pre, len(f), l4s, l4e)
        assert total == km.native_sum(buf, pre, l4s, l4e)
        sa = pre & 3
        proto = f[23]
        skip0 = l4s + (16 if proto == 6 else 6)
        for p in range(skip0, skip0 + (4 if proto == 6 else 2)):
            total -= f[p] << (8 * ((sa + p) & 3))
        lenword = ((struct.unpack(">H", f[16:18])[0] - 4 * ihl) & 0xFFFF) if proto == 6 else struct.unpack(">H", f[l4s + 4 : l4s + 6])[0]
        words = [struct.unpack(">H", f[i : i + 2])[0] for i in (26, 28, 30, 32)] + [proto, lenword]
        for w in words:
            total += w if parity else ((w & 0xFF) << 8) | (w >> 8)
        assert total >= 0
        assert km.fold_native_to_be(total, parity) == got
        checked += 1
    assert checked > 100


def test_block_aligned_rows_vs_zlib():
    # digest_kernel_a<kOps, true>: rows on 64-B blocks, skipped updates past the frame end and
    # the rotated combine reproduce zlib at every block phase, length and start alignment
    rnd = random.Random(12)
    for _ in range(300):
        L = rnd.choice([4, 5, 7, 8, 15, 16, 17, 63, 64, 65, 127, 128, 129, 255, 256, 257, rnd.randrange(4, 1600)])
        pre = rnd.randrange(0, 70)
        buf = rnd.randbytes(pre + L + 8)
        assert km.crc32_model_al(buf, pre, L, rnd.randrange(16)) == zlib.crc32(buf[pre : pre + L])


def test_lane_per_frame_crc_vs_zlib():
    """The small-frame kernel's CRC (one lane per frame, one or two Horner chains) at every start
    alignment and the lengths round the dword and chain boundaries."""
    import random
    import zlib

    from kernel_model import crc32_model_lane

    rnd = random.Random(5)
    buf = bytes(rnd.randrange(256) for _ in range(400))
    for S in range(8):
        for length in list(range(0, 40)) + [47, 60, 64, 65, 127, 128, 129, 200]:
            want = zlib.crc32(buf[S:S + length])
            for chains in (1, 2):
                assert crc32_model_lane(buf, S, length, chains) == want, (S, length, chains)


def test_tile_segments_vs_zlib():
    """The segment kernel's decomposition (km.crc32_tile_segments): random tiles of mixed lengths
    (empty and sub-4-byte frames, gaps, every start alignment and block phase, 1 to 16 groups), the
    C3 tile (64/576/1500/9000 B), and a tile of 64-B frames beside a jumbo frame; and the tail select
    is needed (without it every frame of the C3 tile is wrong)."""
    rnd = random.Random(21)
    for _ in range(60):
        n = rnd.choice([1, 2, 3, 5, 16])
        lens = [rnd.choice([0, 1, 3, 4, 5, 7, 20, 63, 64, 65, 70, 130, 200, 577, 1000]) for _ in range(n)]
        buf = rnd.randbytes(sum(lens) + 4 * n + 64)
        frames, o = [], rnd.randrange(4)
        for ln in lens:
            frames.append((o, ln))
            o += ln + rnd.randrange(4)
        got = km.crc32_tile_segments(buf, frames, rnd.randrange(16), groups=rnd.choice([1, 2, 4, 16]))
        assert got == [zlib.crc32(buf[S:S + ln]) for S, ln in frames]
    buf = rnd.randbytes(50000)
    for lens in ([64, 576, 1500, 9000] * 4, [64] * 15 + [9000]):
        frames, o = [], 0
        for ln in lens:
            frames.append((o, ln))
            o += ln
        exp = [zlib.crc32(buf[S:S + ln]) for S, ln in frames]
        assert km.crc32_tile_segments(buf, frames, 3) == exp
    bad = km.crc32_tile_segments(buf, frames, 3, model_tail_select=False)
    assert sum(g != e for g, e in zip(bad, exp)) > 0
