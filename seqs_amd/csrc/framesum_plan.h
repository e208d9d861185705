// Host-side planning for the framesum entry points, free of HIP so that it compiles on its
// own: the chunks of a host-staged batch (fs_digest_batch_host), the byte-balanced blocks of
// fs_digest_batch_multi, and the round-robin shard maps of fs_digest_batch_sharded and its
// de-interleave kernel. The library includes it; tests/csrc/test_plan.cpp builds it alone
// under ASan + UBSan (sanitizers on the host code) and checks every invariant
// on random, out-of-order, overlapping and edge-case batches.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <numeric>
#include <vector>

namespace framesum {
namespace plan {

// ---------------------------------------------------------------------------------------
// Round-robin shards (eth/crc.go:12-17: CRC791 is per call, so frames are
// independent). Global frame i lives on shard i % N at local index i / N. Shards are padded
// to m = ceil(n / N) rows for the fixed-size RCCL gather; shard k's gathered slab holds its
// m 8-byte digests and then its m verdict bytes, 256-byte aligned.
constexpr uint64_t shard_count(uint64_t n, uint32_t nshards, uint32_t shard) {
    return shard < n ? (n - shard + nshards - 1) / nshards : 0;
}
constexpr uint64_t shard_rows(uint64_t n, uint32_t nshards) { return (n + nshards - 1) / nshards; }
constexpr uint64_t slab_bytes(uint64_t m) { return (9 * m + 255) / 256 * 256; }
// byte offsets, in the gathered buffer of nshards slabs, of global frame i's digest and verdict
constexpr uint64_t gathered_digest_at(uint64_t i, uint32_t nshards, uint64_t m) {
    return (i % nshards) * slab_bytes(m) + 8 * (i / nshards);
}
constexpr uint64_t gathered_status_at(uint64_t i, uint32_t nshards, uint64_t m) {
    return (i % nshards) * slab_bytes(m) + 8 * m + i / nshards;
}

// Chunks of a sharded batch (fs_digest_batch_sharded gathers chunk by chunk, so chunk c's
// transfer overlaps chunk c+1's kernels): chunk c = local rows [c*R, min((c+1)*R, m)) of every
// shard, R a multiple of 256 rows (the digest and verdict pieces stay 256-B aligned in the
// slab). Those rows hold exactly the global frames [c*R*N, min((c+1)*R*N, n)), so the
// de-interleave of a chunk needs only that chunk's pieces.
constexpr uint64_t chunk_rows(uint64_t m, uint32_t nchunks) {
    return nchunks == 0 ? m : ((m + nchunks - 1) / nchunks + 255) / 256 * 256;
}
constexpr uint32_t chunk_count(uint64_t m, uint64_t rows) { return rows == 0 ? 0 : (uint32_t)((m + rows - 1) / rows); }
// shard k's frames in local rows [lo, hi): [lo, min(hi, shard_count))
constexpr uint64_t shard_rows_in(uint64_t n, uint32_t nshards, uint32_t shard, uint64_t lo, uint64_t hi) {
    const uint64_t c = shard_count(n, nshards, shard);
    return (hi < c ? hi : c) > lo ? (hi < c ? hi : c) - lo : 0;
}

// The transfers of one chunk of fs_digest_batch_sharded: for every shard k >= 1 with rows in
// the chunk, its digest piece and its verdict piece go from its own slab (send offsets) to
// slab k of the first device's gather buffer (recv offsets); shard 0's kernel writes in place
// there. The first device then de-interleaves the global frames [g0, g1).
struct Piece {
    uint32_t shard;           // k >= 1
    uint64_t rows;            // rk = shard_rows_in(n, N, k, lo, hi) > 0
    uint64_t send_dig, send_st;  // byte offsets in shard k's slab: 8 lo, 8 m + lo
    uint64_t recv_dig, recv_st;  // byte offsets in the gather buffer: k sb + 8 lo, k sb + 8 m + lo
};
struct ChunkXfer {
    uint64_t lo, hi;   // local rows [lo, hi) of every shard
    uint64_t g0, g1;   // global frames [g0, g1) = [lo N, min(hi N, n))
    std::vector<Piece> pieces;
};
// The chunk plan of a sharded call: nchunks_max chunks at most, about target_rows rows each.
inline void chunk_plan(uint64_t n, uint32_t N, uint32_t nchunks_max, uint64_t target_rows, std::vector<ChunkXfer>& out) {
    out.clear();
    if (N == 0 || n == 0) return;
    const uint64_t m = shard_rows(n, N), sb = slab_bytes(m);
    const uint64_t want = target_rows ? (m + target_rows - 1) / target_rows : 1;
    const uint64_t R = chunk_rows(m, (uint32_t)(want < nchunks_max ? want : nchunks_max));
    const uint32_t C = chunk_count(m, R);
    for (uint32_t c = 0; c < C; ++c) {
        ChunkXfer x;
        x.lo = (uint64_t)c * R;
        x.hi = x.lo + R < m ? x.lo + R : m;
        x.g0 = x.lo * N;
        x.g1 = x.hi * N < n ? x.hi * N : n;
        for (uint32_t k = 1; k < N; ++k) {
            const uint64_t rk = shard_rows_in(n, N, k, x.lo, x.hi);
            if (rk == 0) continue;
            x.pieces.push_back(Piece{k, rk, 8 * x.lo, 8 * m + x.lo, k * sb + 8 * x.lo, k * sb + 8 * m + x.lo});
        }
        out.push_back(x);
    }
}

// ---------------------------------------------------------------------------------------
// Host-staged chunks.

// Index of the first frame that does not lie inside [0, frames_bytes) (overflow-safe), or n.
inline uint32_t first_frame_out_of_range(const uint64_t* offsets, const uint32_t* lengths, uint32_t n,
                                         uint64_t frames_bytes, uint32_t extra = 0, uint32_t* max_len = nullptr) {
    uint32_t mx = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t need = (uint64_t)lengths[i] + extra;
        if (offsets[i] > frames_bytes || need > frames_bytes - offsets[i]) return i;
        mx = lengths[i] > mx ? lengths[i] : mx;
    }
    if (max_len) *max_len = mx;  // (the batch's longest frame, when every frame is in range)
    return n;
}

// One pass over a host batch's descriptors (fs_digest_batch_host): whether every frame lies in
// [0, frames_bytes) (overflow-safe), the longest frame, and the byte span [lo, hi) of the whole
// batch. Branch-free in the loop (the compiler vectorizes it): the host-staged call of a batch of
// short frames walks 65,536 descriptors per call, and two passes of a branchy loop were a sizeable
// part of its host time. bad = the first out-of-range frame, or n.
struct Scan {
    uint32_t bad, max_len, min_len;
    uint64_t lo, hi;
};
// The reductions only (min offset, max offset, max end, max and min length): five independent
// min/max chains the compiler vectorizes. Every frame lies in range iff max offset <= frames_bytes and
// max end + extra <= frames_bytes, as long as no end wraps (frames_bytes < 2^64 - 2^33: a larger
// buffer falls back to the per-frame test).
struct ScanCore {
    uint64_t lo, hi_off, hi_end;
    uint32_t max_len, min_len;
};
inline ScanCore scan_core(const uint64_t* offsets, const uint32_t* lengths, uint32_t n) {
    uint64_t lo = UINT64_MAX, ho = 0, he = 0;
    uint32_t mx = 0, mn = UINT32_MAX;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t o = offsets[i];
        const uint32_t l = lengths[i];
        lo = o < lo ? o : lo;
        ho = o > ho ? o : ho;
        he = o + l > he ? o + l : he;
        mx = l > mx ? l : mx;
        mn = l < mn ? l : mn;
    }
    ScanCore c;
    c.lo = lo;
    c.hi_off = ho;
    c.hi_end = he;
    c.max_len = mx;
    c.min_len = n ? mn : 0;
    return c;
}
inline Scan scan_from(const ScanCore& c, const uint64_t* offsets, const uint32_t* lengths, uint32_t n,
                      uint64_t frames_bytes, uint32_t extra = 0) {
    Scan s;
    const bool exact = frames_bytes < UINT64_MAX - (uint64_t(1) << 33);
    const bool in_range = exact && c.hi_off <= frames_bytes && c.hi_end <= frames_bytes &&
                          frames_bytes - c.hi_end >= extra;
    s.bad = (n == 0 || in_range) ? n : first_frame_out_of_range(offsets, lengths, n, frames_bytes, extra);
    s.max_len = c.max_len;
    s.min_len = c.min_len;
    s.lo = n ? c.lo : 0;
    s.hi = c.hi_end;
    return s;
}
inline Scan scan_batch(const uint64_t* offsets, const uint32_t* lengths, uint32_t n, uint64_t frames_bytes,
                       uint32_t extra = 0) {
    return scan_from(scan_core(offsets, lengths, n), offsets, lengths, n, frames_bytes, extra);
}

struct Chunk {
    uint32_t c0, c1;          // frames [c0, c1)
    uint64_t cpy_lo, cpy_hi;  // host bytes [cpy_lo, cpy_hi) staged for them
};

// The bytes a staged chunk copies for frames spanning [lo, hi): a 16-B aligned start with a
// 16-B prefix (frames under 4 bytes are read from up to 12 bytes before their start), and the
// end rounded up to the dword the engine may read, capped at the buffer.
inline void copy_span(uint64_t lo, uint64_t hi, uint64_t frames_bytes, uint64_t& cpy_lo, uint64_t& cpy_hi) {
    cpy_lo = (lo >= 16 ? lo - 16 : 0) & ~uint64_t(15);
    cpy_hi = (hi + 3) & ~uint64_t(3);
    if (cpy_hi > frames_bytes) cpy_hi = frames_bytes;
    if (cpy_hi < cpy_lo) cpy_hi = cpy_lo;
}

// Cut frames [0, n) into chunks of at most chunk_frames frames whose byte span stays within
// chunk_bytes (a single frame may exceed it). When a chunk would hold fewer than 64 frames
// because the next frame lies far away (frames not stored in index order), the chunk takes
// the rest of the batch instead of a launch per handful of frames. Every frame must already
// lie inside the buffer (first_frame_out_of_range).
inline void host_chunks(const uint64_t* offsets, const uint32_t* lengths, uint32_t n, uint64_t frames_bytes,
                        uint64_t chunk_bytes, uint32_t chunk_frames, std::vector<Chunk>& out) {
    out.clear();
    uint32_t c0 = 0;
    while (c0 < n) {
        uint64_t lo = offsets[c0], hi = offsets[c0] + lengths[c0];
        uint32_t c1 = c0 + 1;
        while (c1 < n && c1 - c0 < chunk_frames) {
            const uint64_t o = offsets[c1], e = o + lengths[c1];
            const uint64_t nlo = o < lo ? o : lo, nhi = e > hi ? e : hi;
            if (nhi - nlo > chunk_bytes) break;
            lo = nlo;
            hi = nhi;
            ++c1;
        }
        if (c1 < n && c1 - c0 < 64 && hi - lo < chunk_bytes / 4) {
            for (; c1 < n; ++c1) {
                const uint64_t o = offsets[c1], e = o + lengths[c1];
                lo = o < lo ? o : lo;
                hi = e > hi ? e : hi;
            }
        }
        Chunk c{c0, c1, 0, 0};
        copy_span(lo, hi, frames_bytes, c.cpy_lo, c.cpy_hi);
        out.push_back(c);
        c0 = c1;
    }
}

// ---------------------------------------------------------------------------------------
// fs_digest_batch_multi blocks: nctx blocks of about equal byte counts. The blocks are
// contiguous runs of the frames in buffer order, so that each context copies only its own
// bytes: `order` is empty when the offsets are already non-decreasing (block k = frames
// [cut[k], cut[k+1])), otherwise it lists the frame indices sorted by offset (stable) and
// block k = order[cut[k] .. cut[k+1]).
struct MultiPlan {
    std::vector<uint32_t> order;
    std::vector<uint32_t> cut;  // nctx + 1 positions, cut[0] = 0, cut[nctx] = n
    uint32_t frame(uint32_t pos) const { return order.empty() ? pos : order[pos]; }
};

inline void multi_blocks(const uint64_t* offsets, const uint32_t* lengths, uint32_t n, int nctx, MultiPlan& p) {
    p.order.clear();
    p.cut.assign((size_t)nctx + 1, n);
    p.cut[0] = 0;
    bool sorted = true;
    for (uint32_t i = 1; i < n && sorted; ++i) sorted = offsets[i] >= offsets[i - 1];
    if (!sorted) {
        p.order.resize(n);
        std::iota(p.order.begin(), p.order.end(), 0u);
        std::stable_sort(p.order.begin(), p.order.end(),
                         [offsets](uint32_t a, uint32_t b) { return offsets[a] < offsets[b]; });
    }
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) total += lengths[i];
    // block k starts at the first position whose running byte count reaches k/nctx of the total
    uint64_t run = 0;
    int k = 1;
    for (uint32_t pos = 0; pos < n && k < nctx; ++pos) {
        while (k < nctx && (unsigned __int128)run * (unsigned)nctx >= (unsigned __int128)total * (unsigned)k)
            p.cut[k++] = pos;
        run += lengths[p.frame(pos)];
    }
}

}  // namespace plan
}  // namespace framesum
