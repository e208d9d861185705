// Host-logic checks of seqs_amd/csrc/framesum_plan.h, built on its own under ASan + UBSan
// (tests/csrc/Makefile, run by tests/test_host_sanitizers.py): the chunks of the
// host-staged path, the blocks of fs_digest_batch_multi and the round-robin shard / gather /
// de-interleave maps, on random batches that are in order, shuffled, sparse, overlapping,
// empty, zero-length, huge-offset, and with more contexts than frames.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../seqs_amd/csrc/framesum_plan.h"

using namespace framesum::plan;

static int g_fail = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            if (++g_fail > 20) std::exit(1);                                  \
        }                                                                     \
    } while (0)

struct Batch {
    std::vector<uint64_t> off;
    std::vector<uint32_t> len;
    uint64_t bytes = 0;
};

static Batch make_batch(std::mt19937_64& rng, uint32_t n, int kind) {
    Batch b;
    b.off.resize(n);
    b.len.resize(n);
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t L = kind == 3 ? 0u : (uint32_t)(rng() % 9100);
        b.len[i] = L;
        if (kind == 2 && rng() % 4 == 0) pos += rng() % (64u << 20);  // sparse: big gaps
        b.off[i] = pos;
        pos += (L + 3) & ~3u;
        if (kind == 4 && i > 0 && rng() % 3 == 0) b.off[i] = b.off[rng() % i];  // overlapping / repeated
    }
    b.bytes = pos + 16;
    if (kind == 1) {  // shuffled: offsets not in index order
        for (uint32_t i = n; i > 1; --i) {
            const uint32_t j = (uint32_t)(rng() % i);
            std::swap(b.off[i - 1], b.off[j]);
            std::swap(b.len[i - 1], b.len[j]);
        }
    }
    return b;
}

static void check_chunks(const Batch& b, uint64_t chunk_bytes, uint32_t chunk_frames) {
    const uint32_t n = (uint32_t)b.len.size();
    CHECK(first_frame_out_of_range(b.off.data(), b.len.data(), n, b.bytes) == n);
    {   // the one-pass scan of the host-staged call: in range, longest frame, byte span
        const Scan sc = scan_batch(b.off.data(), b.len.data(), n, b.bytes);
        uint64_t lo = UINT64_MAX, hi = 0;
        uint32_t mx = 0;
        for (uint32_t i = 0; i < n; ++i) {
            lo = std::min(lo, b.off[i]);
            hi = std::max(hi, b.off[i] + b.len[i]);
            mx = std::max(mx, b.len[i]);
        }
        CHECK(sc.bad == n && sc.max_len == mx && sc.hi == hi && sc.lo == (n ? lo : 0));
    }
    std::vector<Chunk> ch;
    host_chunks(b.off.data(), b.len.data(), n, b.bytes, chunk_bytes, chunk_frames, ch);
    uint32_t next = 0;
    for (const Chunk& c : ch) {
        CHECK(c.c0 == next && c.c1 > c.c0 && c.c1 <= n);
        CHECK(c.cpy_lo % 16 == 0 && c.cpy_lo <= c.cpy_hi && c.cpy_hi <= b.bytes);
        uint64_t lo = UINT64_MAX, hi = 0;
        for (uint32_t i = c.c0; i < c.c1; ++i) {
            // every byte the engine may touch for frame i lies in the staged copy: 12 B before
            // its start (or the buffer start) up to its dword-rounded end (or the buffer end)
            const uint64_t s = b.off[i], e = s + b.len[i];
            CHECK(c.cpy_lo <= (s >= 12 ? s - 12 : 0));
            CHECK(std::min<uint64_t>((e + 3) & ~uint64_t(3), b.bytes) <= c.cpy_hi);
            lo = std::min(lo, s);
            hi = std::max(hi, e);
        }
        const bool single = c.c1 - c.c0 == 1, rest = c.c1 == n;
        CHECK(single || rest || hi - lo <= chunk_bytes);
        CHECK(c.c1 - c.c0 <= chunk_frames || rest);
        next = c.c1;
    }
    CHECK(next == n);
}

static void check_multi(const Batch& b, int nctx) {
    const uint32_t n = (uint32_t)b.len.size();
    MultiPlan p;
    multi_blocks(b.off.data(), b.len.data(), n, nctx, p);
    CHECK((int)p.cut.size() == nctx + 1 && p.cut[0] == 0 && p.cut[nctx] == n);
    for (int k = 0; k < nctx; ++k) CHECK(p.cut[k] <= p.cut[k + 1]);
    std::vector<uint8_t> seen(n, 0);
    uint64_t total = 0, maxlen = 0;
    for (uint32_t pos = 0; pos < n; ++pos) {
        const uint32_t f = p.frame(pos);
        CHECK(f < n);
        if (f < n) seen[f]++;
        if (pos > 0) CHECK(b.off[p.frame(pos - 1)] <= b.off[f]);  // buffer order inside every block
        total += b.len[f];
        maxlen = std::max<uint64_t>(maxlen, b.len[f]);
    }
    for (uint32_t i = 0; i < n; ++i) CHECK(seen[i] == 1);  // a permutation
    for (int k = 0; k < nctx; ++k) {
        uint64_t bytes = 0;
        for (uint32_t pos = p.cut[k]; pos < p.cut[k + 1]; ++pos) bytes += b.len[p.frame(pos)];
        CHECK(bytes * (uint64_t)nctx <= total + (uint64_t)nctx * maxlen);  // byte balance
    }
}

static void check_shards(uint64_t n, uint32_t N) {
    uint64_t sum = 0;
    for (uint32_t k = 0; k < N; ++k) sum += shard_count(n, N, k);
    CHECK(sum == n);
    const uint64_t m = shard_rows(n, N), sb = slab_bytes(m);
    CHECK(sb % 256 == 0 && sb >= 9 * m);
    // simulate: shard k writes local frame j's digest = global index (j*N + k); the gather puts
    // slab k at k*sb; the de-interleave map must give back global order
    std::vector<uint64_t> gathered((N * sb) / 8 + 1, ~0ull);
    std::vector<uint8_t> gst(N * sb, 0xEE);
    for (uint32_t k = 0; k < N; ++k)
        for (uint64_t j = 0; j < shard_count(n, N, k); ++j) {
            const uint64_t at = k * sb + 8 * j;
            CHECK(at % 8 == 0 && at + 8 <= N * sb);
            gathered[at / 8] = j * N + k;
            const uint64_t sat = k * sb + 8 * m + j;
            CHECK(sat < N * sb && sat >= k * sb + 8 * m);
            gst[sat] = (uint8_t)((j * N + k) & 0x7F);
        }
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t at = gathered_digest_at(i, N, m), sat = gathered_status_at(i, N, m);
        CHECK(at % 8 == 0 && at + 8 <= N * sb && sat < N * sb);
        CHECK(gathered[at / 8] == i);
        CHECK(gst[sat] == (uint8_t)(i & 0x7F));
    }
    // chunked gather: chunk c's pieces of every slab hold exactly global frames [c R N, (c+1) R N)
    for (uint32_t nc : {1u, 2u, 3u, 4u, 8u}) {
        const uint64_t R = chunk_rows(m, nc);
        const uint32_t C = chunk_count(m, R);
        CHECK(m == 0 || (R % 256 == 0 && C >= 1 && C <= nc && (uint64_t)C * R >= m && (uint64_t)(C - 1) * R < m));
        std::vector<uint8_t> hit(n, 0);
        for (uint32_t c = 0; c < C; ++c) {
            const uint64_t lo = c * R, hi = std::min<uint64_t>(m, lo + R);
            uint64_t rows = 0;
            for (uint32_t k = 0; k < N; ++k) {
                const uint64_t r = shard_rows_in(n, N, k, lo, hi);
                CHECK(r <= hi - lo);
                rows += r;
                for (uint64_t j = lo; j < lo + r; ++j) {
                    const uint64_t g = j * N + k;
                    CHECK(g < n && g >= lo * N && g < std::min<uint64_t>(n, hi * N));
                    ++hit[g];
                }
                CHECK((8 * lo) % 2048 == 0 && lo % 256 == 0);
            }
            CHECK(rows == (std::min<uint64_t>(n, hi * N) > lo * N ? std::min<uint64_t>(n, hi * N) - lo * N : 0));
        }
        for (uint64_t i = 0; i < n; ++i) CHECK(hit[i] == 1);
    }
}

// The exact chunk loop of fs_digest_batch_sharded (framesum_group.cpp), replayed on the host with
// memcpy standing in for ncclSend/ncclRecv: every shard's kernel writes its chunk rows into its
// slab (shard 0 in place in the gather buffer), every Piece is copied, and each chunk's
// de-interleave then reads only bytes that a kernel or a transfer of that chunk or an earlier one
// has written, getting back global frame order. Ragged n, n < N and empty shards included.
static void replay_chunks(uint64_t n, uint32_t N, uint32_t maxc, uint64_t target) {
    std::vector<ChunkXfer> plan;
    chunk_plan(n, N, maxc, target, plan);
    if (n == 0) {
        CHECK(plan.empty());
        return;
    }
    const uint64_t m = shard_rows(n, N), sb = slab_bytes(m);
    std::vector<std::vector<uint8_t>> send(N, std::vector<uint8_t>(sb, 0xCD));
    std::vector<uint8_t> recv(N * sb, 0xAB), have(N * sb, 0);
    std::vector<uint32_t> wrote(n, 0);
    uint64_t g_next = 0;
    for (const ChunkXfer& x : plan) {
        CHECK(x.lo < x.hi && x.hi <= m && x.g0 == g_next && x.g0 == x.lo * N && x.g1 <= n && x.g0 < x.g1);
        g_next = x.g1;
        // the kernels: shard k writes local rows [lo, lo + rk)
        for (uint32_t k = 0; k < N; ++k) {
            const uint64_t rk = shard_rows_in(n, N, k, x.lo, x.hi);
            uint8_t* slab = k == 0 ? recv.data() : send[k].data();
            for (uint64_t j = x.lo; j < x.lo + rk; ++j) {
                const uint64_t g = j * N + k;
                CHECK(g < n);
                std::memcpy(slab + 8 * j, &g, 8);
                slab[8 * m + j] = (uint8_t)(g * 7 + 1);
                if (k == 0) {
                    std::fill(have.begin() + 8 * j, have.begin() + 8 * j + 8, 1);
                    have[8 * m + j] = 1;
                }
            }
        }
        // the transfers
        uint32_t prev = 0;
        for (const Piece& p : x.pieces) {
            const uint32_t k = p.shard;
            CHECK(k >= 1 && k < N && k > prev);  // one piece per shard, in shard order
            prev = k;
            CHECK(p.rows == shard_rows_in(n, N, k, x.lo, x.hi) && p.rows > 0);
            CHECK(p.send_dig == 8 * x.lo && p.send_st == 8 * m + x.lo);
            CHECK(p.send_dig + 8 * p.rows <= 8 * m && p.send_st + p.rows <= sb);
            CHECK(p.recv_dig == k * sb + p.send_dig && p.recv_st == k * sb + p.send_st);
            CHECK(p.recv_dig + 8 * p.rows <= k * sb + 8 * m && p.recv_st + p.rows <= (k + 1) * sb);
            std::memcpy(recv.data() + p.recv_dig, send[k].data() + p.send_dig, 8 * p.rows);
            std::memcpy(recv.data() + p.recv_st, send[k].data() + p.send_st, p.rows);
            std::fill(have.begin() + p.recv_dig, have.begin() + p.recv_dig + 8 * p.rows, 1);
            std::fill(have.begin() + p.recv_st, have.begin() + p.recv_st + p.rows, 1);
        }
        for (uint32_t k = 1; k < N; ++k) {  // shards with rows in the chunk have a piece
            bool listed = false;
            for (const Piece& p : x.pieces) listed |= p.shard == k;
            CHECK(listed == (shard_rows_in(n, N, k, x.lo, x.hi) > 0));
        }
        // the de-interleave of [g0, g1): only received bytes, global order back
        for (uint64_t g = x.g0; g < x.g1; ++g) {
            const uint64_t at = gathered_digest_at(g, N, m), sat = gathered_status_at(g, N, m);
            bool ok = at + 8 <= recv.size() && sat < recv.size();
            CHECK(ok);
            if (!ok) continue;
            for (int b = 0; b < 8; ++b) CHECK(have[at + b]);
            CHECK(have[sat]);
            uint64_t v = 0;
            std::memcpy(&v, recv.data() + at, 8);
            CHECK(v == g);
            CHECK(recv[sat] == (uint8_t)(g * 7 + 1));
            ++wrote[g];
        }
    }
    CHECK(g_next == n);
    for (uint64_t g = 0; g < n; ++g) CHECK(wrote[g] == 1);
}

int main() {
    std::mt19937_64 rng(12345);
    // chunks: every batch kind, several chunk sizes (small ones force many chunks)
    for (int kind = 0; kind < 5; ++kind)
        for (uint32_t n : {0u, 1u, 2u, 7u, 63u, 64u, 65u, 1000u, 5000u})
            for (uint64_t cb : {uint64_t(4096), uint64_t(65536), uint64_t(16) << 20}) {
                const Batch b = make_batch(rng, n, kind);
                check_chunks(b, cb, kind == 0 ? 100u : (1u << 20));
            }
    // out-of-range detection, including offsets whose end would overflow 64 bits
    {
        std::vector<uint64_t> off = {0, 100, UINT64_MAX - 2, 50};
        std::vector<uint32_t> len = {10, 20, 10, 10};
        CHECK(first_frame_out_of_range(off.data(), len.data(), 4, 1000) == 2);
        CHECK(first_frame_out_of_range(off.data(), len.data(), 2, 1000) == 2);
        CHECK(first_frame_out_of_range(off.data(), len.data(), 2, 120) == 2);
        CHECK(first_frame_out_of_range(off.data(), len.data(), 2, 119) == 1);
        CHECK(first_frame_out_of_range(off.data(), len.data(), 1, 13, 4) == 0);
        CHECK(first_frame_out_of_range(off.data(), len.data(), 1, 14, 4) == 1);
        // scan_batch reports the same first bad frame
        CHECK(scan_batch(off.data(), len.data(), 4, 1000).bad == 2);
        CHECK(scan_batch(off.data(), len.data(), 2, 1000).bad == 2);
        CHECK(scan_batch(off.data(), len.data(), 2, 119).bad == 1);
        CHECK(scan_batch(off.data(), len.data(), 1, 13, 4).bad == 0);
        CHECK(scan_batch(off.data(), len.data(), 1, 14, 4).bad == 1);
        CHECK(scan_batch(off.data(), len.data(), 0, 14).bad == 0);
    }
    // multi blocks: more contexts than frames, empty batches, unordered and overlapping batches
    for (int kind = 0; kind < 5; ++kind)
        for (uint32_t n : {0u, 1u, 3u, 8u, 9u, 100u, 4097u})
            for (int nctx : {1, 2, 3, 8, 16})
                check_multi(make_batch(rng, n, kind), nctx);
    // shard maps for the group entry and the bench's gather
    for (uint32_t N : {1u, 2u, 3u, 4u, 8u})
        for (uint64_t n : {uint64_t(0), uint64_t(1), uint64_t(2), uint64_t(7), uint64_t(8), uint64_t(9),
                           uint64_t(1000), uint64_t(65537), uint64_t(1) << 20})
            check_shards(n, N);
    // the sharded call's chunk loop replayed with memcpy transfers, N = 1..8,
    // ragged n, n < N, empty shards, the library's chunk parameters and small ones (many chunks)
    for (uint32_t N = 1; N <= 8; ++N)
        for (uint64_t n : {uint64_t(0), uint64_t(1), uint64_t(3), uint64_t(7), uint64_t(8), uint64_t(9), uint64_t(255),
                           uint64_t(257), uint64_t(1000), uint64_t(4097), uint64_t(65537), uint64_t(300001)}) {
            replay_chunks(n, N, 8, 32768);
            replay_chunks(n, N, 8, 256);
            replay_chunks(n, N, 3, 1);
        }
    if (g_fail) {
        std::fprintf(stderr, "%d check(s) failed\n", g_fail);
        return 1;
    }
    std::printf("plan checks OK\n");
    return 0;
}
