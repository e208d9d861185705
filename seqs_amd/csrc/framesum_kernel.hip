// framesum digest kernel — CDNA4 / gfx950.
//
// One fused pass per frame over HBM computes
//   * the IEEE CRC-32 of frame[0:len)                     (new: SURVEY.md §0.1)
//   * IPv4Header.CalculateChecksum() of frame[14:34]      (eth/headers.go:333-340)
//   * the TCP/UDP checksum RecvEth verifies + its verdict (stacks/portstack.go:163-308,
//     eth/headers.go:382-393, :510-527, arithmetic of eth/crc.go:13-84)
//
// Work decomposition:
//   * a wave owns a TILE of 16 frames; each frame gets a 4-lane GROUP.
//   * a frame is cut into 64-byte ROWS anchored at its (dword-rounded) END, so
//     the head row is the partial one; lane l of the group loads dwords
//     [4l, 4l+4) of every row with one global_load_dwordx4 (16 B/lane), kPrefetch
//     rows ahead. The row loop depends only on the frame descriptor (offset,
//     length); the frame's first 128 bytes are fetched into LDS by LDS-DMA next to
//     the first rows, and the header parse runs after the first block of rows,
//     hidden behind the rows in flight.
//   * CRC: each lane keeps 4 independent dword STREAMS; a stream's successive
//     dwords are 64 B apart, so its Horner step is  A <- Z64(A) ^ w  with Z64 a
//     fixed GF(2) linear map evaluated by 4 byte-table lookups in LDS. After the
//     last row the 16 streams of a frame are combined in 3 dependent lookups
//     (U = Z12(A0)^Z8(A1)^Z4(A2)^A3 per lane, Z_(16(3-l)) per lane l + DPP
//     quad xor, then a final Z_(4-t) that also removes the t <= 3 zero bytes
//     the dword rounding appended). Leading zero rows do not change a zero-init CRC; the CRC init
//     is applied by XOR-ing the frame's first 4 bytes with 0xFF.
//   * one's-complement sum: the same registers feed v_sad_u16 (acc += lo16 + hi16,
//     one op per dword; congruent mod 65535 to the byte-swapped big-endian word
//     sum) over every frame byte; the group's lane 0 subtracts, in the same
//     domain, the Ethernet + IP header bytes, the excluded words and the Ethernet
//     padding and adds the pseudo-header, then folds with a
//     positive offset so RecvEth's Sum16 result (incl. the 0x0000 / 0xFFFF edge)
//     is reproduced bit for bit.
//   * LDS tables: the hot Z64 (and Z4) tables are stored as 8 copies per table
//     in a [entry][table*8+copy] layout, 256 B per entry. Lane L = c + 8h of a
//     32-lane bank group reads table (k+h)&3 in its k-th lookup, so the 32
//     lanes hit 32 distinct banks: conflict-free ds_read_b32 for any data.
//     One v_perm_b32 forms the LDS address (entry byte | per-lane slot byte).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "framesum_internal.h"

namespace framesum {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

#ifndef FS_PREFETCH
#define FS_PREFETCH 6
#endif
#ifndef FS_NT
#define FS_NT 0  // 1: non-temporal row loads
#endif
#ifndef FS_PRIO
#define FS_PRIO 1  // progress-based s_setprio in the row loop (see stream_rows)
#endif
#ifndef FS_DIAG
#define FS_DIAG 0  // diagnostic builds only: 2 = no CRC lookups in the row loop, 3 = no row loads after the prefetch (wrong results)
#endif

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 16;
constexpr int kThreads = kWave * kWavesPerBlock;
constexpr int kFramesPerTile = 16;
constexpr int kRowDwords = 16;
constexpr int kPrefetch = FS_PREFETCH;
// Header slots: the row loop writes every loaded 16-B chunk that holds frame dwords [0, 28)
// into the group's slot, at the dwords it was loaded from (a clamped head chunk lands at the
// frame start; its bytes before the frame go to the slot's 16-B guard). Slots are 36 dwords
// apart, so the 8 parser lanes of a 32-lane bank group read distinct banks.
constexpr int kHdrDwords = 28;
constexpr uint32_t kHdrSlotBytes = 144;
static_assert(kHdrSlotBytes >= 16 + 4 * (kHdrDwords + 3) + 4, "slot holds the guard + the last chunk");
constexpr uint32_t kHdrWaveBytes = kHdrSlotBytes * kFramesPerTile;
constexpr int kStashBytes = 68;             // the frame's last row (Ethernet padding source); 17-dword stride
constexpr int kFastRel0 = 2;                // rows whose chunks start at dword >= 2 carry no head/init mask

// LDS map (bytes). [0, 100 KB) is the FsTables LDS image: region A built in place from
// the Z64 basis, the plain tables copied by LDS-DMA.
constexpr uint32_t kLdsZ32 = 65536;
constexpr uint32_t kLdsZ16 = kLdsZ32 + 4096;
constexpr uint32_t kLdsZfin = kLdsZ16 + 4096;  // Z4, Z3, Z2, Z1 (4 KB each)
constexpr uint32_t kLdsZ48 = kLdsZfin + 16384;
constexpr uint32_t kLdsZ12 = kLdsZ48 + 4096;
constexpr uint32_t kLdsZ8 = kLdsZ12 + 4096;
constexpr uint32_t kLdsTables = kLdsZ8 + 4096;
constexpr uint32_t kLdsHdr = kLdsTables;
constexpr uint32_t kLdsStash = kLdsHdr + kWavesPerBlock * kHdrWaveBytes;
constexpr uint32_t kLdsBytes = kLdsStash + kWavesPerBlock * kFramesPerTile * kStashBytes;
static_assert(kLdsHdr % 16 == 0 && kLdsStash % 16 == 0, "slots must be 16-B aligned");
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");
static_assert(kTablesLdsBytes == kLdsTables, "FsTables is the LDS image of the tables");
constexpr uint32_t kPlainChunk0 = 65536 / 1024;                     // first 1-KB piece of the plain tables
constexpr uint32_t kPlainChunks = (kLdsTables - 65536) / 1024;      // 36 pieces
constexpr uint32_t kDmaPerWave = (kPlainChunks + kWavesPerBlock - 1) / kWavesPerBlock;

#ifdef FS_STAMPS
// Diagnostic build only: per-wave s_memtime phase stamps, read back by fs_debug_read_stamps().
__device__ unsigned long long g_fs_stamps[8192 * 16];
#define FS_STAMP(k)                                                                          \
    do {                                                                                     \
        __builtin_amdgcn_sched_barrier(0);                                                   \
        unsigned long long t_ = __builtin_amdgcn_s_memtime();                                \
        if (lane == 0 && gwave < 8192u) g_fs_stamps[gwave * 16u + (k)] = t_;                  \
        __builtin_amdgcn_sched_barrier(0);                                                   \
    } while (0)
#define FS_RTSTAMP(k)                                                                        \
    do {                                                                                     \
        __builtin_amdgcn_sched_barrier(0);                                                   \
        unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                            \
        if (lane == 0 && gwave < 8192u) g_fs_stamps[gwave * 16u + (k)] = t_;                  \
        __builtin_amdgcn_sched_barrier(0);                                                   \
    } while (0)
#else
#define FS_STAMP(k) do { } while (0)
#define FS_RTSTAMP(k) do { } while (0)
#endif


// DPP quad_perm controls.
constexpr int kQuadXor1 = 0xB1;  // [1,0,3,2]
constexpr int kQuadXor2 = 0x4E;  // [2,3,0,1]

enum : uint32_t {
    V_OK = 0, V_SMOL = 1, V_MTU = 2, V_NOT_IPV4 = 3, V_ARP = 4, V_IPVER = 5, V_IHL = 6, V_BADLEN = 7,
    V_PROTO = 8, V_SHORT = 9, V_ZEROPORT = 10, V_UDPLEN = 11, V_TCPOFF = 12, V_CSUM = 13
};

__device__ __forceinline__ uint32_t lds32(const char* lds, uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t*>(lds + byte_addr);
}

struct LaneKeys {
    uint32_t cvec;     // byte j = slot byte of table j for this lane (32*j + 4*c)
    uint32_t sel[4];   // v_perm selectors of the 4 lookups
};

// a ^ b ^ c in one VALU op (v_bitop3_b32, truth table 0x96; gfx950 has no v_xor3).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// Z(a) ^ w with Z from replicated region A (off = 0: Z64, off = 128: Z4). Conflict-free.
__device__ __forceinline__ uint32_t zrep(const char* lds, uint32_t a, const LaneKeys& k, uint32_t off, uint32_t w = 0u) {
    uint32_t t0 = lds32(lds, off + __builtin_amdgcn_perm(a, k.cvec, k.sel[0]));
    uint32_t t1 = lds32(lds, off + __builtin_amdgcn_perm(a, k.cvec, k.sel[1]));
    uint32_t t2 = lds32(lds, off + __builtin_amdgcn_perm(a, k.cvec, k.sel[2]));
    uint32_t t3 = lds32(lds, off + __builtin_amdgcn_perm(a, k.cvec, k.sel[3]));
    return xor3(xor3(t0, t1, t2), t3, w);
}

// Z operator from a plain [4][256] table (region B; a few uses per frame).
__device__ __forceinline__ uint32_t zplain(const char* lds, uint32_t a, uint32_t base) {
    return lds32(lds, base + ((a & 0xffu) << 2)) ^ lds32(lds, base + 1024 + (((a >> 8) & 0xffu) << 2)) ^
           lds32(lds, base + 2048 + (((a >> 16) & 0xffu) << 2)) ^ lds32(lds, base + 3072 + ((a >> 24) << 2));
}

template <int kCtrl>
__device__ __forceinline__ uint32_t dpp_quad(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kCtrl, 0xf, 0xf, false);
}

__device__ __forceinline__ uint32_t bswap16(uint32_t v) { return ((v & 0xffu) << 8) | ((v >> 8) & 0xffu); }

// 16 bytes of row data for one lane: dwords [rel, rel+4) relative to the frame's
// first dword. Issued unconditionally (no divergent branch around the load, so
// the prefetch ring keeps kPrefetch-1 loads in flight); rows that start before
// the frame are clamped to `lo` (the frame's first chunk, never below the buffer
// start) and realigned / masked by the slow path. Rows never run past the frame's last dword (see the segments).
__device__ __forceinline__ u32x4 load_chunk(const uint32_t* fb, int rel, int lo) {
    const u32x4_a4* p = reinterpret_cast<const u32x4_a4*>(fb + max(rel, lo));
    if (FS_NT) return __builtin_nontemporal_load(p);  // streamed once: no reuse in L2
    return *p;
}

// One's-complement accumulation: v_sad_u16(x, 0, acc) = acc + x[15:0] + x[31:16] in ONE op.
// x[15:0] + x[31:16] is congruent to the dword's native little-endian value mod 65535 and
// is 0 iff the dword is 0, which is all Sum16's fold needs. A lane adds at
// most 4096 dwords of a 64-KiB frame (< 2^30), so the 32-bit accumulator cannot wrap.
__device__ __forceinline__ uint32_t sad16(uint32_t x, uint32_t acc) { return __builtin_amdgcn_sad_u16(x, 0u, acc); }

// Per-frame row parameters, held by every lane of the frame's group.
struct RowMasks {
    int nd;              // frame dwords (incl. the partial last one); 0 = nothing to stream
    uint32_t head_mask;  // bytes of dword 0 inside the frame; also the CRC init's part in dword 0
    uint32_t init1;      // the CRC init's part in dword 1
    uint32_t tail_mask;  // bytes of dword nd-1 inside the frame
};

__device__ __forceinline__ void process_row(char* lds, const LaneKeys& keys, u32x4 v, int rel, bool fast,
                                            const RowMasks& m, int lo, uint32_t (&A)[4], uint32_t& cs) {
    if (FS_DIAG == 2) {
        A[0] ^= v.x; A[1] ^= v.y; A[2] ^= v.z; A[3] ^= v.w;
        cs = sad16(v.x, cs); cs = sad16(v.y, cs); cs = sad16(v.z, cs); cs = sad16(v.w, cs);
        return;
    }
    if (fast) {
        A[0] = zrep(lds, A[0], keys, 0, v.x);
        A[1] = zrep(lds, A[1], keys, 0, v.y);
        A[2] = zrep(lds, A[2], keys, 0, v.z);
        A[3] = zrep(lds, A[3], keys, 0, v.w);
        cs = sad16(v.x, cs);
        cs = sad16(v.y, cs);
        cs = sad16(v.z, cs);
        cs = sad16(v.w, cs);
    } else {
        const int sh = max(rel, lo) - rel;  // >0 only for a clamped row that starts before the frame
        if (sh > 0 && sh < 4) {
            const u32x4 u = v;
            v.w = (sh == 1) ? u.z : (sh == 2) ? u.y : u.x;
            v.z = (sh == 1) ? u.y : (sh == 2) ? u.x : 0u;
            v.y = (sh == 1) ? u.x : 0u;
            v.x = 0u;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int rj = rel + j;
            uint32_t d = (rj >= 0) ? v[j] : 0u;
            uint32_t x = 0u;
            if (rj == 0) { d &= m.head_mask; x = m.head_mask; }
            if (rj == 1) x = m.init1;
            if (rj == m.nd - 1) d &= m.tail_mask;
            A[j] = zrep(lds, A[j], keys, 0, d ^ x);
            cs = sad16(d, cs);
        }
    }
}

// ---- parser-lane helpers over the LDS header slot (absolute-dword aligned: slot
// dword k = the frame's dword k counted from its first dword, frame byte p at slot byte
// 16 + sa + p). `hb` = the group's slot.
__device__ __forceinline__ uint32_t hdr_dw(const char* lds, uint32_t hb, uint32_t k) {
    return lds32(lds, hb + 16u + 4u * k);
}

// Row data -> header slot: the chunk's 16 bytes are frame dwords [p, p+4), p = max(rel, lo).
__device__ __forceinline__ void capture_header(char* lds, uint32_t hb, int rel, int lo, u32x4 v) {
    const int p = max(rel, lo);
    if (p < kHdrDwords) *reinterpret_cast<u32x4*>(lds + hb + 16u + 4u * (uint32_t)p) = v;
}
// frame bytes [4j, 4j+4) as a little-endian dword
__device__ __forceinline__ uint32_t frame_dw(const char* lds, uint32_t hb, uint32_t sa, uint32_t j) {
    return __builtin_amdgcn_alignbyte(hdr_dw(lds, hb, j + 1), hdr_dw(lds, hb, j), sa);
}
// bytes of absolute dword k that lie in the absolute byte range [a0, a1)
__device__ __forceinline__ uint32_t range_mask(int k, int a0, int a1) {
    const int lo = min(max(a0 - 4 * k, 0), 4), hi = min(max(a1 - 4 * k, 0), 4);
    const uint32_t mhi = (hi >= 4) ? 0xffffffffu : ((1u << (8 * hi)) - 1u);
    const uint32_t mlo = (lo >= 4) ? 0xffffffffu : ((1u << (8 * lo)) - 1u);
    return mhi & ~mlo;
}
// sum, in the accumulator's 16-bit-half domain, of frame bytes [p0, p1) taken from the
// contiguous stash image whose dword 0 is the frame's dword `d0` (= nd - 16). Bytes outside
// the image count 0.
__device__ uint32_t nsum_lds(const char* lds, uint32_t base, int d0, int ndw, uint32_t sa, int p0, int p1) {
    uint32_t s = 0;
    if (p1 <= p0) return s;
    const int a0 = (int)sa + p0, a1 = (int)sa + p1;
    for (int k = a0 >> 2; k <= (a1 - 1) >> 2; ++k) {
        const int i = k - d0;
        if (i >= 0 && i < ndw) s = sad16(lds32(lds, base + 4u * (uint32_t)i) & range_mask(k, a0, a1), s);
    }
    return s;
}
// the same over the header image (frame bytes [p0, p1) with p1 <= 4 * kHdrDwords - sa)
__device__ uint32_t nsum_hdr(const char* lds, uint32_t hb, uint32_t sa, int p0, int p1) {
    uint32_t s = 0;
    if (p1 <= p0) return s;
    const int a0 = (int)sa + p0, a1 = (int)sa + p1;
    for (int k = a0 >> 2; k <= (a1 - 1) >> 2; ++k) s = sad16(hdr_dw(lds, hb, (uint32_t)k) & range_mask(k, a0, a1), s);
    return s;
}

// Header parse result of one frame (frame lane), computed while its rows stream.
struct Parsed {
    uint32_t verdict;   // final unless `compute`
    uint32_t ip_csum;
    uint32_t stored;    // stored L4 checksum (BE)
    int compute;        // the L4 checksum is computed
    int parity;         // absolute parity of the L4 start (1 = odd)
    uint32_t off, end;  // L4 segment [off, end) (frame-relative); Ethernet padding is [end, len)
    int64_t corr;       // checksum corrections except the padding (16-bit-half domain)
    int64_t corr_fixed; // the pseudo-header and excluded-word part of corr
};

// Header parse for one frame (frame lane). Gates follow stacks/portstack.go:163-308
// exactly (oracle/framesum_oracle.c restates them line by line; the parity tests
// compare the two). Reads only the LDS header image.
__device__ Parsed parse_frame(const char* lds, uint32_t hb, uint32_t sa, uint32_t len, uint32_t mtu) {
    Parsed r = {V_OK, 0u, 0u, 0, 0, 0u, 0u, 0, 0};
    if (len < 34u) { r.verdict = V_SMOL; return r; }                          // portstack.go:167-168
    if (mtu != 0 && len > mtu) { r.verdict = V_MTU; return r; }              // :169-172
    uint32_t bs[9];                                                           // bswap32(frame dword j), j = 3..8
#pragma unroll
    for (uint32_t j = 3; j < 9; ++j) bs[j] = __builtin_bswap32(frame_dw(lds, hb, sa, j));
    const uint32_t etype = bs[3] >> 16;                                       // headers.go:209-215
    const uint32_t vihl = (bs[3] >> 8) & 0xffu;
    {   // eth/headers.go:333-340 via Put (:289-301): version forced to 4, checksum zeroed, 20 bytes.
        uint32_t s = ((0x40u | (vihl & 0xfu)) << 8) | (bs[3] & 0xffu);
        s += (bs[4] >> 16) + (bs[4] & 0xffffu) + (bs[5] >> 16) + (bs[5] & 0xffffu) + (bs[6] & 0xffffu) +
             (bs[7] >> 16) + (bs[7] & 0xffffu) + (bs[8] >> 16);
        s = (s & 0xffffu) + (s >> 16);
        s = (s & 0xffffu) + (s >> 16);
        r.ip_csum = (~s) & 0xffffu;
    }
    if (etype != 0x0800u && etype != 0x0806u) { r.verdict = V_NOT_IPV4; return r; }  // :187-188
    if (etype == 0x0806u) { r.verdict = (len < 42u) ? V_SMOL : V_ARP; return r; }     // :191-197
    const uint32_t ipoff = (vihl & 0xfu) * 4u;                                // uint8, <= 60
    const uint32_t off = 14u + ipoff;                                         // :201
    const uint32_t tl = bs[4] >> 16;
    const uint32_t end = (14u + tl) & 0xffffu;                                // :202 uint16 wrap
    if ((vihl >> 4) != 4u) { r.verdict = V_IPVER; return r; }                 // :204
    if (ipoff < 20u) { r.verdict = V_IHL; return r; }                         // :206
    if (off > end || off > len || end > len) { r.verdict = V_BADLEN; return r; }  // :211
    if (mtu != 0 && end > mtu) { r.verdict = V_MTU; return r; }               // :213
    const uint32_t l4len = end - off;
    const uint32_t proto = bs[5] & 0xffu;
    // L4 header: off = 4q + 2 (q = 3 + IHL); frame dwords q .. q+5 cover bytes off-2 .. off+21.
    const uint32_t q = (off - 2u) >> 2;
    uint32_t lb[6];
#pragma unroll
    for (uint32_t i = 0; i < 6; ++i) lb[i] = __builtin_bswap32(frame_dw(lds, hb, sa, q + i));
    const uint32_t sport = lb[0] & 0xffffu, dport = lb[1] >> 16;
    uint32_t lenword, excl;
    if (proto == 17u) {                                                       // :222-244
        if (l4len < 8u) { r.verdict = V_SHORT; return r; }
        const uint32_t ulen = lb[1] & 0xffffu;
        if (sport == 0 || dport == 0) { r.verdict = V_ZEROPORT; return r; }
        if (ulen < 8u) { r.verdict = V_UDPLEN; return r; }
        lenword = ulen;                                                       // headers.go:386-390
        r.stored = lb[2] >> 16;
        excl = 6;                                                             // Checksum (2 bytes)
    } else if (proto == 6u) {                                                 // :283-308
        if (l4len < 20u) { r.verdict = V_SHORT; return r; }
        const uint32_t toff = ((lb[3] >> 12) & 0xfu) * 4u;                    // headers.go:477-485
        if (sport == 0 || dport == 0) { r.verdict = V_ZEROPORT; return r; }
        if (toff < 20u || toff > l4len) { r.verdict = V_TCPOFF; return r; }
        lenword = (tl - ipoff) & 0xffffu;                                     // headers.go:516
        r.stored = lb[4] & 0xffffu;
        excl = 16;                                                            // Checksum + UrgentPtr (:518-526)
    } else {
        r.verdict = V_PROTO;                                                  // :220-221
        return r;
    }
    r.compute = 1;
    r.off = off;
    r.end = end;
    // Total over [off, end) = all streamed frame bytes [0, len) + these corrections (+ the
    // padding correction applied at the end, from the stash), all in the 16-bit-half domain.
    int64_t t = 0;
    t -= (int64_t)nsum_hdr(lds, hb, sa, (int)(off + excl), (int)(off + excl + (proto == 6u ? 4u : 2u)));
    r.parity = (int)((sa + off) & 1u);
    const uint32_t w[6] = {bs[6] & 0xffffu, bs[7] >> 16, bs[7] & 0xffffu, bs[8] >> 16, proto, lenword};
#pragma unroll
    for (int i = 0; i < 6; ++i) t += (int64_t)(r.parity ? w[i] : bswap16(w[i]));
    r.corr_fixed = t;
    t -= (int64_t)nsum_hdr(lds, hb, sa, 0, (int)off);  // the Ethernet + IP header bytes
    r.corr = t;
    return r;
}

// The parse result lives in LDS while the rows stream (it would otherwise hold 11 VGPRs
// across the row loops): dwords 0..13 of the group's header slot, dead after the parse and
// rewritten only by the next tile's rows, after this tile's finish.
// The frame's descriptor (offset, length) is parked next to it (dwords 11..13).
__device__ __forceinline__ void park_parsed(char* lds, uint32_t hb, const Parsed& P, uint64_t S, uint32_t len) {
    const uint32_t v[14] = {P.verdict, P.ip_csum, P.stored, (uint32_t)P.compute, (uint32_t)P.parity, P.off, P.end,
                            (uint32_t)P.corr, (uint32_t)((uint64_t)P.corr >> 32), (uint32_t)P.corr_fixed,
                            (uint32_t)((uint64_t)P.corr_fixed >> 32), (uint32_t)S, (uint32_t)(S >> 32), len};
#pragma unroll
    for (uint32_t k = 0; k < 14; ++k)
        *reinterpret_cast<uint32_t*>(lds + hb + 16u + 4u * k) = v[k];
}
__device__ __forceinline__ Parsed unpark_parsed(const char* lds, uint32_t hb, uint64_t& S, uint32_t& len) {
    uint32_t v[14];
#pragma unroll
    for (uint32_t k = 0; k < 14; ++k) v[k] = hdr_dw(lds, hb, k);
    S = ((uint64_t)v[12] << 32) | v[11];
    len = v[13];
    Parsed P;
    P.verdict = v[0];
    P.ip_csum = v[1];
    P.stored = v[2];
    P.compute = (int)v[3];
    P.parity = (int)v[4];
    P.off = v[5];
    P.end = v[6];
    P.corr = (int64_t)(((uint64_t)v[8] << 32) | v[7]);
    P.corr_fixed = (int64_t)(((uint64_t)v[10] << 32) | v[9]);
    return P;
}

// Final L4 checksum + verdict (frame lane) once the streamed sum is known.
__device__ uint32_t finish_l4(const char* lds, uint32_t stash, const uint32_t* fb, uint32_t sa, uint32_t len,
                              uint32_t nd, const Parsed& P, uint64_t main_sum, uint32_t& verdict) {
    // Every term is congruent (mod 65535) to its exact native contribution, and the true
    // total is > 0 (the pseudo-header protocol word is 6 or 17), so adding 65535 * 2^20
    // keeps t positive and the fold below lands on the same one's-complement value.
    int64_t t = (int64_t)main_sum + P.corr + 65535LL * (1LL << 20);
    if (len >= (1u << 19)) {
        // >= 512 KiB frame (only reachable with a huge Ethernet padding): a lane's streamed
        // 32-bit sum may have wrapped, so sum the L4 segment [off, end) exactly from memory.
        const int a0 = (int)(sa + P.off), a1 = (int)(sa + P.end);
        uint32_t s = 0;
        for (int k = a0 >> 2; k <= (a1 - 1) >> 2; ++k) s = sad16(fb[k] & range_mask(k, a0, a1), s);
        t = (int64_t)s + P.corr_fixed + 65535LL * (1LL << 20);
    } else if (P.end < len) {  // Ethernet padding after the IP datagram
        const int sd0 = (int)nd - 16;
        if ((int)(sa + P.end) >= 4 * sd0) {
            t -= (int64_t)nsum_lds(lds, stash, sd0, 16, sa, (int)P.end, (int)len);
        } else {  // long padding (malformed frame): exact sum straight from global memory
            const int a0 = (int)(sa + P.end), a1 = (int)(sa + len);
            uint32_t s = 0;
            for (int k = a0 >> 2; k <= (a1 - 1) >> 2; ++k) s = sad16(fb[k] & range_mask(k, a0, a1), s);
            t -= (int64_t)s;
        }
    }
    uint64_t x = (uint64_t)t;
    x = (x & 0xffffffffu) + (x >> 32);
    while (x >> 16) x = (x & 0xffffu) + (x >> 16);
    uint32_t l4 = (~(uint32_t)x) & 0xffffu;
    if (!P.parity) l4 = bswap16(l4);
    verdict = (l4 == P.stored) ? V_OK : V_CSUM;
    return l4;
}

// Per-tile state of one wave. Every lane describes its GROUP's frame (the 4 lanes of a
// group load the same descriptor; the group's lane 0 parses, finishes and stores it),
// so no lane-to-lane broadcast is needed anywhere on the tile's critical path.
struct Tile {
    bool fvalid;
    uint32_t fi, len, nd, ndall, sa, te;
    uint64_t E, sdw;
    // row/header load addressing: the group's own frame, or for an empty group (no frame, or
    // a frame under 4 bytes, whose streams are never used) a longest frame of the tile, so
    // that every load -- including the unclamped fast-path refills -- stays inside a frame
    uint64_t ld_sdw;
    int ld_nd, ld_ndall;
    int R, Rp, rel0, lo;
    int Rh;            // wave-uniform: last row holding header dwords [0, kHdrDwords) of any frame
    int RF_lo, RF_hi;  // wave-uniform rows where every lane takes the fast path
    const uint32_t* gfb;
};

__device__ __forceinline__ void tile_descriptors(Tile& T, uint32_t tile, uint32_t grp, uint32_t n,
                                                 const uint64_t* __restrict__ offsets,
                                                 const uint32_t* __restrict__ lengths, uint64_t& S) {
    T.fi = tile * kFramesPerTile + grp;
    T.fvalid = T.fi < n;
    // groups past the batch end read the last frame's descriptor with length 0 (their loads
    // then use a longest frame of the tile, see tile_geometry; `frames` itself may lie
    // outside the allocation: the host-staged path passes staging - first offset)
    const uint32_t fl = T.fvalid ? T.fi : n - 1u;
    // Inline asm: hipcc otherwise sinks the loads into their first use (past the region-A
    // build and the tile branch), serializing two HBM round trips. The values are tied to
    // an explicit wait (descriptors_ready) before use.
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(S) : "v"(offsets + fl));
    asm volatile("global_load_dword %0, %1, off" : "=v"(T.len) : "v"(lengths + fl));
}

// vmcnt(0) tied to the descriptor registers, so no use of them is scheduled above it.
__device__ __forceinline__ void descriptors_ready(Tile& T, uint64_t& S) {
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(S), "+v"(T.len));
    if (!T.fvalid) T.len = 0;
}

// Wave max / min of a value that is uniform within each 4-lane group: two DPP row
// mirrors combine the 4 groups of a 16-lane row, 4 readlanes the rows (no LDS permutes).
template <bool kMax>
__device__ __forceinline__ int group_reduce(int x) {
    int y = __builtin_amdgcn_mov_dpp(x, 0x140, 0xf, 0xf, false);  // row_mirror
    x = kMax ? max(x, y) : min(x, y);
    y = __builtin_amdgcn_mov_dpp(x, 0x141, 0xf, 0xf, false);      // row_half_mirror
    x = kMax ? max(x, y) : min(x, y);
    const int a = __builtin_amdgcn_readlane(x, 0), b = __builtin_amdgcn_readlane(x, 16);
    const int c = __builtin_amdgcn_readlane(x, 32), d = __builtin_amdgcn_readlane(x, 48);
    return kMax ? max(max(a, b), max(c, d)) : min(min(a, b), min(c, d));
}

__device__ __forceinline__ void tile_geometry(Tile& T, uint64_t S, uint32_t gl, const uint8_t* __restrict__ frames) {
    T.E = S + T.len;
    T.sdw = S >> 2;
    T.ndall = (uint32_t)(((T.E + 3u) >> 2) - T.sdw);
    T.nd = (T.fvalid && T.len >= 4u) ? T.ndall : 0u;
    T.sa = (uint32_t)(S & 3u);
    T.te = (uint32_t)(T.E & 3u) ? (uint32_t)(T.E & 3u) : 4u;
    const int nd = (int)T.nd;
    const int rows = (nd + kRowDwords - 1) / kRowDwords;
    T.R = group_reduce<true>(rows);
    {
        const uint64_t ball = __ballot(rows == T.R);  // never 0: some lane holds the maximum
        const int src = (int)__builtin_ctzll(ball);
        const uint32_t s_lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)T.sdw, src);
        const uint32_t s_hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(T.sdw >> 32), src);
        const int s_nd = __builtin_amdgcn_readlane(nd, src);
        const bool borrow = nd == 0;
        T.ld_sdw = borrow ? (((uint64_t)s_hi << 32) | s_lo) : T.sdw;
        T.ld_nd = borrow ? s_nd : nd;
        T.ld_ndall = borrow ? s_nd : (int)T.ndall;
    }
    // Rows padded at the FRONT to a multiple of kPrefetch: leading all-zero rows
    // leave a zero-init CRC stream unchanged, so the loop needs no tail guard.
    T.Rp = (T.R + kPrefetch - 1) / kPrefetch * kPrefetch;
    T.gfb = reinterpret_cast<const uint32_t*>(frames + (T.ld_sdw << 2));
    const int base0 = nd - kRowDwords * T.Rp;  // rel of the group's lane 0 in row 0
    T.rel0 = T.ld_nd - kRowDwords * T.Rp + 4 * (int)gl;
    T.Rh = group_reduce<true>(nd > 0 ? (kHdrDwords - 1 - base0) / kRowDwords : -1);
    // Loads of rows that start before the frame are clamped to the frame's first chunk (its last
    // chunk for frames under 4 dwords), so lanes idling through a tile's longest frame re-read
    // one cached line instead of fetching the bytes that precede their frame; never below frames[0].
    T.lo = max(T.ld_sdw > (1u << 24) ? -(1 << 24) : -(int)T.ld_sdw, min(0, T.ld_nd - 4));
    // Fast rows: every lane's chunk [rel, rel+4) inside [kFastRel0, nd - 1) (no head/tail/init
    // masks, whole chunk streamed into the checksum): lane 0 of the group bounds the start,
    // lane 3 the end. Empty groups stream zeros and never force the slow path.
    int flo = -0x40000000, fhi = 0x40000000;
    if (nd > 0) {
        const int a = kFastRel0 - base0, b = nd - 5 - (base0 + 12);  // rows r with a <= 16 r <= b
        flo = (a <= 0) ? 0 : (a + kRowDwords - 1) / kRowDwords;
        fhi = (b < 0) ? -1 : b / kRowDwords;
    }
    T.RF_lo = group_reduce<true>(flo);
    T.RF_hi = group_reduce<false>(fhi);
}

// Region A in place: thread t builds Z64[b][e] (b = t >> 8, e = t & 255) as the XOR of
// the basis columns of e's set bits and stores its 8 copies (32 contiguous bytes).
// The basis row comes in by a scalar load (lgkmcnt), so waiting for it never waits for the
// descriptors' vector loads issued before it.
__device__ __forceinline__ void build_region_a(const FsTables* __restrict__ tabs, char* lds) {
    typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
    const uint32_t t = threadIdx.x;
    const uint32_t b = __builtin_amdgcn_readfirstlane(t >> 8);  // wave-uniform (64 | 256)
    const uint32_t e = t & 255u;
    const uint64_t a = reinterpret_cast<uint64_t>(&tabs->z64_basis[b][0]);
    const uint64_t sa = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a);
    u32x8 basis;
    asm volatile("s_load_dwordx8 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(basis) : "s"(sa));
    uint32_t v = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        const uint32_t m = 0u - ((e >> j) & 1u);
        v ^= basis[j] & m;
    }
    u32x4* dst = reinterpret_cast<u32x4*>(lds + e * 256u + 32u * b);
    dst[0] = u32x4{v, v, v, v};
    dst[1] = u32x4{v, v, v, v};
}

// The plain tables by LDS-DMA: exactly kDmaPerWave 1-KB pieces per wave (surplus pieces
// re-copy the last one with identical bytes). Inline asm, invisible to hipcc's vmcnt model
// (the builtin makes it drain later LDS reads with vmcnt(0)); unknown VMEM ops only make
// the compiler's own counted waits stricter. Waited for explicitly before the barrier.
// (m0 is reserved to the compiler: this kernel sets it nowhere else, checked in the asm)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void plain_dma(const FsTables* __restrict__ tabs, char* lds, uint32_t wave, uint32_t lane) {
    typedef __attribute__((address_space(3))) char lds_char;
    const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_char*)lds;
    const uint32_t w0 = __builtin_amdgcn_readfirstlane(wave);
#pragma unroll
    for (uint32_t k = 0; k < kDmaPerWave; ++k) {
        const uint32_t c = kPlainChunk0 + min(w0 + k * kWavesPerBlock, kPlainChunks - 1u);
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                     :
                     : "v"(reinterpret_cast<const char*>(tabs) + c * 1024u + lane * 16u),
                       "s"(__builtin_amdgcn_readfirstlane(lds0 + c * 1024u))
                     : "memory", "m0");
    }
}
#pragma clang diagnostic pop

__global__ void __launch_bounds__(kThreads, 1)
digest_kernel(const uint8_t* __restrict__ frames, const uint64_t* __restrict__ offsets,
              const uint32_t* __restrict__ lengths, uint32_t n, uint32_t mtu, const FsTables* __restrict__ tabs,
              uint2* __restrict__ out, uint8_t* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t grp = lane >> 2;   // frame slot of this lane's group
    const uint32_t gl = lane & 3u;    // lane within the group
    const uint32_t gwave = blockIdx.x * kWavesPerBlock + wave;
    const uint32_t nwaves = gridDim.x * kWavesPerBlock;
    const uint32_t ntiles = (n + kFramesPerTile - 1) / kFramesPerTile;
    const uint32_t hdr_wave = kLdsHdr + wave * kHdrWaveBytes;
    const uint32_t stash_base = kLdsStash + wave * (kFramesPerTile * kStashBytes);

    const uint32_t hb = hdr_wave + kHdrSlotBytes * grp;         // the group's header slot
    const uint32_t stash = stash_base + grp * kStashBytes;      // the group's last-row stash
    LaneKeys keys;
    {
        const uint32_t c = lane & 7u, h = (lane >> 3) & 3u;
        keys.cvec = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) keys.cvec |= (32u * j + 4u * c) << (8u * j);
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t b = (k + h) & 3u;
            keys.sel[k] = 0x0c0c0000u | ((4u + b) << 8) | b;
        }
    }

    // Preamble: the first tile's descriptors (one round trip), its geometry, the row
    // prefetch, and only THEN the table LDS-DMA, so that the CU's in-order vector-memory
    // queue serves the descriptors and the first rows before the 100 KB of table pieces;
    // the DMA (L2 hits) then overlaps the rows' HBM latency. hipcc does not count LDS-DMA
    // in its vmcnt model: the DMA is issued last and drained with an explicit vmcnt(0),
    // which the first row needs anyway.
    // Preamble: the first tile's descriptors (the first memory ops, one round trip) while
    // region A is built in place by VALU; geometry; the plain tables' LDS-DMA (36 KB, L2
    // hits); the row prefetch; one barrier once this wave's table pieces have landed.
    uint32_t tile = gwave;
    FS_RTSTAMP(5);
    FS_STAMP(0);
    Tile T;
    uint64_t S;
    u32x4 pf[kPrefetch];
    tile_descriptors(T, tile, grp, n, offsets, lengths, S);
    build_region_a(tabs, lds);
    descriptors_ready(T, S);
#if defined(FS_STAMPS) && FS_STAMPS == 2
    __builtin_amdgcn_s_waitcnt(0x0f70);  // fine-stamp build only: time the descriptor round trip
    FS_STAMP(8);
#endif
    bool rows0 = false;  // the first tile has rows (and so a row prefetch in flight)
    if (__builtin_amdgcn_readfirstlane(tile) < ntiles) {
        tile_geometry(T, S, gl, frames);
        rows0 = T.Rp > 0;
    }
    plain_dma(tabs, lds, wave, lane);
    if (rows0) {  // a tile of frames all under 4 bytes loads no rows (they could lie past the buffer)
#pragma unroll
        for (int i = 0; i < kPrefetch; ++i) pf[i] = load_chunk(T.gfb, T.rel0 + kRowDwords * i, T.lo);
    }
    FS_STAMP(9);
    // the table pieces are older than the rows: vmcnt(kPrefetch) (vmcnt(0) without rows);
    // lgkmcnt(0): this wave's region-A stores
    // s_waitcnt field layout (gfx9): vmcnt[3:0] + vmcnt_hi[15:14], expcnt[6:4], lgkmcnt[11:8]
    if (rows0) __builtin_amdgcn_s_waitcnt(0x0070 | kPrefetch);
    else __builtin_amdgcn_s_waitcnt(0x0070);
    FS_STAMP(10);
    __builtin_amdgcn_s_barrier();  // tables ready (raw barrier: no release fence, no vmcnt(0) drain)
    FS_STAMP(1);

    while (tile < ntiles) {
        RowMasks M;
        M.nd = (int)T.nd;
        M.head_mask = 0xffffffffu << (8u * T.sa);
        M.init1 = (1u << (8u * T.sa)) - 1u;
        M.tail_mask = (T.te == 4u) ? 0xffffffffu : ((1u << (8u * T.te)) - 1u);

        // ---- main loop: rows 0..Rp-1 in blocks of kPrefetch rows with kPrefetch rows in
        // flight; the last block does not refill (nothing lies past the frame end). Blocks
        // whose rows are all fast for every lane run the lean path: four Z64 steps + four
        // v_sad_u16 per row and a refill with an immediate row offset.
        uint32_t A[4] = {0u, 0u, 0u, 0u};
        uint32_t cs = 0u;
        const bool parser = T.fvalid && gl == 0u;  // the group's lane 0 parses, finishes and stores
        // the header parse runs once the block holding row Rh (the last row with header dwords)
        // has been captured, while the ring's loads are in flight
        const uint64_t fS = T.E - T.len;
        const uint32_t fsa = T.sa, flen = T.len;
        auto parse = [&]() {
            if (parser) park_parsed(lds, hb, parse_frame(lds, hb, fsa, flen, mtu), fS, flen);
        };
        auto prio = [&](int r0) {
            // Self-balancing issue priority: the SIMD arbiter favours the oldest wave,
            // a wave with more rows left gets a higher priority.
            if (FS_PRIO == 2) {
                // static, inverted age rank: the SIMD arbiter favours older waves on ties, so
                // the younger waves (higher wave index) get the higher priority
                const uint32_t rank = __builtin_amdgcn_readfirstlane(wave) >> 2;
                if (rank == 3) __builtin_amdgcn_s_setprio(3);
                else if (rank == 2) __builtin_amdgcn_s_setprio(2);
                else if (rank == 1) __builtin_amdgcn_s_setprio(1);
                else __builtin_amdgcn_s_setprio(0);
            } else if (FS_PRIO) {
                const int left4 = (4 * (T.Rp - r0)) / max(T.Rp, 1);  // 4 .. 1
                if (left4 >= 4) __builtin_amdgcn_s_setprio(3);
                else if (left4 == 3) __builtin_amdgcn_s_setprio(2);
                else if (left4 == 2) __builtin_amdgcn_s_setprio(1);
                else __builtin_amdgcn_s_setprio(0);
            }
        };
        // general block: per-row fast/slow (scalar), header capture for rows <= Rh (scalar),
        // clamped refill addresses
        auto block = [&](int r0, auto refill_tag) {
            constexpr bool kRefill = decltype(refill_tag)::value;
            prio(r0);
#pragma unroll
            for (int i = 0; i < kPrefetch; ++i) {
                const int r = r0 + i;
                const int rel = T.rel0 + kRowDwords * r;
                const bool fast = (r >= T.RF_lo) && (r <= T.RF_hi);  // wave-uniform (scalar)
                if (r <= T.Rh) capture_header(lds, hb, rel, T.lo, pf[i]);
                // consume the ring slot, then refill the SAME registers: no copy of an
                // in-flight load, so the compiler keeps kPrefetch-1 loads outstanding
                process_row(lds, keys, pf[i], rel, fast, M, T.lo, A, cs);
                if (kRefill && FS_DIAG != 3) pf[i] = load_chunk(T.gfb, rel + kRowDwords * kPrefetch, T.lo);
            }
        };
        // lean block: every row fast for every lane; the refills of a fast row's successors
        // lie inside the frame, so they need no clamp: one pointer per block, immediate
        // row offsets
        auto lean_block = [&](int r0) {
            prio(r0);
            const uint32_t* pb = T.gfb + (T.rel0 + kRowDwords * (r0 + kPrefetch));
#pragma unroll
            for (int i = 0; i < kPrefetch; ++i) {
                process_row(lds, keys, pf[i], 0, true, M, 0, A, cs);
                if (FS_DIAG != 3) pf[i] = *reinterpret_cast<const u32x4_a4*>(pb + kRowDwords * i);
                // keep consume/refill interleaved per row: unfenced, the scheduler sinks all
                // refills to the block end behind a vmcnt(0), draining the ring every block
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        using Yes = std::true_type;
        using No = std::false_type;
        const int Rc = T.Rp - kPrefetch;
        if (T.Rp > 0) {
            // blocks: [head: general] [body: lean] [tail: general] [last: general, no refill],
            // as three loops in sequence (one code path per loop keeps the ring registers fixed)
            // (a block is lean only past Rh, so the header rows are always in general blocks)
            int r0 = 0;
            for (; r0 < Rc && !(r0 > T.Rh && r0 >= T.RF_lo && r0 + kPrefetch - 1 <= T.RF_hi); r0 += kPrefetch) {
                block(r0, Yes());
                if (T.Rh >= r0 && T.Rh < r0 + kPrefetch) parse();
            }
            for (; r0 < Rc && r0 + kPrefetch - 1 <= T.RF_hi; r0 += kPrefetch) lean_block(r0);
            for (; r0 < Rc; r0 += kPrefetch) block(r0, Yes());
            block(Rc, No());
            if (T.Rh >= Rc) parse();
        } else {
            parse();  // no rows (every frame of the tile under 4 bytes): rejected by length
        }
        FS_STAMP(2);
        // the last ring slot holds the frame's final row: stash it for the padding sum
        *reinterpret_cast<u32x4*>(lds + stash + 16u * gl) = pf[kPrefetch - 1];

        // ---- combine the 16 streams of each frame: C = Z_(4-t)( xor_l Z_16(3-l)( U_l ) ),
        //      U_l = Z12(A0) ^ Z8(A1) ^ Z4(A2) ^ A3   (3 dependent LDS round trips).
        const uint32_t U = zplain(lds, A[0], kLdsZ12) ^ zplain(lds, A[1], kLdsZ8) ^ zplain(lds, A[2], kLdsZfin) ^ A[3];
        const uint32_t ybase = (gl == 0u) ? kLdsZ48 : (gl == 1u) ? kLdsZ32 : kLdsZ16;
        uint32_t Y = zplain(lds, U, ybase);
        if (gl == 3u) Y = U;
        Y ^= dpp_quad<kQuadXor1>(Y);
        Y ^= dpp_quad<kQuadXor2>(Y);
        // checksum partial sum over the 4 lanes of the group (each < 2^30: no u32 overflow)
        cs += dpp_quad<kQuadXor1>(cs);
        cs += dpp_quad<kQuadXor2>(cs);
        const uint64_t csum = cs;

        FS_STAMP(3);
        // ---- the group's lane 0: finish and store (its frame's state comes back from LDS).
        if (parser) {
            uint64_t fS;
            uint32_t flen;
            const Parsed P = unpark_parsed(lds, hb, fS, flen);
            const uint64_t fE = fS + flen, fsdw = fS >> 2;
            const uint32_t fsa = (uint32_t)(fS & 3u), fte = (uint32_t)(fE & 3u) ? (uint32_t)(fE & 3u) : 4u;
            const uint32_t fnd = flen >= 4u ? (uint32_t)(((fE + 3u) >> 2) - fsdw) : 0u;
            const uint32_t fi = tile * kFramesPerTile + grp;
            uint32_t crcv;
            if (flen < 4u) {  // too short for the 4-byte init trick: bytewise CRC-32
                uint32_t c = 0xffffffffu;
                const uint8_t* fbytes = frames + fS;
                for (uint32_t p = 0; p < flen; ++p)
                    c = lds32(lds, kLdsZfin + 3u * 4096u + (((c ^ fbytes[p]) & 0xffu) << 2)) ^ (c >> 8);
                crcv = ~c;
            } else {
                const uint32_t tpad = (4u - fte) & 3u;  // zero bytes appended by the dword rounding
                crcv = ~zplain(lds, Y, kLdsZfin + 4096u * tpad);
            }
            uint32_t verdict = P.verdict, l4 = 0u;
            if (P.compute) {
                const uint32_t* fb = reinterpret_cast<const uint32_t*>(frames + fsdw * 4u);
                l4 = finish_l4(lds, stash, fb, fsa, flen, fnd, P, csum, verdict);
            }
            out[fi] = make_uint2(crcv, P.ip_csum | (l4 << 16));
            if (status) status[fi] = (uint8_t)verdict;
        }
        FS_STAMP(4);
        FS_RTSTAMP(6);
        tile += nwaves;
        if (tile < ntiles) {  // next tile: descriptors, geometry, row prefetch
            tile_descriptors(T, tile, grp, n, offsets, lengths, S);
            descriptors_ready(T, S);
            tile_geometry(T, S, gl, frames);
            if (T.Rp > 0) {
#pragma unroll
                for (int i = 0; i < kPrefetch; ++i) pf[i] = load_chunk(T.gfb, T.rel0 + kRowDwords * i, T.lo);
            }
        }
    }
}

}  // namespace

#ifdef FS_STAMPS
extern "C" int fs_debug_read_stamps(void* host, size_t bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fs_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
#endif

hipError_t launch_digest(const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths, uint32_t n,
                         uint32_t mtu, const FsTables* tables, void* out, uint8_t* status, hipStream_t stream,
                         int num_cus) {
    if (n == 0) return hipSuccess;
    const uint32_t ntiles = (n + kFramesPerTile - 1) / kFramesPerTile;
    uint32_t blocks = (ntiles + kWavesPerBlock - 1) / kWavesPerBlock;
    const uint32_t max_blocks = (uint32_t)(num_cus > 0 ? num_cus : 256);
    if (blocks > max_blocks) blocks = max_blocks;
    hipLaunchKernelGGL(digest_kernel, dim3(blocks), dim3(kThreads), 0, stream, frames, offsets, lengths, n, mtu,
                       tables, reinterpret_cast<uint2*>(out), status);
    return hipGetLastError();
}

}  // namespace framesum
