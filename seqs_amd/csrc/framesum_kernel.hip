// framesum digest kernels — CDNA4 / gfx950.
//
// One fused pass per frame over HBM computes
//   * the IEEE CRC-32 of frame[0:len)                     (new: SURVEY.md §0.1)
//   * IPv4Header.CalculateChecksum() of frame[14:34]      (eth/headers.go:333-340)
//   * the TCP/UDP checksum RecvEth verifies + its verdict (stacks/portstack.go:163-308,
//     eth/headers.go:382-393, :510-527, arithmetic of eth/crc.go:13-84)
// and, as the TX fill (fs_fill_batch), writes the checksums and/or the FCS into the frames.
//
// Two kernels; launch_digest (bottom) picks one per launch, never changing a result:
//   * digest_kernel_a, the ONE-PASS kernel (batches of similar lengths, e.g. C2): a 16-wave
//     workgroup per CU, persistent; a wave owns a TILE of 16 frames, each frame a 4-lane GROUP.
//     Rows are the 64-B blocks (half 128-B lines) that hold the frame, the last one ending on
//     the block boundary after the frame end: lane l of the group loads dwords
//     [4l, 4l+4) of every row with one global_load_dwordx4, kRingA rows ahead. Rows before the
//     frame's first block reload that block (no byte before the frame's page is touched). The
//     frame's first 3 blocks are copied from the first rows into a per-wave LDS header slot as
//     they are consumed (header capture: no extra load), and the parse reads them there.
//   * digest_kernel_ab, the MIXED-LENGTH kernel (e.g. C3): the same rows end-anchored at the
//     frame's dword-rounded end, header slots by dword LDS-DMA, and tiles whose frames differ
//     widely in length cut their long frames into 768-B PIECES spread over the groups the short
//     frames leave idle (mode B), combined per frame with Z768 Horner steps.
// Both:
//   * LEAN rows carry no mask. The head rows (bytes before the frame, the CRC init on frame
//     dwords 0/1) take the masked path; bytes past the frame end in the last row are masked
//     (one-pass) or removed linearly at the combine (mixed).
//   * CRC: each lane keeps 4 independent dword STREAMS; a stream's successive dwords are 64 B
//     apart, so its Horner step is  A <- Z64(A) ^ w  with Z64 a fixed GF(2) linear map evaluated
//     by 4 byte-table lookups in LDS. After the last row the 16 streams of a frame are shifted
//     to the frame end and XOR-ed over the group (DPP). Leading zero rows do not change a
//     zero-init CRC; the init is applied by XOR-ing the frame's first 4 bytes with 0xFF.
//   * one's-complement sum: the same registers feed v_sad_u16 (acc += lo16 + hi16, one op per
//     dword; congruent mod 65535 to the byte-swapped big-endian word sum) over every frame byte;
//     the header parse computes, in the same domain, the sums of the Ethernet + IP header bytes,
//     of the excluded words and of the Ethernet padding (vectorised over the group's 4 lanes)
//     and the pseudo-header, and the finish folds with a positive offset so RecvEth's Sum16
//     result (incl. the 0x0000 / 0xFFFF edge) is reproduced bit for bit.
//   * LDS tables, built in place by VALU from their GF(2) bases (FsTables): the hot Z64 table
//     as 8 copies per byte table in an [entry][table*8+copy] layout, 256 B per entry. Lane
//     L = c + 8h of a 32-lane bank group reads table (k+h)&3 in its k-th lookup, so the 32
//     lanes hit 32 distinct banks: conflict-free ds_read_b32 for any data. One v_perm_b32 forms
//     the LDS address (entry byte | per-lane slot byte). The plain [4][256] tables (combine,
//     finish) follow.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "framesum_internal.h"

namespace framesum {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 16;
constexpr int kThreads = kWave * kWavesPerBlock;
constexpr int kFramesPerTile = 16;
constexpr int kRowDwords = 16;
constexpr int kPrefetch = 6;  // the mixed-length kernel's ring (a divisor of kPieceRows)
// ... with block-aligned rows: an MTU frame (1500 B) spans 24 or 25 blocks, so a tile's rows
// are a multiple of 5 with no padding row
constexpr int kRingA = 5;  // the one-pass kernel's ring
constexpr int kPrioMinRows = 36;  // the one-pass kernel's progress-based priority: tiles of more rows than this

// Header slots: frame dwords [0, 32) of each group's frame, written by 8 dword LDS-DMA
// instructions per wave in the layout [x >> 2][group][x & 3] (256 B per instruction),
// so the DMA destination is lane-linear and both the parser lanes (one per group, same x)
// and the group-vectorised sums (lane gl reads x = 4i + gl) read conflict-free.
constexpr int kHdrDwords = 32;
constexpr uint32_t kHdrWaveBytes = 4u * kHdrDwords * kFramesPerTile;  // 2 KB

// LDS map (bytes). [0, 104 KB) holds the tables: the plain tables first, then region A, both
// built in place by VALU from their GF(2) bases (build_region_a; FsTables keeps the full image
// only as the layout's reference). Every table address is a constant below 64 KB plus a lane-dependent part, so
// hipcc folds the constant into the ds_read offset field instead of holding it in a VGPR.
constexpr uint32_t kLdsZ32 = 0;
constexpr uint32_t kLdsZ16 = kLdsZ32 + 4096;
constexpr uint32_t kLdsZfin = kLdsZ16 + 4096;  // Z4, Z3, Z2, Z1 (4 KB each)
constexpr uint32_t kLdsZ48 = kLdsZfin + 16384;
constexpr uint32_t kLdsZ12 = kLdsZ48 + 4096;
constexpr uint32_t kLdsZ8 = kLdsZ12 + 4096;
constexpr uint32_t kLdsZ768 = kLdsZ8 + 4096;    // Z_768: shift past one full piece (mode B)
constexpr uint32_t kLdsRegionA = kLdsZ768 + 4096;  // 64 KB: [entry][table*8+copy], 256 B per entry
constexpr uint32_t kLdsTables = kLdsRegionA + 65536;
constexpr uint32_t kLdsHdr = kLdsTables;
static_assert(kLdsRegionA < 65536, "ds_read offset field");
// mode B pieces (see "Tiles, pieces and passes")
constexpr int kPieceRows = 12;
constexpr int kPieceDwords = kPieceRows * kRowDwords;  // 192 dwords = 768 bytes
constexpr int kMaxFullPasses = 6;
constexpr uint32_t kWaveScratchBytes = 16u * kFramesPerTile + 8u * kFramesPerTile +
                                       8u * (kFramesPerTile + kFramesPerTile * kMaxFullPasses);
constexpr uint32_t kLdsWave = kLdsHdr + kWavesPerBlock * kHdrWaveBytes;
constexpr uint32_t kLdsBytes = kLdsWave + kWavesPerBlock * kWaveScratchBytes;
static_assert(kWaveScratchBytes >= 3u * 256u, "a parked parse (12 dwords x 16 frames, header-slot layout) fits the wave scratch");
static_assert(kPieceRows % kPrefetch == 0, "a piece is whole blocks of rows");
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");
static_assert(kTablesLdsBytes == kLdsTables, "FsTables is the LDS image of the tables");

// The workgroup's LDS image (static allocation of the digest kernels). Namespace scope, so the
// out-of-line parse routine addresses it as LDS (ds_read), not through a flat pointer.
__shared__ __attribute__((aligned(16))) char g_lds[kLdsBytes];

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
    V_PROTO = 8, V_SHORT = 9, V_ZEROPORT = 10, V_UDPLEN = 11, V_TCPOFF = 12, V_CSUM = 13, V_FCS = 14
};

// Kernel operations (a template parameter: each is its own instantiation, so the plain digest
// carries no code of the others).
//   kOpsDigest : RX digest + verdict (fs_digest_batch)
//   kOpsTx     : TX fill (fs_fill_batch): the runtime `tx` word's kTxFill writes the IPv4 and L4
//                checksums into the frame, kTxAppend the FCS after it; the digest is that of
//                the frame as written
//   kOpsFcs    : RX of wire frames with a trailing FCS (fs_digest_batch_fcs)
enum : uint32_t { kOpsDigest = 0, kOpsTx = 1, kOpsFcs = 2 };
enum : uint32_t { kTxFill = 1, kTxAppend = 2 };

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

// Z64(a) ^ w from replicated region A. Conflict-free.
template <uint32_t kRegion = kLdsRegionA>
__device__ __forceinline__ uint32_t zrep(const char* lds, uint32_t a, const LaneKeys& k, uint32_t w) {
    uint32_t t0 = lds32(lds, kRegion + __builtin_amdgcn_perm(a, k.cvec, k.sel[0]));
    uint32_t t1 = lds32(lds, kRegion + __builtin_amdgcn_perm(a, k.cvec, k.sel[1]));
    uint32_t t2 = lds32(lds, kRegion + __builtin_amdgcn_perm(a, k.cvec, k.sel[2]));
    uint32_t t3 = lds32(lds, kRegion + __builtin_amdgcn_perm(a, k.cvec, k.sel[3]));
    return xor3(xor3(t0, t1, t2), t3, w);
}

// Z operator from a plain [4][256] table (a few uses per frame).
__device__ __forceinline__ uint32_t zplain(const char* lds, uint32_t a, uint32_t base) {
    return lds32(lds, base + ((a & 0xffu) << 2)) ^ lds32(lds, base + 1024 + (((a >> 8) & 0xffu) << 2)) ^
           lds32(lds, base + 2048 + (((a >> 16) & 0xffu) << 2)) ^ lds32(lds, base + 3072 + ((a >> 24) << 2));
}

template <int kCtrl>
__device__ __forceinline__ uint32_t dpp_quad(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kCtrl, 0xf, 0xf, false);
}

__device__ __forceinline__ uint32_t bswap16(uint32_t v) { return ((v & 0xffu) << 8) | ((v >> 8) & 0xffu); }

// One's-complement accumulation: v_sad_u16(x, 0, acc) = acc + x[15:0] + x[31:16] in ONE op.
// x[15:0] + x[31:16] is congruent to the dword's native little-endian value mod 65535 and
// is 0 iff the dword is 0, which is all Sum16's fold needs. It is linear
// over disjoint byte masks (no carry crosses a byte). A lane adds at most 2^15 dwords of a
// frame under 512 KiB, each < 2^17, so the 32-bit accumulator cannot wrap there.
__device__ __forceinline__ uint32_t sad16(uint32_t x, uint32_t acc) { return __builtin_amdgcn_sad_u16(x, 0u, acc); }

// bytes of absolute dword k that lie in the absolute byte range [a0, a1)
__device__ __forceinline__ uint32_t range_mask(int k, int a0, int a1) {
    const int lo = min(max(a0 - 4 * k, 0), 4), hi = min(max(a1 - 4 * k, 0), 4);
    const uint32_t m = (0xffffffffu >> (32 - 8 * (hi - lo))) << (8 * lo);
    return hi > lo ? m : 0u;
}

// ---------------------------------------------------------------------------------------
// Rows.

// A lean row: four Z_stride steps and four v_sad_u16, no masks.
template <uint32_t kRegion = kLdsRegionA>
__device__ __forceinline__ void lean_row(const char* lds, const LaneKeys& k, u32x4 v, uint32_t (&A)[4], uint32_t& cs) {
    A[0] = zrep<kRegion>(lds, A[0], k, v.x);
    A[1] = zrep<kRegion>(lds, A[1], k, v.y);
    A[2] = zrep<kRegion>(lds, A[2], k, v.z);
    A[3] = zrep<kRegion>(lds, A[3], k, v.w);
    cs = sad16(v.x, cs);
    cs = sad16(v.y, cs);
    cs = sad16(v.z, cs);
    cs = sad16(v.w, cs);
}

// A masked row: the chunk was loaded from frame dword p (= rel unless clamped up, see
// load_pos); realign it to [rel, rel+4), zero the dwords before the frame, mask the head and
// tail bytes and apply the CRC init.
// nd: frame dwords (0 = nothing to stream); sa: S & 3; tail_mask: bytes of dword nd-1 inside
// the frame. The head mask (bytes of dword 0 inside the frame) is also the CRC init's part in
// dword 0; its complement is the init's part in dword 1.
template <uint32_t kRegion = kLdsRegionA>
__device__ __forceinline__ void masked_row(const char* lds, const LaneKeys& k, u32x4 u, int rel, int p, int nd,
                                           uint32_t sa, uint32_t tail_mask, uint32_t (&A)[4], uint32_t& cs) {
    const uint32_t head_mask = 0xffffffffu << (8u * sa);
    const int sh = p - rel;  // > 0 only for a clamped chunk; then every dword below p lies before the frame
    uint32_t v[4];
    v[0] = u.x;
    v[1] = (sh == 0) ? u.y : u.x;
    v[2] = (sh == 0) ? u.z : (sh == 1) ? u.y : u.x;
    v[3] = (sh == 0) ? u.w : (sh == 1) ? u.z : (sh == 2) ? u.y : u.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int x = rel + j;
        uint32_t d = (x >= 0) ? v[j] : 0u;
        uint32_t c = 0u;
        if (x == 0) { d &= head_mask; c = head_mask; }
        if (x == 1) c = ~head_mask;
        if (x == nd - 1) d &= tail_mask;
        A[j] = zrep<kRegion>(lds, A[j], k, d ^ c);
        cs = sad16(d, cs);
    }
}

// Block-aligned rows (digest_kernel_a<kOps, true>): a chunk is always loaded where it lies (or,
// wholly before the frame, somewhere irrelevant), so no realignment. Dwords at or past the frame
// end (only in the last row) leave the stream untouched: the combine then shifts that stream
// by its distance to the frame end, which the skipped update would have overshot.
template <uint32_t kRegion = kLdsRegionA>
__device__ __forceinline__ void masked_row_al(const char* lds, const LaneKeys& k, u32x4 u, int rel, int nd,
                                              uint32_t sa, uint32_t tail_mask, uint32_t (&A)[4], uint32_t& cs) {
    const uint32_t head_mask = 0xffffffffu << (8u * sa);
    const uint32_t v[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int x = rel + j;
        uint32_t d = (x >= 0) ? v[j] : 0u;
        uint32_t c = 0u;
        if (x == 0) { d &= head_mask; c = head_mask; }
        if (x == 1) c = ~head_mask;
        if (x == nd - 1) d &= tail_mask;
        const bool in = x < nd;
        const uint32_t a = zrep<kRegion>(lds, A[j], k, d ^ c);
        A[j] = in ? a : A[j];
        cs = sad16(in ? d : 0u, cs);
    }
}
// The last row of block-aligned rows when it is otherwise lean.
template <uint32_t kRegion = kLdsRegionA>
__device__ __forceinline__ void tail_row_al(const char* lds, const LaneKeys& k, u32x4 u, int rel, int nd,
                                            uint32_t tail_mask, uint32_t (&A)[4], uint32_t& cs) {
    const uint32_t v[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int x = rel + j;
        const uint32_t d = (x == nd - 1) ? (v[j] & tail_mask) : v[j];
        const bool in = x < nd;
        const uint32_t a = zrep<kRegion>(lds, A[j], k, d);
        A[j] = in ? a : A[j];
        cs = sad16(in ? d : 0u, cs);
    }
}

// ---------------------------------------------------------------------------------------
// Header slot (frame dwords [0, 32) of the group's frame, layout [x>>2][group][x&3]).

__device__ __forceinline__ uint32_t hdr_at(uint32_t hw, uint32_t g, uint32_t x) {
    return hw + ((x >> 2) << 8) + (g << 4) + ((x & 3u) << 2);
}
__device__ __forceinline__ uint32_t hdr_dw(const char* lds, uint32_t hw, uint32_t g, uint32_t x) {
    return lds32(lds, hdr_at(hw, g, x));
}
// frame bytes [4j, 4j+4) as a little-endian dword (slot dwords are absolute, sa = S & 3). `xo`:
// the slot dword that holds frame dword 0 (0 for the DMA'd slot; the block phase for a slot
// captured from block-aligned rows, which starts at the frame's first 64-B block)
__device__ __forceinline__ uint32_t frame_dw(const char* lds, uint32_t hw, uint32_t g, uint32_t sa, uint32_t j,
                                             uint32_t xo = 0u) {
    return __builtin_amdgcn_alignbyte(hdr_dw(lds, hw, g, xo + j + 1), hdr_dw(lds, hw, g, xo + j), sa);
}

// frame_dw for a slot of kSlotDw dwords: dwords past the slot come from global memory,
// clamped to the frame's last dword `last` as the DMA clamps them.
template <int kSlotDw>
__device__ __forceinline__ uint32_t frame_dw_t(const char* lds, uint32_t hw, uint32_t g, uint32_t sa, uint32_t j,
                                               const uint32_t* fb, uint32_t last, uint32_t xo = 0u) {
    if (kSlotDw >= 32 || j + 1 < (uint32_t)kSlotDw) return frame_dw(lds, hw, g, sa, j, xo);
    const uint32_t a = fb[min(j, last)], b = fb[min(j + 1u, last)];
    return __builtin_amdgcn_alignbyte(b, a, sa);
}

// Sum, in the accumulator's 16-bit-half domain, of frame bytes [p0, p1) held in the slot's
// first 4*nx dwords, split over the group's 4 lanes (lane gl takes dwords 4i + gl) and
// totalled over the group by DPP. Every lane of the group calls it with the same arguments.
__device__ __forceinline__ uint32_t slot_sum(const char* lds, uint32_t hw, uint32_t g, uint32_t gl, uint32_t sa,
                                             int p0, int p1, int nx, uint32_t xo = 0u) {
    const int a0 = (int)sa + p0, a1 = (int)sa + p1;
    uint32_t s = 0;
    for (int i = 0; i < nx; ++i) {
        const int x = 4 * i + (int)gl;
        s = sad16(hdr_dw(lds, hw, g, xo + (uint32_t)x) & range_mask(x, a0, a1), s);
    }
    s += dpp_quad<kQuadXor1>(s);
    s += dpp_quad<kQuadXor2>(s);
    return s;
}

// exact sum of frame bytes [p0, p1) straight from global memory (rare paths)
// (through a global-address-space pointer: inside the out-of-line parse a plain pointer argument
// is generic, and a flat load there made hipcc's wait counting fall back to vmcnt(0))
typedef __attribute__((address_space(1))) const uint32_t gcu32;
__device__ __forceinline__ uint32_t global_sum(const uint32_t* fb, uint32_t sa, int p0, int p1) {
    uint32_t s = 0;
    if (p1 <= p0) return s;
    const int a0 = (int)sa + p0, a1 = (int)sa + p1;
    gcu32* gfb = reinterpret_cast<gcu32*>(reinterpret_cast<uintptr_t>(fb));
    for (int k = a0 >> 2; k <= (a1 - 1) >> 2; ++k) s = sad16(gfb[k] & range_mask(k, a0, a1), s);
    return s;
}

// Header parse result of one frame (parser lane), computed while its rows stream.
struct Parsed {
    uint32_t verdict;   // final unless `compute`
    uint32_t ip_csum;
    uint32_t stored;    // stored L4 checksum (BE)
    int compute;        // the L4 checksum is computed
    int parity;         // absolute parity of the L4 start (1 = odd)
    uint32_t off, end;  // L4 segment [off, end) (frame-relative)
    int64_t corr;       // every checksum correction (16-bit-half domain)
    int64_t corr_fixed; // the pseudo-header and excluded-word part of corr
    uint32_t aux;       // kOpsTx: stored IPv4 checksum | L4 checksum field offset << 16
};

// Header parse for one frame (parser lane). Gates follow stacks/portstack.go:163-308
// exactly (oracle/framesum_oracle.c restates them line by line; the parity tests
// compare the two). Reads only the LDS header slot; `hsum` = sum of frame bytes [0, off)
// and `pad` = sum of the Ethernet padding [end, len), both from the group-vectorised sums
// (pad < 0: the padding lies past the slot, summed here from global memory).
template <uint32_t kOps, int kSlotDw = kHdrDwords>
__device__ __forceinline__ Parsed parse_frame(const char* lds, uint32_t hw, uint32_t g, uint32_t sa, uint32_t len, uint32_t mtu,
                              uint32_t hsum, int64_t pad, const uint32_t* fb, uint32_t xo = 0u) {
    Parsed r = {V_OK, 0u, 0u, 0, 0, 0u, 0u, 0, 0, 0u};
    if (len < 34u) { r.verdict = V_SMOL; return r; }                          // portstack.go:167-168
    if (mtu != 0 && len > mtu) { r.verdict = V_MTU; return r; }              // :169-172
    uint32_t bs[9];                                                           // bswap32(frame dword j), j = 3..8
#pragma unroll
    for (uint32_t j = 3; j < 9; ++j) bs[j] = __builtin_bswap32(frame_dw(lds, hw, g, sa, j, xo));
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
    for (uint32_t i = 0; i < 6; ++i)
        lb[i] = __builtin_bswap32(frame_dw_t<kSlotDw>(lds, hw, g, sa, q + i, fb, ((sa + len + 3u) >> 2) - 1u, xo));
    const uint32_t sport = lb[0] & 0xffffu, dport = lb[1] >> 16;
    uint32_t lenword;
    if (proto == 17u) {                                                       // :222-244
        if (l4len < 8u) { r.verdict = V_SHORT; return r; }
        const uint32_t ulen = lb[1] & 0xffffu;
        if (sport == 0 || dport == 0) { r.verdict = V_ZEROPORT; return r; }
        if (ulen < 8u) { r.verdict = V_UDPLEN; return r; }
        lenword = ulen;                                                       // headers.go:386-390
        r.stored = lb[2] >> 16;
    } else if (proto == 6u) {                                                 // :283-308
        if (l4len < 20u) { r.verdict = V_SHORT; return r; }
        const uint32_t toff = ((lb[3] >> 12) & 0xfu) * 4u;                    // headers.go:477-485
        if (sport == 0 || dport == 0) { r.verdict = V_ZEROPORT; return r; }
        if (toff < 20u || toff > l4len) { r.verdict = V_TCPOFF; return r; }
        lenword = (tl - ipoff) & 0xffffu;                                     // headers.go:516
        r.stored = lb[4] & 0xffffu;
    } else {
        r.verdict = V_PROTO;                                                  // :220-221
        return r;
    }
    r.compute = 1;
    r.off = off;
    r.end = end;
    if (kOps == kOpsTx) r.aux = (bs[6] >> 16) | ((off + (proto == 6u ? 16u : 6u)) << 16);
    // Total over [off, end) = all streamed frame bytes [0, len) + these corrections, in the
    // 16-bit-half domain: a big-endian word at frame offset p (even) weighs 256^((sa + p) & 1),
    // i.e. it enters as itself when the L4 start is odd, byte-swapped when even.
    r.parity = (int)((sa + off) & 1u);
    const bool odd = r.parity != 0;
    // excluded words: the stored checksum (UDP headers.go:386-390; TCP :518-526) and, for
    // TCP, the urgent pointer (:518-526 never adds it)
    int64_t t = -(int64_t)(odd ? r.stored : bswap16(r.stored));
    if (proto == 6u) {
        const uint32_t urg = lb[5] >> 16;
        t -= (int64_t)(odd ? urg : bswap16(urg));
    }
    const uint32_t w[6] = {bs[6] & 0xffffu, bs[7] >> 16, bs[7] & 0xffffu, bs[8] >> 16, proto, lenword};
#pragma unroll
    for (int i = 0; i < 6; ++i) t += (int64_t)(odd ? w[i] : bswap16(w[i]));
    r.corr_fixed = t;
    t -= (int64_t)hsum;  // the Ethernet + IP header bytes [0, off)
    if (end < len) t -= (pad >= 0) ? pad : (int64_t)global_sum(fb, sa, (int)end, (int)len);
    r.corr = t;
    return r;
}

// The parse result lives in LDS while the rows stream (it would otherwise hold 11 VGPRs
// across the row loops): dwords 0..10 of the group's header slot, dead after the parse and
// rewritten only by the next tile's header DMA, after this tile's finish.
template <uint32_t kOps>
__device__ __forceinline__ void park_parsed(char* lds, uint32_t hw, uint32_t g, const Parsed& P) {
    constexpr uint32_t kN = kOps == kOpsTx ? 12 : 11;
    const uint32_t v[12] = {P.verdict, P.ip_csum, P.stored, (uint32_t)P.compute, (uint32_t)P.parity, P.off, P.end,
                            (uint32_t)P.corr, (uint32_t)((uint64_t)P.corr >> 32), (uint32_t)P.corr_fixed,
                            (uint32_t)((uint64_t)P.corr_fixed >> 32), P.aux};
#pragma unroll
    for (uint32_t k = 0; k < kN; ++k) *reinterpret_cast<uint32_t*>(lds + hdr_at(hw, g, k)) = v[k];
}
template <uint32_t kOps>
__device__ __forceinline__ Parsed unpark_parsed(const char* lds, uint32_t hw, uint32_t g) {
    constexpr uint32_t kN = kOps == kOpsTx ? 12 : 11;
    uint32_t v[12];
    v[11] = 0u;
#pragma unroll
    for (uint32_t k = 0; k < kN; ++k) v[k] = hdr_dw(lds, hw, g, k);
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
    P.aux = v[11];
    return P;
}

// The whole header parse of a tile, out of line so that its registers are allocated apart
// from the row loop's (it needs fewer than the 40 VGPRs below the callee-saved range, so the
// call saves nothing). Every lane takes part: group-vectorised sums over the header slot
// (the bytes [0, off) of the Ethernet + IP headers; the Ethernet padding [end, len) when it
// lies in the slot), then the parser lane's gates and corrections, parked in LDS.
// `pk`: where the parse result is parked (the header slot itself).
template <uint32_t kOps, int kSlotDw = kHdrDwords>
__device__ __attribute__((noinline)) void parse_tile(uint32_t hw, uint32_t grp, uint32_t gl, uint32_t sa, uint32_t len,
                                                     uint32_t mtu, const uint32_t* fbs, bool parser, uint32_t pk,
                                                     uint32_t xo = 0u) {
    const char* lds = g_lds;
    const uint32_t d3 = __builtin_bswap32(frame_dw(lds, hw, grp, sa, 3, xo));
    const uint32_t off = 14u + ((d3 >> 8) & 0xfu) * 4u;
    const uint32_t tl = __builtin_bswap32(frame_dw(lds, hw, grp, sa, 4, xo)) >> 16;
    const uint32_t end = (14u + tl) & 0xffffu;
    // [0, off) spans at most 3 + 74 bytes: absolute dwords < 20 (a 16-dword slot holds [0, 64 - sa);
    // longer IP headers are summed from global memory)
    const uint32_t h1 = min(off, len);
    uint32_t hsum = slot_sum(lds, hw, grp, gl, sa, 0, (int)h1, min(5, kSlotDw / 4), xo);
    if (kSlotDw < 32 && sa + h1 > 4u * kSlotDw) hsum = global_sum(fbs, sa, 0, (int)h1);
    const bool pad_in_slot = sa + len <= 4u * kSlotDw;
    int64_t pad = -1;
    if (__ballot(len >= 34u && end < len && pad_in_slot) != 0) {
        const uint32_t ps = slot_sum(lds, hw, grp, gl, sa, (int)min(end, len), (int)len, kSlotDw / 4, xo);
        if (pad_in_slot) pad = (int64_t)ps;
    }
    if (parser)
        park_parsed<kOps>(g_lds, pk, grp, parse_frame<kOps, kSlotDw>(lds, hw, grp, sa, len, mtu, hsum, pad, fbs, xo));
}

// Final L4 checksum + verdict (parser lane) once the streamed sum is known.
__device__ __forceinline__ uint32_t finish_l4(const uint32_t* fb, uint32_t sa, uint32_t len, const Parsed& P, uint64_t main_sum,
                              uint32_t& verdict) {
    // Every term is congruent (mod 65535) to its exact native contribution, and the true
    // total is > 0 (the pseudo-header protocol word is 6 or 17), so adding 65535 * 2^20
    // keeps t positive and the fold below lands on the same one's-complement value.
    int64_t t = (int64_t)main_sum + P.corr + 65535LL * (1LL << 20);
    if (len >= (1u << 19)) {
        // >= 512 KiB frame (only reachable with a huge Ethernet padding): a lane's streamed
        // 32-bit sum may have wrapped, so sum the L4 segment [off, end) exactly from memory.
        t = (int64_t)global_sum(fb, sa, (int)P.off, (int)P.end) + P.corr_fixed + 65535LL * (1LL << 20);
    }
    uint64_t x = (uint64_t)t;
    x = (x & 0xffffffffu) + (x >> 32);
    while (x >> 16) x = (x & 0xffffu) + (x >> 16);
    uint32_t l4 = (~(uint32_t)x) & 0xffffu;
    if (!P.parity) l4 = bswap16(l4);
    verdict = (l4 == P.stored) ? V_OK : V_CSUM;
    return l4;
}

// Z_k(v) for any k (one lane, a few uses per frame): Z768 and Z64 steps, then the sub-64
// tables (Z48/Z32/Z16, Z12/Z8/Z4, Z3/Z2/Z1). Z64 reads region A's copy 0 (entry e, table b:
// byte e*256 + 32*b).
__device__ __forceinline__ uint32_t zshift(const char* lds, uint32_t v, uint32_t k) {
    for (; k >= 768u; k -= 768u) v = zplain(lds, v, kLdsZ768);
    for (; k >= 64u; k -= 64u)
        v = lds32(lds, kLdsRegionA + ((v & 0xffu) << 8)) ^ lds32(lds, kLdsRegionA + (((v >> 8) & 0xffu) << 8) + 32u) ^
            lds32(lds, kLdsRegionA + (((v >> 16) & 0xffu) << 8) + 64u) ^ lds32(lds, kLdsRegionA + ((v >> 24) << 8) + 96u);
    if (k >= 48u) { v = zplain(lds, v, kLdsZ48); k -= 48u; }
    else if (k >= 32u) { v = zplain(lds, v, kLdsZ32); k -= 32u; }
    else if (k >= 16u) { v = zplain(lds, v, kLdsZ16); k -= 16u; }
    if (k >= 12u) { v = zplain(lds, v, kLdsZ12); k -= 12u; }
    else if (k >= 8u) { v = zplain(lds, v, kLdsZ8); k -= 8u; }
    else if (k >= 4u) { v = zplain(lds, v, kLdsZfin); k -= 4u; }
    if (k > 0u) v = zplain(lds, v, kLdsZfin + 4096u * (4u - k));  // zfin[t] = Z_(4-t)
    return v;
}

// A byte store into a frame (TX; hipcc merges neighbours into short/dword stores). Non-temporal
// stores measured no faster: the cost of these writes is the dirty lines' write-back.
__device__ __forceinline__ void st8(uint8_t* p, uint32_t v) { *p = (uint8_t)v; }

// The parser lane's finish of one frame: CRC-32 from the combined register Y, L4 checksum and
// verdict from the streamed sum `cs` and the parked parse, then the op's writes and stores.
// `len` is the frame length the rows streamed (kOpsFcs: without the FCS).
// The table layout the finish reads.
struct LayoutA {
    static constexpr uint32_t kZfin = kLdsZfin;
    __device__ static __forceinline__ uint32_t shift(const char* lds, uint32_t v, uint32_t k) { return zshift(lds, v, k); }
    // Z_(4-t)(v): the final step (t = bytes of dword rounding)
    __device__ static __forceinline__ uint32_t fin(const char* lds, uint32_t v, uint32_t t) {
        return zplain(lds, v, kZfin + 4096u * t);
    }
    // the standard CRC-32 byte table (Z_1's byte table 0)
    __device__ static __forceinline__ uint32_t byte1(const char* lds, uint32_t i) { return lds32(lds, kZfin + 3u * 4096u + (i << 2)); }
};

template <uint32_t kOps, class L = LayoutA>
__device__ __forceinline__ void finish_frame(const char* lds, const Parsed& P, uint64_t S, uint32_t len,
                                             uint32_t te, uint32_t Y, uint32_t cs, const uint8_t* frames,
                                             uint8_t* wframes, const uint32_t* lengths, uint32_t fi, uint2* out,
                                             uint8_t* status, uint32_t tx) {
    uint32_t fcs = 0u;
    if (kOps == kOpsFcs) {  // the FCS bytes [len, len+4): issued first, used last
        const uint8_t* fp = frames + S + len;
        fcs = (uint32_t)fp[0] | ((uint32_t)fp[1] << 8) | ((uint32_t)fp[2] << 16) | ((uint32_t)fp[3] << 24);
    }
    const uint32_t sa = (uint32_t)S & 3u;
    const uint32_t* fbs = reinterpret_cast<const uint32_t*>(frames + ((S >> 2) << 2));
    uint32_t crcv;
    if (len < 4u) {  // too short for the 4-byte init trick: bytewise CRC-32
        uint32_t c = 0xffffffffu;
        const uint8_t* fbytes = frames + S;
        for (uint32_t p = 0; p < len; ++p)
            c = L::byte1(lds, (c ^ fbytes[p]) & 0xffu) ^ (c >> 8);
        crcv = ~c;
    } else {
        const uint32_t tpad = (4u - te) & 3u;  // zero bytes appended by the dword rounding
        crcv = ~L::fin(lds, Y, tpad);
    }
    uint32_t verdict = P.verdict, l4 = 0u;
    if (P.compute) l4 = finish_l4(fbs, sa, len, P, cs, verdict);
    if constexpr (kOps == kOpsTx) {
        uint8_t* wf = wframes + S;
        if ((tx & kTxFill) && P.compute) {
            // write the IPv4 checksum at [24, 26) and the L4 checksum at its field, big-endian;
            // the CRC of the written frame differs from the streamed one by the CRC (zero init)
            // of the two 16-bit XOR deltas: Z_(len-p2)( Z_(p2-24)(d_ip) ^ d_l4 ), d as LE bytes
            const uint32_t ipc = P.ip_csum, old_ip = P.aux & 0xffffu, p2 = P.aux >> 16;
            {
                const uint32_t d = L::shift(lds, bswap16(old_ip ^ ipc), p2 - 24u) ^ bswap16(P.stored ^ l4);
                crcv ^= L::shift(lds, d, len - p2);
            }
            st8(wf + 24, ipc >> 8);
            st8(wf + 25, ipc);
            st8(wf + p2, l4 >> 8);
            st8(wf + p2 + 1, l4);
            verdict = V_OK;  // the written field now holds the computed checksum
        }
        if (tx & kTxAppend) {
            st8(wf + len, crcv);
            st8(wf + len + 1, crcv >> 8);
            st8(wf + len + 2, crcv >> 16);
            st8(wf + len + 3, crcv >> 24);
        }
    }
    if (kOps == kOpsFcs) {
        // len 0 covers wire frames of 0..4 bytes: only those of 4 carry an FCS
        const bool present = len > 0u || lengths[fi] >= 4u;
        if (!present || fcs != crcv) verdict = V_FCS;
    }
    out[fi] = make_uint2(crcv, P.ip_csum | (l4 << 16));
    if (status) status[fi] = (uint8_t)verdict;
}

// ---------------------------------------------------------------------------------------
// Tiles, pieces and passes.
//
// A tile's 16 frames run in PASSES of lockstep rows. MODE A (one pass): every group streams
// its whole frame, rows end-anchored at the pass end -- the lean choice when the frames have
// similar lengths. MODE B, for tiles whose lengths differ widely: a frame of nd stream dwords
// is cut into a HEAD piece of nd0 = nd - 192 (npc - 1) dwords (2 <= nd0 <= 193) and npc - 1
// FULL pieces of 192 dwords (12 rows, kPieceRows) that follow it; pass 0 streams every
// group's head piece exactly as mode A streams whole frames; passes 1.. stream the tile's F
// full pieces, 16 per pass (full piece q -> group q mod 16 of pass 1 + q / 16), all lean.
// Each pass ends with the 16-stream combine of every group's piece into one register value
// Y and a checksum partial, parked in a per-wave LDS slot; a frame's CRC register is then
// the Horner fold C = Z768(C) ^ Y over its pieces (a piece's value is its contribution as
// if the frame ended with it; Z768 shifts it past one full piece). Every pass runs the same
// row loop; the next pass's first rows are prefetched before the current pass's combine.

// The group's own frame (parse and finish). Every lane describes its GROUP's frame (the 4
// lanes of a group load the same descriptor; the group's lane 0 parses, finishes and stores).
struct Tile {
    uint64_t S;     // frame offset
    uint32_t len;   // frame length (0 for groups past the batch end)
    int npass;      // wave-uniform: 1 (mode A) or 1 + ceil(F / 16) (mode B)
    int F;          // wave-uniform: full pieces of the tile (mode B)
    __device__ __forceinline__ uint32_t sa() const { return (uint32_t)S & 3u; }
    __device__ __forceinline__ uint64_t sdw() const { return S >> 2; }
    // dwords the frame touches (incl. frames under 4 bytes)
    __device__ __forceinline__ int ndall() const { return (int)((sa() + len + 3u) >> 2); }
    // stream dwords (0: empty group -- past the batch end, or a frame under 4 bytes)
    __device__ __forceinline__ int nd() const { return len >= 4u ? ndall() : 0; }
    __device__ __forceinline__ uint32_t te() const {
        const uint32_t e = (sa() + len) & 3u;
        return e ? e : 4u;
    }
    __device__ __forceinline__ uint32_t tail_mask() const {
        const uint32_t t = te();
        return t == 4u ? 0xffffffffu : ((1u << (8u * t)) - 1u);
    }
};

__device__ __forceinline__ int pieces_of(int nd) { return nd <= 1 ? 1 : (nd - 1 + kPieceDwords - 1) / kPieceDwords; }

// The rows one pass streams.
struct Unit {
    const uint32_t* gfb;  // frame dword 0 of the lane's rows (a longest frame's for an empty group)
    int rel0;   // frame dword of this lane's chunk in row 0
    int lo;     // lowest frame dword a clamped row load may start at
    int P;      // wave-uniform: rows (a multiple of kPrefetch; 0 = no rows)
    int H;      // wave-uniform: leading rows that take the masked path
    // mode B: bit 31 valid piece, bit 30 the frame's last piece (its last dword carries the
    // dword-rounding junk), bits 28-29 the frame's end byte in its last dword, bits 0-15 slot
    uint32_t info;
};

__device__ __forceinline__ void tile_descriptors(uint32_t tile, uint32_t grp, uint32_t n,
                                                 const uint64_t* __restrict__ offsets,
                                                 const uint32_t* __restrict__ lengths, uint64_t& S, uint32_t& len,
                                                 uint32_t fpt = kFramesPerTile) {
    const uint32_t fi = tile * fpt + grp;
    // groups past the batch end (or past the tile's fpt frames) read the last frame's
    // descriptor (their length is zeroed)
    const uint32_t fl = (grp < fpt && fi < n) ? fi : n - 1u;
    // Inline asm: hipcc otherwise sinks the loads into their first use, serializing two HBM
    // round trips. The values are tied to an explicit wait (descriptors_ready) before use.
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(S) : "v"(offsets + fl));
    asm volatile("global_load_dword %0, %1, off" : "=v"(len) : "v"(lengths + fl));
}

// vmcnt(0) tied to the descriptor registers, so no use of them is scheduled above it.
// kOpsFcs: the rows stream the frame without its trailing FCS.
template <uint32_t kOps>
__device__ __forceinline__ void descriptors_ready(uint64_t& S, uint32_t& len) {
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(S), "+v"(len));
    if (kOps == kOpsFcs) len = len >= 4u ? len - 4u : 0u;
}

// Wave max (sum) of a value that is uniform within each 4-lane group: two DPP row mirrors
// combine the 4 groups of a 16-lane row, 4 readlanes the rows (no LDS permutes).
__device__ __forceinline__ int group_max(int x) {
    int y = __builtin_amdgcn_mov_dpp(x, 0x140, 0xf, 0xf, false);  // row_mirror
    x = max(x, y);
    y = __builtin_amdgcn_mov_dpp(x, 0x141, 0xf, 0xf, false);      // row_half_mirror
    x = max(x, y);
    const int a = __builtin_amdgcn_readlane(x, 0), b = __builtin_amdgcn_readlane(x, 16);
    const int c = __builtin_amdgcn_readlane(x, 32), d = __builtin_amdgcn_readlane(x, 48);
    return max(max(a, b), max(c, d));
}
__device__ __forceinline__ int group_sum(int x) {
    x += __builtin_amdgcn_mov_dpp(x, 0x140, 0xf, 0xf, false);  // lane i + lane 15-i: two groups
    x += __builtin_amdgcn_mov_dpp(x, 0x141, 0xf, 0xf, false);  // lanes 0-7: all four groups of the row
    return __builtin_amdgcn_readlane(x, 0) + __builtin_amdgcn_readlane(x, 16) + __builtin_amdgcn_readlane(x, 32) +
           __builtin_amdgcn_readlane(x, 48);
}

// Per-wave LDS scratch of mode B: the tile's frame table (offset, length) for the full-piece
// passes, the per-group full-piece counts, their inclusive prefix, and the piece slots.
struct WaveScratch {
    uint32_t ftab;   // [16] x {S_lo, S_hi, len, -}
    uint32_t dpc;    // [16] pieces - 1
    uint32_t epre;   // [16] inclusive prefix of dpc
    uint32_t slots;  // [16 + 16 * kMaxFullPasses] x {Y, csum}
};

// Pass-0 rows over `ndp` stream dwords per group (whole frames in mode A, head pieces in mode B).
__device__ __forceinline__ void pass0_unit(Unit& U, const Tile& T, int ndp, uint32_t gl,
                                           const uint8_t* __restrict__ frames) {
    const int rows0 = (ndp + kRowDwords - 1) / kRowDwords;
    const int R0 = group_max(rows0);
    U.P = (R0 + kPrefetch - 1) / kPrefetch * kPrefetch;
    uint64_t ld_sdw = T.sdw();
    int ld_nd = ndp;
    {
        const uint64_t ball = __ballot(rows0 == R0);  // never 0: some lane holds the maximum
        const int src = (int)__builtin_ctzll(ball);
        const uint32_t s_lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ld_sdw, src);
        const uint32_t s_hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(ld_sdw >> 32), src);
        const int s_nd = __builtin_amdgcn_readlane(ndp, src);
        if (ndp == 0) {
            ld_sdw = ((uint64_t)s_hi << 32) | s_lo;
            ld_nd = s_nd;
        }
    }
    U.gfb = reinterpret_cast<const uint32_t*>(frames + (ld_sdw << 2));
    U.rel0 = ld_nd - kRowDwords * U.P + 4 * (int)gl;
    // Loads of rows that start before the frame are clamped to the frame's first chunk (its last
    // chunk for frames under 4 dwords), so lanes idling through a tile's longest frame re-read
    // one cached line instead of fetching the bytes that precede their frame; a chunk that
    // straddles the frame start is loaded where it lies unless that is below frames[0].
    U.lo = max(ld_sdw > (1u << 24) ? -(1 << 24) : -(int)ld_sdw, min(0, ld_nd - 4));
    // Masked rows: those holding, for some lane, a frame dword < 2 (head bytes, CRC init) or a
    // dword before the frame. The group's lane 0 has the lowest rel: row r is lean for the
    // group once ndp - 16 P + 16 r >= 2.
    const int need = 2 - (ndp - kRowDwords * U.P);
    const int h = (ndp > 0 && need > 0) ? (need + kRowDwords - 1) / kRowDwords : 0;
    U.H = min(group_max(h), U.P);
    U.info = 0u;
}

__device__ __forceinline__ void tile_geometry(Tile& T, Unit& U, uint32_t tile, uint32_t grp, uint32_t gl, uint32_t n,
                                              uint64_t S, uint32_t len, const uint8_t* __restrict__ frames,
                                              char* lds, const WaveScratch& ws, uint32_t fpt) {
    T.len = (grp < fpt && tile * fpt + grp < n) ? len : 0u;
    T.S = S;
    const int nd = T.nd();
    const int rows = (nd + kRowDwords - 1) / kRowDwords;
    const int RA = (group_max(rows) + kPrefetch - 1) / kPrefetch * kPrefetch;
    // mode B: pass 0 over the head pieces, then ceil(F / 16) full-piece passes of 12 rows, each
    // about 2 rows' worth of combine; taken when that beats one pass over the longest frame
    const int npc = nd > 0 ? pieces_of(nd) : 1;
    const int nd0 = nd - kPieceDwords * (npc - 1);
    const int P0B = (group_max((nd0 + kRowDwords - 1) / kRowDwords) + kPrefetch - 1) / kPrefetch * kPrefetch;
    const int F = group_sum(npc - 1);
    const int fullp = (F + kFramesPerTile - 1) / kFramesPerTile;
    const bool modeB = F > 0 && fullp <= kMaxFullPasses && P0B + (kPieceRows + 2) * fullp < RA;
    T.F = modeB ? F : 0;
    T.npass = modeB ? 1 + fullp : 1;
    if (modeB) {
        // frame table, full-piece counts and their inclusive prefix (same wave: LDS in order)
        if (gl == 0u) {
            *reinterpret_cast<u32x4*>(lds + ws.ftab + 16u * grp) = u32x4{(uint32_t)S, (uint32_t)(S >> 32), T.len, 0u};
            *reinterpret_cast<uint32_t*>(lds + ws.dpc + 4u * grp) = (uint32_t)(npc - 1);
        }
        int e = 0;
#pragma unroll
        for (uint32_t j = 0; j < kFramesPerTile; j += 4) {
            const u32x4 d = *reinterpret_cast<const u32x4*>(lds + ws.dpc + 4u * j);
            e += (j + 0 <= grp ? (int)d.x : 0) + (j + 1 <= grp ? (int)d.y : 0) + (j + 2 <= grp ? (int)d.z : 0) +
                 (j + 3 <= grp ? (int)d.w : 0);
        }
        if (gl == 0u) *reinterpret_cast<uint32_t*>(lds + ws.epre + 4u * grp) = (uint32_t)e;
    }
    pass0_unit(U, T, modeB ? nd0 : nd, gl, frames);
}

// The full piece a group streams in pass p >= 1 (mode B): q = 16 (p - 1) + group; groups past
// the tile's F pieces re-stream piece F - 1 (valid addresses) and discard it.
__device__ __forceinline__ void full_piece_unit(Unit& U, const char* lds, const WaveScratch& ws,
                                                const uint8_t* __restrict__ frames, int F, int p, uint32_t grp,
                                                uint32_t gl) {
    const int q0 = kFramesPerTile * (p - 1) + (int)grp;
    const int q = min(q0, F - 1);
    // frame i = #{j : E_j <= q}; its first full piece is number E_(i-1) = max{E_j : E_j <= q}
    int i = 0, ebefore = 0;
#pragma unroll
    for (uint32_t j = 0; j < kFramesPerTile; j += 4) {
        const u32x4 e = *reinterpret_cast<const u32x4*>(lds + ws.epre + 4u * j);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int ej = (int)e[c];
            i += ej <= q ? 1 : 0;
            ebefore = ej <= q ? max(ebefore, ej) : ebefore;
        }
    }
    const u32x4 fr = *reinterpret_cast<const u32x4*>(lds + ws.ftab + 16u * (uint32_t)i);
    const uint64_t S = ((uint64_t)fr.y << 32) | fr.x;
    const uint32_t len = fr.z, sa = (uint32_t)S & 3u;
    const int nd = (int)((sa + len + 3u) >> 2);
    const int npc = pieces_of(nd);
    const int k = q - ebefore + 1;                 // 1 .. npc - 1
    U.gfb = reinterpret_cast<const uint32_t*>(frames + ((S >> 2) << 2));
    U.rel0 = nd - kPieceDwords * (npc - k) + 4 * (int)gl;  // the piece's first dword + the lane's chunk
    U.lo = 0;
    U.P = kPieceRows;
    U.H = 0;
    U.info = (q0 < F ? 0x80000000u : 0u) | (k == npc - 1 ? 0x40000000u : 0u) | (((sa + len) & 3u) << 28) |
             (uint32_t)(kFramesPerTile + q);
}

// How the tile's lengths mix (the report that steers the automatic choice): 0 similar lengths (the
// one-pass kernel), 1 mode B pays (the decision of tile_geometry: the mixed-length kernel), 2 a frame
// longer than mode B's passes cover beside frames at least 4 rows shorter (the segment kernel).
constexpr uint32_t kMixNone = 0u, kMixPieces = 1u, kMixGiant = 2u;
__device__ __forceinline__ uint32_t mixed_class(int nd) {
    const int rows = (nd + kRowDwords - 1) / kRowDwords;
    const int rmax = group_max(rows);
    // a tile whose frames differ by under 4 rows (256 B) has nothing for pieces to fill: the
    // common case of uniform batches skips the piece arithmetic (it only steers the choice)
    if (rmax + group_max(-rows) < 4) return kMixNone;
    const int RA = (rmax + kPrefetch - 1) / kPrefetch * kPrefetch;
    const int npc = nd > 0 ? pieces_of(nd) : 1;
    const int nd0 = nd - kPieceDwords * (npc - 1);
    const int P0B = (group_max((nd0 + kRowDwords - 1) / kRowDwords) + kPrefetch - 1) / kPrefetch * kPrefetch;
    const int F = group_sum(npc - 1);
    const int fullp = (F + kFramesPerTile - 1) / kFramesPerTile;
    if (F > 0 && fullp > kMaxFullPasses) return kMixGiant;
    return F > 0 && P0B + (kPieceRows + 2) * fullp < RA ? kMixPieces : kMixNone;
}

// ---- the mode-A-only kernel's tile state: the group's own frame and its single pass
struct TileA {
    uint64_t S;     // frame offset
    uint32_t len;   // frame length (0 for groups past the batch end)
    // row addressing: the group's own frame, or for an empty group a longest frame of the
    // tile, so that every row load -- including the unclamped lean refills -- stays inside a frame
    const uint32_t* gfb;
    int rel0;   // frame dword of this lane's chunk in row 0
    int lo;     // lowest frame dword a clamped row load may start at
    int P;      // wave-uniform: rows of the tile (a multiple of kPrefetch; 0 = no rows)
    int H;      // wave-uniform: leading rows that take the masked path
    uint32_t ph;  // block-aligned rows: absolute 64-B block phase (in dwords) of frame dword 0
    int r0f;      // block-aligned rows: the row of the frame's first block (large for an empty group)
    int cap;      // wave-uniform: every frame's first 3 blocks lie in the first block of rows (captured there)
    // derived per use (they would otherwise hold VGPRs across the row loop)
    __device__ __forceinline__ uint32_t sa() const { return (uint32_t)S & 3u; }
    // block-aligned rows: dwords past the frame end in its last row (the row ends on a 64-B block)
    __device__ __forceinline__ int ealign() const { return (16 - (int)((ph + (uint32_t)nd()) & 15u)) & 15; }
    __device__ __forceinline__ uint64_t sdw() const { return S >> 2; }
    // dwords the frame touches (incl. frames under 4 bytes)
    __device__ __forceinline__ int ndall() const { return (int)((sa() + len + 3u) >> 2); }
    // stream dwords (0: empty group -- past the batch end, or a frame under 4 bytes)
    __device__ __forceinline__ int nd() const { return len >= 4u ? ndall() : 0; }
    __device__ __forceinline__ uint32_t te() const {
        const uint32_t e = (sa() + len) & 3u;
        return e ? e : 4u;
    }
    __device__ __forceinline__ uint32_t tail_mask() const {
        const uint32_t t = te();
        return t == 4u ? 0xffffffffu : ((1u << (8u * t)) - 1u);
    }
};

// BLOCK-ALIGNED rows: each frame's rows are the 64-B blocks (half 128-B lines) that hold it, the
// last one ending on the block boundary after the frame end (nd + ealign() dwords from frame
// dword 0), so a row load never straddles a line.
// The tile's masked-row count H and its capture flag (the last part of tile_geometry_a; the first
// tile computes them after its first rows are issued, kDeferTail).
template <int kCapBlocks = 3>
__device__ __forceinline__ void tile_geometry_a_tail(TileA& T) {
    const int nd = T.nd();
    const int ndb = nd > 0 ? nd + T.ealign() : nd;
    T.cap = __ballot(nd > 0 && min(T.r0f + kCapBlocks, T.P) > kRingA) == 0;
    // Masked rows: those holding, for some lane, a frame dword < 2 (head bytes, CRC init) or a
    // dword before the frame. The group's lane 0 has the lowest rel: row r is lean for the
    // group once nd - 16 P + 16 r >= 2.
    const int need = 2 - (ndb - kRowDwords * T.P);
    const int h = (nd > 0 && need > 0) ? (need + kRowDwords - 1) / kRowDwords : 0;
    T.H = min(group_max(h), T.P);
}
template <int kCapBlocks = 3, bool kDeferTail = false>
__device__ __forceinline__ void tile_geometry_a(TileA& T, uint32_t tile, uint32_t grp, uint32_t gl, uint32_t n,
                                              uint64_t S, uint32_t len, const uint8_t* __restrict__ frames,
                                              uint32_t fpt) {
    T.len = (grp < fpt && tile * fpt + grp < n) ? len : 0u;
    T.S = S;
    T.ph = (uint32_t)((reinterpret_cast<uint64_t>(frames) >> 2) + T.sdw()) & 15u;
    const int nd = T.nd();
    const int ndb = nd > 0 ? nd + T.ealign() : nd;  // stream dwords up to the last row's end
    const int rows = (int)((T.ph + (uint32_t)ndb) >> 4) * (nd > 0);
    const int R = group_max(rows);
    T.P = (R + kRingA - 1) / kRingA * kRingA;
    T.r0f = nd > 0 ? T.P - rows : (1 << 20);
    uint64_t ld_sdw = T.sdw();
    int ld_nd = ndb;
    uint32_t ld_ph = T.ph;
    {
        const uint64_t ball = __ballot(rows == R);  // never 0: some lane holds the maximum
        const int src = (int)__builtin_ctzll(ball);
        const uint32_t s_lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ld_sdw, src);
        const uint32_t s_hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(ld_sdw >> 32), src);
        const int s_nd = __builtin_amdgcn_readlane(ndb, src);
        const uint32_t s_ph = (uint32_t)__builtin_amdgcn_readlane((int)ld_ph, src);
        if (nd == 0) {
            ld_sdw = ((uint64_t)s_hi << 32) | s_lo;
            ld_nd = s_nd;
            ld_ph = s_ph;
        }
    }
    T.gfb = reinterpret_cast<const uint32_t*>(frames + (ld_sdw << 2));
    T.rel0 = ld_nd - kRowDwords * T.P + 4 * (int)gl;
    // Loads of rows that start before the frame's first block (lo = the frame dword where that
    // block starts) reload the lane's chunk of that block, so lanes idling through a tile's longest
    // frame re-read one cached line instead of fetching the bytes that precede their frame (a row
    // inside a block that holds a frame byte never leaves that byte's page: no other clamp).
    T.lo = -(int)ld_ph;
    if (!kDeferTail) tile_geometry_a_tail<kCapBlocks>(T);
}

// Frame dword at which a masked row's chunk is loaded: where it lies, unless it starts
// before the frame's first chunk (then the frame's first chunk: its dwords are all masked
// or realigned) or below frames[0].
__device__ __forceinline__ int load_pos(int rel, int lo) { return rel <= -4 ? lo : max(rel, lo); }

__device__ __forceinline__ u32x4 load_row(const uint32_t* fb, int pos) {
    return *reinterpret_cast<const u32x4_a4*>(fb + pos);
}

__device__ __forceinline__ void prefetch_unit(const Unit& U, u32x4 (&pf)[kPrefetch]) {
    if (U.P > 0) {  // a tile of frames all under 4 bytes loads no rows (they could lie past the buffer)
#pragma unroll
        for (int i = 0; i < kPrefetch; ++i) {
            const int rel = U.rel0 + kRowDwords * i;
            pf[i] = load_row(U.gfb, i < U.H ? load_pos(rel, U.lo) : rel);
        }
    }
}

// The tables in place. Region A: thread t builds the 16-B chunk k = t & 7 of entry rows
// e = t >> 3 and e + 128 (the chunk holds 4 of table b = k >> 1's 8 copies of Z64[b][e], the XOR
// of the basis columns of e's set bits; the two entries differ in bit 7 only). An 8-lane
// ds_write_b128 group so writes one entry's 128 contiguous bytes: 8 distinct bank quads (one
// thread per (b, e) writing its 32 B put every lane of a group on the same 4 banks: 8-way).
// The plain tables: wave w builds the 1-KB pieces p = w, w + 16, w + 32 (< 40) of the
// 40 [4][256] tables the same way, lane l the entries 4l .. 4l + 3 (one ds_write_b128): no
// LDS-DMA in the preamble's vector-memory burst, no wait for table pieces at the barrier.
// The bases come in by scalar loads (lgkmcnt), all issued before one wait, so waiting for them
// never waits for the descriptors' vector loads issued before them.
__device__ __forceinline__ uint64_t sgpr_addr(const void* p) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a);
}
__device__ __forceinline__ void build_region_a(const FsTables* __restrict__ tabs, char* lds) {
    typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
    const uint32_t t = threadIdx.x;
    const uint32_t w = __builtin_amdgcn_readfirstlane(t >> 6);
    const uint32_t lane = t & 63u;
    const uint64_t sz = sgpr_addr(&tabs->z64_basis[0][0]);
    const uint64_t s0 = sgpr_addr(&tabs->plain_basis[w][0]);
    const uint64_t s1 = sgpr_addr(&tabs->plain_basis[w + 16u][0]);
    const uint64_t s2 = sgpr_addr(&tabs->plain_basis[min(w + 32u, 39u)][0]);
    u32x8 z0, z1, z2, z3, pb0, pb1, pb2;
    asm volatile(
        "s_load_dwordx8 %0, %7, 0x0\n\ts_load_dwordx8 %1, %7, 0x20\n\ts_load_dwordx8 %2, %7, 0x40\n\t"
        "s_load_dwordx8 %3, %7, 0x60\n\ts_load_dwordx8 %4, %8, 0x0\n\ts_load_dwordx8 %5, %9, 0x0\n\t"
        "s_load_dwordx8 %6, %10, 0x0\n\ts_waitcnt lgkmcnt(0)"
        : "=&s"(z0), "=&s"(z1), "=&s"(z2), "=&s"(z3), "=&s"(pb0), "=&s"(pb1), "=&s"(pb2)
        : "s"(sz), "s"(s0), "s"(s1), "s"(s2));
    const uint32_t k = t & 7u, b = k >> 1, e = t >> 3;  // e < 128
    uint32_t v = 0, top = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        const uint32_t lo = (b & 1u) ? z1[j] : z0[j];
        const uint32_t hi = (b & 1u) ? z3[j] : z2[j];
        const uint32_t bj = (b & 2u) ? hi : lo;
        if (j < 7) v ^= bj & (0u - ((e >> j) & 1u));
        else top = bj;
    }
    *reinterpret_cast<u32x4*>(lds + kLdsRegionA + e * 256u + 16u * k) = u32x4{v, v, v, v};
    v ^= top;
    *reinterpret_cast<u32x4*>(lds + kLdsRegionA + (e + 128u) * 256u + 16u * k) = u32x4{v, v, v, v};
    auto piece = [&](const u32x8& pb, uint32_t p) {
        uint32_t x = 0;
#pragma unroll
        for (uint32_t j = 2; j < 8; ++j) x ^= pb[j] & (0u - ((lane >> (j - 2u)) & 1u));
        const uint32_t x1 = x ^ pb[0];
        *reinterpret_cast<u32x4*>(lds + 1024u * p + 16u * lane) = u32x4{x, x1, x ^ pb[1], x1 ^ pb[1]};
    };
    piece(pb0, w);
    piece(pb1, w + 16u);
    if (w + 32u < 40u) piece(pb2, w + 32u);
}
// LDS-DMA by inline asm: invisible to hipcc's vmcnt model (the builtin makes it drain later
// LDS reads with vmcnt(0)); unknown VMEM ops only make the compiler's own counted waits
// stricter (loads retire in order). Every use is covered by an explicit counted wait.
// (m0 is reserved to the compiler: it is written in the same statement that uses it)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma_x4(const void* src, uint32_t lds_dst) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 :
                 : "v"(src), "s"(lds_dst)
                 : "memory", "m0");
}
__device__ __forceinline__ void dma_x1(const void* src, uint32_t lds_dst) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off"
                 :
                 : "v"(src), "s"(lds_dst)
                 : "memory", "m0");
}
#pragma clang diagnostic pop

__device__ __forceinline__ uint32_t lds_base(const char* lds) {
    typedef __attribute__((address_space(3))) const char lds_char;
    return (uint32_t)(uintptr_t)(lds_char*)lds;
}

// The tile's header slots: 8 dword DMAs; instruction i writes frame dword x = 4i + gl of
// every group (lane-linear: LDS byte hw + 256 i + 4 lane). Sources are clamped to the
// frame's last dword (never past it).
// When every frame of the tile spans the whole slot (>= 32 dwords), 2 dwordx4 DMAs do it
// instead: lane L = g + 16 q loads frame dwords [4c, 4c + 4), c = q + 4 k, of group g's frame
// (instruction k; lane-linear 16 B per lane: the same [x >> 2][group][x & 3] layout). The
// tile start is VMEM-issue-bound (16 waves' descriptor, header, table and row loads through
// one CU), so 6 fewer instructions per wave start the row loops earlier.
// Returns whether the dwordx4 form was used (wave-uniform: 2 instructions, else 8). kX4 = false
// (the mixed-length kernel: its tiles hold short frames, and the permutes cost it registers)
// always takes the dword form.
template <bool kX4, int kSlot = kHdrDwords, class TileT>
__device__ __forceinline__ bool header_dma(const TileT& T, const uint8_t* __restrict__ frames, const char* lds,
                                           uint32_t hw, uint32_t gl, uint32_t lane) {
    static_assert(kSlot == 16 || kSlot == 32, "header slot: 16 or 32 dwords");
    const uint32_t hdr0 = __builtin_amdgcn_readfirstlane(lds_base(lds) + hw);
    const int last = T.ndall() - 1;
    const bool own = T.len > 0u;
    const uint64_t fa = reinterpret_cast<uint64_t>(frames + (T.sdw() << 2));
    if (kX4 && __ballot(own && last < kSlot - 1) == 0) {
        const int src = (int)((lane & 15u) << 4);  // group (lane & 15)'s lane 0
        const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)fa);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(fa >> 32));
        const uint32_t lg = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)T.len);
        const uint32_t* fb = reinterpret_cast<const uint32_t*>(((uint64_t)hi << 32) | lo);
        const uint32_t q = lane >> 4;
        if (lg > 0u) {
            dma_x4(fb + 4u * q, hdr0);
            if (kSlot > 16) dma_x4(fb + 4u * (q + 4u), hdr0 + 1024u);
        }
        return true;
    }
    if (own) {  // exec-masked: a group with no frame bytes writes nothing (its slot is never used)
        const uint32_t* fbs = reinterpret_cast<const uint32_t*>(fa);
#pragma unroll
        for (int i = 0; i < kSlot / 4; ++i) dma_x1(fbs + min(4 * i + (int)gl, last), hdr0 + 256u * i);
    }
    return false;
}

// The preamble's wait: the table pieces (issued before the header DMA and the rows) have
// landed -- vmcnt(rows + header DMAs) -- and lgkmcnt(0): this wave's region-A stores.
// s_waitcnt field layout (gfx9): vmcnt[3:0] + vmcnt_hi[15:14], expcnt[6:4], lgkmcnt[11:8]
template <int kPf, int kSlot = kHdrDwords>
__device__ __forceinline__ void tables_landed(bool first, bool rows, bool x4) {
    constexpr int kX4n = kSlot / 16, kX1n = kSlot / 4;  // header DMA instructions of either form
    if (first && rows && x4) __builtin_amdgcn_s_waitcnt(0x0070 | (kPf + kX4n));
    else if (first && rows) __builtin_amdgcn_s_waitcnt(0x0070 | (kPf + kX1n));
    else if (first && x4) __builtin_amdgcn_s_waitcnt(0x0070 | kX4n);
    else if (first) __builtin_amdgcn_s_waitcnt(0x0070 | kX1n);
    else __builtin_amdgcn_s_waitcnt(0x0070);
}

// 16-stream combine of a group's piece: U_l = Z12(A0) ^ Z8(A1) ^ Z4(A2) ^ A3 per lane (minus the
// junk the piece's last dword may carry, lane 3), Y = xor_l Z_16(3-l)(U_l) over the group by
// DPP; the checksum partial folded mod 65535 (every partial < 2^18) and summed over the group.
__device__ __forceinline__ void combine_piece(const char* lds, uint32_t gl, const uint32_t (&A)[4], uint32_t cs,
                                              uint32_t junk, uint32_t& Y, uint32_t& csum) {
    const uint32_t U =
        zplain(lds, A[0], kLdsZ12) ^ zplain(lds, A[1], kLdsZ8) ^ zplain(lds, A[2], kLdsZfin) ^ A[3] ^ junk;
    cs -= sad16(junk, 0u);
    const uint32_t ybase = (gl == 0u) ? kLdsZ48 : (gl == 1u) ? kLdsZ32 : kLdsZ16;
    uint32_t y = zplain(lds, U, ybase);
    if (gl == 3u) y = U;
    y ^= dpp_quad<kQuadXor1>(y);
    y ^= dpp_quad<kQuadXor2>(y);
    cs = (cs & 0xffffu) + (cs >> 16);
    cs += dpp_quad<kQuadXor1>(cs);
    cs += dpp_quad<kQuadXor2>(cs);
    Y = y;
    csum = cs;
}

// The one-pass kernel's LDS layout: one 16-wave workgroup per CU (region A and the plain tables
// built in place), 3-block captured header slots per wave.
struct LayA1 : LayoutA {
    static constexpr uint32_t kRegion = kLdsRegionA;
    static constexpr uint32_t kHdr = kLdsHdr;
    static constexpr uint32_t kCapStride = 3072;
    static constexpr int kCapBlocks = 3;
    // Z_(16a)(v), a = 0..3 (the lookups run for a = 0 too; the select drops them)
    __device__ static __forceinline__ uint32_t z16a(const char* lds, uint32_t v, uint32_t a) {
        const uint32_t y = zplain(lds, v, a == 1u ? kLdsZ16 : a == 2u ? kLdsZ32 : kLdsZ48);
        return a ? y : v;
    }
};

// The 16 streams of a group combined to the frame's last dword, at block position q = 15 - ealign
// of the last row (the block-aligned combine). Stream j of lane gl (row position
// 4 gl + j) is shifted by its distance in dwords to q: s = (K - j) mod 16 with K = (q - 4 gl) mod 16
// = 4 a + C (the streams past q skipped the last row). Streams j <= C need Z_(16 a) Z_(4 (C - j)),
// the others Z_(16 ((a - 1) & 3)) Z_(4 (4 + C - j)). Sorted by their Z4 class c (B_c = A_((C - c) & 3):
// the registers reversed, then rotated by C), that is one round of Z4 / Z8 / Z12 with a fixed table
// per register and one round of Z_(16 a) per class: 5 lookups in 2 dependent rounds, then the XOR
// over the group's 4 lanes by DPP (tests/kernel_model.py).
template <class Lay>
__device__ __forceinline__ uint32_t combine_to_end(const char* lds, const uint32_t (&A)[4], int ealign, uint32_t gl) {
    const uint32_t K = (uint32_t)(15 - ealign - 4 * (int)gl) & 15u;
    const uint32_t a = K >> 2, C = K & 3u;
    uint32_t Y;
    {
        const bool r1 = (C & 1u) != 0u, r2 = (C & 2u) != 0u;
        // reversed: (A0, A3, A2, A1); rotated by 1 then by 2 where C has those bits
        const uint32_t x0 = r1 ? A[1] : A[0], x1 = r1 ? A[0] : A[3], x2 = r1 ? A[3] : A[2], x3 = r1 ? A[2] : A[1];
        const uint32_t b0 = r2 ? x2 : x0, b1 = r2 ? x3 : x1, b2 = r2 ? x0 : x2, b3 = r2 ? x1 : x3;
        const uint32_t t1 = zplain(lds, b1, kLdsZfin);  // Z4
        const uint32_t t2 = zplain(lds, b2, kLdsZ8);
        const uint32_t t3 = zplain(lds, b3, kLdsZ12);
        const uint32_t v1 = b0 ^ (C >= 1u ? t1 : 0u) ^ (C >= 2u ? t2 : 0u) ^ (C == 3u ? t3 : 0u);
        const uint32_t v2 = xor3(b0 ^ t1, t2, t3) ^ v1;
        Y = Lay::z16a(lds, v1, a) ^ Lay::z16a(lds, v2, (a - 1u) & 3u);
    }
    Y ^= dpp_quad<kQuadXor1>(Y);
    Y ^= dpp_quad<kQuadXor2>(Y);
    return Y;
}

// `report` = the host-mapped report block's address in bits 0..46, the watch flag in bit 47, the launch
// id in bits 48..63
// (one kernel argument, loaded where it is used: nothing of it stays live through the tile loop).
template <int kWord = kReportLatest>
__device__ __forceinline__ void post_report(uint64_t report, uint32_t bits = 0u) {
    asm volatile("" : "+s"(report));  // split here, not hoisted into a register held by the whole kernel
    // a GLOBAL store (address space 1), not a flat one: hipcc's wait counting treats any pending
    // flat op as able to complete out of order with the vector memory operations, so every vmcnt
    // wait after it became vmcnt(0) -- the first block of rows waited for the whole ring
    typedef __attribute__((address_space(1))) uint32_t gu32;
    *reinterpret_cast<gu32*>((report & kReportAddrMask) + 4u * kWord) = (uint32_t)(report >> 48) | bits;
}
// Bit 47 of `report`: the host is counting short launches (or a long report is news to it), so every
// wave reports its long tiles; otherwise only the grid's first wave does, in its "ran" post (uniform
// long traffic then costs one post per launch, not one per tile).
__device__ __forceinline__ bool report_watch(uint64_t report) { return ((report >> 47) & 1u) != 0u; }

// A wave's posts for a tile of frames of `len` (group-uniform; 0 for an empty group), issued at the
// tile's start, after its row prefetch. A store to host memory counts in vmcnt until it lands (~PCIe
// latency): a wait for any load issued after it waits for the store too. Each post costs its launch
// about 0.25 us (C2: one store from the grid's first wave; placements tried, same box: at the first
// tile's start +0.25 us, just before the tile's last block about the same but +18 VGPRs in the
// one-pass kernel, after the wave's own work +0.27 us on C2 and +1.1 us on C3), hence the sampled
// asks (kAskRan, kAskMixed). The grid's first tile posts "ran" with its own long flag in the same
// word (kReportRanLong), so a launch it saw long never reads as short, whatever order posts land in.
// What a tile posts (wave-uniform bits), computed apart from the stores so that a wave's first tile
// computes them while its rows load and stores them after its counted wait (computing them after the
// wait put the wave's barrier arrival ~0.1 us later on C2). kMixedOnAsk: mixed tiles are posted only
// when the launch asks (kAskMixed; the mixed-length kernel).
constexpr uint32_t kPostMixed = 1u, kPostRan = 2u, kPostRanLong = 4u, kPostLong = 8u, kPostGiant = 16u;
template <bool kMixedOnAsk>
__device__ __forceinline__ uint32_t tile_posts(uint64_t report, uint32_t len, uint32_t mix, bool first_tile_of_grid) {
    // the bit tests here, per tile: hoisted out of the tile loop, hipcc kept each flag as a live
    // 64-bit mask and spilled SGPRs (the mixed-length kernel 24 against 14, C3 +1.1 us per launch)
    asm volatile("" : "+s"(report));
    const bool mixed = mix != kMixNone && (!kMixedOnAsk || (report & kAskMixed) != 0u);
    const bool ran = first_tile_of_grid && (report & kAskRan) != 0u;
    const bool lng = (ran || report_watch(report)) && __ballot(len > kSmallMaxLen) != 0u;
    return (mixed ? (mix == kMixGiant ? kPostMixed | kPostGiant : kPostMixed) : 0u) |
           (ran ? (lng ? kPostRan | kPostRanLong : kPostRan) : (lng ? kPostLong : 0u));
}
__device__ __forceinline__ void post_tile(uint64_t report, uint32_t posts, uint32_t lane) {
    if (posts == 0u || lane != 0u) return;
    if (posts & kPostMixed) post_report<kReportLatest>(report, (posts & kPostGiant) ? kReportMixedGiant : 0u);
    if (posts & kPostRan) post_report<kReportRan>(report, (posts & kPostRanLong) ? kReportRanLong : 0u);
    if (posts & kPostLong) post_report<kReportLong>(report);
}
// The wave's first tile (later tiles: + all waves): wave-major, so a workgroup's waves read tiles
// spread over the batch and neighbouring workgroups (on different XCDs) neighbouring tiles.
__device__ __forceinline__ uint32_t first_tile(uint32_t wave) { return wave * gridDim.x + blockIdx.x; }

// The kernel for batches of similar lengths: every tile in one pass over block-aligned rows. It
// reports in `report` whether any tile would have run better in mode B, so that the host launches
// digest_kernel_ab next time (launch_digest).
template <uint32_t kOps>
__global__ void __launch_bounds__(kThreads, 1)
digest_kernel_a(const uint8_t* __restrict__ frames, const uint64_t* __restrict__ offsets,
                const uint32_t* __restrict__ lengths, uint32_t n, uint32_t mtu, const FsTables* __restrict__ tabs,
                uint2* __restrict__ out, uint8_t* __restrict__ status, uint64_t report, uint8_t* wframes, uint32_t tx, uint32_t fpt) {
    using Lay = LayA1;
    char* lds = g_lds;
    constexpr int kPfA = kRingA;

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t grp = lane >> 2;   // frame slot of this lane's group
    const uint32_t gl = lane & 3u;    // lane within the group
    const uint32_t gwave = first_tile(wave);
    const uint32_t nwaves = gridDim.x * kWavesPerBlock;
    // fpt: frames per tile (16, or 8 / 4 for batches too small to give every wave a tile;
    // the other groups stay empty)
    fpt = __builtin_amdgcn_readfirstlane(fpt);
    const uint32_t ntiles = (n + fpt - 1) / fpt;
    // Header slots captured from the rows: the first block of rows holds every frame's first 3
    // blocks (checked per tile: T.cap), and each of those rows is written to the slot as it is
    // consumed -- cell 4k + gl of the slot holds the lane's 16 B of the frame's block k, so slot
    // dword s is frame dword s - ph (the parse's `xo`). 3 KB per wave (12 cells), overlapping the
    // wave scratch this kernel leaves unused.
    static_assert(Lay::kHdr + kWavesPerBlock * Lay::kCapStride <= kLdsBytes, "captured header slots fit");
    static_assert(4u * Lay::kCapBlocks * 256u <= Lay::kCapStride, "a wave's captured cells fit its stride");
    const uint32_t hw = Lay::kHdr + wave * Lay::kCapStride;  // this wave's header slots (and parked parse)
    // where a masked row's chunk is loaded: where it lies, or wholly before the frame's first
    // block, the lane's chunk of that block
    auto lpos = [&](int rel, int lo) -> int { return rel >= lo ? rel : lo + 4 * (int)gl; };
    // the slots of a tile whose frames start too late for the capture: plain loads (rare: mixed lengths)
    auto tile_header = [&](const TileA& Tt) {
        if (!Tt.cap) {
            const int rows = Tt.P - Tt.r0f;
            const uint32_t* fb = reinterpret_cast<const uint32_t*>(frames + (Tt.sdw() << 2));
#pragma unroll
            for (int k = 0; k < Lay::kCapBlocks; ++k) {
                if (Tt.len >= 4u && k < rows) {
                    const u32x4 v = load_row(fb, -(int)Tt.ph + 16 * k + 4 * (int)gl);
                    *reinterpret_cast<u32x4*>(lds + hw + (uint32_t)(4 * k + (int)gl) * 256u + grp * 16u) = v;
                }
            }
        }
    };

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

    // Preamble: the first tile's descriptors (the first memory ops, one round trip) while the
    // tables are built in place by VALU; geometry; the first rows; the masked-row count and the
    // capture flag; one barrier once this wave's table stores are done.
    // (round 4 built a pipelined tile transition -- the next tile's descriptors during the rows, its
    // first rows in the last block -- and measured it 3-5% slower on two-tile batches and 1-2% on C4,
    // equal on C2: DESIGN.md §3.11; this loop stays)
    uint32_t tile = gwave;
    FS_RTSTAMP(5);
    FS_STAMP(0);
    TileA T;
    u32x4 pf[kPfA];
    const bool first = __builtin_amdgcn_readfirstlane(tile) < ntiles;
    {
        uint64_t S;
        uint32_t len;
        tile_descriptors(tile, grp, n, offsets, lengths, S, len, fpt);
        build_region_a(tabs, lds);
        FS_STAMP(7);
        descriptors_ready<kOps>(S, len);
        FS_STAMP(8);
        T.P = 0;
        if (first) tile_geometry_a<Lay::kCapBlocks, true>(T, tile, grp, gl, n, S, len, frames, fpt);
        FS_STAMP(11);
        FS_STAMP(12);
    }
    if (first && T.P > 0) {  // a tile of frames all under 4 bytes loads no rows (they could lie past the buffer)
#pragma unroll
        for (int i = 0; i < kPfA; ++i) pf[i] = load_row(T.gfb, lpos(T.rel0 + kRowDwords * i, T.lo));
    }
    if (first) tile_geometry_a_tail<Lay::kCapBlocks>(T);
    const uint32_t posts0 = first && report ? tile_posts<false>(report, T.len, mixed_class(T.nd()), gwave == 0u) : 0u;
    if (first) tile_header(T);
    FS_STAMP(13);
    FS_STAMP(9);
    // the tables are this wave's own LDS stores: only the rows stay in flight
    if (first && T.P > 0) __builtin_amdgcn_s_waitcnt(0x0070 | kPfA);
    else __builtin_amdgcn_s_waitcnt(0x0070);
    // (after the counted wait above, younger than the rows)
    post_tile(report, posts0, lane);
    FS_STAMP(10);
    __builtin_amdgcn_s_barrier();  // tables ready (raw barrier: no release fence, no vmcnt(0) drain)
    // two-level age priority: the SIMD's younger half (waves 8..15) outranks the older (round 2:
    // -0.35..-0.55 us per launch)
    if ((__builtin_amdgcn_readfirstlane(wave) >> 3) != 0u) __builtin_amdgcn_s_setprio(1);
    FS_STAMP(1);

    while (tile < ntiles) {

        uint32_t A[4] = {0u, 0u, 0u, 0u};
        uint32_t cs = 0u;
        const bool fvalid = grp < fpt && tile * fpt + grp < n;
        const bool parser = fvalid && gl == 0u;  // the group's lane 0 parses, finishes and stores
        const int Rc = T.P - kPfA;  // first row of the last block

        // ---- header parse: after the first block of rows (the captured slot is this wave's own
        // LDS writes), while the ring's loads are in flight
        auto parse = [&]() {
            parse_tile<kOps, kHdrDwords>(hw, grp, gl, T.sa(), T.len, mtu,
                                         reinterpret_cast<const uint32_t*>(frames + (T.sdw() << 2)), parser, hw, T.ph);
        };
        auto prio = [&](int r0) {
            // Self-balancing issue priority for long tiles (C2-size tiles run faster without): the
            // SIMD arbiter favours the oldest wave, a wave with more rows left gets a higher priority.
            if (T.P > kPrioMinRows) {
                const int left4 = (4 * (T.P - r0)) / max(T.P, 1);  // 4 .. 1
                if (left4 >= 4) __builtin_amdgcn_s_setprio(3);
                else if (left4 == 3) __builtin_amdgcn_s_setprio(2);
                else if (left4 == 2) __builtin_amdgcn_s_setprio(1);
                else __builtin_amdgcn_s_setprio(0);
            }
        };
        // general block: rows below H take the masked path (scalar branch per row); refills of
        // rows below H are clamped. kRefill: this tile's rows kPfA ahead (false: the last block).
        auto block = [&](int r0, auto refill_tag) {
            constexpr bool kRefill = decltype(refill_tag)::value;
            prio(r0);
#pragma unroll
            for (int i = 0; i < kPfA; ++i) {
                const int r = r0 + i;
                const int rel = T.rel0 + kRowDwords * r;
                // consume the ring slot, then refill the SAME registers: no copy of an
                // in-flight load, so the compiler keeps kPfA-1 loads outstanding
                if (r < T.H) masked_row_al<Lay::kRegion>(lds, keys, pf[i], rel, T.nd(), T.sa(), T.tail_mask(), A, cs);
                else if (!kRefill && i == kPfA - 1) tail_row_al<Lay::kRegion>(lds, keys, pf[i], rel, T.nd(), T.tail_mask(), A, cs);
                else lean_row<Lay::kRegion>(lds, keys, pf[i], A, cs);
                if (r0 == 0 && T.cap) {  // the frame's first blocks into the header slot
                    const uint32_t k = (uint32_t)(i - T.r0f);
                    if (k < (uint32_t)Lay::kCapBlocks) {
                        // two 8-B stores, the odd group lanes writing their upper half first: a
                        // group's 4 lanes write the same 16-B column of 4 cells 256 B apart, so one
                        // 16-B store each hits one bank quad 4 times; this way 2 lanes share banks
                        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
                        const u32x4 v = pf[i];
                        const bool s1 = (gl & 1u) != 0u;
                        const u32x2 h0 = s1 ? u32x2{v.z, v.w} : u32x2{v.x, v.y};
                        const u32x2 h1 = s1 ? u32x2{v.x, v.y} : u32x2{v.z, v.w};
                        const uint32_t cb = hw + (4u * k + gl) * 256u + grp * 16u + ((gl & 1u) << 3);
                        *reinterpret_cast<u32x2*>(lds + cb) = h0;
                        *reinterpret_cast<u32x2*>(lds + (cb ^ 8u)) = h1;
                    }
                }
                if (kRefill) {
                    const int rn = rel + kRowDwords * kPfA;
                    pf[i] = load_row(T.gfb, r + kPfA < T.H ? lpos(rn, T.lo) : rn);
                }
            }
        };
        // lean block: every row lean for every lane; the refills lie inside the frame, so they
        // need no clamp: one pointer per block, immediate row offsets
        auto lean_block = [&](int r0, auto refill_tag) {
            constexpr bool kRefill = decltype(refill_tag)::value;
            prio(r0);
            const uint32_t* pb = T.gfb + (T.rel0 + kRowDwords * (r0 + kPfA));
#pragma unroll
            for (int i = 0; i < kPfA; ++i) {
                if (!kRefill && i == kPfA - 1)
                    tail_row_al<Lay::kRegion>(lds, keys, pf[i], T.rel0 + kRowDwords * (r0 + i), T.nd(), T.tail_mask(), A, cs);
                else lean_row<Lay::kRegion>(lds, keys, pf[i], A, cs);
                if (kRefill) pf[i] = *reinterpret_cast<const u32x4_a4*>(pb + kRowDwords * i);
                // keep consume/refill interleaved per row: unfenced, the scheduler sinks all
                // refills to the block end behind a vmcnt(0), draining the ring every block
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        using Yes = std::true_type;
        using No = std::false_type;
        if (T.P > 0) {
            // [first block] parse [head blocks: general] [body: lean] [last block: no refill]
            if (Rc > 0) {
                if (T.H > 0) block(0, Yes());
                else lean_block(0, Yes());
                parse();
                int r0 = kPfA;
                for (; r0 < Rc && r0 < T.H; r0 += kPfA) block(r0, Yes());
                for (; r0 < Rc; r0 += kPfA) lean_block(r0, Yes());
                if (Rc < T.H) block(Rc, No());
                else lean_block(Rc, No());
            } else {
                if (T.H > 0) block(0, No());
                else lean_block(0, No());
                parse();
            }
        } else {
            parse();  // no rows (every frame of the tile under 4 bytes): rejected by length
        }
        FS_STAMP(2);

        // ---- combine the 16 streams of each frame to its last dword (combine_to_end).
        // The parked parse, read by every lane now: its LDS round trip overlaps the combine's.
        const Parsed P = unpark_parsed<kOps>(lds, hw, grp);
        const uint32_t Y = combine_to_end<Lay>(lds, A, T.ealign(), gl);
        // checksum over the 4 lanes of the group, each lane first folded mod 65535 (the finish
        // only needs the total mod 65535; the fold keeps every partial < 2^18)
        cs = (cs & 0xffffu) + (cs >> 16);
        cs += dpp_quad<kQuadXor1>(cs);
        cs += dpp_quad<kQuadXor2>(cs);
        FS_STAMP(3);
        // ---- the group's lane 0: finish and store (its frame's parse comes back from LDS).
        if (parser)
            finish_frame<kOps, Lay>(lds, P, T.S, T.len, T.te(), Y, cs, frames, wframes, lengths, tile * fpt + grp, out,
                                    status, tx);
        FS_STAMP(4);
        FS_RTSTAMP(6);
        tile += nwaves;
        if (tile < ntiles) {  // next tile: descriptors, geometry, row prefetch, header slots
            uint64_t S;
            uint32_t len;
            tile_descriptors(tile, grp, n, offsets, lengths, S, len, fpt);
            descriptors_ready<kOps>(S, len);
            tile_geometry_a<Lay::kCapBlocks>(T, tile, grp, gl, n, S, len, frames, fpt);
            if (T.P > 0) {
#pragma unroll
                for (int i = 0; i < kPfA; ++i) {
                    const int rel = T.rel0 + kRowDwords * i;
                    pf[i] = load_row(T.gfb, i < T.H ? lpos(rel, T.lo) : rel);
                }
            }
            if (report) post_tile(report, tile_posts<false>(report, T.len, mixed_class(T.nd()), false), lane);
            tile_header(T);
        }
    }
}

// The kernel for batches with mixed lengths: tiles in mode A or mode B, per tile.
template <uint32_t kOps>
__global__ void __launch_bounds__(kThreads, 1)
digest_kernel_ab(const uint8_t* __restrict__ frames, const uint64_t* __restrict__ offsets,
                 const uint32_t* __restrict__ lengths, uint32_t n, uint32_t mtu, const FsTables* __restrict__ tabs,
                 uint2* __restrict__ out, uint8_t* __restrict__ status, uint64_t report, uint8_t* wframes, uint32_t tx,
                 uint32_t fpt) {
    char* lds = g_lds;

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: SGPR addresses
    const uint32_t grp0 = lane >> 2;   // frame slot of this lane's group
    const uint32_t gl0 = lane & 3u;    // lane within the group
    const uint32_t gwave = first_tile(wave);
    const uint32_t nwaves = gridDim.x * kWavesPerBlock;
    fpt = __builtin_amdgcn_readfirstlane(fpt);  // frames per tile (16, 8 or 4; see launch_digest)
    const uint32_t ntiles = (n + fpt - 1) / fpt;
    const uint32_t hw = kLdsHdr + wave * kHdrWaveBytes;  // this wave's header slots
    WaveScratch ws;
    ws.ftab = kLdsWave + wave * kWaveScratchBytes;
    ws.dpc = ws.ftab + 16u * kFramesPerTile;
    ws.epre = ws.dpc + 4u * kFramesPerTile;
    ws.slots = ws.epre + 4u * kFramesPerTile;

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

    // Preamble: the first tile's descriptors (the first memory ops, one round trip) while the
    // tables are built in place by VALU; geometry; the row prefetch; the header DMA; one barrier
    // once the header DMA has landed.
    uint32_t tile = gwave;
    FS_RTSTAMP(5);
    FS_STAMP(0);
    Tile T;
    Unit U;
    u32x4 pf[kPrefetch];
    const bool first = __builtin_amdgcn_readfirstlane(tile) < ntiles;
    {
        uint64_t S;
        uint32_t len;
        tile_descriptors(tile, grp0, n, offsets, lengths, S, len, fpt);
        build_region_a(tabs, lds);
        descriptors_ready<kOps>(S, len);
        U.P = 0;
        if (first) tile_geometry(T, U, tile, grp0, gl0, n, S, len, frames, lds, ws, fpt);
    }
    bool x4 = false;
    // the first rows ahead of the header DMA (still older than the first block's refills, which
    // is all the parse's vmcnt(kPrefetch) needs)
    if (first) prefetch_unit(U, pf);
    if (first) x4 = header_dma<false>(T, frames, lds, hw, gl0, lane);
    // (the mixed class only when the launch asks: a giant tile runs mode A here, so the pass count cannot tell)
    const uint32_t posts0 = first && report ? tile_posts<true>(report, T.len, (report & kAskMixed) ? mixed_class(T.nd()) : kMixNone, gwave == 0u) : 0u;
    FS_STAMP(9);
    tables_landed<kPrefetch>(first, U.P > 0, x4);
    post_tile(report, posts0, lane);  // (after the counted wait, younger than the rows)
    FS_STAMP(10);
    __builtin_amdgcn_s_barrier();  // tables ready (raw barrier: no release fence, no vmcnt(0) drain)
    if ((wave >> 3) != 0u) __builtin_amdgcn_s_setprio(1);  // two-level age priority: the SIMD's younger half first
    FS_STAMP(1);

    while (tile < ntiles) {
        // The lane indices recomputed per tile from mbcnt (no register of the kernel's start
        // stays live for them: they used to be spilled, and their reload at the loop head
        // waited vmcnt(0), draining the tile's prefetched rows).
        uint32_t ln;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
        uint32_t grp = ln >> 2, gl = ln & 3u;
        const bool fvalid = grp < fpt && tile * fpt + grp < n;
        const bool parser = fvalid && gl == 0u;  // the group's lane 0 parses, finishes and stores
        const int npass = T.npass;

        // ---- header parse: after the first block of rows, while the ring's loads are in flight.
        // The header DMA was issued before the tile's rows; vmcnt(kPrefetch) retires it once the
        // first block's refills are the only younger loads.
        auto parse = [&](bool refilled) {
            if (refilled) __builtin_amdgcn_s_waitcnt(0x0070 | kPrefetch);
            else __builtin_amdgcn_s_waitcnt(0x0070);
            parse_tile<kOps>(hw, grp, gl, T.sa(), T.len, mtu, reinterpret_cast<const uint32_t*>(frames + (T.sdw() << 2)),
                       parser, hw);
        };
        uint32_t Y = 0u, csum = 0u;  // the frame's combined register value and sum (mode A)
        for (int pass = 0; pass < npass; ++pass) {
            // (opaque per pass too: lane-derived row constants are rematerialized per pass)
            asm volatile("" : "+v"(grp), "+v"(gl));
            uint32_t A[4] = {0u, 0u, 0u, 0u};
            uint32_t cs = 0u;
            // general block: rows below H take the masked path (scalar branch per row); refills
            // of rows below H are clamped
            auto block = [&](int r0, auto refill_tag) {
                constexpr bool kRefill = decltype(refill_tag)::value;
#pragma unroll
                for (int i = 0; i < kPrefetch; ++i) {
                    const int r = r0 + i;
                    const int rel = U.rel0 + kRowDwords * r;
                    // consume the ring slot, then refill the SAME registers: no copy of an
                    // in-flight load, so the compiler keeps kPrefetch-1 loads outstanding
                    if (r < U.H) masked_row(lds, keys, pf[i], rel, load_pos(rel, U.lo), T.nd(), T.sa(), T.tail_mask(), A, cs);
                    else lean_row(lds, keys, pf[i], A, cs);
                    if (kRefill) {
                        const int rn = rel + kRowDwords * kPrefetch;
                        pf[i] = load_row(U.gfb, r + kPrefetch < U.H ? load_pos(rn, U.lo) : rn);
                    }
                }
            };
            // lean block: every row lean for every lane; the refills lie inside the frame, so they
            // need no clamp: one pointer per block, immediate row offsets
            auto lean_block = [&](int r0, auto refill_tag) {
                constexpr bool kRefill = decltype(refill_tag)::value;
                const uint32_t* pb = U.gfb + (U.rel0 + kRowDwords * (r0 + kPrefetch));
#pragma unroll
                for (int i = 0; i < kPrefetch; ++i) {
                    lean_row(lds, keys, pf[i], A, cs);
                    if (kRefill) pf[i] = *reinterpret_cast<const u32x4_a4*>(pb + kRowDwords * i);
                    // keep consume/refill interleaved per row: unfenced, the scheduler sinks all
                    // refills to the block end behind a vmcnt(0), draining the ring every block
                    __builtin_amdgcn_sched_barrier(0);
                }
            };
            using Yes = std::true_type;
            using No = std::false_type;
            const int Rc = U.P - kPrefetch;  // first row of the last block
            if (U.P > 0) {
                // [first block] (pass 0: parse) [head blocks: general] [body: lean] post [last block]
                if (Rc > 0) {
                    if (U.H > 0) block(0, Yes());
                    else lean_block(0, Yes());
                    if (pass == 0) parse(true);
                    int r0 = kPrefetch;
                    for (; r0 < Rc && r0 < U.H; r0 += kPrefetch) block(r0, Yes());
                    for (; r0 < Rc; r0 += kPrefetch) lean_block(r0, Yes());
                    if (Rc < U.H) block(Rc, No());
                    else lean_block(Rc, No());
                } else {
                    if (U.H > 0) block(0, No());
                    else lean_block(0, No());
                    if (pass == 0) parse(false);
                }
            } else {
                parse(false);  // no rows (every frame of the tile under 4 bytes): rejected by length
            }
            FS_STAMP(2);
            // Opaque frame descriptor: what the combine and the finish derive from it is
            // recomputed here rather than kept (and spilled) across the row loop.
            asm volatile("" : "+v"(T.S), "+v"(T.len));
            // The pass's last row was lean (unless every row was masked): if it ends the frame,
            // its last dword -- lane 3's 4th -- still holds the up to 3 bytes past the frame end.
            // Their CRC contribution is that junk itself (the last dword enters the combine
            // unshifted) and their sum is sad16 of it: combine_piece removes both.
            uint32_t junk = 0u;
            if (pass == 0) {
                // mode B: a head piece ends the frame only when it is the whole frame
                const bool ends = npass == 1 || pieces_of(T.nd()) == 1;
                if (U.P > 0 && U.H < U.P && gl == 3u && T.nd() > 0 && ends) junk = pf[kPrefetch - 1].w & ~T.tail_mask();
            } else if ((U.info & 0x40000000u) && gl == 3u) {
                const uint32_t t = (U.info >> 28) & 3u;
                junk = pf[kPrefetch - 1].w & ~(t == 0u ? 0xffffffffu : ((1u << (8u * t)) - 1u));
            }
            const uint32_t info = U.info;
            // the next pass's piece and its first rows, in flight during this pass's combine
            if (pass + 1 < npass) {
                full_piece_unit(U, lds, ws, frames, T.F, pass + 1, grp, gl);
                prefetch_unit(U, pf);
            }
            uint32_t y, c;
            combine_piece(lds, gl, A, cs, junk, y, c);
            if (npass == 1) {
                Y = y;
                csum = c;
            } else if (gl == 0u && (pass == 0 || (info >> 31))) {
                const uint32_t slot = pass == 0 ? grp : (info & 0xffffu);
                *reinterpret_cast<uint2*>(lds + ws.slots + 8u * slot) = make_uint2(y, c);
            }
        }
        FS_STAMP(3);
        // ---- the group's lane 0: (mode B) Horner over the frame's pieces, finish and store
        // (its frame's parse comes back from LDS).
        if (parser) {
            if (npass > 1) {
                const uint2 h = *reinterpret_cast<const uint2*>(lds + ws.slots + 8u * grp);
                Y = h.x;
                csum = h.y;
                const int npc = pieces_of(T.nd());
                // the frame's first full piece: the exclusive prefix of the groups' full pieces
                const int e0 = (int)lds32(lds, ws.epre + 4u * grp) - (npc - 1);
                for (int k = 1; k < npc; ++k) {
                    const uint2 sl = *reinterpret_cast<const uint2*>(lds + ws.slots + 8u * (kFramesPerTile + e0 + k - 1));
                    Y = zplain(lds, Y, kLdsZ768) ^ sl.x;
                    csum += sl.y;
                }
            }
            finish_frame<kOps>(lds, unpark_parsed<kOps>(lds, hw, grp), T.S, T.len, T.te(), Y, csum, frames, wframes,
                               lengths,
                               tile * fpt + grp, out, status, tx);
        }
        FS_STAMP(4);
        FS_RTSTAMP(6);
        tile += nwaves;
        if (tile < ntiles) {  // next tile: descriptors, geometry, header DMA, row prefetch
            uint64_t S;
            uint32_t len;
            tile_descriptors(tile, grp, n, offsets, lengths, S, len, fpt);
            descriptors_ready<kOps>(S, len);
            tile_geometry(T, U, tile, grp, gl, n, S, len, frames, lds, ws, fpt);
            header_dma<false>(T, frames, lds, hw, gl, lane);
            prefetch_unit(U, pf);
            if (report)
                post_tile(report, tile_posts<true>(report, T.len, (report & kAskMixed) ? mixed_class(T.nd()) : kMixNone, false), lane);
        }
    }
}


// =======================================================================================
// The SEGMENT kernel (digest_kernel_g, variant 3, round 6): mixed lengths on
// the one-pass kernel's block-aligned rows, with no idle group and no pass. A tile's frames, as the
// 64-B blocks that hold them, are concatenated in frame order (a frame with no stream dword takes no
// block; the others are numbered by RANK) into T virtual blocks, cut into 16 CHUNKS of
// L = ceil(T / 16) blocks, one per 4-lane group: every group streams L rows back to back through one
// ring, crossing frame boundaries. A SEGMENT is the part of one frame inside one chunk. The row that
// ends a segment (the frame's last block, or the chunk's last) PARKS the group's 16 streams in LDS
// and restarts them from zero, so the row loop never combines; a frame's head rows (its first block,
// and its second when frame dword 1 lies there) mask the bytes before the frame and apply the CRC
// init; its last block masks the bytes past its end and leaves the streams past its last dword as
// they were (the one-pass tail row). Those rows are EVENTS of the lanes they concern: a divergent
// branch before and after the row's lean update, which the wave runs when any of its lanes has an
// event (about 30 rows of a C3 tile's 45). A tile has at most 16 + 15 = 31 segments, and segment
// (rank k, group g) parks in slot k + g: no per-tile bound, no fallback. After the rows group
// s mod 16 combines slot s as the one-pass kernel combines a frame (to the frame's last dword for
// the segment that ends the frame, to the block end for one cut by its chunk) and shifts it by its
// distance to the frame end; a frame's register is the XOR of its segments' values and its sum the
// sum of theirs (tests/kernel_model.py: crc32_tile_segments).
constexpr int kRingG = 5;
constexpr int kSlotG = 16;  // header slot dwords (1 KB per wave; longer headers come from memory)
constexpr uint32_t kHdrWaveG = 4u * kSlotG * kFramesPerTile;
constexpr uint32_t kLdsHdrG = kLdsTables;
constexpr uint32_t kLdsWaveG = kLdsHdrG + kWavesPerBlock * kHdrWaveG;
// Per-wave scratch: the frame table by rank (16 B: {delta lo, delta hi, vend, info}; block v of the
// tile lies at delta + 64 v), the rank-indexed vend table (~0 past the last rank: the walks' starting
// search), the parked checksums (one per slot, folded over the group; a combined slot's {value, sum}
// after the combine), the slot meta (the rank of the frame parked there; ~0 = unused), and each
// group's frame (read back by the parse and the finish: no register holds it through the rows).
constexpr uint32_t kGFtab = 0, kGVend = 256, kGPcs = 320, kGMeta = 576, kGFrame = 704;
constexpr uint32_t kGScratch = 960;
constexpr uint32_t kSegSlots = 2u * kFramesPerTile - 1u;
static_assert(kLdsWaveG + kWavesPerBlock * kGScratch <= kLdsBytes, "segment kernel LDS");
static_assert(kGPcs - kGVend >= 4u * kFramesPerTile && kGMeta - kGPcs >= 8u * (kSegSlots + 1u) &&
                  kGFrame - kGMeta >= 4u * (kSegSlots + 1u) && kGScratch - kGFrame >= 16u * kFramesPerTile,
              "segment scratch");
// Parked streams: region A's upper halves (bytes 128..255 of its 256-B entries, which no lookup
// reads): wave w owns entries 16 w .. 16 w + 15, two 64-B slots each.
__device__ __forceinline__ uint32_t park_at(uint32_t wave, uint32_t s) {
    return kLdsRegionA + (16u * wave + (s >> 1)) * 256u + 128u + 64u * (s & 1u);
}
// frame info word: block phase of frame dword 0 | start alignment << 4 | block position of the last
// dword << 8 | bytes of the last dword << 12
__device__ __forceinline__ uint32_t head_rows(uint32_t info) {  // head rows after the first: 1 when dword 1 lies in the 2nd block
    return ((info & 15u) == 15u && ((info >> 4) & 3u) != 0u) ? 1u : 0u;
}
// bytes of a dword at byte x of it and after (x <= 0: all, x >= 4: none)
__device__ __forceinline__ uint32_t from_byte(int x) {
    return (uint32_t)(0xffffffffull << ((uint32_t)min(max(x, 0), 4) * 8u));
}
// Inclusive scan over the wave's 16 groups of a group-uniform value: DPP row shifts by one and two
// groups inside each 16-lane row, then the rows' totals by readlane.
__device__ __forceinline__ uint32_t group_scan(uint32_t x, uint32_t lane) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane((int)x, 15);
    const uint32_t t1 = (uint32_t)__builtin_amdgcn_readlane((int)x, 31);
    const uint32_t t2 = (uint32_t)__builtin_amdgcn_readlane((int)x, 47);
    const uint32_t row = lane >> 4;
    return x + (row >= 1u ? t0 : 0u) + (row >= 2u ? t1 : 0u) + (row >= 3u ? t2 : 0u);
}
__device__ __forceinline__ LaneKeys lane_keys(uint32_t lane) {
    LaneKeys keys;
    const uint32_t c = lane & 7u, h = (lane >> 3) & 3u;
    keys.cvec = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) keys.cvec |= (32u * j + 4u * c) << (8u * j);
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t b = (k + h) & 3u;
        keys.sel[k] = 0x0c0c0000u | ((4u + b) << 8) | b;
    }
    return keys;
}

typedef __attribute__((address_space(1))) const u32x4_a4 gu32x4;

// A segment-kernel tile: the chunk a group streams and the two walks along it: the REFILL walk (the
// frame of the row being loaded, kRingG rows ahead) and the CONSUME walk (the frame of the row being
// streamed: its head rows and its segment's last row). The group's own frame lives in LDS (kGFrame).
struct TileG {
    uint64_t S;        // the group's frame (the tile's start only: header DMA, posts)
    uint32_t len;      // (0: a group past the batch end)
    uint32_t T, L;     // wave-uniform: the tile's blocks, rows (the chunk length)
    uint32_t v0;       // the chunk [v0, min(v0 + L, T)) of the tile's blocks (empty when v0 >= T)
    uint32_t vlast;    // the last block a load may address (the chunk's last; 0 for an empty chunk)
    uint64_t rdelta;   // refill walk: block v of its frame at rdelta + 64 v (+ this lane's 16 B)
    uint32_t rvend, rk;
    uint32_t ck, cvs, cvend, cinfo, clast, chd;  // consume walk: rank, blocks [cvs, cvend), info, segment end, head rows
    __device__ __forceinline__ uint32_t sa() const { return (uint32_t)S & 3u; }
    __device__ __forceinline__ uint64_t sdw() const { return S >> 2; }
    __device__ __forceinline__ int ndall() const { return (int)((sa() + len + 3u) >> 2); }
    __device__ __forceinline__ uint32_t v1() const { return min(v0 + L, T); }
};

// The tile's geometry (every lane, before any row): blocks, ranks and the frame table, the chunk,
// and both walks at the chunk's first block.
__device__ __forceinline__ void tile_geometry_g(TileG& G, uint32_t tile, uint32_t grp, uint32_t gl, uint32_t lane,
                                                uint32_t n, uint64_t S, uint32_t len,
                                                const uint8_t* __restrict__ frames, char* lds, uint32_t sc,
                                                uint32_t fpt) {
    G.len = (grp < fpt && tile * fpt + grp < n) ? len : 0u;
    G.S = S;
    const uint32_t sa = G.sa();
    const uint32_t nd = G.len >= 4u ? (sa + G.len + 3u) >> 2 : 0u;
    const uint32_t ph = ((uint32_t)(reinterpret_cast<uint64_t>(frames) >> 2) + (uint32_t)G.sdw()) & 15u;
    const uint32_t nb = nd ? (ph + nd + 15u) >> 4 : 0u;
    const uint32_t incl = group_scan(nb, lane);
    const uint32_t has = nb ? 1u : 0u;
    const uint32_t rincl = group_scan(has, lane);
    const uint32_t vs = incl - nb, rank = rincl - has;
    G.T = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    G.L = (G.T + 15u) >> 4;
    // the tables (this wave's scratch; LDS ops of one wave complete in order)
    if (lane < 16u) *reinterpret_cast<uint32_t*>(lds + sc + kGVend + 4u * lane) = ~0u;
    if (lane < 32u) *reinterpret_cast<uint32_t*>(lds + sc + kGMeta + 4u * lane) = ~0u;
    if (gl == 0u && nb) {
        const uint32_t e = ((sa + G.len) & 3u) ? ((sa + G.len) & 3u) : 4u;
        const uint32_t info = ph | (sa << 4) | (((ph + nd - 1u) & 15u) << 8) | (e << 12);
        const uint64_t delta = reinterpret_cast<uint64_t>(frames) + 4ull * G.sdw() - 4u * ph - 64ull * vs;
        *reinterpret_cast<u32x4*>(lds + sc + kGFtab + 16u * rank) =
            u32x4{(uint32_t)delta, (uint32_t)(delta >> 32), vs + nb, info};
        *reinterpret_cast<uint32_t*>(lds + sc + kGVend + 4u * rank) = vs + nb;
    }
    if (gl == 0u)
        *reinterpret_cast<u32x4*>(lds + sc + kGFrame + 16u * grp) =
            u32x4{(uint32_t)S, (uint32_t)(S >> 32), G.len, rank | (has << 8)};
    G.v0 = grp * G.L;
    const uint32_t v1 = G.v1();
    const bool empty = G.v0 >= v1;
    // the rank holding block v0: #{k : vend_k <= v0}
    uint32_t k0 = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const u32x4 e = *reinterpret_cast<const u32x4*>(lds + sc + kGVend + 16u * j);
        k0 += (e.x <= G.v0 ? 1u : 0u) + (e.y <= G.v0 ? 1u : 0u) + (e.z <= G.v0 ? 1u : 0u) + (e.w <= G.v0 ? 1u : 0u);
    }
    if (empty) k0 = 0u;  // (an empty chunk loads rank 0's first block: a valid address)
    const u32x4 e0 = *reinterpret_cast<const u32x4*>(lds + sc + kGFtab + 16u * k0);
    const uint32_t vs0 = k0 ? lds32(lds, sc + kGVend + 4u * (k0 - 1u)) : 0u;
    G.vlast = empty ? 0u : v1 - 1u;
    G.rk = k0;
    G.rdelta = (((uint64_t)e0.y << 32) | e0.x) + 16u * gl;
    G.rvend = e0.z;
    G.ck = k0;
    G.cvs = empty ? ~0u : vs0;
    G.cvend = e0.z;
    G.cinfo = e0.w;
    G.clast = empty ? ~0u : min(e0.z, v1) - 1u;
    G.chd = empty ? 0u : head_rows(e0.w);
}

template <uint32_t kOps>
__global__ void __launch_bounds__(kThreads, 1)
digest_kernel_g(const uint8_t* __restrict__ frames, const uint64_t* __restrict__ offsets,
                const uint32_t* __restrict__ lengths, uint32_t n, uint32_t mtu, const FsTables* __restrict__ tabs,
                uint2* __restrict__ out, uint8_t* __restrict__ status, uint64_t report, uint8_t* wframes, uint32_t tx,
                uint32_t fpt) {
    char* lds = g_lds;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: SGPR addresses
    const uint32_t grp = lane >> 2, gl = lane & 3u;
    const uint32_t gwave = first_tile(wave);
    const uint32_t nwaves = gridDim.x * kWavesPerBlock;
    fpt = __builtin_amdgcn_readfirstlane(fpt);
    const uint32_t ntiles = (n + fpt - 1) / fpt;
    const uint32_t hw = kLdsHdrG + wave * kHdrWaveG;    // this wave's header slots (and parked parse)
    const uint32_t sc = kLdsWaveG + wave * kGScratch;  // this wave's scratch
    const LaneKeys keys = lane_keys(lane);

    TileG G;
    u32x4 pf[kRingG];
    // the row a refill loads: chunk row r (clamped to the chunk's last block) through the refill walk;
    // `nx` = the frame table entry of the walk's next rank, read at the start of the row (every row,
    // so that no branch waits for an LDS read)
    struct Next {
        uint64_t delta;
        uint32_t vend;
    };
    auto row_addr = [&](uint32_t r, const Next& nx) __attribute__((always_inline)) -> gu32x4* {
        const uint32_t vn = min(G.v0 + r, G.vlast);
        if (vn >= G.rvend) {  // the chunk's next frame (ranks are consecutive)
            G.rk += 1u;
            G.rdelta = nx.delta + 16u * gl;
            G.rvend = nx.vend;
        }
        return reinterpret_cast<gu32x4*>(G.rdelta + ((uint64_t)vn << 6));
    };
    auto next_entry = [&](uint32_t k) __attribute__((always_inline)) -> Next {
        const uint32_t e = sc + kGFtab + 16u * min(k + 1u, kFramesPerTile - 1u);
        return Next{*reinterpret_cast<const uint64_t*>(lds + e), lds32(lds, e + 8u)};
    };
    auto prefetch = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < kRingG; ++i) pf[i] = *row_addr((uint32_t)i, next_entry(G.rk));
    };
    auto posts_of = [&](bool first_of_grid) __attribute__((always_inline)) -> uint32_t {
        const bool ask_mixed = (report & kAskMixed) != 0u;
        const int nd = G.len >= 4u ? G.ndall() : 0;
        return tile_posts<false>(report, G.len, ask_mixed ? mixed_class(nd) : kMixNone, first_of_grid);
    };

    // Preamble: the first tile's descriptors while the tables are built in place; geometry; the first
    // rows; the header DMA; one barrier.
    uint32_t tile = gwave;
    FS_RTSTAMP(5);
    FS_STAMP(0);
    const bool first = __builtin_amdgcn_readfirstlane(tile) < ntiles;
    {
        uint64_t S;
        uint32_t len;
        tile_descriptors(tile, grp, n, offsets, lengths, S, len, fpt);
        build_region_a(tabs, lds);
        descriptors_ready<kOps>(S, len);
        G.L = 0;
        if (first) tile_geometry_g(G, tile, grp, gl, lane, n, S, len, frames, lds, sc, fpt);
    }
    if (first && G.L > 0u) prefetch();
    bool x4 = false;
    if (first) x4 = header_dma<true, kSlotG>(G, frames, lds, hw, gl, lane);
    const uint32_t posts0 = first && report ? posts_of(gwave == 0u) : 0u;
    tables_landed<kRingG, kSlotG>(first, G.L > 0u, x4);
    post_tile(report, posts0, lane);  // (after the counted wait, younger than the rows)
    __builtin_amdgcn_s_barrier();     // tables ready (raw barrier: no release fence, no vmcnt(0) drain)
    if ((wave >> 3) != 0u) __builtin_amdgcn_s_setprio(1);  // two-level age priority: the SIMD's younger half first
    FS_STAMP(1);

    while (tile < ntiles) {
        const bool fvalid = grp < fpt && tile * fpt + grp < n;
        const bool parser = fvalid && gl == 0u;  // the group's lane 0 parses, finishes and stores
        uint32_t A[4] = {0u, 0u, 0u, 0u};
        uint32_t cs = 0u;

        // ---- one row of the chunk from ring slot w: its events, the lean update, the segment's park
        auto consume = [&](const u32x4& w, uint32_t r, const uint2& cn) __attribute__((always_inline)) {
            const uint32_t vr = G.v0 + r;
            const uint32_t hrow = vr - G.cvs;
            const bool head = hrow <= G.chd;
            const bool park = vr == G.clast;
            const bool tail = park && vr + 1u == G.cvend;
            // the streams past a frame's last dword keep their value: saved before the update
            uint32_t As[4];
            if (tail) {
#pragma unroll
                for (int j = 0; j < 4; ++j) As[j] = A[j];
            }
            lean_row(lds, keys, w, A, cs);
            // The event fixes, after the update (which fed w unmasked; it is linear in w): the bytes
            // before the frame (head) and past it (tail) XOR-ed back out of the streams and subtracted
            // from the sum (disjoint byte masks, so sad16 splits), the CRC init XOR-ed in on frame
            // bytes [0, 4), and the streams past the last dword restored.
            if (head || park) {
                if (head) {
                    const uint32_t ci = G.cinfo;
                    const int b0 = 4 * (int)(ci & 15u) + (int)((ci >> 4) & 3u) - 64 * (int)hrow - 16 * (int)gl;
                    int fix = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t k = from_byte(b0 - 4 * j);
                        const uint32_t junk = w[j] & ~k;
                        A[j] ^= junk ^ (k & ~from_byte(b0 + 4 - 4 * j));
                        fix += (int)sad16(junk, 0u);
                    }
                    cs -= (uint32_t)fix;
                }
                if (tail) {
                    const uint32_t ci = G.cinfo;
                    const int eb = 4 * (int)((ci >> 8) & 15u) + (int)((ci >> 12) & 7u) - 16 * (int)gl;
                    int fix = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t junk = w[j] & from_byte(eb - 4 * j);
                        A[j] = (eb - 4 * j > 0) ? (A[j] ^ junk) : As[j];
                        fix += (int)sad16(junk, 0u);
                    }
                    cs -= (uint32_t)fix;
                }
                if (park) {  // the segment (rank ck, group grp) into slot ck + grp; the streams restart
                    const uint32_t s = G.ck + grp;
                    *reinterpret_cast<u32x4*>(lds + park_at(wave, s) + 16u * gl) = u32x4{A[0], A[1], A[2], A[3]};
                    uint32_t c = (cs & 0xffffu) + (cs >> 16);
                    c += dpp_quad<kQuadXor1>(c);
                    c += dpp_quad<kQuadXor2>(c);
                    if (gl == 0u) {
                        *reinterpret_cast<uint32_t*>(lds + sc + kGPcs + 8u * s) = c;
                        *reinterpret_cast<uint32_t*>(lds + sc + kGMeta + 4u * s) = G.ck;
                    }
                    A[0] = A[1] = A[2] = A[3] = 0u;
                    cs = 0u;
                    if (tail) {  // the chunk's next frame
                        G.ck += 1u;
                        G.cvs = G.cvend;
                        G.cvend = cn.x;
                        G.cinfo = cn.y;
                        G.clast = min(cn.x, G.v1()) - 1u;
                        G.chd = head_rows(cn.y);
                    } else {  // the chunk's end: no event after it
                        G.clast = ~0u;
                        G.cvs = ~0u;
                        G.chd = 0u;
                    }
                }
            }
        };
        auto block = [&](uint32_t r0, auto refill_tag) __attribute__((always_inline)) {
            constexpr bool kRefill = decltype(refill_tag)::value;
#pragma unroll
            for (int i = 0; i < kRingG; ++i) {
                // both walks' next frame-table entries, read ahead of the row's lookups
                const uint2 cn = *reinterpret_cast<const uint2*>(
                    lds + sc + kGFtab + 16u * min(G.ck + 1u, kFramesPerTile - 1u) + 8u);
                Next rn;
                if (kRefill) rn = next_entry(G.rk);
                consume(pf[i], r0 + (uint32_t)i, cn);
                if (kRefill) pf[i] = *row_addr(r0 + (uint32_t)(i + kRingG), rn);
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        // header parse: after the first block of rows; the header DMA was issued behind the tile's
        // first rows, so vmcnt(kRingG) retires it once the block's refills are the only younger loads
        auto parse = [&](bool refilled) __attribute__((always_inline)) {
            if (refilled) __builtin_amdgcn_s_waitcnt(0x0070 | kRingG);
            else __builtin_amdgcn_s_waitcnt(0x0070);
            const u32x4 fr = *reinterpret_cast<const u32x4*>(lds + sc + kGFrame + 16u * grp);
            const uint64_t S = ((uint64_t)fr.y << 32) | fr.x;
            parse_tile<kOps, kSlotG>(hw, grp, gl, (uint32_t)S & 3u, fr.z, mtu,
                                     reinterpret_cast<const uint32_t*>(frames + ((S >> 2) << 2)), parser, hw);
        };
        using Yes = std::true_type;
        using No = std::false_type;
        const uint32_t R = G.L;
        if (R > (uint32_t)kRingG) {
            block(0u, Yes());
            parse(true);
            uint32_t r0 = kRingG;
            for (; r0 + kRingG < R; r0 += kRingG) block(r0, Yes());
            block(r0, No());
        } else if (R > 0u) {
            block(0u, No());
            parse(false);
        } else {
            parse(false);  // no rows (every frame of the tile under 4 bytes): rejected by length
        }
        FS_STAMP(2);

        // ---- the parked segments: slot s combined by group s mod 16 (both rounds in one pass): to the
        // frame's last dword for the segment that ends the frame, else to the end of the chunk's last
        // block and then shifted by the bytes from there to the frame's last dword
        const uint32_t T = G.T, L = G.L;
#pragma unroll
        for (uint32_t h = 0; h < 2; ++h) {
            const uint32_t s = grp + 16u * h;
            const uint32_t k = s < kSegSlots ? lds32(lds, sc + kGMeta + 4u * s) : ~0u;
            if (k != ~0u) {
                const u32x4 a4 = *reinterpret_cast<const u32x4*>(lds + park_at(wave, s) + 16u * gl);
                const uint32_t c = lds32(lds, sc + kGPcs + 8u * s);
                const uint2 ve = *reinterpret_cast<const uint2*>(lds + sc + kGFtab + 16u * k + 8u);  // {vend, info}
                const uint32_t v1g = min((s - k + 1u) * L, T), dblk = ve.x > v1g ? ve.x - v1g : 0u;
                const int ealign = 15 - (int)((ve.y >> 8) & 15u);
                const uint32_t Aa[4] = {a4.x, a4.y, a4.z, a4.w};
                uint32_t Y = combine_to_end<LayA1>(lds, Aa, dblk ? 0 : ealign, gl);
                if (dblk) Y = zshift(lds, Y, 64u * dblk - 4u * (uint32_t)ealign);
                if (gl == 0u) *reinterpret_cast<uint2*>(lds + sc + kGPcs + 8u * s) = make_uint2(Y, c);
            }
        }
        FS_STAMP(3);
        // ---- the group's lane 0: its frame's segments (slots rank + the chunks of its first and last
        // block), finish and store
        if (parser) {
            const u32x4 fr = *reinterpret_cast<const u32x4*>(lds + sc + kGFrame + 16u * grp);
            const uint64_t S = ((uint64_t)fr.y << 32) | fr.x;
            const uint32_t len = fr.z, rank = fr.w & 0xffu;
            uint32_t Y = 0u, c = 0u;
            if (fr.w >> 8) {
                const uint32_t vend = lds32(lds, sc + kGVend + 4u * rank);
                const uint32_t vs = rank ? lds32(lds, sc + kGVend + 4u * (rank - 1u)) : 0u;
                const uint32_t f = rank + vs / L, l = min(rank + (vend - 1u) / L, kSegSlots - 1u);
                for (uint32_t s = f; s <= l; ++s) {
                    const uint2 rs = *reinterpret_cast<const uint2*>(lds + sc + kGPcs + 8u * s);
                    Y ^= rs.x;
                    c += rs.y;
                }
            }
            const uint32_t e = ((uint32_t)S + len) & 3u;
            finish_frame<kOps>(lds, unpark_parsed<kOps>(lds, hw, grp), S, len, e ? e : 4u, Y, c, frames, wframes,
                               lengths, tile * fpt + grp, out, status, tx);
        }
        FS_STAMP(4);
        FS_RTSTAMP(6);
        tile += nwaves;
        if (tile < ntiles) {  // next tile: descriptors, geometry, row prefetch, header DMA
            uint64_t S;
            uint32_t len;
            tile_descriptors(tile, grp, n, offsets, lengths, S, len, fpt);
            descriptors_ready<kOps>(S, len);
            tile_geometry_g(G, tile, grp, gl, lane, n, S, len, frames, lds, sc, fpt);
            if (G.L > 0u) prefetch();
            header_dma<true, kSlotG>(G, frames, lds, hw, gl, lane);
            if (report) post_tile(report, posts_of(false), lane);
        }
    }
}

// =======================================================================================
// The small-frame kernel (digest_kernel_s, variant 8): ONE LANE PER FRAME,
// 64 frames per wave, for batches of short frames (the reference's own benchmark sends 47-byte
// UDP frames, stacks/benchmark_test.go:12-46). The 4-lane kernels spend a 104-KB table image,
// a workgroup barrier and one 16-wave workgroup per CU on every launch; on 47-byte frames that
// fixed cost is the whole launch. Here a workgroup is 4 waves with 52 KB of LDS (the Z_4..Z_1
// tables, 16 KB, built in place from their bases, and the header slots), so three fit a CU and
// consecutive launches overlap. Per lane: the frame's descriptor, its 16-B aligned chunks
// (whole chunks never leave the pages that hold frame bytes) into the lane's header slot, then
// the CRC as a Horner chain P <- Z4(P) ^ d over the frame's dwords read back from the slot (the
// CRC init XOR-ed into frame bytes 0..3, as the 4-lane kernels do), the one's-complement sum,
// the RecvEth parse and the finish of the 4-lane kernels (parse_frame, finish_frame).
// Frames longer than the slot (~130 B) stay correct -- their dwords past the slot come from
// global memory -- but slow: the variant is for short-frame traffic (fs_ctx_set_kernel).
constexpr int kSmallWaves = 4;
constexpr int kSmallSlotRows = 9;  // 36 dwords per frame: frame dwords [0, 33) at any chunk phase
constexpr uint32_t kSmallQuad = kSmallSlotRows * 256u;  // 16 frames' slots ([x >> 2][frame][x & 3])
constexpr uint32_t kSmallWave = 4u * kSmallQuad;
constexpr uint32_t kSmallTables = 16384u;  // zfin: Z_4, Z_3, Z_2, Z_1 ([4][256] each)
constexpr uint32_t kSmallLdsBytes = kSmallTables + kSmallWaves * kSmallWave;
static_assert(kSmallLdsBytes <= 53248, "three small-kernel workgroups fit a CU's LDS");
__shared__ __attribute__((aligned(16))) char s_lds[kSmallLdsBytes];

struct LayoutS {
    __device__ static __forceinline__ uint32_t fin(const char* lds, uint32_t v, uint32_t t) {
        return zplain(lds, v, 4096u * t);
    }
    __device__ static __forceinline__ uint32_t byte1(const char* lds, uint32_t i) { return lds32(lds, 3u * 4096u + (i << 2)); }
    __device__ static __forceinline__ uint32_t shift(const char*, uint32_t v, uint32_t) { return v; }  // (no TX op)
};

// sum of frame bytes [p0, p1) from the lane's slot (chunk phase xo), in the 16-bit-half domain
__device__ __forceinline__ uint32_t lane_slot_sum(const char* lds, uint32_t hw, uint32_t g, uint32_t sa, uint32_t xo,
                                                  int p0, int p1) {
    uint32_t s = 0;
    if (p1 <= p0) return s;
    const int a0 = (int)sa + p0, a1 = (int)sa + p1;
    for (int k = a0 >> 2; k <= (a1 - 1) >> 2; ++k) s = sad16(hdr_dw(lds, hw, g, xo + (uint32_t)k) & range_mask(k, a0, a1), s);
    return s;
}

template <uint32_t kOps>
__global__ void __launch_bounds__(kWave * kSmallWaves)
digest_kernel_s(const uint8_t* __restrict__ frames, const uint64_t* __restrict__ offsets,
                const uint32_t* __restrict__ lengths, uint32_t n, uint32_t mtu, const FsTables* __restrict__ tabs,
                uint2* __restrict__ out, uint8_t* __restrict__ status, uint64_t report) {
    static_assert(kOps != kOpsTx, "the small-frame kernel has no TX fill");
    char* lds = s_lds;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t g = lane & 15u;
    const uint32_t hw = kSmallTables + wave * kSmallWave + (lane >> 4) * kSmallQuad;  // this lane's slot set
    const uint32_t nwaves = gridDim.x * kSmallWaves;
    const uint32_t ntiles = (n + 63u) / 64u;
    uint32_t tile = __builtin_amdgcn_readfirstlane(blockIdx.x * kSmallWaves + wave);

    // the first tile's descriptors, then the tables while they fly
    auto desc = [&](uint32_t t, uint64_t& S, uint32_t& len) {
        const uint32_t fi = t * 64u + lane;
        const uint32_t fc = fi < n ? fi : n - 1u;
        S = offsets[fc];
        len = fi < n ? lengths[fc] : 0u;
    };
    uint64_t S = 0;
    uint32_t len = 0;
    if (tile < ntiles) desc(tile, S, len);
    {   // Z_4, Z_3, Z_2, Z_1 (plain pieces 8..23 of the 4-lane layout) in place: wave w builds
        // pieces 8 + w + 4k, lane l the entries 4l .. 4l + 3 of each
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t p = 8u + wave + 4u * k;
            const uint32_t* pb = tabs->plain_basis[p];
            uint32_t x = 0;
#pragma unroll
            for (uint32_t j = 2; j < 8; ++j) x ^= pb[j] & (0u - ((lane >> (j - 2u)) & 1u));
            const uint32_t x1 = x ^ pb[0];
            *reinterpret_cast<u32x4*>(lds + 1024u * (p - 8u) + 16u * lane) = u32x4{x, x1, x ^ pb[1], x1 ^ pb[1]};
        }
    }
    __syncthreads();

    bool long_posted = false;
    for (; tile < ntiles; tile += nwaves) {
        const uint32_t fi = tile * 64u + lane;
        const bool valid = fi < n;
        // a frame too long for this kernel's slot: report it (once per wave), so the launches that
        // follow run the 4-lane kernels (launch_digest); this one stays correct, only slower
        if (report && !long_posted && __ballot(valid && len > kSmallMaxLen) != 0u) {
            if (lane == 0u) post_report<kReportLong>(report);
            long_posted = true;
        }
        if (kOps == kOpsFcs) len = len >= 4u ? len - 4u : 0u;
        // 16-B chunks at ABSOLUTE 16-B boundaries (frames is only 4-byte aligned): a chunk that
        // holds a frame byte never leaves that byte's page
        const uint64_t fa = reinterpret_cast<uint64_t>(frames) + S;
        const uint32_t sa = (uint32_t)fa & 3u;        // = S & 3 (frames is 4-byte aligned)
        const uint32_t xo = (uint32_t)(fa >> 2) & 3u;  // frame dword 0's place in its 16-B chunk
        const uint32_t nd = (sa + len + 3u) >> 2;     // dwords holding frame bytes
        const uint32_t nch = valid && len > 0u ? (xo + nd + 3u) >> 2 : 0u;
        const u32x4* cb = reinterpret_cast<const u32x4*>(fa & ~(uint64_t)15u);
        // the frame's chunks into the slot (the chunks past the slot come from memory below)
        u32x4 v[kSmallSlotRows];
#pragma unroll
        for (int c = 0; c < kSmallSlotRows; ++c)
            if ((uint32_t)c < nch) v[c] = cb[c];
#pragma unroll
        for (int c = 0; c < kSmallSlotRows; ++c)
            if ((uint32_t)c < nch) *reinterpret_cast<u32x4*>(lds + hw + (uint32_t)c * 256u + g * 16u) = v[c];
        // the next tile's descriptors, behind this tile's chunks
        uint64_t Sn = 0;
        uint32_t lenn = 0;
        if (tile + nwaves < ntiles) desc(tile + nwaves, Sn, lenn);

        // CRC (pending-register Horner, zero init; the init XOR-ed into frame bytes 0..3) and the
        // one's-complement sum over the frame's dwords [0, nd) (head and tail bytes masked)
        const uint32_t head = 0xffffffffu << (8u * sa);
        const uint32_t te = ((sa + len) & 3u) ? ((sa + len) & 3u) : 4u;
        const uint32_t tailm = te == 4u ? 0xffffffffu : ((1u << (8u * te)) - 1u);
        const uint32_t* fb = reinterpret_cast<const uint32_t*>(frames + ((S >> 2) << 2));
        uint32_t P = 0u, cs = 0u;
        const uint32_t lim = valid && len >= 4u ? nd : 0u;
        const uint32_t lim1 = min(lim, 4u * kSmallSlotRows - xo);  // the dwords in the slot
        for (uint32_t x = 0; x < lim1; ++x) {
            uint32_t d = hdr_dw(lds, hw, g, xo + x);
            if (x == 0u) d &= head;
            if (x + 1u == nd) d &= tailm;
            cs = sad16(d, cs);
            const uint32_t c = x == 0u ? head : x == 1u ? ~head : 0u;
            P = zplain(lds, P, 0u) ^ d ^ c;  // Z_4 (zfin[0]) of the pending register
        }
        // a frame longer than the slot: its remaining 16-B chunks from memory, 4 in flight (correct
        // for any length, but one lane streams the frame: the variant is for short frames)
        for (uint32_t c = kSmallSlotRows; c < (lim ? nch : 0u); c += 4u) {
            u32x4 u[4];
#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i)
                if (c + i < nch) u[i] = cb[c + i];
#pragma unroll
            for (uint32_t i = 0; i < 4u; ++i) {
#pragma unroll
                for (uint32_t k = 0; k < 4u; ++k) {
                    const uint32_t x = 4u * (c + i) + k - xo;
                    if (c + i < nch && x < nd) {
                        uint32_t d = u[i][k];
                        if (x + 1u == nd) d &= tailm;
                        cs = sad16(d, cs);
                        P = zplain(lds, P, 0u) ^ d;
                    }
                }
            }
        }

        // header parse (RecvEth's gates and the checksum corrections) from the slot, and the finish
        if (valid) {
            uint32_t hsum = 0;
            int64_t pad = -1;
            if (len >= 34u) {
                const uint32_t d3 = __builtin_bswap32(frame_dw(lds, hw, g, sa, 3, xo));
                const uint32_t off = 14u + ((d3 >> 8) & 0xfu) * 4u;
                const uint32_t tl = __builtin_bswap32(frame_dw(lds, hw, g, sa, 4, xo)) >> 16;
                const uint32_t end = (14u + tl) & 0xffffu;
                hsum = lane_slot_sum(lds, hw, g, sa, xo, 0, (int)min(off, len));
                if (end < len && xo + nd <= 4u * kSmallSlotRows) pad = (int64_t)lane_slot_sum(lds, hw, g, sa, xo, (int)end, (int)len);
            }
            const Parsed Pr = parse_frame<kOps, 32>(lds, hw, g, sa, len, mtu, hsum, pad, fb, xo);
            finish_frame<kOps, LayoutS>(lds, Pr, S, len, te, P, cs, frames, nullptr, lengths, fi, out, status, 0u);
        }
        S = Sn;
        len = lenn;
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
                         int num_cus, volatile uint32_t* report_host, uint32_t* report_dev, uint32_t* next_id,
                         int force, FsOp op, uint8_t* wframes, uint32_t tx) {
    if (n == 0) return hipSuccess;
    const uint32_t max_blocks = (uint32_t)(num_cus > 0 ? num_cus : 256);
    // The report of the launches before (the latest launch id that met a mixed-length tile):
    // launches are enqueued ahead of the GPU, so a report arrives several launches late; the
    // mixed kernel stays chosen for kStickyLaunches launches after the latest report (it keeps
    // reporting while the traffic is mixed, on every kMixedSample-th launch). A heuristic only:
    // never a result.
    // Launch ids are 16-bit (they travel in the report pointer's top bits; 0 = never reported).
    // The window is timed on the host instead: `next_id` is the context's 32-bit launch sequence,
    // and the host notes the sequence at which it first saw the report word change (host-only
    // words kReportSeen / kReportSeenSeq), so a report stays recent for kStickyLaunches of this
    // context's launches and never aliases an old one after the 16-bit ids wrap.
    constexpr uint32_t kStickyLaunches = 4096;
    // (the counter is the context's: another context's launches never shift this one's window;
    // a context is used from one thread at a time, include/framesum.h)
    const uint32_t seq = (*next_id)++;
    uint32_t id = seq & 0xFFFFu;
    if (id == 0u) id = 0x8000u;  // (0 means "never reported"; any non-zero tag will do)
    const uint64_t rdev = reinterpret_cast<uint64_t>(report_dev);
    const bool can_report = report_host && rdev != 0u && (rdev & ~kReportAddrMask) == 0u;  // (64-B aligned too)
    uint64_t report = can_report ? rdev | ((uint64_t)id << 48) : 0u;
    bool mixed = false, giant = false;
    if (can_report) {
        const uint32_t latest = report_host[kReportLatest];
        giant = (latest & kReportMixedGiant) != 0u;
        if (latest != report_host[kReportSeen]) {
            report_host[kReportSeen] = latest;
            report_host[kReportSeenSeq] = seq;
        }
        mixed = latest != 0u && seq - report_host[kReportSeenSeq] <= kStickyLaunches;
        // the mixed-length kernel's own posts only refresh the window: sampled (kMixedSample)
        if (latest == 0u || seq % kMixedSample == 0u) report |= kAskMixed;
        // A context's first launches run the mixed-length kernel: it reports its own mode-B tiles,
        // so mixed traffic keeps it from the first batch on (the one-pass kernel's report would
        // arrive launches late, after slow first batches), and uniform traffic moves to the
        // one-pass kernel once the window ends (host-only word: the device never writes it).
        const uint32_t left = report_host[kReportInitial];
        if (left != 0u) {
            report_host[kReportInitial] = left - 1u;
            mixed = true;
        }
    }
    // fs_ctx_set_kernel: 2 the mixed-length kernel (digest_kernel_ab, pieces), 4 the one-pass kernel, 3 the
    // segment kernel (digest_kernel_g: another mixed-length decomposition, slower on C3)
    if (force == 2 || force == 3 || force == 4) mixed = force != 4;
    if (force == kForceUniformHost) mixed = false;
    // the automatic choice runs the segment kernel while the latest mixed report saw a giant tile
    const bool segments = force == 3 || (mixed && giant && (force == 0 || force == kForceNoSmall || force == 8));
    // The small-frame kernel (RX digest and FCS verify; a TX fill keeps the 4-lane choice above).
    // The kernels report launches that met a frame longer than kSmallMaxLen (kReportLong), and the
    // 4-lane kernels, when asked (kAskRan), that a launch ran (kReportRan, with the grid's first
    // tile's own long flag in the same word, kReportRanLong); the host counts the launches it sees
    // run since the latest long report. Variant 0
    // moves to the small-frame kernel after kShortLaunchesAuto of them; variant 8 runs it until a
    // long report arrives, then the 4-lane choice until kShortLaunchesSmall launches ran short
    // again. The reports come launches late, so a long frame can still meet the small-frame kernel:
    // it stays correct there, only slower (one lane streams it). kForceSmallExact: the host-staged
    // path, which has seen every length.
    bool small = false;
    // kForceNoSmall (a host-staged batch with a long frame) reports as the automatic choice does, so
    // its long frames end a short streak; it only never picks the small-frame kernel itself
    const bool autov = force == 0 || force == kForceNoSmall || force == kForceUniformHost;
    if (can_report) {
        const uint32_t lng = report_host[kReportLong], rw = report_host[kReportRan], ran = rw & 0xFFFFu;
        const bool ran_new = ran != report_host[kReportRanSeen];
        if (lng != report_host[kReportLongSeen] || (ran_new && (rw & kReportRanLong) != 0u)) {
            report_host[kReportLongSeen] = lng;
            report_host[kReportShort] = 0u;
            report_host[kReportLongEver] = 1u;
        } else if (ran_new && ran != lng && report_host[kReportShort] < (1u << 30)) {
            report_host[kReportShort] = report_host[kReportShort] + 1u;
        }
        report_host[kReportRanSeen] = ran;
        const uint32_t streak = report_host[kReportShort];
        if (force == 0) small = streak >= kShortLaunchesAuto;
        if (force == 8) small = report_host[kReportLongEver] == 0u || streak >= kShortLaunchesSmall;
        // every workgroup reports its long frames while the host counts short launches
        if ((autov || force == 8) && streak > 0u) report |= 1ull << 47;
        // "ran": variant 0 samples it on long traffic and asks every launch while it counts short
        // ones; variant 8 (short traffic expected: back to the small-frame kernel after 2 short
        // launches) asks every launch
        if (force == 8 || (autov && (streak > 0u || seq % kRanSample == 0u))) report |= kAskRan;
    } else if (force == 8) {
        small = true;  // no report block: the caller's choice as it stands
    }
    if (force == kForceSmallExact) small = true;
    if (force == kForceNoSmall || force == kForceUniformHost || op == FsOp::kFill) small = false;
    if (small) mixed = false;
    // the variant this launch runs, for fs_ctx_last_kernel (host-only word)
    auto chosen = [&](uint32_t v) {
        if (report_host) report_host[kReportChosen] = v;
    };
    // Fewer frames per tile (8, then 4) while 16 would leave waves without a tile: a small
    // batch still spreads over every CU. The groups past a tile's frames stay empty in the
    // one-pass kernel; the mixed-length kernel gives them pieces of the tile's long frames.
    uint32_t fpt = kFramesPerTile;
    const uint32_t waves = max_blocks * (uint32_t)kWavesPerBlock;
    while (fpt > 4u && (n + fpt - 1) / fpt < waves) fpt >>= 1;
    const uint32_t tiles = (n + fpt - 1) / fpt;
    uint32_t blocks = (tiles + kWavesPerBlock - 1) / kWavesPerBlock;
    if (blocks > max_blocks) blocks = max_blocks;
    uint2* o = reinterpret_cast<uint2*>(out);
#define FS_LAUNCH(K)                                                                                        \
    hipLaunchKernelGGL(K, dim3(blocks), dim3(kThreads), 0, stream, frames, offsets, lengths, n, mtu, \
                       tables, o, status, report, wframes, tx, fpt)
    chosen(small ? 8u : mixed ? (segments ? 3u : 2u) : 4u);
    if (small) {
        const uint32_t stiles = (n + 63u) / 64u;  // 64 frames (one per lane) per wave
        uint32_t sb = (stiles + kSmallWaves - 1u) / kSmallWaves;
        if (sb > 2u * max_blocks) sb = 2u * max_blocks;
        if (op == FsOp::kFcs)
            hipLaunchKernelGGL((digest_kernel_s<kOpsFcs>), dim3(sb), dim3(kWave * kSmallWaves), 0, stream, frames,
                               offsets, lengths, n, mtu, tables, reinterpret_cast<uint2*>(out), status, report);
        else
            hipLaunchKernelGGL((digest_kernel_s<kOpsDigest>), dim3(sb), dim3(kWave * kSmallWaves), 0, stream, frames,
                               offsets, lengths, n, mtu, tables, reinterpret_cast<uint2*>(out), status, report);
        return hipGetLastError();
    }
    switch (op) {
    case FsOp::kDigest:
        if (mixed && segments) FS_LAUNCH((digest_kernel_g<kOpsDigest>));
        else if (mixed) FS_LAUNCH((digest_kernel_ab<kOpsDigest>));
        else FS_LAUNCH((digest_kernel_a<kOpsDigest>));
        break;
    case FsOp::kFill:
        if (mixed && segments) FS_LAUNCH((digest_kernel_g<kOpsTx>));
        else if (mixed) FS_LAUNCH((digest_kernel_ab<kOpsTx>));
        else FS_LAUNCH((digest_kernel_a<kOpsTx>));
        break;
    case FsOp::kFcs:
        if (mixed && segments) FS_LAUNCH((digest_kernel_g<kOpsFcs>));
        else if (mixed) FS_LAUNCH((digest_kernel_ab<kOpsFcs>));
        else FS_LAUNCH((digest_kernel_a<kOpsFcs>));
        break;
    }
#undef FS_LAUNCH
    return hipGetLastError();
}

}  // namespace framesum
