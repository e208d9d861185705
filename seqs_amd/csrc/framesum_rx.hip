// framesum streaming kernel — CDNA4 / gfx950. The engine's kernel for every operation
// (RX digest, TX fill, FCS verify).
//
// One fused HBM pass per frame computes
//   * the IEEE CRC-32 of frame[0:len)                        (new: SURVEY.md §0.1)
//   * IPv4Header.CalculateChecksum() of frame[14:34]         (eth/headers.go:333-340)
//   * the TCP/UDP checksum RecvEth verifies + its verdict    (stacks/portstack.go:163-308,
//     eth/headers.go:382-393, :510-527; the arithmetic of eth/crc.go:13-84)
//
// Decomposition:
//   * a wave owns TILES of 16 consecutive frames; its 64 lanes are 4 GROUPS of 16.
//   * a frame streams as PIECES of up to 6 ROWS of 256 B, anchored at its stream end Ed (its end
//     rounded down to a dword): the last piece ends at Ed, each earlier one 1536 B before it, and
//     the HEAD piece keeps the 1..6 rows that remain. Lane l of a group loads bytes [16l, 16l+16)
//     of a row with one global_load_dwordx4, so a wave instruction reads 4 x 256 contiguous bytes.
//   * a STEP gives every group one piece. A tile runs its head pieces first, ordered by rows (a
//     step's pieces have about equal rows), then its other pieces round by round (round p: piece p
//     of every frame that has one), so no two groups of a step share a frame.
//   * the row ring (6 x 16 B per lane) runs one step ahead, across steps and tiles: while a step's
//     6 rows are consumed, the next step's 6 rows are loaded into the same registers.
//   * CRC-32 is linear over GF(2); feeding k zero bytes is a linear map Z_k. Each lane keeps 4 dword
//     STREAMS (its chunk's dwords 0..3); a stream's dwords are 256 B apart, so its Horner step is
//     A <- Z256(A) ^ w: 4 byte-table lookups in LDS (8 copies per byte table, lane-rotated:
//     conflict-free for any data). A piece's 64 streams combine as U = Z4(Z4(Z4(A0)^A1)^A2)^A3 per
//     lane, Z_(16(3-r)) per lane r of a quad + DPP quad xor, Z_(64(3-q)) per quad q + DPP row xor;
//     a frame's pieces fold C <- Z1536(C) ^ W. The CRC init is applied by XOR-ing the frame's first
//     4 bytes with 0xFF (leading zeros do not change a zero-init CRC).
//   * one's-complement sum: v_sad_u16 over the same registers, in the 16-bit-half domain (the
//     byte-swapped big-endian word sum, mod 65535).
//   * the head piece's first chunks (frame dwords [0, 25)) are written to a per-frame LDS header
//     slot as they stream; the parse and the finish run once per tile, one lane per frame.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "framesum_internal.h"

namespace framesum {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef __attribute__((address_space(1))) const u32x4_a4 gu32x4;  // global (not flat) row loads

constexpr int kWave = 64;
constexpr int kWaves = 8;  // waves per workgroup: two workgroups (80 KB LDS each) fit a CU
constexpr int kThreads = kWave * kWaves;
constexpr int kPR = 6;                         // rows per piece = ring depth = positions per step
constexpr uint32_t kPieceBytes = 256u * kPR;   // 1536
constexpr int kTile = 16;                      // frames per tile
constexpr int kSlotDw = 28;                    // header slot: 7 chunks of 16 B
constexpr uint32_t kSlotBytes = 4u * kSlotDw;
// per-wave LDS area: 16 header slots, the frames' pending CRC registers and sums, the step order
constexpr uint32_t kWC = kTile * kSlotBytes;
constexpr uint32_t kWS = kWC + 4u * kTile;
constexpr uint32_t kWO = kWS + 4u * kTile;
constexpr uint32_t kWaveBytes = kWO + 16u;
constexpr uint32_t kLdsWaves = 65536u;  // [0, 64 KB): the table region
constexpr uint32_t kLdsBytes = kLdsWaves + kWaves * kWaveBytes;
static_assert(2u * kLdsBytes <= 160u * 1024u, "two workgroups per CU");
static_assert(kWaveBytes % 16u == 0u && kSlotBytes % 16u == 0u, "16-B aligned header chunks");

__shared__ __attribute__((aligned(16))) char g_lds[kLdsBytes];

// section markers in the assembly (diagnostic builds only: -DFS_MARKS; tools/asm_sections.py)
#ifdef FS_MARKS
#define FS_MARK(name) asm volatile("; @@" name ::: "memory")
#else
#define FS_MARK(name) do { } while (0)
#endif

// the plain tables (FsTablesRx::plain_basis order, kRxPlain shifts)
enum : uint32_t { kT4 = 0, kT16 = 1, kT32 = 2, kT48 = 3, kT64 = 4, kT128 = 5, kT192 = 6, kT1536 = 7 };

enum : uint32_t {
    V_OK = 0, V_SMOL = 1, V_MTU = 2, V_NOT_IPV4 = 3, V_ARP = 4, V_IPVER = 5, V_IHL = 6, V_BADLEN = 7,
    V_PROTO = 8, V_SHORT = 9, V_ZEROPORT = 10, V_UDPLEN = 11, V_TCPOFF = 12, V_CSUM = 13, V_FCS = 14
};
// operations (a template parameter: each is its own instantiation)
enum : uint32_t { kOpsDigest = 0, kOpsTx = 1, kOpsFcs = 2 };
enum : uint32_t { kTxFill = 1, kTxAppend = 2 };

__device__ __forceinline__ uint32_t lds32(uint32_t a) { return *reinterpret_cast<const uint32_t*>(g_lds + a); }
__device__ __forceinline__ void sts32(uint32_t a, uint32_t v) { *reinterpret_cast<uint32_t*>(g_lds + a) = v; }

// a ^ b ^ c in one VALU op (v_bitop3_b32, truth table 0x96; gfx950 has no v_xor3)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// acc + x[15:0] + x[31:16] in one op: the one's-complement accumulation
__device__ __forceinline__ uint32_t sad16(uint32_t x, uint32_t acc) { return __builtin_amdgcn_sad_u16(x, 0u, acc); }
__device__ __forceinline__ uint32_t fold16(uint32_t x) { return (x & 0xffffu) + (x >> 16); }
__device__ __forceinline__ uint32_t bswap16(uint32_t v) { return ((v & 0xffu) << 8) | ((v >> 8) & 0xffu); }

template <int kCtrl>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kCtrl, 0xf, 0xf, false);
}
constexpr int kQuadXor1 = 0xB1, kQuadXor2 = 0x4E, kRowRor4 = 0x124, kRowRor8 = 0x128;

// ---------------------------------------------------------------------------------------
// Tables.
//
// Region row e (256 B at LDS e * 256): slots 0..31 hold Z256[b][e] at slot 8b + c (c = copy).
// Lane L = c + 8h (within its 32-lane half) reads byte table (k + h) & 3 in its k-th lookup: the
// 32 lanes hit 32 distinct banks whatever the data. One v_perm_b32 forms the address (the data
// byte as bits 8..15, the lane's slot byte as bits 0..7).
struct Keys {
    uint32_t cvec;   // byte j = the lane's slot byte for byte table j (32 j + 4 c)
    uint32_t s[4];   // v_perm selectors of the 4 lookups
};
__device__ __forceinline__ Keys lane_keys(uint32_t lane) {
    const uint32_t c = lane & 7u, h = (lane >> 3) & 3u;
    Keys k;
    k.cvec = 0x60402000u + 0x04040404u * c;
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
        const uint32_t b = (i + h) & 3u;
        k.s[i] = 0x0C0C0000u | ((4u + b) << 8) | b;
    }
    return k;
}
// Z256(a) ^ w (the row step)
__device__ __forceinline__ uint32_t zrow(uint32_t a, const Keys& k, uint32_t w) {
    const uint32_t t0 = lds32(__builtin_amdgcn_perm(a, k.cvec, k.s[0]));
    const uint32_t t1 = lds32(__builtin_amdgcn_perm(a, k.cvec, k.s[1]));
    const uint32_t t2 = lds32(__builtin_amdgcn_perm(a, k.cvec, k.s[2]));
    const uint32_t t3 = lds32(__builtin_amdgcn_perm(a, k.cvec, k.s[3]));
    return xor3(xor3(t0, t1, t2), t3, w);
}
// Slots 32..63: plain table t, byte b, entry e at slot 32 + ((4t + b) ^ (e >> 3)) (the XOR spreads
// a table's entries over the banks). cst byte b = 128 + 4 (4t + b): x = (e << 8) | cst_b, and
// (x >> 9) & 0x7C = (e >> 3) << 2 supplies the swizzle.
__host__ __device__ constexpr uint32_t pcst(uint32_t t) { return 0x8C888480u + 0x10101010u * t; }
__device__ __forceinline__ uint32_t paddr(uint32_t v, uint32_t cst, uint32_t b) {
    const uint32_t x = __builtin_amdgcn_perm(v, cst, 0x0C0C0000u | ((4u + b) << 8) | b);
    return x ^ ((x >> 9) & 0x7Cu);
}
__device__ __forceinline__ uint32_t zt(uint32_t v, uint32_t cst) {
    return lds32(paddr(v, cst, 0)) ^ lds32(paddr(v, cst, 1)) ^ lds32(paddr(v, cst, 2)) ^ lds32(paddr(v, cst, 3));
}
// the standard CRC-32 byte table (Z4's byte-3 table)
__device__ __forceinline__ uint32_t tbyte(uint32_t i) {
    return lds32((i << 8) + 128u + ((((kT4 << 2) + 3u) ^ (i >> 3)) << 2));
}
// Z256 from copy 0 of the row tables (a few uses per frame)
__device__ __forceinline__ uint32_t z256(uint32_t v) {
    return lds32((v & 0xffu) << 8) ^ lds32((((v >> 8) & 0xffu) << 8) + 32u) ^ lds32((((v >> 16) & 0xffu) << 8) + 64u) ^
           lds32(((v >> 24) << 8) + 96u);
}
// Z_k(v) for any k (TX corrections)
__device__ __forceinline__ uint32_t zshift(uint32_t v, uint32_t k) {
    for (; k >= 1536u; k -= 1536u) v = zt(v, pcst(kT1536));
    for (; k >= 256u; k -= 256u) v = z256(v);
    if (k >= 192u) { v = zt(v, pcst(kT192)); k -= 192u; }
    else if (k >= 128u) { v = zt(v, pcst(kT128)); k -= 128u; }
    else if (k >= 64u) { v = zt(v, pcst(kT64)); k -= 64u; }
    if (k >= 48u) { v = zt(v, pcst(kT48)); k -= 48u; }
    else if (k >= 32u) { v = zt(v, pcst(kT32)); k -= 32u; }
    else if (k >= 16u) { v = zt(v, pcst(kT16)); k -= 16u; }
    for (; k >= 4u; k -= 4u) v = zt(v, pcst(kT4));
    for (; k > 0u; --k) v = (v >> 8) ^ tbyte(v & 0xffu);
    return v;
}

// The workgroup's LDS image, by VALU from the bases (scalar loads; no vector-memory traffic).
// Row tables: thread t builds Z256[b][e] for e = t & 255, b = 2 (t >> 8), 2 (t >> 8) + 1, 8 copies
// each. Plain tables: wave w builds q = w + 8 i (i = 0..3), lane l the entries 4l .. 4l + 3.
__device__ __forceinline__ uint64_t sgpr_addr(const void* p) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a);
}
__device__ __forceinline__ void build_tables(const FsTablesRx* __restrict__ tabs, uint32_t wave, uint32_t lane) {
    typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
    const uint32_t t = wave * 64u + lane;
    const uint32_t hb = wave >> 2;  // wave-uniform
    const uint32_t e = t & 255u;
    const uint64_t a0 = sgpr_addr(&tabs->z256_basis[2u * hb][0]), a1 = sgpr_addr(&tabs->z256_basis[2u * hb + 1u][0]);
    const uint64_t q0 = sgpr_addr(&tabs->plain_basis[wave][0]), q1 = sgpr_addr(&tabs->plain_basis[wave + 8u][0]);
    const uint64_t q2 = sgpr_addr(&tabs->plain_basis[wave + 16u][0]), q3 = sgpr_addr(&tabs->plain_basis[wave + 24u][0]);
    u32x8 z0, z1, p0, p1, p2, p3;
    asm volatile(
        "s_load_dwordx8 %0, %6, 0x0\n\ts_load_dwordx8 %1, %7, 0x0\n\ts_load_dwordx8 %2, %8, 0x0\n\t"
        "s_load_dwordx8 %3, %9, 0x0\n\ts_load_dwordx8 %4, %10, 0x0\n\ts_load_dwordx8 %5, %11, 0x0\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&s"(z0), "=&s"(z1), "=&s"(p0), "=&s"(p1), "=&s"(p2), "=&s"(p3)
        : "s"(a0), "s"(a1), "s"(q0), "s"(q1), "s"(q2), "s"(q3));
    uint32_t v0 = 0, v1 = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        const uint32_t m = 0u - ((e >> j) & 1u);
        v0 ^= z0[j] & m;
        v1 ^= z1[j] & m;
    }
    u32x4* dst = reinterpret_cast<u32x4*>(g_lds + e * 256u + 64u * hb);
    dst[0] = u32x4{v0, v0, v0, v0};
    dst[1] = u32x4{v0, v0, v0, v0};
    dst[2] = u32x4{v1, v1, v1, v1};
    dst[3] = u32x4{v1, v1, v1, v1};
    auto piece = [&](const u32x8& pb, uint32_t q) {
        uint32_t x = 0;
#pragma unroll
        for (uint32_t j = 2; j < 8; ++j) x ^= pb[j] & (0u - ((lane >> (j - 2u)) & 1u));
        const uint32_t x1 = x ^ pb[0];
        const uint32_t xv[4] = {x, x1, x ^ pb[1], x1 ^ pb[1]};
        const uint32_t slot = 32u + (q ^ (lane >> 1));  // e >> 3 for e = 4 lane + i
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) sts32(((4u * lane + i) << 8) + (slot << 2), xv[i]);
    };
    piece(p0, wave);
    piece(p1, wave + 8u);
    piece(p2, wave + 16u);
    piece(p3, wave + 24u);
}

// ---------------------------------------------------------------------------------------
// Rows.

// A lean row: four Z256 steps and four v_sad_u16, no masks.
#ifndef FS_RX_DIAG
#define FS_RX_DIAG 0
#endif
__device__ __forceinline__ void lean_row(const Keys& k, u32x4 v, uint32_t (&A)[4], uint32_t& cs) {
    if (FS_RX_DIAG & 8) {
        A[0] ^= v.x; A[1] ^= v.y; A[2] ^= v.z; A[3] ^= v.w; cs += v.x;
        return;
    }
    A[0] = zrow(A[0], k, v.x);
    A[1] = zrow(A[1], k, v.y);
    A[2] = zrow(A[2], k, v.z);
    A[3] = zrow(A[3], k, v.w);
    cs = sad16(v.x, cs);
    cs = sad16(v.y, cs);
    cs = sad16(v.z, cs);
    cs = sad16(v.w, cs);
}

// A head row (the rows that hold bytes before the frame or its first two dwords). x: frame dword
// (relative to F4 = S & ~3) of the chunk's dword 0. Bytes before the frame are zeroed, and the CRC
// init XORs 0xFF into frame bytes [0, 4): for dword j, t = the bytes of it before S (clamped to
// 0..4); keep(t) = the bytes at or after S, and the init bytes are keep(t) & ~keep(t + 4).
__device__ __forceinline__ uint32_t keep_mask(int t) {
    const int c = min(max(t, 0), 4);
    return (uint32_t)(0xffffffffull << (8 * c));
}
__device__ __forceinline__ void head_row(const Keys& k, const uint32_t (&v)[4], int x, uint32_t sa, uint32_t (&A)[4],
                                         uint32_t& cs) {
    const int b0 = (int)sa - 4 * x;  // chunk byte at which the frame starts
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t keep = keep_mask(b0 - 4 * j), init = keep & ~keep_mask(b0 - 4 * j + 4);
        const uint32_t d = v[j] & keep;
        A[j] = zrow(A[j], k, d ^ init);
        cs = sad16(d, cs);
    }
}
// The header slot: the chunks holding frame dwords [-xo, 28 - xo) (xo: frame dword 0's place in its
// chunk) are copied to the frame's slot as they stream.
__device__ __forceinline__ void capture(uint32_t slot, int x, int xo, const uint32_t (&v)[4]) {
    const int c = x + xo;  // a multiple of 4
    if (c >= 0 && c < kSlotDw) *reinterpret_cast<u32x4*>(g_lds + slot + 4u * (uint32_t)c) = u32x4{v[0], v[1], v[2], v[3]};
}

// ---------------------------------------------------------------------------------------
// Frames of a tile. Lane L holds frame L & 15 of the tile (the 4 groups hold the same copy).
// The head piece's geometry is derived here once per tile, so a step's assignment is a few
// permutes and adds.
struct Frames {
    uint32_t slo, shi;    // frame offset
    uint32_t slen;        // streamed length (kOpsFcs: without the FCS; 0 past the batch end)
    uint32_t npc;         // pieces (0 = no rows: under 4 bytes past the first dword)
    uint32_t pelo, pehi;  // absolute end of the head piece: frames + Ed - 1536 (npc - 1)
    uint32_t meta;        // Dh (head piece dwords, 1..384) | dP << 9 | sa << 20
    uint32_t tail;        // the dword at Ed (bytes [Ed, E) are the frame's tail; kOpsFcs: also FCS bytes)
    uint32_t tail2;       // kOpsFcs: the dword after it
    __device__ __forceinline__ uint64_t S() const { return ((uint64_t)shi << 32) | slo; }
};
// dP: where the head piece's grid (its 1536 B before pe) enters the memory page that holds the
// frame's first byte, counted from the grid start (0: the grid lies in that page). Chunks before
// dP load from the page start instead (realigned): reading before a frame never leaves the page of
// its first byte. (Rows end at Ed, never past the frame.)
__device__ __forceinline__ uint32_t meta_dh(uint32_t m) { return m & 511u; }
__device__ __forceinline__ uint32_t meta_dp(uint32_t m) { return (m >> 9) & 2047u; }
__device__ __forceinline__ uint32_t meta_sa(uint32_t m) { return (m >> 20) & 3u; }

// Raw descriptors of a tile: plain loads, issued an assign call ahead of their use (a loop
// iteration later, so hipcc cannot sink them; its counted wait lets the row ring run on).
__device__ __forceinline__ void load_raw(uint32_t tile, uint32_t fl, uint32_t n, const uint64_t* __restrict__ offsets,
                                         const uint32_t* __restrict__ lengths, uint64_t& S, uint32_t& L) {
    const uint32_t fi = tile * 16u + fl;
    const uint32_t fc = fi < n ? fi : n - 1u;
    S = offsets[fc];
    L = lengths[fc];
}

template <uint32_t kOps>
__device__ __forceinline__ Frames derive(uint64_t S, uint32_t L, bool valid, const uint8_t* __restrict__ frames) {
    Frames f;
    f.slo = (uint32_t)S;
    f.shi = (uint32_t)(S >> 32);
    uint32_t slen = valid ? L : 0u;
    if (kOps == kOpsFcs) slen = slen >= 4u ? slen - 4u : 0u;
    f.slen = slen;
    const uint64_t E = S + slen, Ed = E & ~3ull, F4 = S & ~3ull;
    f.npc = 0u;
    f.meta = 0u;
    const uint64_t base = reinterpret_cast<uint64_t>(frames);
    if (slen >= 4u && Ed >= S + 4u) {
        const uint32_t D = (uint32_t)((Ed - F4) >> 2);
        const uint32_t npc = (((D + 63u) >> 6) + kPR - 1u) / kPR;
        const uint32_t Dh = D - 384u * (npc - 1u);
        const uint64_t pe = base + Ed - (uint64_t)kPieceBytes * (npc - 1u);
        const uint64_t page = (base + S) & ~4095ull, g0 = pe - kPieceBytes;
        const uint32_t dP = page > g0 ? (uint32_t)(page - g0) : 0u;
        f.npc = npc;
        f.pelo = (uint32_t)pe;
        f.pehi = (uint32_t)(pe >> 32);
        f.meta = Dh | (dP << 9) | (((uint32_t)S & 3u) << 20);
    }
    // the tail dword and (FCS) the one after it: dword-aligned dwords that hold a byte of the
    // frame (or of its FCS), so they never leave the frame's memory pages
    const uint32_t t = (uint32_t)(E - Ed);
    f.tail = 0u;
    f.tail2 = 0u;
    const uint32_t* tp = reinterpret_cast<const uint32_t*>(frames + Ed);
    const bool fcs = kOps == kOpsFcs && valid && L >= 4u;
    if (f.npc != 0u && (t > 0u || fcs)) f.tail = tp[0];
    if (f.npc != 0u && fcs && t > 0u) f.tail2 = tp[1];
    return f;
}

// ---------------------------------------------------------------------------------------
// Steps.
struct Step {
    uint64_t base;  // address of this lane's chunk at position 0 (piece end - 1536 + 16 gl)
    int rel0;       // frame dword (relative to F4) of that chunk's dword 0
    uint32_t info;  // frame (0..15) | active << 4 | sa << 5 | xo << 7 | dP << 9
    __device__ __forceinline__ uint32_t f() const { return info & 15u; }
    __device__ __forceinline__ bool active() const { return (info >> 4) & 1u; }
    __device__ __forceinline__ uint32_t sa() const { return (info >> 5) & 3u; }
    __device__ __forceinline__ int xo() const { return (int)((info >> 7) & 3u); }
    __device__ __forceinline__ uint32_t dP() const { return info >> 9; }
};
// wave-uniform step parameters
struct StepU {
    int kind;         // 1 head pieces, 0 other pieces, -1 none (the wave is done)
    int start;        // first consumed position
    int mask_until;   // positions <= this take the head-row path
    int cap_until;    // positions <= this may hold header-slot chunks
    int clamp_until;  // rare: loads at positions <= this are clamped into the frame's page (realigned)
    int last;         // the last step of its tile: the tile is finished after it
};

// The row loads of one step (unconditional: one load per position, so the ring's wait counts are static).
__device__ __forceinline__ u32x4 load_pos(const Step& s, const StepU& su, int u, uint32_t gl) {
    uint64_t a = s.base + 256u * (uint32_t)u;
    if (u <= su.clamp_until) {  // rare: the head grid starts in the page before the frame's first byte
        const uint64_t lo = s.base - 16u * gl + s.dP();
        a = a < lo ? lo : a;
    }
    return *reinterpret_cast<gu32x4*>(a);
}
// A clamped chunk realigned to where it belongs (rare path): sh dwords of shift, zeros before.
__device__ __forceinline__ void realign(uint32_t (&v)[4], int sh) {
    const uint32_t u0 = v[0], u1 = v[1], u2 = v[2], u3 = v[3];
    v[0] = sh == 0 ? u0 : 0u;
    v[1] = sh == 0 ? u1 : sh == 1 ? u0 : 0u;
    v[2] = sh == 0 ? u2 : sh == 1 ? u1 : sh == 2 ? u0 : 0u;
    v[3] = sh == 0 ? u3 : sh == 1 ? u2 : sh == 2 ? u1 : sh == 3 ? u0 : 0u;
}

// ---------------------------------------------------------------------------------------
// Parse and finish (one lane per frame).

// A frame's header slot: frame dword x (relative to F4) is slot dword x + xo while x < D (the
// stream dwords); dword D is the tail dword, later ones are past the frame.
struct Slot {
    uint32_t sb;
    int xo, D;
    uint32_t tail, sa;
    __device__ __forceinline__ uint32_t dw(int x) const {
        if (x >= D) return x == D ? tail : 0u;
        return lds32(sb + 4u * (uint32_t)(x + xo));
    }
    // frame bytes [4j, 4j + 4) as a little-endian dword
    __device__ __forceinline__ uint32_t fdw(int j) const { return __builtin_amdgcn_alignbyte(dw(j + 1), dw(j), sa); }
};

// bytes of dword x (frame bytes [4x - sa, 4x + 4 - sa)) that lie in [a0, a1), a0/a1 counted from F4
__device__ __forceinline__ uint32_t range_mask(int x, int a0, int a1) {
    const int lo = min(max(a0 - 4 * x, 0), 4), hi = min(max(a1 - 4 * x, 0), 4);
    const uint32_t m = (0xffffffffu >> (32 - 8 * (hi - lo))) << (8 * lo);
    return hi > lo ? m : 0u;
}
// exact sum of frame bytes [p0, p1) from global memory (rare paths; at most 64 KB)
__device__ __forceinline__ uint32_t global_sum(const uint32_t* fb, uint32_t sa, int p0, int p1) {
    uint32_t s = 0;
    if (p1 <= p0) return s;
    const int a0 = (int)sa + p0, a1 = (int)sa + p1;
    for (int k = a0 >> 2; k <= (a1 - 1) >> 2; ++k) s = sad16(fb[k] & range_mask(k, a0, a1), s);
    return s;
}

struct Parsed {
    uint32_t verdict;   // final unless `compute`
    uint32_t ip_csum;
    uint32_t stored;    // stored L4 checksum (BE)
    int compute;        // the L4 checksum is computed
    int parity;         // absolute parity of the L4 start (1 = odd)
    int direct;         // l4sum is the L4 segment's own sum (huge Ethernet padding)
    uint32_t off, end;  // L4 segment [off, end) (frame-relative)
    uint32_t l4sum;
    int64_t corr;       // every checksum correction (16-bit-half domain)
    int64_t corr_fixed; // the pseudo-header and excluded-word part of corr
    uint32_t aux;       // kOpsTx: stored IPv4 checksum | L4 checksum field offset << 16
};

// Header parse of one frame. The gates follow stacks/portstack.go:163-308 exactly
// (oracle/framesum_oracle.c restates them line by line; the parity tests compare the two).
template <uint32_t kOps>
__device__ __forceinline__ Parsed parse_frame(const Slot& V, uint32_t len, uint32_t mtu, const uint32_t* fb) {
    Parsed r = {V_OK, 0u, 0u, 0, 0, 0, 0u, 0u, 0u, 0, 0, 0u};
    if (len < 34u) { r.verdict = V_SMOL; return r; }                          // portstack.go:167-168
    if (mtu != 0 && len > mtu) { r.verdict = V_MTU; return r; }              // :169-172
    uint32_t bs[9];                                                           // bswap32(frame dword j), j = 3..8
#pragma unroll
    for (int j = 3; j < 9; ++j) bs[j] = __builtin_bswap32(V.fdw(j));
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
    const int q = (int)((off - 2u) >> 2);
    uint32_t lb[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) lb[i] = __builtin_bswap32(V.fdw(q + i));
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
    r.parity = (int)((V.sa + off) & 1u);
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
    // the Ethernet + IP header bytes [0, off): big-endian words (off = 4q + 2: frame dwords 0 .. q-1
    // and the high half of dword q), moved into the 16-bit-half domain as the words above
    {
        uint32_t s = 0;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const uint32_t d = __builtin_bswap32(V.fdw(j));
            s += (d >> 16) + (d & 0xffffu);
        }
#pragma unroll
        for (int j = 3; j < 9; ++j) s += j < q ? (bs[j] >> 16) + (bs[j] & 0xffffu) : 0u;
        for (int j = 9; j < q; ++j) {  // IP options past dword 8 (rare)
            const uint32_t d = __builtin_bswap32(V.fdw(j));
            s += (d >> 16) + (d & 0xffffu);
        }
        s += lb[0] >> 16;
        s = fold16(fold16(s));
        t -= (int64_t)(odd ? s : bswap16(s));
    }
    if (end < len) {  // Ethernet padding [end, len)
        const int a0 = (int)(V.sa + end), a1 = (int)(V.sa + len);
        if (a1 <= 4 * (kSlotDw - V.xo)) {
            uint32_t s = 0;
            for (int x = a0 >> 2; x <= (a1 - 1) >> 2; ++x) s = sad16(V.dw(x) & range_mask(x, a0, a1), s);
            t -= (int64_t)s;
        } else if (len - end <= end - off) {
            t -= (int64_t)global_sum(fb, V.sa, (int)end, (int)len);
        } else {  // a padding larger than the segment: sum the segment itself (at most 64 KB)
            r.direct = 1;
            r.l4sum = global_sum(fb, V.sa, (int)off, (int)end);
        }
    }
    r.corr = t;
    return r;
}

// Final L4 checksum + verdict once the streamed sum is known.
__device__ __forceinline__ uint32_t finish_l4(const Parsed& P, uint32_t main_sum, uint32_t& verdict) {
    // Every term is congruent (mod 65535) to its exact native contribution, and the true total is
    // > 0 (the pseudo-header protocol word is 6 or 17), so adding 65535 * 2^20 keeps t positive and
    // the fold lands on the same one's-complement value (the Sum16 edge 0x0000 / 0xFFFF included).
    int64_t t = P.direct ? (int64_t)P.l4sum + P.corr_fixed : (int64_t)main_sum + P.corr;
    t += 65535LL * (1LL << 20);
    uint64_t x = (uint64_t)t;
    x = (x & 0xffffffffu) + (x >> 32);  // < 2^33
    x = (x & 0xffffu) + (x >> 16);      // < 2^18
    x = (x & 0xffffu) + (x >> 16);      // < 2^16 + 4
    x = (x & 0xffffu) + (x >> 16);      // <= 0xFFFF
    uint32_t l4 = (~(uint32_t)x) & 0xffffu;
    if (!P.parity) l4 = bswap16(l4);
    verdict = (l4 == P.stored) ? V_OK : V_CSUM;
    return l4;
}

// A byte store into a frame (TX; hipcc merges neighbours into wider stores).
__device__ __forceinline__ void st8(uint8_t* p, uint32_t v) { *p = (uint8_t)v; }

// Finish a frame with no stream dwords (under 4 bytes past its first dword): bytewise from memory.
template <uint32_t kOps>
__device__ __forceinline__ void finish_tiny(const Frames& F, uint32_t fi, const uint8_t* __restrict__ frames,
                                            uint8_t* __restrict__ wframes, const uint32_t* __restrict__ lengths,
                                            uint2* __restrict__ out, uint8_t* __restrict__ status, uint32_t tx) {
    const uint64_t S = F.S();
    const uint32_t slen = F.slen;
    uint32_t c = 0xffffffffu;
    const uint8_t* fp = frames + S;
    for (uint32_t p = 0; p < slen; ++p) c = tbyte((c ^ fp[p]) & 0xffu) ^ (c >> 8);
    const uint32_t crcv = ~c;
    uint32_t verdict = V_SMOL;  // slen < 34 (portstack.go:167-168)
    if (kOps == kOpsTx && (tx & kTxAppend)) {
        uint8_t* wf = wframes + S;
        st8(wf + slen, crcv);
        st8(wf + slen + 1, crcv >> 8);
        st8(wf + slen + 2, crcv >> 16);
        st8(wf + slen + 3, crcv >> 24);
    }
    if (kOps == kOpsFcs) {
        // slen 0 covers wire frames of 0..4 bytes: only those of 4 carry an FCS
        const bool present = slen > 0u || lengths[fi] >= 4u;
        uint32_t fcs = 0u;
        if (present)
            fcs = (uint32_t)fp[slen] | ((uint32_t)fp[slen + 1] << 8) | ((uint32_t)fp[slen + 2] << 16) |
                  ((uint32_t)fp[slen + 3] << 24);
        if (!present || fcs != crcv) verdict = V_FCS;
    }
    out[fi] = make_uint2(crcv, 0u);
    if (status) status[fi] = (uint8_t)verdict;
}

// Finish one frame (frame lane): CRC-32 from the frame's pending register, checksum + verdict from
// its sum and its header slot, the operation's writes, the stores.
template <uint32_t kOps>
__device__ __forceinline__ void finish_frame(const Frames& F, uint32_t fi, uint32_t wb, uint32_t i, uint32_t mtu,
                                             const uint8_t* __restrict__ frames, uint8_t* __restrict__ wframes,
                                             const uint32_t* __restrict__ lengths, uint2* __restrict__ out,
                                             uint8_t* __restrict__ status, uint32_t tx) {
    const uint64_t S = F.S();
    const uint32_t slen = F.slen, sa = (uint32_t)S & 3u;
    const uint64_t E = S + slen, Ed = E & ~3ull, F4 = S & ~3ull;
    const uint32_t t = (uint32_t)(E - Ed);
    const uint32_t* fb = reinterpret_cast<const uint32_t*>(frames + F4);
    if (F.npc == 0u) {
        finish_tiny<kOps>(F, fi, frames, wframes, lengths, out, status, tx);
        return;
    }
    uint32_t crcv, fcs = 0u, cs = 0u;
    Parsed P;
    {
        const uint32_t npc = F.npc;
        Slot V;
        V.sb = wb + i * kSlotBytes;
        V.xo = (int)((0u - meta_dh(F.meta)) & 3u);
        V.D = (int)((Ed - F4) >> 2);
        V.tail = F.tail;
        V.sa = sa;
        // the pending register and its tail bytes
        uint32_t reg = zt(lds32(wb + kWC + 4u * i), pcst(kT4));
        if (npc > 1u && (uint32_t)V.D - 384u * (npc - 1u) == 1u && sa != 0u) {
            // frame dword 1 opens piece 1 (a one-dword head piece): its part of the CRC init (the
            // frame bytes [4 - sa, 4) XOR 0xFF) was not applied by the rows; it is linear, added here
            reg ^= zshift(zt(~(0xffffffffu << (8u * sa)), pcst(kT4)), 4u * (uint32_t)V.D - 8u);
        }
        for (uint32_t b = 0; b < t; ++b) reg = (reg >> 8) ^ tbyte((reg ^ (F.tail >> (8u * b))) & 0xffu);
        crcv = ~reg;
        cs = lds32(wb + kWS + 4u * i);
        if (t) cs = sad16(F.tail & ((1u << (8u * t)) - 1u), cs);
        if (kOps == kOpsFcs) fcs = __builtin_amdgcn_alignbyte(F.tail2, F.tail, t);
        P = parse_frame<kOps>(V, slen, mtu, fb);
    }
    uint32_t verdict = P.verdict, l4 = 0u;
    if (P.compute) l4 = finish_l4(P, cs, verdict);
    if constexpr (kOps == kOpsTx) {
        uint8_t* wf = wframes + S;
        if ((tx & kTxFill) && P.compute) {
            // write the IPv4 checksum at [24, 26) and the L4 checksum at its field, big-endian; the
            // CRC of the written frame differs from the streamed one by the CRC (zero init) of the two
            // 16-bit XOR deltas: Z_(len-p2)( Z_(p2-24)(d_ip) ^ d_l4 ), d as little-endian bytes
            const uint32_t ipc = P.ip_csum, old_ip = P.aux & 0xffffu, p2 = P.aux >> 16;
            const uint32_t d = zshift(bswap16(old_ip ^ ipc), p2 - 24u) ^ bswap16(P.stored ^ l4);
            crcv ^= zshift(d, slen - p2);
            st8(wf + 24, ipc >> 8);
            st8(wf + 25, ipc);
            st8(wf + p2, l4 >> 8);
            st8(wf + p2 + 1, l4);
            verdict = V_OK;  // the written field now holds the computed checksum
        }
        if (tx & kTxAppend) {
            st8(wf + slen, crcv);
            st8(wf + slen + 1, crcv >> 8);
            st8(wf + slen + 2, crcv >> 16);
            st8(wf + slen + 3, crcv >> 24);
        }
    }
    if (kOps == kOpsFcs) {
        // slen 0 covers wire frames of 0..4 bytes: only those of 4 carry an FCS
        const bool present = slen > 0u || lengths[fi] >= 4u;
        if (!present || fcs != crcv) verdict = V_FCS;
    }
    out[fi] = make_uint2(crcv, P.ip_csum | (l4 << 16));
    if (status) status[fi] = (uint8_t)verdict;
}

// ---------------------------------------------------------------------------------------
// The kernel.
//
// Per wave: an assigner that runs one step ahead of the consumer. The assigner walks its tile's
// head steps then its rounds, reading the tile's frames from T1; when they are exhausted it moves
// T1 on to the wave's next tile. The consumer finishes its tile (T0, a copy of T1 taken when the
// consumer reached that tile) after the tile's last step.
template <uint32_t kOps>
__global__ void __launch_bounds__(kThreads, 4)
rx_kernel(const uint8_t* __restrict__ frames, const uint64_t* __restrict__ offsets, const uint32_t* __restrict__ lengths,
          uint32_t n, uint32_t mtu, const FsTablesRx* __restrict__ tabs, uint2* __restrict__ out,
          uint8_t* __restrict__ status, uint8_t* __restrict__ wframes, uint32_t tx) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t grp = lane >> 4, gl = lane & 15u;
    // wave-major tiles: a workgroup's waves read tiles spread over the batch, neighbouring
    // workgroups (different XCDs) neighbouring tiles
    const uint32_t gwave = wave * gridDim.x + blockIdx.x;
    const uint32_t nwaves = gridDim.x * kWaves;
    const uint32_t ntiles = (n + 15u) >> 4;
    const uint32_t wb = kLdsWaves + wave * kWaveBytes;

    uint64_t rS = 0;
    uint32_t rL = 0;
    if (gwave < ntiles) load_raw(gwave, gl, n, offsets, lengths, rS, rL);
    build_tables(tabs, wave, lane);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (gwave >= ntiles) return;

    const Keys keys = lane_keys(lane);
    const uint32_t cq = pcst((gl & 3u) == 0u ? kT48 : (gl & 3u) == 1u ? kT32 : kT16);
    const uint32_t cr = pcst((gl >> 2) == 0u ? kT192 : (gl >> 2) == 1u ? kT128 : kT64);

    // ---- the assigner's state (wave-uniform)
    uint32_t a_tile = 0;             // its tile
    uint32_t a_next = gwave;         // the tile whose raw descriptors are in (rS, rL)
    int a_done = 0, a_pend = 0;      // a_pend: its tile's last step is out, advance at the next call
    int a_phase = 0, a_k = 0, a_p = 0, a_nh = 0, a_cnt = 0, a_maxnpc = 0;
    Frames T0, T1;                   // the consumer's tile, the assigner's tile
    uint32_t c_tile = 0;             // the consumer's tile index

    // The head order of T1's tile (frames with rows, by head rows descending, then index) into the
    // wave's order bytes; returns the number of frames with rows.
    auto schedule = [&]() __attribute__((always_inline)) -> int {
        const uint32_t npc = T1.npc, dh = meta_dh(T1.meta);
        const uint32_t h = (dh + 63u) >> 6;
        const uint32_t mR = (uint32_t)__ballot(npc > 0u) & 0xffffu;
        a_nh = __builtin_popcount(mR);
        // the pieces of the longest frame: a max over the row of 16 frames
        uint32_t m = npc;
        m = max(m, dpp<0x121>(m));
        m = max(m, dpp<0x122>(m));
        m = max(m, dpp<0x124>(m));
        m = max(m, dpp<0x128>(m));
        a_maxnpc = (int)__builtin_amdgcn_readfirstlane(m);
        uint32_t rank;
        const uint32_t h0 = mR ? __builtin_amdgcn_readlane(h, __builtin_ctz(mR)) : 0u;
        if (((uint32_t)__ballot(npc > 0u && h == h0) & 0xffffu) == mR) {
            rank = __builtin_amdgcn_mbcnt_lo(mR, 0u);  // one head length (a uniform batch): index order
        } else {
            rank = 0u;
            for (uint32_t mm = mR; mm; mm &= mm - 1u) {
                const uint32_t j = __builtin_ctz(mm);
                const uint32_t hj = __builtin_amdgcn_readlane(h, j);
                rank += (hj > h || (hj == h && j < gl)) ? 1u : 0u;
            }
        }
        if (lane < 16u && npc > 0u) g_lds[wb + kWO + rank] = (char)lane;
        a_phase = 0;
        a_k = 0;
        return a_nh;
    };
    // Move the assigner to the wave's next tile that has steps (into T1); tiles whose frames are all
    // under the stream minimum are finished right here. Returns false when the wave has no tile
    // left. Called one assign call after the previous tile's last step was produced: by then the
    // consumer has copied T1 (a tile of one step is consumed right after the step before it).
    auto advance = [&]() __attribute__((always_inline)) -> bool {
        FS_MARK("advance");
        if (a_next >= ntiles) return false;
        a_tile = a_next;
        T1 = derive<kOps>(rS, rL, a_tile * 16u + gl < n, frames);  // (rS, rL): loaded a block ago
        a_next = a_tile + nwaves;
        if (schedule() > 0) return true;
        // rare: tiles with no rows at all (frames under 4 bytes past their first dword)
        for (;;) {
            if (lane < 16u && a_tile * 16u + lane < n)
                finish_tiny<kOps>(T1, a_tile * 16u + lane, frames, wframes, lengths, out, status, tx);
            if (a_next >= ntiles) return false;
            a_tile = a_next;
            uint64_t S;
            uint32_t L;
            load_raw(a_tile, gl, n, offsets, lengths, S, L);
            T1 = derive<kOps>(S, L, a_tile * 16u + gl < n, frames);
            a_next = a_tile + nwaves;
            if (schedule() > 0) return true;
        }
    };

    // Produce the assigner's next step (its params for this lane's group) and advance it.
    auto assign = [&](Step& s, StepU& su, const Step& prev, const StepU& prevu) __attribute__((always_inline)) {
        if (a_pend) {
            a_pend = 0;
            if (!advance()) a_done = 1;
        }
        if (a_done) {
            s = prev;
            su = prevu;
            su.kind = -1;
            su.last = 0;
            return;
        }
        FS_MARK("produce");
        const int k = a_k;
        int p = 0, count;
        if (a_phase == 0) {
            count = a_nh;
        } else {
            p = a_p;
            if (a_k == 0) {  // a round starts: the frames with a piece p, in index order
                const uint32_t mP = (uint32_t)__ballot(T1.npc > (uint32_t)p) & 0xffffu;
                a_cnt = __builtin_popcount(mP);
                const uint32_t pos = __builtin_amdgcn_mbcnt_lo(mP, 0u);
                if (lane < 16u && T1.npc > (uint32_t)p) g_lds[wb + kWO + pos] = (char)lane;
            }
            count = a_cnt;
        }
        const int sidx = 4 * k + (int)grp;
        const bool act = sidx < count;
        const uint32_t f = (uint32_t)(uint8_t)g_lds[wb + kWO + (act ? sidx : 4 * k)];
        const int src = (int)((grp * 16u + f) << 2);
        const uint32_t pelo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)T1.pelo);
        const uint32_t pehi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)T1.pehi);
        const uint32_t meta = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)T1.meta);
        const uint32_t dh = meta_dh(meta), sa = meta_sa(meta);
        // chunk at position 0: piece end (head + 1536 p) - 1536 + 16 gl
        const int off0 = 1536 * (p - 1) + 16 * (int)gl;
        s.base = (((uint64_t)pehi << 32) | pelo) + (uint64_t)(int64_t)off0;
        s.rel0 = (int)dh - 384 + 384 * p + 4 * (int)gl;
        s.info = f | (act ? 16u : 0u) | (sa << 5) | (((0u - dh) & 3u) << 7) | (p == 0 ? (meta_dp(meta) << 9) : 0u);
        int last;
        su.start = 0;
        su.mask_until = -1;
        su.cap_until = -1;
        su.clamp_until = -1;
        if (a_phase == 0) {
            // per group: its head rows, the row of frame dword 1 (0: S is dword aligned; the
            // init and the masks end there), the row of the last header-slot dword, the clamp
            const int glast = min(3, a_nh - 1 - 4 * k);
            int hmax = 0, mrow = -1, crow = -1, clamp = -1;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                if (g > glast) break;
                const uint32_t mg = __builtin_amdgcn_readlane(meta, 16 * g);
                const int dg = (int)meta_dh(mg);
                const int xm = meta_sa(mg) ? 1 : 0;
                const int xo = (int)((0u - (uint32_t)dg) & 3u);
                hmax = max(hmax, (dg + 63) >> 6);
                mrow = max(mrow, (xm + 384 - dg) >> 6);
                crow = max(crow, (kSlotDw - 1 - xo + 384 - dg) >> 6);
                const int dp = (int)meta_dp(mg);
                if (dp > 0) clamp = max(clamp, (dp - 1) >> 8);
            }
            su.kind = 1;
            su.start = kPR - hmax;
            su.mask_until = min(kPR - 1, mrow);
            su.cap_until = min(kPR - 1, crow);
            su.clamp_until = clamp;
            ++a_k;
            if (4 * a_k >= a_nh) {  // the head steps are done
                a_phase = 1;
                a_p = 1;
                a_k = 0;
            }
            last = (a_phase == 1 && a_maxnpc <= 1) ? 1 : 0;
        } else {
            su.kind = 0;
            // round 1: header-slot chunks past a short head piece (in piece 1's first row)
            su.cap_until = p == 1 ? 0 : -1;
            ++a_k;
            last = 0;
            if (4 * a_k >= a_cnt) {
                a_k = 0;
                ++a_p;
                if (a_p >= a_maxnpc) last = 1;
            }
        }
        su.last = last;
        a_pend = last;
    };

    // ---- prologue: the first tile, the first step's rows
    Step cur, nxt;
    StepU cu, nu;
    u32x4 ring[kPR];
    if (!advance()) return;
    T0 = T1;
    c_tile = a_tile;
    // the descriptors of the assigner's next tile, reloaded at one place per block (unconditional,
    // so the row ring's waits are static and no merge copies a pending register)
    load_raw(min(a_next, ntiles - 1u), gl, n, offsets, lengths, rS, rL);
    {
        Step z{};
        StepU zu{};
        assign(nxt, nu, z, zu);
    }
#pragma unroll
    for (int u = 0; u < kPR; ++u) ring[u] = load_pos(nxt, nu, u, gl);
    cur = nxt;
    cu = nu;
    assign(nxt, nu, cur, cu);

    while (cu.kind >= 0) {
        uint32_t A[4] = {0u, 0u, 0u, 0u};
        uint32_t cs = 0u;
        const uint32_t slot = wb + cur.f() * kSlotBytes;
#pragma unroll
        for (int u = 0; u < kPR; ++u) {
            if (u >= cu.start) {
                uint32_t v[4] = {ring[u].x, ring[u].y, ring[u].z, ring[u].w};
                const int x = cur.rel0 + 64 * u;
                if (!(FS_RX_DIAG & 4) && u <= cu.clamp_until) {  // rare: chunks loaded from the frame's page start
                    FS_MARK("realign");
                    realign(v, min(max(((int)cur.dP() - 256 * u - 16 * (int)gl) >> 2, 0), 4));
                }
                if (!(FS_RX_DIAG & 4) && u <= cu.cap_until) capture(slot, x, cur.xo(), v);
                if (!(FS_RX_DIAG & 4) && u <= cu.mask_until) {
                    FS_MARK("head_row");
                    head_row(keys, v, x, cur.sa(), A, cs);
                } else {
                    FS_MARK("lean_row");
                    lean_row(keys, ring[u], A, cs);
                }
            }
            FS_MARK("load");
            ring[u] = load_pos(nxt, nu, u, gl);
            FS_MARK("pos_end");
        }
        // ---- combine the group's piece: W (its pending CRC register) and its sum
        FS_MARK("combine");
        if (FS_RX_DIAG & 2) {
            if (gl == 0u && cur.active()) sts32(wb + kWC + 4u * cur.f(), A[0] ^ A[1] ^ A[2] ^ A[3] ^ cs);
        } else {
            const uint32_t c4 = pcst(kT4);
            uint32_t U = zt(A[0], c4) ^ A[1];
            U = zt(U, c4) ^ A[2];
            U = zt(U, c4) ^ A[3];
            uint32_t V = zt(U, cq);
            V = (gl & 3u) == 3u ? U : V;
            V ^= dpp<kQuadXor1>(V);
            V ^= dpp<kQuadXor2>(V);
            uint32_t W = zt(V, cr);
            W = (gl >> 2) == 3u ? V : W;
            W ^= dpp<kRowRor4>(W);
            W ^= dpp<kRowRor8>(W);
            cs = fold16(cs);
            cs += dpp<kQuadXor1>(cs);
            cs += dpp<kQuadXor2>(cs);
            cs += dpp<kRowRor4>(cs);
            cs += dpp<kRowRor8>(cs);
            if (gl == 0u && cur.active()) {
                const uint32_t ca = wb + kWC + 4u * cur.f(), sa = wb + kWS + 4u * cur.f();
                if (cu.kind == 1) {
                    sts32(ca, W);
                    sts32(sa, cs);
                } else {
                    sts32(ca, zt(lds32(ca), pcst(kT1536)) ^ W);
                    sts32(sa, fold16(lds32(sa) + cs));
                }
            }
        }
        FS_MARK("after_combine");
        if (cu.last) {
            FS_MARK("finish");
            // ---- the consumer's tile is complete: parse and finish its frames
            if (FS_RX_DIAG & 1) {
                if (lane < 16u && c_tile * 16u + lane < n)
                    out[c_tile * 16u + lane] = make_uint2(lds32(wb + kWC + 4u * lane), T0.meta);
            } else if (lane < 16u && c_tile * 16u + lane < n)
                finish_frame<kOps>(T0, c_tile * 16u + lane, wb, lane, mtu, frames, wframes, lengths, out, status, tx);
            T0 = T1;
            c_tile = a_tile;
        }
        FS_MARK("assign");
        cur = nxt;
        cu = nu;
        assign(nxt, nu, cur, cu);
        load_raw(min(a_next, ntiles - 1u), gl, n, offsets, lengths, rS, rL);
        FS_MARK("loop_end");
    }
}

}  // namespace

hipError_t launch_rx(const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths, uint32_t n, uint32_t mtu,
                     const FsTablesRx* tables, void* out, uint8_t* status, hipStream_t stream, int num_cus,
                     int grid_per_cu, int op, uint8_t* wframes, uint32_t tx) {
    if (n == 0) return hipSuccess;
    const uint32_t cus = (uint32_t)(num_cus > 0 ? num_cus : 256);
    const uint32_t per = (uint32_t)(grid_per_cu == 2 ? 2 : 1);
    const uint32_t tiles = (n + 15u) / 16u;
    uint32_t blocks = (tiles + kWaves - 1u) / kWaves;
    if (blocks > per * cus) blocks = per * cus;
    uint2* o = reinterpret_cast<uint2*>(out);
#define FS_LAUNCH(OPS)                                                                                      \
    hipLaunchKernelGGL((rx_kernel<OPS>), dim3(blocks), dim3(kThreads), 0, stream, frames, offsets, lengths, n, mtu, \
                       tables, o, status, wframes, tx)
    switch (op) {
    case 1: FS_LAUNCH(kOpsTx); break;
    case 2: FS_LAUNCH(kOpsFcs); break;
    default: FS_LAUNCH(kOpsDigest); break;
    }
#undef FS_LAUNCH
    return hipGetLastError();
}

}  // namespace framesum
