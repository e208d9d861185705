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
//     [4l, 4l+4) of every row with one global_load_dwordx4 (16 B/lane).
//   * CRC: each lane keeps 4 independent dword STREAMS; a stream's successive
//     dwords are 64 B apart, so its Horner step is  A <- Z64(A) ^ w  with Z64 a
//     fixed GF(2) linear map evaluated by 4 byte-table lookups in LDS. After the
//     last row the 16 streams of a frame are combined (intra-lane Z4 Horner,
//     then a 2-level lane tree with Z32/Z16 over DPP quad permutes).
//     Leading zero rows do not change a zero-init CRC, and the <=3 zero bytes
//     the dword rounding appends are removed by an exact one-byte inverse step.
//   * one's-complement sum: the same registers are summed as dwords into a
//     64-bit accumulator (exact integer, so RecvEth's Sum16 fold is reproduced
//     bit for bit, incl. the 0x0000 / 0xFFFF edge); header bytes, the
//     pseudo-header and the excluded words are applied by the frame's lane.
//   * LDS tables: the hot Z64 (and Z4) tables are stored as 8 copies per table
//     in a [entry][table*8+copy] layout, 256 B per entry. Lane L = c + 8h of a
//     32-lane bank group reads table (k+h)&3 in its k-th lookup, so the 32
//     lanes hit 32 distinct banks: conflict-free ds_read_b32 for any data.
//     One v_perm_b32 forms the LDS address (entry byte | per-lane slot byte).
#include <hip/hip_runtime.h>
#include <stdint.h>

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
constexpr int kPrefetch = 4;
constexpr int kHdrChunks = 7;               // 7 x 16 B staged header bytes per frame
constexpr int kHdrBytes = kHdrChunks * 16;  // 112

// LDS map (bytes).
constexpr uint32_t kLdsZ32 = 65536;
constexpr uint32_t kLdsZ16 = kLdsZ32 + 4096;
constexpr uint32_t kLdsT1 = kLdsZ16 + 4096;
constexpr uint32_t kLdsInv = kLdsT1 + 1024;
constexpr uint32_t kLdsHdr = kLdsInv + 256;
constexpr uint32_t kLdsBytes = kLdsHdr + kWavesPerBlock * kFramesPerTile * kHdrBytes;
static_assert(kLdsHdr % 16 == 0, "header slots must be 16-B aligned");
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");

constexpr uint32_t kZ4Off = 128;  // Z4 copies sit in slots 32..63 of each region-A entry row

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
__device__ __forceinline__ uint32_t lds8(const char* lds, uint32_t byte_addr) {
    return *reinterpret_cast<const uint8_t*>(lds + byte_addr);
}

struct LaneKeys {
    uint32_t cvec;     // byte j = slot byte of table j for this lane (32*j + 4*c)
    uint32_t sel[4];   // v_perm selectors of the 4 lookups
};

// Z operator from replicated region A (off = 0: Z64, off = 128: Z4). Conflict-free.
__device__ __forceinline__ uint32_t zrep(const char* lds, uint32_t a, const LaneKeys& k, uint32_t off) {
    uint32_t t0 = lds32(lds, off + __builtin_amdgcn_perm(a, k.cvec, k.sel[0]));
    uint32_t t1 = lds32(lds, off + __builtin_amdgcn_perm(a, k.cvec, k.sel[1]));
    uint32_t t2 = lds32(lds, off + __builtin_amdgcn_perm(a, k.cvec, k.sel[2]));
    uint32_t t3 = lds32(lds, off + __builtin_amdgcn_perm(a, k.cvec, k.sel[3]));
    return t0 ^ t1 ^ t2 ^ t3;
}

// Z operator from a plain [4][256] table (region B; used twice per frame).
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
// the prefetch ring keeps kPrefetch loads in flight); rows that start before
// the frame are clamped to `lo` (>= the buffer start) and fixed up / masked by
// the slow path.
__device__ __forceinline__ u32x4 load_chunk(const uint32_t* fb, int rel, int lo) {
    return *reinterpret_cast<const u32x4_a4*>(fb + max(rel, lo));
}

// Per-frame row-mask parameters, held by every lane of the frame's group.
struct RowMasks {
    int nd;              // frame dwords (incl. the partial last one); 0 = nothing to stream
    int in_lo, in_hi;    // dwords [in_lo, in_hi) lie fully inside the L4 checksum range
    int fast_lo, fast_hi;
    uint32_t head_mask, init0, init1, tail_mask;
};

__device__ __forceinline__ void process_row(const char* lds, const LaneKeys& keys, u32x4 v, int rel, bool fast,
                                            const RowMasks& m, int lo, uint32_t (&A)[4], uint64_t& cs) {
    if (fast) {
        A[0] = zrep(lds, A[0], keys, 0) ^ v.x;
        A[1] = zrep(lds, A[1], keys, 0) ^ v.y;
        A[2] = zrep(lds, A[2], keys, 0) ^ v.z;
        A[3] = zrep(lds, A[3], keys, 0) ^ v.w;
        cs += (uint64_t)v.x + v.y + (uint64_t)v.z + v.w;
    } else {
        const int sh = max(rel, lo) - rel;  // >0 only when the load was clamped at the buffer start
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
            const uint32_t d = v[j];
            uint32_t mk = 0xffffffffu, x = 0u;
            if (rj == 0) { mk &= m.head_mask; x ^= m.init0; }
            if (rj == 1) x ^= m.init1;
            if (rj == m.nd - 1) mk &= m.tail_mask;
            const uint32_t dc = (rj >= 0) ? ((d & mk) ^ x) : 0u;
            const uint32_t ds = ((uint32_t)(rj - m.in_lo) < (uint32_t)(m.in_hi - m.in_lo)) ? d : 0u;
            A[j] = zrep(lds, A[j], keys, 0) ^ dc;
            cs += ds;
        }
    }
}

// Header parse of one frame from its LDS staging slot (frame byte p at slot[sa + p]).
struct Parsed {
    uint32_t verdict;
    uint32_t ip_csum;
    uint32_t stored;     // stored L4 checksum word (BE value)
    int compute;         // 0 none, 1 L4 checksum computed
    int use_main;        // add the streamed inside-dword sum
    int in_lo, in_hi;
    int parity;          // absolute parity of the L4 start (1 = odd)
    int64_t corr;        // exact native-domain corrections
    int tail_nb;         // bytes of the partial dword at in_hi that belong to L4 (0 = none)
};

__device__ __forceinline__ uint32_t hb(const char* lds, uint32_t slot, uint32_t p) { return lds8(lds, slot + p); }
__device__ __forceinline__ uint32_t hbe16(const char* lds, uint32_t slot, uint32_t p) {
    return (hb(lds, slot, p) << 8) | hb(lds, slot, p + 1);
}

__device__ Parsed parse_frame(const char* lds, uint32_t slot /* byte addr of frame byte 0 */, uint32_t sa,
                              uint32_t len, uint32_t mtu) {
    Parsed r;
    r.verdict = V_OK;
    r.ip_csum = 0;
    r.stored = 0;
    r.compute = 0;
    r.use_main = 0;
    r.in_lo = 0;
    r.in_hi = 0;
    r.parity = 0;
    r.corr = 0;
    r.tail_nb = 0;
    if (len < 34) { r.verdict = V_SMOL; return r; }                       // portstack.go:167-168
    if (mtu != 0 && len > mtu) { r.verdict = V_MTU; return r; }           // :169-172
    {   // eth/headers.go:333-340 via Put (:289-301): version forced to 4, checksum zeroed, 20 bytes.
        uint32_t s = (((0x40u | (hb(lds, slot, 14) & 0xfu)) << 8) | hb(lds, slot, 15));
#pragma unroll
        for (uint32_t p = 16; p < 34; p += 2)
            if (p != 24) s += hbe16(lds, slot, p);
        s = (s & 0xffffu) + (s >> 16);
        s = (s & 0xffffu) + (s >> 16);
        r.ip_csum = (~s) & 0xffffu;
    }
    const uint32_t etype = hbe16(lds, slot, 12);
    if (etype != 0x0800u && etype != 0x0806u) { r.verdict = V_NOT_IPV4; return r; }  // :187-188
    if (etype == 0x0806u) { r.verdict = (len < 42) ? V_SMOL : V_ARP; return r; }     // :191-197
    const uint32_t vihl = hb(lds, slot, 14);
    const uint32_t ipoff = (vihl & 0xfu) * 4u;                            // uint8, <= 60
    const uint32_t off = 14u + ipoff;                                     // :201
    const uint32_t tl = hbe16(lds, slot, 16);
    const uint32_t end = (14u + tl) & 0xffffu;                            // :202 uint16 wrap
    if ((vihl >> 4) != 4u) { r.verdict = V_IPVER; return r; }             // :204
    if (ipoff < 20u) { r.verdict = V_IHL; return r; }                     // :206
    if (off > end || off > len || end > len) { r.verdict = V_BADLEN; return r; }  // :211
    if (mtu != 0 && end > mtu) { r.verdict = V_MTU; return r; }           // :213
    const uint32_t l4len = end - off;
    const uint32_t proto = hb(lds, slot, 23);
    uint32_t lenword, skip0;
    if (proto == 17u) {                                                   // :222-244
        if (l4len < 8u) { r.verdict = V_SHORT; return r; }
        const uint32_t sport = hbe16(lds, slot, off), dport = hbe16(lds, slot, off + 2);
        const uint32_t ulen = hbe16(lds, slot, off + 4);
        if (sport == 0 || dport == 0) { r.verdict = V_ZEROPORT; return r; }
        if (ulen < 8u) { r.verdict = V_UDPLEN; return r; }
        lenword = ulen;                                                   // headers.go:386-390
        skip0 = off + 6;
        r.stored = hbe16(lds, slot, off + 6);
    } else if (proto == 6u) {                                             // :283-308
        if (l4len < 20u) { r.verdict = V_SHORT; return r; }
        const uint32_t sport = hbe16(lds, slot, off), dport = hbe16(lds, slot, off + 2);
        const uint32_t toff = (hbe16(lds, slot, off + 12) >> 12) * 4u;    // headers.go:477-485
        if (sport == 0 || dport == 0) { r.verdict = V_ZEROPORT; return r; }
        if (toff < 20u || toff > l4len) { r.verdict = V_TCPOFF; return r; }
        lenword = (tl - ipoff) & 0xffffu;                                 // headers.go:516
        skip0 = off + 16;                                                 // Checksum + UrgentPtr (:518-526)
        r.stored = hbe16(lds, slot, off + 16);
    } else {
        r.verdict = V_PROTO;                                              // :220-221
        return r;
    }
    r.compute = 1;
    // Native (little-endian dword) domain: byte at absolute address a weighs 256^(a mod 4).
    const uint32_t a_s = sa + off, a_e = sa + end;
    r.parity = (int)(a_s & 1u);
    int in_lo = (int)((a_s + 3u) >> 2), in_hi = (int)(a_e >> 2);
    int64_t corr = 0;
    if (in_lo < in_hi) {
        for (uint32_t p = off; sa + p < 4u * (uint32_t)in_lo; ++p) corr += (int64_t)(hb(lds, slot, p) << (8u * ((sa + p) & 3u)));
        r.tail_nb = (int)(a_e & 3u);
        r.use_main = 1;
    } else {
        for (uint32_t p = off; p < end; ++p) corr += (int64_t)(hb(lds, slot, p) << (8u * ((sa + p) & 3u)));
        in_lo = in_hi = 0;
    }
    // Excluded words (UDP: Checksum; TCP: Checksum + UrgentPtr), exact contributions.
    const uint32_t nskip = (proto == 6u) ? 4u : 2u;
    for (uint32_t p = skip0; p < skip0 + nskip; ++p) corr -= (int64_t)(hb(lds, slot, p) << (8u * ((sa + p) & 3u)));
    // Pseudo-header words (BE values), mapped to the native domain.
    const uint32_t w[6] = {hbe16(lds, slot, 26), hbe16(lds, slot, 28), hbe16(lds, slot, 30), hbe16(lds, slot, 32),
                           proto, lenword};
#pragma unroll
    for (int i = 0; i < 6; ++i) corr += (int64_t)(r.parity ? w[i] : bswap16(w[i]));
    r.corr = corr;
    r.in_lo = in_lo;
    r.in_hi = in_hi;
    return r;
}

__global__ void __launch_bounds__(kThreads, 1)
digest_kernel(const uint8_t* __restrict__ frames, const uint64_t* __restrict__ offsets,
              const uint32_t* __restrict__ lengths, uint32_t n, uint32_t mtu, const FsTables* __restrict__ tabs,
              uint2* __restrict__ out, uint8_t* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];

    // ---- LDS table fill: region A (replicated Z64 | Z4), region B (Z32, Z16, T1, inv).
    for (uint32_t w = threadIdx.x; w < 4096u; w += kThreads) {
        const uint32_t e = w >> 4, slot0 = (w & 15u) * 4u;
        const uint32_t b = (slot0 & 31u) >> 3;
        const uint32_t val = (slot0 < 32u) ? tabs->zrow[b][e] : tabs->z4[b][e];
        u32x4 v4 = {val, val, val, val};
        *reinterpret_cast<u32x4*>(lds + e * 256u + slot0 * 4u) = v4;
    }
    {
        const uint32_t* src = &tabs->z32[0][0];  // z32, z16, t1, inv are contiguous
        uint32_t* dst = reinterpret_cast<uint32_t*>(lds + kLdsZ32);
        for (uint32_t i = threadIdx.x; i < (kLdsHdr - kLdsZ32) / 4u; i += kThreads) dst[i] = src[i];
    }
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t grp = lane >> 2;   // frame slot of this lane's group
    const uint32_t gl = lane & 3u;    // lane within the group
    const uint32_t gwave = blockIdx.x * kWavesPerBlock + wave;
    const uint32_t nwaves = gridDim.x * kWavesPerBlock;
    const uint32_t ntiles = (n + kFramesPerTile - 1) / kFramesPerTile;
    const uint32_t hdr_base = kLdsHdr + wave * (kFramesPerTile * kHdrBytes);

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

    for (uint32_t tile = gwave; tile < ntiles; tile += nwaves) {
        // ---- frame lanes (0..15): descriptor, header staging.
        const uint32_t fi = tile * kFramesPerTile + lane;
        const bool fvalid = lane < (uint32_t)kFramesPerTile && fi < n;
        uint64_t S = 0;
        uint32_t len = 0;
        if (fvalid) {
            S = offsets[fi];
            len = lengths[fi];
        }
        const uint64_t E = S + len;
        const uint64_t sdw = S >> 2;
        const uint32_t ndall = (uint32_t)(((E + 3u) >> 2) - sdw);
        const uint32_t nd = (fvalid && len >= 4u) ? ndall : 0u;
        const uint32_t sa = (uint32_t)(S & 3u);
        const uint32_t te = (uint32_t)(E & 3u) ? (uint32_t)(E & 3u) : 4u;  // valid bytes in last dword
        const uint32_t* fb = reinterpret_cast<const uint32_t*>(frames + sdw * 4u);
        const uint32_t slot = hdr_base + (lane & 15u) * kHdrBytes;
        if (fvalid) {
#pragma unroll
            for (uint32_t k = 0; k < (uint32_t)kHdrChunks; ++k) {
                const uint32_t d0 = 4u * k;
                if (d0 < ndall) {
                    u32x4 v = {0u, 0u, 0u, 0u};
                    if (d0 + 4u <= ndall) {
                        v = *reinterpret_cast<const u32x4_a4*>(fb + d0);
                    } else {
                        v.x = fb[d0];
                        if (d0 + 1u < ndall) v.y = fb[d0 + 1];
                        if (d0 + 2u < ndall) v.z = fb[d0 + 2];
                    }
                    *reinterpret_cast<u32x4*>(lds + slot + 16u * k) = v;
                }
            }
        }

        // ---- group lanes: frame geometry from the frame lane, wave row count.
        // (rebuilt from the kernel argument so the loads stay global_load, not flat_load)
        const uint32_t sdw_lo = (uint32_t)__shfl((int)(uint32_t)sdw, (int)grp);
        const uint32_t sdw_hi = (uint32_t)__shfl((int)(uint32_t)(sdw >> 32), (int)grp);
        const uint32_t* gfb = reinterpret_cast<const uint32_t*>(frames + ((((uint64_t)sdw_hi << 32) | sdw_lo) << 2));
        const int g_nd = __shfl((int)nd, (int)grp);
        const uint32_t g_sa = (uint32_t)__shfl((int)sa, (int)grp);
        const uint32_t g_te = (uint32_t)__shfl((int)te, (int)grp);

        uint32_t rows = (lane < (uint32_t)kFramesPerTile) ? (nd + kRowDwords - 1) / kRowDwords : 0u;
#pragma unroll
        for (int m = 8; m >= 1; m >>= 1) rows = max(rows, (uint32_t)__shfl_xor((int)rows, m));
        const int R = __builtin_amdgcn_readfirstlane((int)rows);
        // Rows padded at the FRONT to a multiple of kPrefetch: leading all-zero rows
        // leave a zero-init CRC stream unchanged, so the loop needs no tail guard.
        const int Rp = (R + kPrefetch - 1) / kPrefetch * kPrefetch;
        const int rel0 = g_nd - kRowDwords * Rp + 4 * (int)gl;
        // lowest dword index a load may touch: the buffer start (frames[0])
        const int lo = (sdw_hi != 0 || sdw_lo > (1u << 24)) ? -(1 << 24) : -(int)sdw_lo;

        u32x4 pf[kPrefetch];
#pragma unroll
        for (int i = 0; i < kPrefetch; ++i) pf[i] = load_chunk(gfb, rel0 + kRowDwords * i, lo);

        // ---- frame lanes: header parse (LDS slot), tail partial dword of the L4 range.
        Parsed P;
        uint32_t tail_word = 0;
        if (fvalid) {
            P = parse_frame(lds, slot + sa, sa, len, mtu);
            if (P.compute && P.tail_nb) tail_word = fb[P.in_hi] & ((1u << (8u * (uint32_t)P.tail_nb)) - 1u);
        } else {
            P.verdict = V_OK; P.ip_csum = 0; P.stored = 0; P.compute = 0; P.use_main = 0;
            P.in_lo = 0; P.in_hi = 0; P.parity = 0; P.corr = 0; P.tail_nb = 0;
        }
        const int use_lo = P.use_main ? P.in_lo : 0;
        const int use_hi = P.use_main ? P.in_hi : (int)nd;

        RowMasks M;
        M.nd = g_nd;
        M.in_lo = __shfl(use_lo, (int)grp);
        M.in_hi = __shfl(use_hi, (int)grp);
        if (g_nd > 0) {
            M.fast_lo = max(2, M.in_lo);
            M.fast_hi = min(g_nd - 5, M.in_hi - 4);
        } else {  // empty group: every row streams zeros
            M.fast_lo = -0x40000000;
            M.fast_hi = 0x40000000;
        }
        M.head_mask = 0xffffffffu << (8u * g_sa);
        M.init0 = M.head_mask;
        M.init1 = (1u << (8u * g_sa)) - 1u;
        M.tail_mask = (g_te == 4u) ? 0xffffffffu : ((1u << (8u * g_te)) - 1u);

        // ---- main loop: rows 0..Rp-1, kPrefetch rows in flight.
        uint32_t A[4] = {0u, 0u, 0u, 0u};
        uint64_t cs = 0;
        const int rel_last = rel0 + kRowDwords * (Rp - 1);
        for (int r0 = 0; r0 < Rp; r0 += kPrefetch) {
#pragma unroll
            for (int i = 0; i < kPrefetch; ++i) {
                const int rel = rel0 + kRowDwords * (r0 + i);
                const u32x4 v = pf[i];
                pf[i] = load_chunk(gfb, min(rel + kRowDwords * kPrefetch, rel_last), lo);
                const bool lane_fast = rel >= M.fast_lo && rel <= M.fast_hi;
                const bool fast = __all(lane_fast);
                process_row(lds, keys, v, rel, fast, M, lo, A, cs);
            }
        }

        // ---- combine the 16 streams of each frame (see header comment).
        uint32_t U = zrep(lds, A[0], keys, kZ4Off) ^ A[1];
        U = zrep(lds, U, keys, kZ4Off) ^ A[2];
        U = zrep(lds, U, keys, kZ4Off) ^ A[3];
        uint32_t V = zplain(lds, U, kLdsZ32) ^ dpp_quad<kQuadXor2>(U);
        uint32_t W = zplain(lds, V, kLdsZ16) ^ dpp_quad<kQuadXor1>(V);
        const uint32_t C = zrep(lds, W, keys, kZ4Off);
        uint32_t cs_lo = (uint32_t)cs, cs_hi = (uint32_t)(cs >> 32);
        {   // 64-bit sum over the 4 lanes of the group
            uint64_t t = ((uint64_t)dpp_quad<kQuadXor1>(cs_hi) << 32) | dpp_quad<kQuadXor1>(cs_lo);
            cs += t;
            cs_lo = (uint32_t)cs;
            cs_hi = (uint32_t)(cs >> 32);
            t = ((uint64_t)dpp_quad<kQuadXor2>(cs_hi) << 32) | dpp_quad<kQuadXor2>(cs_lo);
            cs += t;
        }
        const uint32_t src = (lane & 15u) * 4u;
        uint32_t crcv = (uint32_t)__shfl((int)C, (int)src);
        const uint64_t csum =
            ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(cs >> 32), (int)src) << 32) |
            (uint32_t)__shfl((int)(uint32_t)cs, (int)src);

        // ---- frame lanes: finalize + store.
        if (fvalid) {
            if (len < 4u) {  // too short for the 4-byte init trick: bytewise CRC-32
                uint32_t c = 0xffffffffu;
                for (uint32_t p = 0; p < len; ++p)
                    c = lds32(lds, kLdsT1 + (((c ^ lds8(lds, slot + sa + p)) & 0xffu) << 2)) ^ (c >> 8);
                crcv = ~c;
            } else {
                uint32_t c = crcv;
                const uint32_t t = (4u - (uint32_t)(E & 3u)) & 3u;  // zero bytes appended by dword rounding
                for (uint32_t k = 0; k < t; ++k) {
                    const uint32_t j = lds8(lds, kLdsInv + (c >> 24));
                    c = ((c ^ lds32(lds, kLdsT1 + (j << 2))) << 8) | j;
                }
                crcv = ~c;
            }
            uint32_t verdict = P.verdict, l4 = 0;
            if (P.compute) {
                uint64_t x = (uint64_t)((int64_t)(P.use_main ? csum : 0u) + P.corr) + tail_word;
                x = (x & 0xffffffffu) + (x >> 32);
                while (x >> 16) x = (x & 0xffffu) + (x >> 16);
                l4 = (~(uint32_t)x) & 0xffffu;
                if (!P.parity) l4 = bswap16(l4);
                verdict = (l4 == P.stored) ? V_OK : V_CSUM;
            }
            out[fi] = make_uint2(crcv, P.ip_csum | (l4 << 16));
            if (status) status[fi] = (uint8_t)verdict;
        }
    }
}

}  // namespace

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
