// Internal declarations shared by the framesum HIP kernel and the C-ABI host code.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace framesum {

// CRC-32 "zero-shift" operator tables, built on the host once per context
// (framesum_tables.cpp) in the kernel's LDS layout.
// Z_k[b][v] = register value after feeding k zero bytes to a reflected
// CRC-32 register holding (v << 8b)  -- i.e. multiplication by x^(8k) mod P.
// Each workgroup builds region A itself from `z64_basis` (VALU + ds_write, no memory
// traffic ahead of the first rows) and copies the plain tables by LDS-DMA behind its
// first rows; they are only needed by the per-frame combine.
struct FsTables {
    // Region A (64 KB): 256 entry rows x 64 dword slots. Slot 8*b + c (c = 0..7) holds
    // Z_64[b][e] (one 64-byte frame-row of stream stride); the 8 copies make the kernel's
    // lookups LDS-bank-conflict-free (the 256-B entry stride lets one v_perm_b32 form the
    // address). Slots 32..63 are unused (the captured header slots do not overlap them).
    uint32_t region_a[256][64];
    uint32_t z32[4][256];      // Z_32 : lane-tree level 1 (lanes l, l+2)
    uint32_t z16[4][256];      // Z_16 : lane-tree level 2 (lanes l, l+1)
    uint32_t zfin[4][4][256];  // Z_4, Z_3, Z_2, Z_1 : final step Z_(4-t) (t = bytes of dword rounding); Z_4 also
                               // serves the intra-lane combine
    uint32_t z48[4][256];      // Z_48 : lane 0 of the flattened lane tree
    uint32_t z12[4][256];      // Z_12 : stream 0 of the flattened intra-lane combine
    uint32_t z8[4][256];       // Z_8  : stream 1
    uint32_t z768[4][256];     // Z_768: one full piece (mode B Horner over a frame's pieces)
    // --- not part of the LDS image ---
    uint32_t z64_basis[4][8];  // Z_64[b][1 << j]: region A's entries are XORs of these
    // T[b][1 << j] of the 40 plain [4][256] tables above, in LDS-image order (piece p = 4 t + b is the
    // 1-KB piece at LDS byte 1024 p): the kernels build them in place by VALU, as region A
    uint32_t plain_basis[40][8];
};
constexpr uint32_t kTablesLdsBytes = 65536 + 4096 * 10;  // the LDS image: everything before z64_basis
static_assert(offsetof(FsTables, z64_basis) == kTablesLdsBytes, "FsTables layout");
static_assert(offsetof(FsTables, z32) == 65536 && offsetof(FsTables, plain_basis) == kTablesLdsBytes + 128,
              "FsTables layout: the plain tables are 40 1-KB pieces after region A");

void build_tables(FsTables* t);

// Launch the digest kernel. `num_cus` sizes the persistent grid. `report` (nullable) is a
// host-mapped word: a kernel writes its launch id there when its batch has tiles of widely
// mixed frame lengths; launches within a window after such a report use the kernel variant
// that can split long frames into pieces (mode B), others the leaner one-pass variant. The choice never changes a
// result, only the speed. `force`: 0 = that choice, 2 / 3 / 4 / 8 = always the mixed-length / segment /
// one-pass kernel, the small-frame kernel preferred (fs_ctx_set_kernel; tests run every case through
// each), or one of the host-staged path's kForce* values below. `next_id`: the
// context's launch counter (the ids its launches report under).
// `op`: the RX digest; the TX fill (`wframes` = the same frames, writable; `tx` = FS_FILL_* flags:
// checksums written into the frames and/or the FCS appended after them); or the RX digest of
// wire frames whose lengths include a trailing FCS.
enum class FsOp { kDigest, kFill, kFcs };
// The context's host-mapped report block (64 B): word kReportLatest is written by the device (the
// latest launch id that met mixed-length tiles); the others only by the host: the launches left in
// the context's initial mixed-kernel window, and the variant of its latest launch.
// kReportSeen / kReportSeenSeq (host-only): the report word's value as the host last saw it
// change, and the context's launch sequence at that moment (the sticky window's clock).
constexpr int kReportLatest = 0, kReportInitial = 1, kReportChosen = 2, kReportSeen = 3, kReportSeenSeq = 4;
constexpr uint32_t kInitialMixedLaunches = 16;
// The short-frame choice (the small-frame kernel, variant 8, for traffic of frames <= kSmallMaxLen
// bytes): kReportLong and kReportRan are written by the device -- the latest launch
// id that met a frame longer than kSmallMaxLen, and the latest launch id that ran a 4-lane kernel
// (posted by the grid's first wave, with kReportRanLong set when its own tile held such a frame);
// kReportLongSeen, kReportRanSeen, kReportShort and kReportLongEver only by the host: the two words
// as it last saw them, the number of launches seen to run since the latest long report, and whether
// any long report has arrived (launch_digest).
constexpr int kReportLong = 5, kReportRan = 6, kReportLongSeen = 7, kReportRanSeen = 8, kReportShort = 9;
constexpr int kReportLongEver = 10;
constexpr uint32_t kReportRanLong = 1u << 16;
// ... and in the kReportLatest word, the posting tile held a frame longer than the mixed-length kernel's
// pieces cover (kMaxFullPasses passes of 16 pieces) beside short ones: the automatic choice then runs
// the segment kernel (variant 3), which splits any frame into equal chunks
constexpr uint32_t kReportMixedGiant = 1u << 16;
constexpr uint32_t kSmallMaxLen = 128;
// the kernels' `report` argument: the report block's device address in bits 6..46 (host-mapped
// memory sits below 2^47; the block is 64-B aligned), a watch flag in bit 47, the launch id in bits
// 48..63, and in bits 0..1 what this launch is asked to post: kAskRan (the grid's first tile posts
// kReportRan) and kAskMixed (the mixed-length kernel posts its mixed tiles; the one-pass kernel
// always does). Each post costs the launch ~0.28 us (C2), so steady traffic is sampled: "ran" on
// every kRanSample-th launch under variant 0 (every launch while the host counts short launches,
// and every launch under variant 8), "mixed" from the
// mixed-length kernel on every kMixedSample-th launch (and until the first report).
constexpr uint64_t kReportAddrMask = ((1ull << 47) - 1u) & ~63ull;
constexpr uint64_t kAskRan = 1u, kAskMixed = 2u;
constexpr uint32_t kRanSample = 4, kMixedSample = 32;
// launches seen to run without a long frame before variant 0 moves to the small-frame kernel, and
// before a variant-8 context that met long frames goes back to it
constexpr uint32_t kShortLaunchesAuto = 16, kShortLaunchesSmall = 2;
// launch_digest's force values for the host-staged path, which knows every length: the small-frame
// kernel unconditionally (every frame <= kSmallMaxLen), or the automatic choice among the 4-lane
// kernels only (a frame is longer: however short the context's recent traffic, the small-frame
// kernel would stream that frame with one lane)
constexpr int kForceSmallExact = 16;
constexpr int kForceNoSmall = 17;
// ... and for a host batch whose lengths all lie within kUniformSpan bytes (no tile can differ by the
// 4 rows a mixed-length tile needs), the one-pass kernel from the context's first call: the initial
// mixed-kernel window (kInitialMixedLaunches) is for device-resident batches, whose lengths the host
// never sees
constexpr int kForceUniformHost = 18;
constexpr uint32_t kUniformSpan = 256;
hipError_t launch_digest(const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths, uint32_t n,
                         uint32_t mtu, const FsTables* tables, void* out, uint8_t* status, hipStream_t stream,
                         int num_cus, volatile uint32_t* report_host, uint32_t* report_dev, uint32_t* next_id,
                         int force = 0, FsOp op = FsOp::kDigest, uint8_t* wframes = nullptr, uint32_t tx = 0);

// Restore global frame order from nshards gathered round-robin slabs (framesum_plan.h layout):
// out[i] = slab[i % nshards].digest[i / nshards], status likewise (nullable), for global frames
// [i0, min(i1, n)) of the n-frame batch. framesum_shard.hip.
hipError_t launch_deinterleave(const uint8_t* gathered, uint32_t nshards, uint64_t n, void* out, uint8_t* status,
                               hipStream_t stream, uint64_t i0 = 0, uint64_t i1 = ~0ull);

}  // namespace framesum
