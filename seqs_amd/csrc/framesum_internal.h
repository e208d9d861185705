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
    // address). Slots 32..63 hold 8 plain tables for the two-workgroups-per-CU kernel, which
    // copies region A as it is: slot 32 + ((4 t + b) ^ (e & 31)) = T_t[b][e] for the tables
    // kA2Tables (the XOR spreads one table's entries over the banks as a plain [4][256] table's).
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
    // T_(kA2Tables[q >> 2])[q & 3][1 << j]: the bases of region A's upper-half plain tables (LayA2)
    uint32_t a2_basis[32][8];
};
constexpr uint32_t kTablesLdsBytes = 65536 + 4096 * 10;  // the LDS image: everything before z64_basis
// region A's plain tables (slots 32..63): the zero shift in bytes of table t = 0..7
constexpr int kA2Tables[8] = {4, 8, 12, 16, 32, 48, 2, 1};
static_assert(offsetof(FsTables, z64_basis) == kTablesLdsBytes, "FsTables layout");
static_assert(offsetof(FsTables, z32) == 65536 && offsetof(FsTables, plain_basis) == kTablesLdsBytes + 128,
              "FsTables layout: the plain tables are 40 1-KB pieces after region A");

void build_tables(FsTables* t);

// The 16-lane kernel's tables (digest_kernel_w): a frame streams as 16 lanes, each folding its
// 4 dwords of every 256-byte row into one accumulator, A <- Z4(Z4(Z4(Z244(A) ^ w0) ^ w1) ^ w2) ^ w3;
// region A holds Z_244 and Z_4 (8 copies each, conflict-free). The combine's lane shifts use
// Z_16..Z_48 (within a quad of lanes) and Z_64..Z_192 (across the 4 quads). LDS image: the 11
// plain [4][256] tables (copied by LDS-DMA) then region A (built in place from the bases).
struct FsTablesW {
    uint32_t z16[4][256];
    uint32_t z32[4][256];
    uint32_t z48[4][256];
    uint32_t z64[4][256];
    uint32_t z128[4][256];
    uint32_t z192[4][256];
    uint32_t zfin[4][4][256];  // Z_4, Z_3, Z_2, Z_1 (zfin[t] = Z_(4-t))
    uint32_t z1024[4][256];    // TX fill: long CRC corrections
    uint32_t region_a[256][64];  // [entry][op*32 + table*8 + copy], op 0 = Z_244, op 1 = Z_4
    // --- not part of the LDS image ---
    uint32_t basis[2][4][8];   // op, byte table, bit: region A's entries are XORs of these
};
constexpr uint32_t kTablesWPlainBytes = 11u * 4096u;
constexpr uint32_t kTablesWLdsBytes = kTablesWPlainBytes + 65536u;
static_assert(offsetof(FsTablesW, region_a) == kTablesWPlainBytes, "FsTablesW layout");
static_assert(offsetof(FsTablesW, basis) == kTablesWLdsBytes, "FsTablesW layout");

void build_tables_w(FsTablesW* t);

// The streaming kernel's tables (framesum_rx.hip). Each workgroup builds its 64-KB LDS image from
// these bases (every table is GF(2)-linear in its byte): entry row e (256 B) holds, in dword slots
// 0..31, Z_256[b][e] for slot 8b + c (8 copies per byte table: the row lookups are conflict-free),
// and in slots 32..63 the 8 plain tables kRxPlain, T_t[b][e] at slot 32 + ((4t + b) ^ (e >> 3)).
constexpr int kRxPlain[8] = {4, 16, 32, 48, 64, 128, 192, 1536};
struct FsTablesRx {
    uint32_t z256_basis[4][8];   // Z_256[b][1 << j]
    uint32_t plain_basis[32][8]; // q = 4t + b: T_t[b][1 << j]
};
void build_tables_rx(FsTablesRx* t);
// the LDS image those bases describe (host reference, for the CPU tests of the layout)
void rx_region_image(const FsTablesRx* t, uint32_t region[256][64]);

// Launch the streaming kernel (every operation). `grid_per_cu`: workgroups per CU (1 = one
// 8-wave workgroup per CU, so consecutive launches co-reside; 2 = the whole CU for one launch).
hipError_t launch_rx(const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths, uint32_t n, uint32_t mtu,
                     const FsTablesRx* tables, void* out, uint8_t* status, hipStream_t stream, int num_cus,
                     int grid_per_cu, int op, uint8_t* wframes, uint32_t tx);

// Launch the digest kernel. `num_cus` sizes the persistent grid. `report` (nullable) is a
// host-mapped word: a kernel writes its launch id there when its batch has tiles of widely
// mixed frame lengths; launches within a window after such a report use the kernel variant
// that can split long frames into pieces (mode B), others the leaner one-pass variant. The choice never changes a
// result, only the speed. `force`: 0 = that choice, 1 = always the one-pass kernel, 2 = always
// the mixed-length kernel (fs_ctx_set_kernel; tests run every case through both).
// `op`: the RX digest; the TX fill (`wframes` = the same frames, writable; `tx` = FS_FILL_* flags:
// checksums written into the frames and/or the FCS appended after them); or the RX digest of
// wire frames whose lengths include a trailing FCS.
enum class FsOp { kDigest, kFill, kFcs };
// force 5 = the same kernel as two 8-wave workgroups per CU (LayA2: RX ops; the fill runs force 4's);
// force 4 = the one-pass kernel with block-aligned rows (what force 0 uses for the one-pass choice;
// force 1 keeps the end-anchored rows).
// `tables_w`: the 16-lane kernel's tables; force 3 = the 16-lane kernel (an experimental variant,
// parity-tested like the others; slower than the 4-lane kernels on the benchmark configs).
// The context's host-mapped report block (64 B): word kReportLatest is written by the device (the
// latest launch id that met mixed-length tiles); the others only by the host: the launches left in
// the context's initial mixed-kernel window, and the variant of its latest launch.
constexpr int kReportLatest = 0, kReportInitial = 1, kReportChosen = 2;
constexpr uint32_t kInitialMixedLaunches = 16;
hipError_t launch_digest(const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths, uint32_t n,
                         uint32_t mtu, const FsTables* tables, void* out, uint8_t* status, hipStream_t stream,
                         int num_cus, volatile uint32_t* report_host, uint32_t* report_dev, int force = 0,
                         FsOp op = FsOp::kDigest, uint8_t* wframes = nullptr, uint32_t tx = 0,
                         const FsTablesW* tables_w = nullptr);

// Restore global frame order from nshards gathered round-robin slabs (framesum_plan.h layout):
// out[i] = slab[i % nshards].digest[i / nshards], status likewise (nullable), for global frames
// [i0, min(i1, n)) of the n-frame batch. framesum_shard.hip.
hipError_t launch_deinterleave(const uint8_t* gathered, uint32_t nshards, uint64_t n, void* out, uint8_t* status,
                               hipStream_t stream, uint64_t i0 = 0, uint64_t i1 = ~0ull);

}  // namespace framesum
