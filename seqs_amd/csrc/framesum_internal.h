// Internal declarations shared by the framesum HIP kernel and the C-ABI host code.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace framesum {

// CRC-32 "zero-shift" operator tables, built on the host once per context
// (framesum_tables.cpp) directly in the kernel's LDS layout, so every workgroup
// fills its LDS with plain 1-KB LDS-DMA copies (global_load_lds_dwordx4).
// Z_k[b][v] = register value after feeding k zero bytes to a reflected
// CRC-32 register holding (v << 8b)  -- i.e. multiplication by x^(8k) mod P.
struct FsTables {
    // Region A (64 KB): 256 entry rows x 64 dword slots. Slot 8*b + c (c = 0..7) holds
    // Z_64[b][e] (one 64-byte frame-row of stream stride), slot 32 + 8*b + c holds
    // Z_4[b][e]; the 8 copies make the kernel's lookups LDS-bank-conflict-free.
    uint32_t region_a[256][64];
    uint32_t z32[4][256];      // Z_32 : lane-tree level 1 (lanes l, l+2)
    uint32_t z16[4][256];      // Z_16 : lane-tree level 2 (lanes l, l+1)
    uint32_t zfin[4][4][256];  // Z_4, Z_3, Z_2, Z_1 : final step Z_(4-t) (t = bytes of dword rounding)
    uint32_t z48[4][256];      // Z_48 : lane 0 of the flattened lane tree
    uint32_t z12[4][256];      // Z_12 : stream 0 of the flattened intra-lane combine
    uint32_t z8[4][256];       // Z_8  : stream 1
};
static_assert(sizeof(FsTables) == 65536 + 4096 * 9, "FsTables is the LDS image (100 KB)");

void build_tables(FsTables* t);

// Launch the digest kernel. `num_cus` sizes the persistent grid.
hipError_t launch_digest(const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths, uint32_t n,
                         uint32_t mtu, const FsTables* tables, void* out, uint8_t* status, hipStream_t stream,
                         int num_cus);

}  // namespace framesum
