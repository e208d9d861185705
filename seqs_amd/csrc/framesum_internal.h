// Internal declarations shared by the framesum HIP kernel and the C-ABI host code.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace framesum {

// CRC-32 "zero-shift" operator tables, built on the host once per context
// (framesum_tables.cpp) and copied into LDS by every workgroup.
// Z_k[b][v] = register value after feeding k zero bytes to a reflected
// CRC-32 register holding (v << 8b)  -- i.e. multiplication by x^(8k) mod P.
struct FsTables {
    uint32_t zrow[4][256];  // Z_64 : one 64-byte frame-row (4 lanes x 16 B) of stream stride
    uint32_t z4[4][256];    // Z_4  : one dword (intra-lane Horner + final step)
    uint32_t z32[4][256];   // Z_32 : lane-tree level 1 (lanes l, l+2)
    uint32_t z16[4][256];   // Z_16 : lane-tree level 2 (lanes l, l+1)
    uint32_t t1[256];       // Z_1 byte table (standard CRC-32 table)
    uint32_t inv[64];       // 256 bytes: inv[t1[j] >> 24] = j (one-byte un-shift)
};

void build_tables(FsTables* t);

// Launch the digest kernel. `num_cus` sizes the persistent grid.
hipError_t launch_digest(const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths, uint32_t n,
                         uint32_t mtu, const FsTables* tables, void* out, uint8_t* status, hipStream_t stream,
                         int num_cus);

}  // namespace framesum
