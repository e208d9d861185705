// De-interleave of round-robin shard results — CDNA4 / gfx950.
//
// After the RCCL gather of fs_digest_batch_sharded (or a torch.distributed gather into one
// buffer, bench.py --config c4), the root device holds nshards slabs back to back: slab k =
// shard k's m 8-byte digests, then its m verdict bytes (framesum_plan.h). Global frame i is
// local frame i / N of shard i % N, so out[i] = slab[i % N].digest[i / N]. One thread per
// global frame: the 8-byte writes are coalesced, the reads are N contiguous streams.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "framesum_internal.h"
#include "framesum_plan.h"

namespace framesum {
namespace {

__global__ void __launch_bounds__(256) deinterleave_kernel(const uint8_t* __restrict__ gathered, uint32_t nshards,
                                                          uint64_t i0, uint64_t i1, uint64_t m,
                                                          uint2* __restrict__ out, uint8_t* __restrict__ status) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = i0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < i1; i += stride) {
        out[i] = *reinterpret_cast<const uint2*>(gathered + plan::gathered_digest_at(i, nshards, m));
        if (status) status[i] = gathered[plan::gathered_status_at(i, nshards, m)];
    }
}

}  // namespace

hipError_t launch_deinterleave(const uint8_t* gathered, uint32_t nshards, uint64_t n, void* out, uint8_t* status,
                               hipStream_t stream, uint64_t i0, uint64_t i1) {
    if (i1 > n) i1 = n;
    if (i0 >= i1) return hipSuccess;
    const uint64_t m = plan::shard_rows(n, nshards);
    uint64_t blocks = (i1 - i0 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(deinterleave_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, gathered, nshards, i0, i1, m,
                       reinterpret_cast<uint2*>(out), status);
    return hipGetLastError();
}

}  // namespace framesum
