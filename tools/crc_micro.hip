// Microbenchmark of the digest kernel's row-compute loop (measurement tool).
// Data comes from registers (no global loads), 16 waves per block, one block per CU,
// region-A-style replicated LDS tables. Reports cycles per row per wave and the
// implied per-CU byte rate (1 KB per wave-row: 16 frames x 64 B).
//  v0: 4 streams x 16 B per lane-row (current kernel fast path)
//  v1: no LDS lookups (perm + xor only)
//  v2: 8 streams (two 16-B chunks per lane-row, i.e. 32 B/lane/row, 2 frames per group)
//  v3: v0 with all 16 lookups issued before any xor (explicit ILP)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ uint32_t ld(const char* lds, uint32_t a) { return *reinterpret_cast<const uint32_t*>(lds + a); }

struct Keys { uint32_t cvec, s0, s1, s2, s3; };

__device__ __forceinline__ uint32_t z(const char* lds, uint32_t a, const Keys& k) {
    return ld(lds, __builtin_amdgcn_perm(a, k.cvec, k.s0)) ^ ld(lds, __builtin_amdgcn_perm(a, k.cvec, k.s1)) ^
           ld(lds, __builtin_amdgcn_perm(a, k.cvec, k.s2)) ^ ld(lds, __builtin_amdgcn_perm(a, k.cvec, k.s3));
}

template <int V>
__global__ void __launch_bounds__(1024, 1) k_rows(int rows, uint32_t seed, uint32_t* out, unsigned long long* cyc) {
    __shared__ __attribute__((aligned(16))) char lds[65536];
    for (uint32_t i = threadIdx.x; i < 16384; i += 1024) reinterpret_cast<uint32_t*>(lds)[i] = i * 2654435761u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    Keys k;
    {
        const uint32_t c = lane & 7u, h = (lane >> 3) & 3u;
        k.cvec = 0;
        for (uint32_t j = 0; j < 4; ++j) k.cvec |= (32u * j + 4u * c) << (8u * j);
        uint32_t s[4];
        for (uint32_t q = 0; q < 4; ++q) { uint32_t b = (q + h) & 3u; s[q] = 0x0c0c0000u | ((4u + b) << 8) | b; }
        k.s0 = s[0]; k.s1 = s[1]; k.s2 = s[2]; k.s3 = s[3];
    }
    uint32_t A[8] = {seed ^ lane, seed * 3, lane * 7, seed + lane, 1, 2, 3, 4};
    uint32_t w0 = seed ^ (threadIdx.x * 0x9e3779b9u), w1 = w0 * 5, w2 = w0 * 7, w3 = w0 * 11;
    uint32_t lo = 0, hi = 0;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < rows; ++r) {
        if (V == 0) {
            A[0] = z(lds, A[0], k) ^ w0; A[1] = z(lds, A[1], k) ^ w1;
            A[2] = z(lds, A[2], k) ^ w2; A[3] = z(lds, A[3], k) ^ w3;
        } else if (V == 1) {
            A[0] = (__builtin_amdgcn_perm(A[0], k.cvec, k.s0) ^ __builtin_amdgcn_perm(A[0], k.cvec, k.s1) ^ __builtin_amdgcn_perm(A[0], k.cvec, k.s2) ^ __builtin_amdgcn_perm(A[0], k.cvec, k.s3)) ^ w0;
            A[1] = (__builtin_amdgcn_perm(A[1], k.cvec, k.s0) ^ __builtin_amdgcn_perm(A[1], k.cvec, k.s1) ^ __builtin_amdgcn_perm(A[1], k.cvec, k.s2) ^ __builtin_amdgcn_perm(A[1], k.cvec, k.s3)) ^ w1;
            A[2] = (__builtin_amdgcn_perm(A[2], k.cvec, k.s0) ^ __builtin_amdgcn_perm(A[2], k.cvec, k.s1) ^ __builtin_amdgcn_perm(A[2], k.cvec, k.s2) ^ __builtin_amdgcn_perm(A[2], k.cvec, k.s3)) ^ w2;
            A[3] = (__builtin_amdgcn_perm(A[3], k.cvec, k.s0) ^ __builtin_amdgcn_perm(A[3], k.cvec, k.s1) ^ __builtin_amdgcn_perm(A[3], k.cvec, k.s2) ^ __builtin_amdgcn_perm(A[3], k.cvec, k.s3)) ^ w3;
        } else if (V == 2) {
#pragma unroll
            for (int q = 0; q < 8; ++q) A[q] = z(lds, A[q], k) ^ (w0 + q);
        } else {
            uint32_t t[16];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                t[4 * q + 0] = ld(lds, __builtin_amdgcn_perm(A[q], k.cvec, k.s0));
                t[4 * q + 1] = ld(lds, __builtin_amdgcn_perm(A[q], k.cvec, k.s1));
                t[4 * q + 2] = ld(lds, __builtin_amdgcn_perm(A[q], k.cvec, k.s2));
                t[4 * q + 3] = ld(lds, __builtin_amdgcn_perm(A[q], k.cvec, k.s3));
            }
            A[0] = t[0] ^ t[1] ^ t[2] ^ t[3] ^ w0; A[1] = t[4] ^ t[5] ^ t[6] ^ t[7] ^ w1;
            A[2] = t[8] ^ t[9] ^ t[10] ^ t[11] ^ w2; A[3] = t[12] ^ t[13] ^ t[14] ^ t[15] ^ w3;
        }
        unsigned int c;
        lo = __builtin_addc(lo, w0, 0u, &c); hi += c;
        lo = __builtin_addc(lo, w1, 0u, &c); hi += c;
        lo = __builtin_addc(lo, w2, 0u, &c); hi += c;
        lo = __builtin_addc(lo, w3, 0u, &c); hi += c;
        w0 += A[0]; w1 ^= A[1]; w2 += A[2]; w3 ^= A[3];
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t r = A[0] ^ A[1] ^ A[2] ^ A[3] ^ A[4] ^ A[5] ^ A[6] ^ A[7] ^ lo ^ hi;
    out[blockIdx.x * 1024 + threadIdx.x] = r;
    if (lane == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int V>
void run(const char* name, int blocks, int rows, double bytes_per_lane_row) {
    uint32_t* out; unsigned long long* cyc;
    CHECK(hipMalloc(&out, blocks * 1024 * 4));
    CHECK(hipMalloc(&cyc, blocks * 16 * 8));
    hipLaunchKernelGGL(k_rows<V>, dim3(blocks), dim3(1024), 0, 0, rows, 1u, out, cyc);
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(k_rows<V>, dim3(blocks), dim3(1024), 0, 0, rows, 2u, out, cyc);
    CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
    float ms; CHECK(hipEventElapsedTime(&ms, a, b));
    unsigned long long* h = (unsigned long long*)malloc(blocks * 16 * 8);
    CHECK(hipMemcpy(h, cyc, blocks * 16 * 8, hipMemcpyDeviceToHost));
    double s = 0; for (int i = 0; i < blocks * 16; ++i) s += h[i];
    double cpr = s / (blocks * 16) / rows;
    double clk = s / (blocks * 16) / (ms * 1e-3);  // memtime ticks per second
    double per_cu = 16.0 * 64 * bytes_per_lane_row / cpr;  // bytes per tick per CU
    printf("%-40s blocks=%4d  %7.1f ticks/row/wave  %5.2f B/tick/CU  (%.2f GHz memtime)  chip %.0f GB/s\n", name, blocks,
           cpr, per_cu, clk / 1e9, per_cu * clk * blocks / 1e9);
    free(h); CHECK(hipFree(out)); CHECK(hipFree(cyc));
}

int main() {
    hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
    int cus = p.multiProcessorCount;
    for (int blocks : {1, cus}) {
        run<0>("v0 4 streams/lane (kernel fast path)", blocks, 4000, 16);
        run<1>("v1 perm+xor only (no LDS)", blocks, 4000, 16);
        run<2>("v2 8 streams/lane (32 B/lane/row)", blocks, 2000, 32);
        run<3>("v3 4 streams, 16 lookups batched", blocks, 4000, 16);
    }
    return 0;
}
