// Row-compute microbenchmark (measurement tool): the digest kernel's lean row (Z64 Horner
// via replicated LDS table + v_sad_u16) with data from registers, at W waves per CU (one
// 100 KB-LDS block per CU) and K independent tiles interleaved per wave (4K streams/lane).
// Reports ticks per row per wave and the implied per-CU byte rate (1 KB per tile-row).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ uint32_t ld(const char* lds, uint32_t a) { return *reinterpret_cast<const uint32_t*>(lds + a); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
struct Keys { uint32_t cvec, s[4]; };
__device__ __forceinline__ uint32_t z(const char* lds, uint32_t a, const Keys& k, uint32_t w) {
    uint32_t t0 = ld(lds, __builtin_amdgcn_perm(a, k.cvec, k.s[0]));
    uint32_t t1 = ld(lds, __builtin_amdgcn_perm(a, k.cvec, k.s[1]));
    uint32_t t2 = ld(lds, __builtin_amdgcn_perm(a, k.cvec, k.s[2]));
    uint32_t t3 = ld(lds, __builtin_amdgcn_perm(a, k.cvec, k.s[3]));
    return xor3(xor3(t0, t1, t2), t3, w);
}

template <int K>
__global__ void k_rows(int rows, uint32_t seed, uint32_t* out, unsigned long long* cyc) {
    __shared__ __attribute__((aligned(16))) char lds[100 * 1024];
    for (uint32_t i = threadIdx.x; i < 16384; i += blockDim.x) reinterpret_cast<uint32_t*>(lds)[i] = i * 2654435761u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    Keys k;
    {
        const uint32_t c = lane & 7u, h = (lane >> 3) & 3u;
        k.cvec = 0;
        for (uint32_t j = 0; j < 4; ++j) k.cvec |= (32u * j + 4u * c) << (8u * j);
        for (uint32_t q = 0; q < 4; ++q) { uint32_t b = (q + h) & 3u; k.s[q] = 0x0c0c0000u | ((4u + b) << 8) | b; }
    }
    uint32_t A[4 * K], w[4 * K], cs[K];
#pragma unroll
    for (int q = 0; q < 4 * K; ++q) { A[q] = seed ^ (lane * (q + 1)); w[q] = seed * (q + 3) ^ threadIdx.x; }
#pragma unroll
    for (int t = 0; t < K; ++t) cs[t] = 0;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < rows; ++r) {
#pragma unroll
        for (int t = 0; t < K; ++t) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                A[4 * t + j] = z(lds, A[4 * t + j], k, w[4 * t + j]);
                cs[t] = __builtin_amdgcn_sad_u16(w[4 * t + j], 0u, cs[t]);
            }
        }
#pragma unroll
        for (int q = 0; q < 4 * K; ++q) w[q] += 0x9e3779b9u;  // fresh data each row (1 op per dword, like a load)
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t r = 0;
#pragma unroll
    for (int q = 0; q < 4 * K; ++q) r ^= A[q];
#pragma unroll
    for (int t = 0; t < K; ++t) r ^= cs[t];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (lane == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int K>
void run(int blocks, int waves, int rows) {
    uint32_t* out; unsigned long long* cyc;
    CHECK(hipMalloc(&out, blocks * 1024 * 4));
    CHECK(hipMalloc(&cyc, blocks * 16 * 8));
    hipLaunchKernelGGL(k_rows<K>, dim3(blocks), dim3(64 * waves), 0, 0, rows, 1u, out, cyc);
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(k_rows<K>, dim3(blocks), dim3(64 * waves), 0, 0, rows, 2u, out, cyc);
    CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
    float ms; CHECK(hipEventElapsedTime(&ms, a, b));
    unsigned long long* h = (unsigned long long*)malloc(blocks * 16 * 8);
    CHECK(hipMemcpy(h, cyc, blocks * 16 * 8, hipMemcpyDeviceToHost));
    double s = 0, mx = 0; int cnt = 0;
    for (int bl = 0; bl < blocks; ++bl) for (int wv = 0; wv < waves; ++wv) { double v = h[bl * 16 + wv]; s += v; mx = v > mx ? v : mx; ++cnt; }
    double cpr = s / cnt / rows;  // ticks per row per wave (K tile-rows)
    double per_cu = waves * 1024.0 * K / cpr;
    double clk = (s / cnt) / (ms * 1e-3);
    printf("waves/CU=%2d K=%d  %7.1f ticks/row/wave (max wave %.1f)  %5.2f B/tick/CU  clk %.2f GHz  chip %.1f TB/s\n",
           waves, K, cpr, mx / rows, per_cu, clk / 1e9, per_cu * clk * blocks / 1e12);
    free(h); CHECK(hipFree(out)); CHECK(hipFree(cyc));
}

int main() {
    hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
    int cus = p.multiProcessorCount;
    for (int waves : {4, 8, 16}) {
        run<1>(cus, waves, 2000);
        run<2>(cus, waves, 1000);
        if (waves <= 8) run<4>(cus, waves, 500);
    }
    return 0;
}
