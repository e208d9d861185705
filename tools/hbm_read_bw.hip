// HBM read-bandwidth microbenchmark for the framesum access pattern (measurement tool).
//  k_stream : grid-stride global_load_dwordx4, 16 B/lane, fully coalesced (chip ceiling)
//  k_frames : the digest kernel's pattern without compute — 16 frames per wave,
//             4 lanes per frame, 64-B end-anchored rows, kPF rows in flight
//  k_frames_al : the same with rows aligned to 64 or 128 B in memory
// Both rotate NB distinct 98.3 MB buffers (> 256 MiB Infinity Cache).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <chrono>
#include <string>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <bool NT>
__device__ __forceinline__ u32x4 ld4(const u32x4* p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}

template <bool NT>
__global__ void k_stream(const u32x4* __restrict__ p, size_t n16, uint32_t* out) {
    uint32_t acc = 0;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        u32x4 a = ld4<NT>(p + i), b = ld4<NT>(p + i + stride), c = ld4<NT>(p + i + 2 * stride), d = ld4<NT>(p + i + 3 * stride);
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
    }
    for (; i < n16; i += stride) { u32x4 a = p[i]; acc ^= a.x ^ a.y ^ a.z ^ a.w; }
    if (acc == 0x12345678u) out[0] = acc;
}

// G lanes per frame (64/G frames per wave), rows of G*16 bytes anchored at the frame end.
template <int kPF, int G, bool NT = false, int WPB = 16>
__global__ void __launch_bounds__(64 * WPB) k_frames(const uint8_t* __restrict__ base, uint32_t nframes, uint32_t flen,
                                                     uint32_t* out) {
    constexpr int FPW = 64 / G, RD = 4 * G;  // frames per wave, row dwords
    const uint32_t lane = threadIdx.x & 63, grp = lane / G, gl = lane % G;
    const uint32_t gwave = blockIdx.x * WPB + (threadIdx.x >> 6), nwaves = gridDim.x * WPB;
    const uint32_t ntiles = (nframes + FPW - 1) / FPW;
    uint32_t acc = 0;
    for (uint32_t t = gwave; t < ntiles; t += nwaves) {
        uint32_t f = t * FPW + grp;
        if (f >= nframes) f = nframes - 1;
        const uint64_t S = (uint64_t)f * flen, E = S + flen;
        const uint64_t sdw = S >> 2;
        const int nd = (int)(((E + 3) >> 2) - sdw);
        const int R = (nd + RD - 1) / RD;
        const int Rp = (R + kPF - 1) / kPF * kPF;
        const int rel0 = nd - RD * Rp + 4 * (int)gl;
        const int rel_last = rel0 + RD * (Rp - 1);
        const uint32_t* fb = reinterpret_cast<const uint32_t*>(base + sdw * 4);
        const int lo = -(int)min(sdw, (uint64_t)(1 << 24));
        u32x4 pf[kPF];
#pragma unroll
        for (int i = 0; i < kPF; ++i) pf[i] = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4_a4*>(fb + max(rel0 + RD * i, lo))) : *reinterpret_cast<const u32x4_a4*>(fb + max(rel0 + RD * i, lo));
        for (int r0 = 0; r0 < Rp; r0 += kPF) {
#pragma unroll
            for (int i = 0; i < kPF; ++i) {
                const int rel = rel0 + RD * (r0 + i);
                acc = (acc * 3) ^ pf[i].x ^ pf[i].y ^ pf[i].z ^ pf[i].w;
                const u32x4_a4* q = reinterpret_cast<const u32x4_a4*>(fb + max(min(rel + RD * kPF, rel_last), lo));
                pf[i] = NT ? __builtin_nontemporal_load(q) : *q;
            }
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// Same as k_frames but rows are 64-B aligned in memory (no row straddles a 128-B line):
// a frame covers blocks [S>>6, (E-1)>>6]; the partial head/tail blocks would be masked.
template <int kPF, int WPB = 16, int RB = 64>
__global__ void __launch_bounds__(64 * WPB) k_frames_al(const uint8_t* __restrict__ base, uint32_t nframes, uint32_t flen,
                                                        uint32_t* out) {
    constexpr int G = RB / 16, FPW = 64 / G;
    const uint32_t lane = threadIdx.x & 63, grp = lane / G, gl = lane % G;
    const uint32_t gwave = blockIdx.x * WPB + (threadIdx.x >> 6), nwaves = gridDim.x * WPB;
    const uint32_t ntiles = (nframes + FPW - 1) / FPW;
    uint32_t acc = 0;
    for (uint32_t t = gwave; t < ntiles; t += nwaves) {
        uint32_t f = t * FPW + grp;
        if (f >= nframes) f = nframes - 1;
        const uint64_t S = (uint64_t)f * flen, E = S + flen;
        const uint64_t b0 = S / RB, b1 = (E - 1) / RB;
        const int R = (int)(b1 - b0 + 1);
        const int Rp = (R + kPF - 1) / kPF * kPF;
        // row r (0..Rp-1) reads block b1 - (Rp-1-r), clamped to b0
        const u32x4* bl = reinterpret_cast<const u32x4*>(base) + b1 * (RB / 16) + gl;
        const int first = -(Rp - 1);  // relative block of row 0
        const int lo = -(R - 1);
        u32x4 pf[kPF];
#pragma unroll
        for (int i = 0; i < kPF; ++i) pf[i] = bl[(RB / 16) * max(first + i, lo)];
        for (int r0 = 0; r0 < Rp; r0 += kPF) {
#pragma unroll
            for (int i = 0; i < kPF; ++i) {
                const int rel = first + r0 + i;
                acc = (acc * 3) ^ pf[i].x ^ pf[i].y ^ pf[i].z ^ pf[i].w;
                pf[i] = bl[(RB / 16) * max(min(rel + kPF, 0), lo)];
            }
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// The frames pattern behind a descriptor load (offsets read from memory, as the digest
// kernel's first dependent round trip), with LDS reserved per workgroup so that 1 or 2
// workgroups fit a CU: for back-to-back launches on several streams, does a second
// resident workgroup hide one launch's start and tail behind another's rows?
template <int kPF, int WPB>
__global__ void __launch_bounds__(64 * WPB) k_frames_desc(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
                                                          uint32_t nframes, uint32_t flen, uint32_t* out) {
    extern __shared__ uint32_t lds_res[];
    constexpr int G = 4, FPW = 16, RD = 16;
    const uint32_t lane = threadIdx.x & 63, grp = lane / G, gl = lane % G;
    const uint32_t gwave = blockIdx.x * WPB + (threadIdx.x >> 6), nwaves = gridDim.x * WPB;
    const uint32_t ntiles = (nframes + FPW - 1) / FPW;
    uint32_t acc = 0;
    lds_res[threadIdx.x] = threadIdx.x;
    for (uint32_t t = gwave; t < ntiles; t += nwaves) {
        uint32_t f = t * FPW + grp;
        if (f >= nframes) f = nframes - 1;
        const uint64_t S = offs[f], E = S + flen;
        const uint64_t sdw = S >> 2;
        const int nd = (int)(((E + 3) >> 2) - sdw);
        const int R = (nd + RD - 1) / RD;
        const int Rp = (R + kPF - 1) / kPF * kPF;
        const int rel0 = nd - RD * Rp + 4 * (int)gl;
        const int rel_last = rel0 + RD * (Rp - 1);
        const uint32_t* fb = reinterpret_cast<const uint32_t*>(base + sdw * 4);
        const int lo = -(int)min(sdw, (uint64_t)(1 << 24));
        u32x4 pf[kPF];
#pragma unroll
        for (int i = 0; i < kPF; ++i) pf[i] = *reinterpret_cast<const u32x4_a4*>(fb + max(rel0 + RD * i, lo));
        for (int r0 = 0; r0 < Rp; r0 += kPF) {
#pragma unroll
            for (int i = 0; i < kPF; ++i) {
                const int rel = rel0 + RD * (r0 + i);
                acc = (acc * 3) ^ pf[i].x ^ pf[i].y ^ pf[i].z ^ pf[i].w;
                pf[i] = *reinterpret_cast<const u32x4_a4*>(fb + max(min(rel + RD * kPF, rel_last), lo));
            }
        }
    }
    __syncthreads();
    if (acc == 0x12345678u) out[0] = acc + lds_res[(threadIdx.x + 1) % (64 * WPB)];
}

// k_frames_al's aligned rows behind the same descriptor load, for the multi-stream runs.
template <int kPF, int WPB, int RB>
__global__ void __launch_bounds__(64 * WPB) k_frames_desc_al(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
                                                             uint32_t nframes, uint32_t flen, uint32_t* out) {
    extern __shared__ uint32_t lds_res[];
    constexpr int G = RB / 16, FPW = 64 / G;
    const uint32_t lane = threadIdx.x & 63, grp = lane / G, gl = lane % G;
    const uint32_t gwave = blockIdx.x * WPB + (threadIdx.x >> 6), nwaves = gridDim.x * WPB;
    const uint32_t ntiles = (nframes + FPW - 1) / FPW;
    uint32_t acc = 0;
    lds_res[threadIdx.x] = threadIdx.x;
    for (uint32_t t = gwave; t < ntiles; t += nwaves) {
        uint32_t f = t * FPW + grp;
        if (f >= nframes) f = nframes - 1;
        const uint64_t S = offs[f], E = S + flen;
        const uint64_t b0 = S / RB, b1 = (E - 1) / RB;
        const int R = (int)(b1 - b0 + 1);
        const int Rp = (R + kPF - 1) / kPF * kPF;
        const u32x4* bl = reinterpret_cast<const u32x4*>(base) + b1 * (RB / 16) + gl;
        const int first = -(Rp - 1), lo = -(R - 1);
        u32x4 pf[kPF];
#pragma unroll
        for (int i = 0; i < kPF; ++i) pf[i] = bl[(RB / 16) * max(first + i, lo)];
        for (int r0 = 0; r0 < Rp; r0 += kPF) {
#pragma unroll
            for (int i = 0; i < kPF; ++i) {
                const int rel = first + r0 + i;
                acc = (acc * 3) ^ pf[i].x ^ pf[i].y ^ pf[i].z ^ pf[i].w;
                pf[i] = bl[(RB / 16) * max(min(rel + kPF, 0), lo)];
            }
        }
    }
    __syncthreads();
    if (acc == 0x12345678u) out[0] = acc + lds_res[(threadIdx.x + 1) % (64 * WPB)];
}

int main(int argc, char** argv) {
    const size_t nbytes = argc > 1 ? (size_t)atoll(argv[1]) : 98304000;
    const int NB = (int)((1200000000ull + nbytes - 1) / nbytes) < 4 ? 4 : (int)((1200000000ull + nbytes - 1) / nbytes);
    const int iters = 50;
    std::vector<uint8_t*> bufs(NB);
    for (auto& b : bufs) {
        CHECK(hipMalloc(&b, nbytes + 4096));
        CHECK(hipMemset(b, 0x5a, nbytes + 4096));
    }
    uint32_t* out;
    CHECK(hipMalloc(&out, 64));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    int cus = prop.multiProcessorCount;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    printf("buffer %zu bytes, %d rotated\n", nbytes, NB);
    if (argc > 2 && std::string(argv[2]) == "streams") {
        // back-to-back launches of the descriptor-led pattern on 4 streams
        const uint32_t fl = 1500, nf = (uint32_t)(nbytes / fl);
        std::vector<uint64_t> h(nf);
        for (uint32_t i = 0; i < nf; ++i) h[i] = (uint64_t)i * fl;
        uint64_t* d_offs;
        CHECK(hipMalloc(&d_offs, nf * 8ull));
        CHECK(hipMemcpy(d_offs, h.data(), nf * 8ull, hipMemcpyHostToDevice));
        hipStream_t st[4];
        for (auto& x : st) CHECK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
        auto run = [&](auto kern, int wpb, int grid, size_t lds, int nstreams, const char* name) {
            CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            const int reps = 400;
            for (int pass = 0; pass < 2; ++pass) {
                CHECK(hipDeviceSynchronize());
                auto t0 = std::chrono::steady_clock::now();
                for (int i = 0; i < reps; ++i)
                    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * wpb), lds, st[i % nstreams], bufs[i % NB], d_offs, nf, fl, out);
                CHECK(hipDeviceSynchronize());
                const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
                if (pass) printf("%-52s %9.2f us/step  %8.1f GB/s whole job\n", name, us, nbytes / (us * 1e-6) / 1e9);
            }
        };
        for (int ns : {1, 4}) {
            char nm[160];
            snprintf(nm, sizeof nm, "desc 16 waves/WG, 150 KB LDS (1 WG/CU), %d stream(s)", ns);
            run(k_frames_desc<6, 16>, 16, cus, 150 * 1024, ns, nm);
            snprintf(nm, sizeof nm, "desc  8 waves/WG,  76 KB LDS (2 WG/CU), %d stream(s)", ns);
            run(k_frames_desc<6, 8>, 8, 2 * cus, 76 * 1024, ns, nm);
            snprintf(nm, sizeof nm, "desc  8 waves/WG, 150 KB LDS (1 WG/CU), %d stream(s)", ns);
            run(k_frames_desc<6, 8>, 8, 2 * cus, 150 * 1024, ns, nm);
            snprintf(nm, sizeof nm, "desc  4 waves/WG,  38 KB LDS (4 WG/CU), %d stream(s)", ns);
            run(k_frames_desc<6, 4>, 4, 4 * cus, 38 * 1024, ns, nm);
            snprintf(nm, sizeof nm, "desc aligned64 16 waves/WG, 150 KB LDS, %d stream(s)", ns);
            run(k_frames_desc_al<6, 16, 64>, 16, cus, 150 * 1024, ns, nm);
            snprintf(nm, sizeof nm, "desc aligned128 16 waves/WG, 150 KB LDS, %d stream(s)", ns);
            run(k_frames_desc_al<4, 16, 128>, 16, cus, 150 * 1024, ns, nm);
        }
        for (int ns : {1, 4}) {
            const int reps = 400;
            for (int pass = 0; pass < 2; ++pass) {
                CHECK(hipDeviceSynchronize());
                auto t0 = std::chrono::steady_clock::now();
                for (int i = 0; i < reps; ++i)
                    hipLaunchKernelGGL(k_stream<false>, dim3(cus * 2), dim3(256), 0, st[i % ns], (const u32x4*)bufs[i % NB], nbytes / 16, out);
                CHECK(hipDeviceSynchronize());
                const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
                if (pass) printf("stream dwordx4 grid=%dx256, %d stream(s)                %9.2f us/step  %8.1f GB/s whole job\n", cus * 2, ns, us, nbytes / (us * 1e-6) / 1e9);
            }
        }
        return 0;
    }
    auto timeit = [&](auto launch, const char* name) {
        for (int i = 0; i < 10; ++i) launch(i);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        for (int i = 0; i < iters; ++i) launch(i);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        double us = ms * 1e3 / iters;
        printf("%-44s %9.2f us/launch  %8.1f GB/s\n", name, us, nbytes / (us * 1e-6) / 1e9);
    };
    for (int mult : {2, 4, 8}) {
        char nm[128];
        snprintf(nm, sizeof nm, "stream dwordx4 grid=%dx%d", cus * mult, 256);
        timeit([&](int i) { hipLaunchKernelGGL(k_stream<false>, dim3(cus * mult), dim3(256), 0, 0,
                                               (const u32x4*)bufs[i % NB], nbytes / 16, out); }, nm);
        snprintf(nm, sizeof nm, "stream dwordx4 nt grid=%dx%d", cus * mult, 256);
        timeit([&](int i) { hipLaunchKernelGGL(k_stream<true>, dim3(cus * mult), dim3(256), 0, 0,
                                               (const u32x4*)bufs[i % NB], nbytes / 16, out); }, nm);
    }
    const uint32_t fl = 1500, nf = (uint32_t)(nbytes / fl);
#define FR(PF, G, NT, GRID, NAME) timeit([&](int i) { hipLaunchKernelGGL((k_frames<PF, G, NT>), dim3(GRID), dim3(1024), 0, 0, bufs[i % NB], nf, fl, out); }, NAME)
    FR(6, 1, false, cus, "frames G=1  PF=6");
    FR(8, 1, false, cus, "frames G=1  PF=8");
    FR(12, 1, false, cus, "frames G=1  PF=12");
    FR(6, 2, false, cus, "frames G=2  PF=6");
    FR(6, 4, false, cus, "frames G=4  PF=6");
    FR(6, 4, true, cus, "frames G=4  PF=6 nt");
    FR(4, 16, false, cus, "frames G=16 PF=4");
    FR(4, 16, true, cus, "frames G=16 PF=4 nt");
    FR(2, 64, false, cus, "frames G=64 PF=2");
    FR(2, 64, true, cus, "frames G=64 PF=2 nt");
    // fewer waves per CU (one block of WPB waves per CU), deeper rings
#define FRW(PF, WPB, NAME) timeit([&](int i) { hipLaunchKernelGGL((k_frames<PF, 4, false, WPB>), dim3(cus), dim3(64 * WPB), 0, 0, bufs[i % NB], nf, fl, out); }, NAME)
    FRW(6, 16, "frames G=4  PF=6  16 waves/CU");
    FRW(12, 8, "frames G=4  PF=12 8 waves/CU");
    FRW(8, 8, "frames G=4  PF=8  8 waves/CU");
    FRW(6, 8, "frames G=4  PF=6  8 waves/CU");
    FRW(16, 4, "frames G=4  PF=16 4 waves/CU");
    FRW(12, 12, "frames G=4  PF=12 12 waves/CU");
#define FRA(PF, WPB, RB, NAME) timeit([&](int i) { hipLaunchKernelGGL((k_frames_al<PF, WPB, RB>), dim3(cus), dim3(64 * WPB), 0, 0, bufs[i % NB], nf, fl, out); }, NAME)
    FRA(6, 16, 64, "aligned64 G=4 PF=6 16 waves/CU");
    FRA(8, 16, 64, "aligned64 G=4 PF=8 16 waves/CU");
    FRA(4, 16, 64, "aligned64 G=4 PF=4 16 waves/CU");
    FRA(12, 8, 64, "aligned64 G=4 PF=12 8 waves/CU");
    FRA(4, 16, 128, "aligned128 G=8 PF=4 16 waves/CU");
    FRA(3, 16, 128, "aligned128 G=8 PF=3 16 waves/CU");
    FRA(6, 8, 128, "aligned128 G=8 PF=6 8 waves/CU");
    FRW(6, 16, "frames G=4  PF=6  16 waves/CU (again)");
    return 0;
}
