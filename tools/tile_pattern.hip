// Access-pattern microbenchmark for the digest kernel's decomposition (measurement tool, no
// CRC compute): persistent waves stream tiles of 64/G consecutive 1500-B frames (packed back
// to back, as the C2/C4 batches), G lanes per frame, rows of 16*G bytes, a ring of PF row
// loads per wave that runs on across tiles (no drain at tile ends). Rows either aligned to
// their size in memory (AL = 1: full 128-B lines for G >= 8; the partial head and tail rows'
// lanes outside the frame issue no load; AL = 2: whole blocks, every lane loads -- the one-pass
// kernel's block-aligned rows for G = 4) or anchored at the frame end (AL = 0, the end-anchored
// rows). Compared with a plain grid-stride stream, on a 98.3 MB C2 batch (one launch) and a
// 1.57 GB C4 batch (steady state), on 1 and 4 streams. `tile_pattern calib`: the FETCH_SIZE
// calibration set (run under rocprofv3 --pmc FETCH_SIZE).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) {                                                            \
            printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__);                     \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

// MAP 0: a wave's tiles are grid-strided (tile gwave + k nwaves); MAP 1: a wave's tiles are
// consecutive (the wave's share of the batch, 4 consecutive tiles per wave for C2 with G = 16)
template <int G, int PF, int AL, int WPB, int MAP = 0>
__global__ void __launch_bounds__(64 * WPB) k_tiles(const uint8_t* __restrict__ base, uint32_t nframes, uint32_t flen,
                                                    uint32_t* out, uint32_t delay_10ns = 0) {
    constexpr int FPT = 64 / G;
    if (delay_10ns) {  // `ovl`: a start phase of this length (the digest kernel's tables and geometry)
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < delay_10ns) __builtin_amdgcn_s_sleep(2);
    }
    constexpr uint32_t RB = 16u * G;
    const uint32_t lane = threadIdx.x & 63u, grp = lane / G, gl = lane % G;
    const uint32_t gwave = (threadIdx.x >> 6) * gridDim.x + blockIdx.x;  // wave-major
    const uint32_t nwaves = gridDim.x * WPB;
    const uint32_t ntiles = (nframes + FPT - 1) / FPT;
    const uint32_t my_tiles = gwave < ntiles ? (ntiles - gwave + nwaves - 1) / nwaves : 0;
    // AL 4 (G = 16): 256-B rows of 4 whole 64-B blocks, the last row ending with the frame's last
    // block (the one-pass kernel's block-aligned rows, 4 blocks per row); blocks before the frame's
    // first block reload that block's chunk, as the kernel's clamped loads do
    const int Rmax = AL == 4 ? (int)(((flen + 63) / 64 + 1 + 3) / 4)
                     : AL ? (int)((flen + RB - 1) / RB + 1) : (int)((flen + RB - 1) / RB);
    const int nq = (int)my_tiles * Rmax;
    // address of flattened row q for this lane; false if the lane loads nothing
    auto addr = [&](int q, const u32x4_a4*& p) -> bool {
        const int k = q / Rmax, r = q - k * Rmax;
        const uint32_t f = (MAP ? gwave * my_tiles + (uint32_t)k : gwave + (uint32_t)k * nwaves) * FPT + grp;
        if (f >= nframes) return false;
        const uint64_t S = (uint64_t)f * flen, E = S + flen;
        uint64_t a;
        if (AL == 4) {
            const int64_t b0 = (int64_t)(S / 64), b1 = (int64_t)((E - 1) / 64);
            const int64_t b = b1 - 4 * (Rmax - 1 - r) - 3 + (int64_t)(gl >> 2);
            a = (uint64_t)(b < b0 ? b0 : b) * 64u + 16u * (gl & 3u);
        } else if (AL) {
            const uint64_t b0 = S / RB, b1 = (E - 1) / RB;
            if (b0 + (uint64_t)r > b1) return false;
            // AL 3: whole blocks, the odd groups' frames read backwards (last block first), so the
            // 128-B line a frame shares with the next one is read by both at the same time
            a = ((AL == 3 && (grp & 1u)) ? b1 - r : b0 + r) * RB + 16u * gl;
            if (AL == 1 && (a + 16 <= S || a >= E)) return false;  // AL 2: whole blocks, as the kernel loads
        } else {
            const uint64_t E4 = (E + 3) & ~uint64_t(3);
            const int64_t s = (int64_t)E4 - (int64_t)RB * (Rmax - r) + 16 * (int64_t)gl;
            if (s + 16 <= (int64_t)S) return false;
            a = (uint64_t)(s < (int64_t)S ? (int64_t)(S & ~uint64_t(3)) : s);
        }
        p = reinterpret_cast<const u32x4_a4*>(base + a);
        return true;
    };
    uint32_t acc = 0;
    u32x4 pf[PF];
#pragma unroll
    for (int i = 0; i < PF; ++i) {
        const u32x4_a4* p;
        pf[i] = (i < nq && addr(i, p)) ? *p : u32x4{0, 0, 0, 0};
    }
    for (int q0 = 0; q0 < nq; q0 += PF) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            acc = (acc * 3u) ^ pf[i].x ^ pf[i].y ^ pf[i].z ^ pf[i].w;
            const int qn = q0 + i + PF;
            const u32x4_a4* p;
            if (qn < nq && addr(qn, p)) pf[i] = *p;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// `burst`: the one-pass kernel's pattern (4 lanes per frame, 64-B block-aligned whole blocks,
// AL 2) with the ring refilled in BURSTS: H slices of B rows; a slice's B rows are consumed,
// then re-issued back to back, so each frame's next B blocks (64 B each) reach the memory system
// together. B = 1 is the per-row refill the kernel uses (ring H rows).
template <int B, int H, int WPB>
__global__ void __launch_bounds__(64 * WPB) k_burst(const uint8_t* __restrict__ base, uint32_t nframes, uint32_t flen,
                                                    uint32_t* out) {
    constexpr int G = 4, FPT = 16, PF = B * H;
    constexpr uint32_t RB = 64u;
    const uint32_t lane = threadIdx.x & 63u, grp = lane / G, gl = lane % G;
    const uint32_t gwave = (threadIdx.x >> 6) * gridDim.x + blockIdx.x;
    const uint32_t nwaves = gridDim.x * WPB;
    const uint32_t ntiles = (nframes + FPT - 1) / FPT;
    const uint32_t my_tiles = gwave < ntiles ? (ntiles - gwave + nwaves - 1) / nwaves : 0;
    const int Rmax = (int)((flen + RB - 1) / RB + 1);
    const int nq = (int)my_tiles * Rmax;
    auto addr = [&](int q, const u32x4_a4*& p) -> bool {
        const int k = q / Rmax, r = q - k * Rmax;
        const uint32_t f = (gwave + (uint32_t)k * nwaves) * FPT + grp;
        if (f >= nframes) return false;
        const uint64_t S = (uint64_t)f * flen, E = S + flen;
        const uint64_t b0 = S / RB, b1 = (E - 1) / RB;
        if (b0 + (uint64_t)r > b1) return false;
        p = reinterpret_cast<const u32x4_a4*>(base + (b0 + r) * RB + 16u * gl);
        return true;
    };
    uint32_t acc = 0;
    u32x4 pf[PF];
#pragma unroll
    for (int i = 0; i < PF; ++i) {
        const u32x4_a4* p;
        pf[i] = (i < nq && addr(i, p)) ? *p : u32x4{0, 0, 0, 0};
    }
    for (int q0 = 0; q0 < nq; q0 += PF) {
#pragma unroll
        for (int h = 0; h < H; ++h) {
#pragma unroll
            for (int b = 0; b < B; ++b) {
                const u32x4 v = pf[h * B + b];
                acc = (acc * 3u) ^ v.x ^ v.y ^ v.z ^ v.w;
            }
#pragma unroll
            for (int b = 0; b < B; ++b) {
                const int qn = q0 + h * B + b + PF;
                const u32x4_a4* p;
                if (qn < nq && addr(qn, p)) pf[h * B + b] = *p;
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// `super`: 16 frames per wave as the kernel, but LOADED 16 lanes per frame: a super-row is 4
// blocks (256 B) of each of the 16 frames, 4 load instructions, instruction i covering frames
// 4i .. 4i+3 (lane L: frame 4i + L/16, block 4r + (L%16)/4 from the frame's first block, chunk
// L%4; blocks past the frame's last reload it). TR = 1 transposes each super-row through LDS
// (ds_write_b128 lane-linear, ds_read_b128) into the 4-lanes-per-frame layout the digest
// kernel computes on (register b, lane 16k + 4j + gl = frame 4k + j, block b, chunk gl).
// S super-rows in flight.
template <int S, int TR>
__global__ void __launch_bounds__(1024) k_super(const uint8_t* __restrict__ base, uint32_t nframes, uint32_t flen,
                                                uint32_t* out) {
    __shared__ u32x4 stage[16][4][64];
    constexpr int FPT = 16;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t gwave = wave * gridDim.x + blockIdx.x;
    const uint32_t nwaves = gridDim.x * 16u;
    const uint32_t ntiles = (nframes + FPT - 1) / FPT;
    const uint32_t my_tiles = gwave < ntiles ? (ntiles - gwave + nwaves - 1) / nwaves : 0;
    const int Rs = (int)(((flen + 63u) / 64u + 1u + 3u) / 4u);  // super-rows per tile (max blocks / 4)
    const int nq = (int)my_tiles * Rs;
    const uint32_t fq = lane >> 4, blk = (lane >> 2) & 3u, ch = lane & 3u;
    auto addr = [&](int q, int i, const u32x4_a4*& p) -> bool {
        const int k = q / Rs, r = q - k * Rs;
        const uint32_t f = (gwave + (uint32_t)k * nwaves) * FPT + 4u * (uint32_t)i + fq;
        if (f >= nframes) return false;
        const uint64_t S0 = (uint64_t)f * flen, E = S0 + flen;
        const uint64_t b0 = S0 / 64u, b1 = (E - 1) / 64u;
        uint64_t b = b0 + 4u * (uint64_t)r + blk;
        if (b > b1) b = b1;
        p = reinterpret_cast<const u32x4_a4*>(base + b * 64u + 16u * ch);
        return true;
    };
    uint32_t acc = 0;
    u32x4 pf[S][4];
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const u32x4_a4* p;
            pf[s][i] = (s < nq && addr(s, i, p)) ? *p : u32x4{0, 0, 0, 0};
        }
    for (int q0 = 0; q0 < nq; q0 += S) {
#pragma unroll
        for (int s = 0; s < S; ++s) {
            if (TR) {
#pragma unroll
                for (int i = 0; i < 4; ++i) stage[wave][i][lane] = pf[s][i];
                // R_b at lane 16k + 4j + gl <- X_k at lane 16j + 4b + gl
                const uint32_t k = lane >> 4, j = (lane >> 2) & 3u, gl = lane & 3u;
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const u32x4 v = stage[wave][k][16u * j + 4u * (uint32_t)b + gl];
                    acc = (acc * 3u) ^ v.x ^ v.y ^ v.z ^ v.w;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) acc = (acc * 3u) ^ pf[s][i].x ^ pf[s][i].y ^ pf[s][i].z ^ pf[s][i].w;
            }
            const int qn = q0 + s + S;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const u32x4_a4* p;
                if (qn < nq && addr(qn, i, p)) pf[s][i] = *p;
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int PF, int WPB>
__global__ void __launch_bounds__(64 * WPB) k_stream(const u32x4* __restrict__ p, size_t n16, uint32_t* out) {
    uint32_t acc = 0;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (PF - 1) * stride < n16; i += PF * stride) {
        u32x4 v[PF];
#pragma unroll
        for (int k = 0; k < PF; ++k) v[k] = p[i + k * stride];
#pragma unroll
        for (int k = 0; k < PF; ++k) acc = (acc * 3u) ^ v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    for (; i < n16; i += stride) {
        const u32x4 a = p[i];
        acc ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
    // `dir [flen]`: forward-only (AL 2) against alternating-direction (AL 3) whole blocks
    const bool dir = argc > 1 && std::string(argv[1]).rfind("dir", 0) == 0;
    const uint32_t flen = dir && argc > 2 ? (uint32_t)atoi(argv[2]) : 1500;
    const bool big = argc > 1 && std::string(argv[1]) == "c4";
    const uint32_t nf = big ? (1u << 20) : (uint32_t)(98304000ull / flen);
    const size_t nbytes = (size_t)nf * flen;
    const bool calib = argc > 1 && std::string(argv[1]) == "calib";
    const int NB = big ? 2 : 6;
    std::vector<uint8_t*> bufs(NB);
    for (auto& b : bufs) {
        CHECK(hipMalloc(&b, nbytes + 4096));
        CHECK(hipMemset(b, 0x5a, nbytes + 4096));
    }
    uint32_t* out;
    CHECK(hipMalloc(&out, 64));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    hipStream_t st[5];
    for (auto& x : st) CHECK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    printf("batch %u x %u B = %zu bytes, %d rotated, %d CUs\n", nf, flen, nbytes, NB, cus);
    const bool dircal = argc > 1 && std::string(argv[1]) == "dircal";
    const int reps = big ? 40 : (calib || dircal) ? 20 : 400;
    auto run = [&](auto launch, const char* name) {
        double res[2];
        int k = 0;
        for (int ns : {1, 4}) {
            for (int pass = 0; pass < 2; ++pass) {
                CHECK(hipDeviceSynchronize());
                auto t0 = std::chrono::steady_clock::now();
                for (int i = 0; i < reps; ++i) launch(i, st[i % ns]);
                CHECK(hipDeviceSynchronize());
                res[k] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
            }
            ++k;
        }
        printf("%-44s 1 stream %9.2f us %7.0f GB/s | 4 streams %9.2f us %7.0f GB/s\n", name, res[0],
               nbytes / (res[0] * 1e-6) / 1e9, res[1], nbytes / (res[1] * 1e-6) / 1e9);
    };
#define TILES(G, PF, AL, WPB) TILESX(G, PF, AL, WPB, 1)
#define TILESX(G, PF, AL, WPB, GM)                                                                        \
    run([&](int i, hipStream_t s) {                                                                       \
        hipLaunchKernelGGL((k_tiles<G, PF, AL, WPB>), dim3(cus * GM), dim3(64 * WPB), 0, s, bufs[i % NB], nf, flen, out); \
    }, "tiles G=" #G " PF=" #PF " AL=" #AL " waves/WG=" #WPB " WG/CU=" #GM)
#define STREAM(PF, WPB, GRIDMUL)                                                                          \
    run([&](int i, hipStream_t s) {                                                                       \
        hipLaunchKernelGGL((k_stream<PF, WPB>), dim3(cus * GRIDMUL), dim3(64 * WPB), 0, s,                \
                           (const u32x4*)bufs[i % NB], nbytes / 16, out);                                 \
    }, "stream PF=" #PF " waves/WG=" #WPB " WG/CU=" #GRIDMUL)
    if (argc > 1 && std::string(argv[1]) == "ovl") {
        // overlap of consecutive launches when a start phase precedes the rows: one 16-wave
        // workgroup per CU (LDS-bound, as the digest kernel) against two 8-wave workgroups
        auto ovl = [&](int wpb, size_t lds, uint32_t delay, const char* name) {
            double res[2];
            int k = 0;
            for (int ns : {1, 5}) {
                for (int pass = 0; pass < 2; ++pass) {
                    CHECK(hipDeviceSynchronize());
                    auto t0 = std::chrono::steady_clock::now();
                    for (int i = 0; i < reps; ++i) {
                        if (wpb == 16)
                            hipLaunchKernelGGL((k_tiles<4, 5, 2, 16>), dim3(cus), dim3(1024), lds, st[i % ns],
                                               bufs[i % NB], nf, flen, out, delay);
                        else
                            hipLaunchKernelGGL((k_tiles<4, 5, 2, 8>), dim3(cus * 2), dim3(512), lds, st[i % ns],
                                               bufs[i % NB], nf, flen, out, delay);
                    }
                    CHECK(hipDeviceSynchronize());
                    res[k] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
                }
                ++k;
            }
            printf("%-44s 1 stream %9.2f us %7.0f GB/s | 5 streams %9.2f us %7.0f GB/s\n", name, res[0],
                   nbytes / (res[0] * 1e-6) / 1e9, res[1], nbytes / (res[1] * 1e-6) / 1e9);
        };
        CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_tiles<4, 5, 2, 16>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
        CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_tiles<4, 5, 2, 8>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024));
        for (int rep = 0; rep < 2; ++rep) {
            for (uint32_t d : {0u, 300u, 500u}) {
                char nm[96];
                snprintf(nm, sizeof nm, "16 waves, 150 KB, 1 WG/CU, start %u ns", d * 10);
                ovl(16, 150 * 1024, d, nm);
                snprintf(nm, sizeof nm, "8 waves, 80 KB, 2 WG/CU, start %u ns", d * 10);
                ovl(8, 80 * 1024, d, nm);
            }
        }
        return 0;
    }
#define TILESM(G, PF, AL, MAP)                                                                             \
    run([&](int i, hipStream_t s) {                                                                       \
        hipLaunchKernelGGL((k_tiles<G, PF, AL, 16, MAP>), dim3(cus), dim3(1024), 0, s, bufs[i % NB], nf, flen, out); \
    }, "tiles G=" #G " PF=" #PF " AL=" #AL " MAP=" #MAP)
    if (argc > 1 && std::string(argv[1]) == "map") {
        for (int rep = 0; rep < 2; ++rep) {
            STREAM(4, 16, 1);
            TILESM(4, 5, 2, 0);
            TILESM(16, 6, 0, 0);
            TILESM(16, 6, 0, 1);
            TILESM(16, 5, 0, 0);
            TILESM(16, 5, 0, 1);
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "w4") {
        // round 4: 16 lanes per frame with rows of 4 whole 64-B blocks end-anchored at the frame's
        // last block (AL 4), against the one-pass kernel's pattern and 256-B end-anchored rows
        for (int rep = 0; rep < 2; ++rep) {
            STREAM(4, 16, 1);
            TILESM(4, 5, 2, 0);
            TILESM(16, 6, 0, 0);
            TILESM(16, 5, 4, 0);
            TILESM(16, 6, 4, 0);
            TILESM(16, 7, 4, 0);
            TILESM(16, 8, 4, 0);
            TILESM(16, 7, 4, 1);
            TILESM(16, 7, 2, 0);
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "super") {
#define SUPER(S, TR)                                                                                        \
    run([&](int i, hipStream_t s) {                                                                       \
        hipLaunchKernelGGL((k_super<S, TR>), dim3(cus), dim3(1024), 0, s, bufs[i % NB], nf, flen, out); \
    }, "super S=" #S " TR=" #TR)
        for (int rep = 0; rep < 2; ++rep) {
            STREAM(4, 16, 1);
            TILES(4, 5, 2, 16);
            TILES(16, 6, false, 16);
            SUPER(1, 0);
            SUPER(2, 0);
            SUPER(3, 0);
            SUPER(1, 1);
            SUPER(2, 1);
            SUPER(3, 1);
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "burst") {
#define BURST(B, H)                                                                                        \
    run([&](int i, hipStream_t s) {                                                                       \
        hipLaunchKernelGGL((k_burst<B, H, 16>), dim3(cus), dim3(1024), 0, s, bufs[i % NB], nf, flen, out); \
    }, "burst B=" #B " H=" #H " (ring " #B "x" #H ")")
        for (int rep = 0; rep < 2; ++rep) {
            STREAM(4, 16, 1);
            TILES(4, 5, 2, 16);
            BURST(1, 5);
            BURST(5, 2);
            BURST(4, 2);
            BURST(3, 2);
            BURST(2, 3);
            BURST(2, 4);
            BURST(4, 3);
            BURST(8, 2);
        }
        return 0;
    }
    if (dir) {
        STREAM(4, 16, 1);
        TILES(4, 5, 2, 16);
        TILES(4, 5, 3, 16);
        TILES(4, 5, 2, 16);
        TILES(4, 5, 3, 16);
        return 0;
    }
    if (calib) {  // FETCH_SIZE calibration under rocprofv3 (98,304,000 B per launch)
        STREAM(4, 16, 1);
        TILES(4, 5, 2, 16);
        TILES(4, 6, 0, 16);
        return 0;
    }
    STREAM(4, 4, 2);
    STREAM(4, 16, 1);
    TILES(4, 5, 2, 16);
    TILES(4, 6, false, 16);
    TILES(4, 5, true, 16);
    TILESX(4, 5, true, 16, 2);
    TILESX(4, 5, true, 8, 2);
    TILESX(4, 5, true, 8, 4);
    TILES(4, 10, true, 16);
    TILESX(4, 10, true, 8, 2);
    TILESX(4, 5, false, 16, 2);
    TILES(16, 6, false, 16);
    TILESX(16, 4, false, 16, 2);
    return 0;
}
