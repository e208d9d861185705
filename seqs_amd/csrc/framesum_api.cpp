// framesum C ABI (include/framesum.h) — context management, device-resident and
// host-staged batch entry points. No CPU fallback: every digest is computed by
// the gfx950 kernel (framesum_kernel.hip); a missing/unsupported device is an error.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <system_error>
#include <string>
#include <thread>
#include <vector>

#include "../../include/framesum.h"
#include "framesum_internal.h"
#include "framesum_plan.h"

using framesum::FsTables;

// Host-staged path: the batch is cut into chunks of about kChunkBytes of frame bytes,
// staged through kHostSlots device buffers. The whole batch's descriptors go first, in one
// H2D copy; the chunks' frame bytes then alternate between two copy streams (two DMA queues
// keep the PCIe link busier than one: no gap between one chunk's copy and the next); kernels
// and the small D2H copies run on a compute stream. Events order each chunk's kernel after
// its copy (`copied`) and the reuse of a slot by chunk c + kHostSlots after chunk c's kernel
// (`consumed`), so chunk c+1's H2D overlaps chunk c's kernel and D2H.
constexpr int kHostSlots = 3;
constexpr uint64_t kChunkBytes = 16ull << 20;
constexpr uint32_t kChunkFrames = 1u << 20;
// Frames per call: tile and frame indices are 32-bit in the kernel (n + 15 must not wrap).
constexpr uint32_t kMaxFrames = 1u << 31;

struct HostSlot {
    hipEvent_t copied = nullptr, consumed = nullptr, landed = nullptr;  // landed: the chunk's results are in the mirror
    bool used = false;
    uint8_t* d_frames = nullptr;
    uint64_t cap_frames = 0;
    uint64_t* d_offsets = nullptr;
    uint32_t* d_lengths = nullptr;
    fs_digest* d_out = nullptr;
    uint8_t* d_status = nullptr;
    uint32_t cap_n = 0;
};

struct fs_ctx {
    int device = 0;
    int num_cus = 0;
    FsTables* d_tables = nullptr;
    // fault injection for the host-staged pipeline's tests, settable only through the test
    // library's fs_test_set_fault (-DFS_TEST_HOOKS): fs_digest_batch_host fails with FS_E_NOMEM at
    // chunk k, after the earlier chunks' work and chunk k's copy are queued. -1 in the product.
    long fault_chunk = -1;
    // the path the latest fs_digest_batch_host took (fs_test_last_host_path): 1 staged in one
    // chunk, 2 read in place, 3 chunked
    int last_host_path = 0;
    // host-mapped word the kernels set when a batch has widely mixed lengths (launch_digest)
    volatile uint32_t* h_report = nullptr;
    uint32_t* d_report = nullptr;
    int force_kernel = 0;  // fs_ctx_set_kernel
    int workgroups = 0;    // fs_ctx_set_workgroups (0: one per CU)
    uint32_t next_launch_id = 1;  // the context's launch sequence (launch_digest: report ids, sticky window)
    HostSlot slot[kHostSlots];
    hipStream_t copy_stream = nullptr, compute_stream = nullptr;
    hipStream_t copy_stream2 = nullptr;  // the odd chunks' frame copies
    hipEvent_t desc_copied = nullptr;    // the batch's descriptors are on the device
    hipEvent_t host_done = nullptr;      // a host-staged call's last device work (polled, host_wait)
    // a host-staged call left work in flight (it failed half-way): the next one drains the
    // context's streams first (quiesce_host_streams); a call that returns FS_SUCCESS leaves none
    bool host_dirty = false;
    uint8_t* d_desc = nullptr;           // the batch's offsets (8 n) then lengths (4 n)
    uint64_t cap_desc_n = 0;
    // pinned host mirrors of the descriptors and results, so every per-chunk copy is
    // asynchronous even when the caller's arrays are pageable (Go slices, numpy)
    uint8_t* h_pin = nullptr;
    uint8_t* d_pin = nullptr;  // h_pin as the device addresses it (mapped): kernels write results there
    uint64_t cap_pin_n = 0;
    std::string err;
};

namespace {

thread_local std::string g_create_err;

fs_status set_err(fs_ctx* ctx, fs_status code, const std::string& msg) {
    if (ctx) ctx->err = msg;
    else g_create_err = msg;
    return code;
}

fs_status hip_err(fs_ctx* ctx, hipError_t e, const char* what) {
    return set_err(ctx, FS_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define FS_HIP(ctx, call)                                   \
    do {                                                    \
        hipError_t e_ = (call);                             \
        if (e_ != hipSuccess) return hip_err(ctx, e_, #call); \
    } while (0)

// Grow-only staging of one slot; a slot being regrown first waits for its last kernel.
fs_status ensure_slot(fs_ctx* ctx, HostSlot& sl, uint64_t frame_bytes, uint32_t n) {
    if (frame_bytes > sl.cap_frames) {
        if (sl.used) FS_HIP(ctx, hipEventSynchronize(sl.consumed));
        (void)hipFree(sl.d_frames);
        sl.d_frames = nullptr;
        sl.cap_frames = 0;
        const uint64_t cap = frame_bytes + 256;
        if (hipMalloc(&sl.d_frames, cap) != hipSuccess) return set_err(ctx, FS_E_NOMEM, "hipMalloc frames staging");
        sl.cap_frames = cap;
    }
    if (n > sl.cap_n) {
        if (sl.used) FS_HIP(ctx, hipEventSynchronize(sl.consumed));
        (void)hipFree(sl.d_offsets);
        (void)hipFree(sl.d_lengths);
        (void)hipFree(sl.d_out);
        (void)hipFree(sl.d_status);
        sl.d_offsets = nullptr;
        sl.d_lengths = nullptr;
        sl.d_out = nullptr;
        sl.d_status = nullptr;
        sl.cap_n = 0;
        if (hipMalloc(&sl.d_offsets, (size_t)n * 8) != hipSuccess || hipMalloc(&sl.d_lengths, (size_t)n * 4) != hipSuccess ||
            hipMalloc(&sl.d_out, (size_t)n * (sizeof(fs_digest) + 1)) != hipSuccess ||
            hipMalloc(&sl.d_status, (size_t)n) != hipSuccess)
            return set_err(ctx, FS_E_NOMEM, "hipMalloc descriptor staging");
        sl.cap_n = n;
    }
    return FS_SUCCESS;
}

// h_pin layout for n frames: offsets (8n) | lengths (4n) | digests (8n) | status (n)
fs_status ensure_desc(fs_ctx* ctx, uint32_t n) {
    if (n <= ctx->cap_desc_n) return FS_SUCCESS;
    (void)hipFree(ctx->d_desc);  // the previous call's kernels have ended (callers synchronize first)
    ctx->d_desc = nullptr;
    ctx->cap_desc_n = 0;
    if (hipMalloc(&ctx->d_desc, (size_t)n * 12 + 64) != hipSuccess) return set_err(ctx, FS_E_NOMEM, "hipMalloc descriptors");
    ctx->cap_desc_n = n;
    return FS_SUCCESS;
}

fs_status ensure_pinned(fs_ctx* ctx, uint32_t n) {
    if (n <= ctx->cap_pin_n) return FS_SUCCESS;
    if (ctx->h_pin) FS_HIP(ctx, hipHostFree(ctx->h_pin));
    ctx->h_pin = nullptr;
    ctx->d_pin = nullptr;
    ctx->cap_pin_n = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&ctx->h_pin), (size_t)n * 21 + 64, hipHostMallocMapped) != hipSuccess)
        return set_err(ctx, FS_E_NOMEM, "hipHostMalloc descriptor mirror");
    if (hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->d_pin), ctx->h_pin, 0) != hipSuccess) {
        (void)hipHostFree(ctx->h_pin);
        ctx->h_pin = nullptr;
        return set_err(ctx, FS_E_HIP, "hipHostGetDevicePointer of the descriptor mirror");
    }
    ctx->cap_pin_n = n;
    return FS_SUCCESS;
}

// Every host-staged entry point starts here: the pinned mirrors and the staging slots are free
// only once the context's compute stream AND both copy streams are idle (a host-staged call that
// failed half-way may have left odd-chunk copies in flight on copy_stream2 that would otherwise
// write a slot while the next call stages into it). A call that succeeded left nothing in flight
// (its results were waited for), so the three synchronizes (~3 us each when idle) run only after
// a failed call.
fs_status quiesce_host_streams(fs_ctx* ctx) {
    if (!ctx->host_dirty) return FS_SUCCESS;
    FS_HIP(ctx, hipStreamSynchronize(ctx->compute_stream));
    FS_HIP(ctx, hipStreamSynchronize(ctx->copy_stream));
    FS_HIP(ctx, hipStreamSynchronize(ctx->copy_stream2));
    ctx->host_dirty = false;
    return FS_SUCCESS;
}

// A host-staged call that fails after it has enqueued work drains the context's streams before it
// returns (best effort), so that nothing of it still reads the caller's buffers or writes the
// caller's result arrays (the kernel writes them in place when they are pinned) after the error.
void drain_host_streams(fs_ctx* ctx) {
    const bool ok = hipStreamSynchronize(ctx->compute_stream) == hipSuccess &&
                    hipStreamSynchronize(ctx->copy_stream) == hipSuccess &&
                    hipStreamSynchronize(ctx->copy_stream2) == hipSuccess;
    if (ok) ctx->host_dirty = false;
}
#define FS_HIP_DRAIN(ctx, call)                  \
    do {                                         \
        hipError_t e_ = (call);                  \
        if (e_ != hipSuccess) {                  \
            drain_host_streams(ctx);             \
            return hip_err(ctx, e_, #call);      \
        }                                        \
    } while (0)

// Wait on the host for `ev` by polling: HIP's blocking wait wakes the host about 25 us after the
// work ends, a third of a short host-staged call. After 2 ms of polling (a long
// batch) it falls back to the blocking wait instead of burning the core.
hipError_t host_wait(hipEvent_t ev) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e != hipErrorNotReady) return e;
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) return hipEventSynchronize(ev);
    }
}

// Is [p, p + bytes) inside ONE page-locked host allocation the GPU can copy from / to asynchronously
// (fs_host_alloc, hipHostMalloc, hipHostRegister)? Then a host-staged call copies straight from / to
// it, or has the kernel read or write it in place, instead of going through the context's pinned
// mirror. The whole span is checked, not only its start: a DMA or a kernel access past the end of a
// pinned allocation would fault the GPU, where the mirror path's host memcpy stays on the host.
bool is_pinned(const void* p, size_t bytes) {
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: not an error of the call
        return false;
    }
    if (a.type != hipMemoryTypeHost) return false;
    void* start = nullptr;
    size_t size = 0;
    if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, const_cast<void*>(p)) != hipSuccess ||
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, const_cast<void*>(p)) != hipSuccess) {
        (void)hipGetLastError();
        return false;  // the span cannot be checked: take the mirror path
    }
    const uintptr_t b = reinterpret_cast<uintptr_t>(start), q = reinterpret_cast<uintptr_t>(p);
    return q >= b && bytes <= size && q - b <= size - bytes;
}

// One launch of the context's kernel choice.
// `force` < 0: the context's kernel choice (fs_ctx_set_kernel).
hipError_t launch(fs_ctx* ctx, const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths, uint32_t n,
                  uint32_t mtu, fs_digest* out, uint8_t* status, hipStream_t stream, framesum::FsOp op,
                  uint8_t* wframes, uint32_t tx, int force = -1) {
    const int wgs = ctx->workgroups > 0 && ctx->workgroups < ctx->num_cus ? ctx->workgroups : ctx->num_cus;
    return framesum::launch_digest(frames, offsets, lengths, n, mtu, ctx->d_tables, out, status, stream, wgs,
                                   ctx->h_report, ctx->d_report, &ctx->next_launch_id,
                                   force >= 0 ? force : ctx->force_kernel, op, wframes, tx);
}

// The host-staged digest sees the batch's lengths on the host: with the automatic choice (0) or the
// short-frame preference (8), a batch whose frames are all this short runs the small-frame kernel
// (one lane per frame; its header slot holds frames up to ~130 B), and any other batch the
// automatic choice between the 4-lane kernels. (A device-resident batch's lengths are in device
// memory: there launch_digest chooses from the kernels' reports.)
constexpr uint32_t kSmallAutoMaxLen = framesum::kSmallMaxLen;
int host_force(const fs_ctx* ctx, uint32_t max_len, uint32_t min_len) {
    if (ctx->force_kernel != 0 && ctx->force_kernel != 8) return ctx->force_kernel;
    if (max_len <= kSmallAutoMaxLen) return framesum::kForceSmallExact;
    // a longer frame: the 4-lane choice, never the small-frame kernel, even after a
    // streak of short device-resident launches; lengths within kUniformSpan: the one-pass kernel from
    // the first call (a short-lived RecvEthBatch context)
    return max_len - min_len < framesum::kUniformSpan ? framesum::kForceUniformHost : framesum::kForceNoSmall;
}

}  // namespace

extern "C" {

uint32_t fs_abi_version(void) { return FRAMESUM_ABI_VERSION; }

int fs_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

fs_status fs_ctx_create(int device, fs_ctx** out) {
    if (!out) return set_err(nullptr, FS_E_INVALID, "fs_ctx_create: out is NULL");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return set_err(nullptr, FS_E_NODEVICE, "fs_ctx_create: no such HIP device");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess)
        return set_err(nullptr, FS_E_NODEVICE, "fs_ctx_create: hipGetDeviceProperties failed");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return set_err(nullptr, FS_E_NODEVICE, std::string("fs_ctx_create: device is ") + prop.gcnArchName +
                                                   ", this build targets gfx950 only");
    fs_ctx* ctx = new (std::nothrow) fs_ctx();
    if (!ctx) return set_err(nullptr, FS_E_NOMEM, "fs_ctx_create: out of host memory");
    ctx->device = device;
    ctx->num_cus = prop.multiProcessorCount;
    hipError_t e = hipSetDevice(device);
    FsTables* h = new (std::nothrow) FsTables;
    if (e != hipSuccess || !h) {
        delete h;
        delete ctx;
        return set_err(nullptr, FS_E_HIP, "fs_ctx_create: hipSetDevice / table alloc failed");
    }
    framesum::build_tables(h);
    e = hipMalloc(&ctx->d_tables, sizeof(FsTables));
    if (e == hipSuccess) e = hipMemcpy(ctx->d_tables, h, sizeof(FsTables), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        void* hp = nullptr;
        e = hipHostMalloc(&hp, 64, hipHostMallocMapped);
        if (e == hipSuccess) {
            ctx->h_report = static_cast<volatile uint32_t*>(hp);
            ctx->h_report[framesum::kReportLatest] = 0u;
            ctx->h_report[framesum::kReportInitial] = framesum::kInitialMixedLaunches;
            ctx->h_report[framesum::kReportChosen] = 0u;
            ctx->h_report[framesum::kReportSeen] = 0u;
            ctx->h_report[framesum::kReportSeenSeq] = 0u;
            for (int w : {framesum::kReportLong, framesum::kReportRan, framesum::kReportLongSeen,
                          framesum::kReportRanSeen, framesum::kReportShort, framesum::kReportLongEver})
                ctx->h_report[w] = 0u;
            e = hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->d_report), hp, 0);
        }
    }
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->compute_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->copy_stream2, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->desc_copied, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->host_done, hipEventDisableTiming);
    for (int k = 0; k < kHostSlots && e == hipSuccess; ++k) {
        e = hipEventCreateWithFlags(&ctx->slot[k].copied, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->slot[k].consumed, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->slot[k].landed, hipEventDisableTiming);
    }
    delete h;
    if (e != hipSuccess) {
        std::string msg = std::string("fs_ctx_create: ") + hipGetErrorString(e);
        fs_ctx_destroy(ctx);
        return set_err(nullptr, FS_E_HIP, msg);
    }
    *out = ctx;
    return FS_SUCCESS;
}

fs_status fs_ctx_destroy(fs_ctx* ctx) {
    if (!ctx) return FS_E_INVALID;
    ctx->err.clear();
    (void)hipSetDevice(ctx->device);
    if (ctx->copy_stream) (void)hipStreamSynchronize(ctx->copy_stream);
    if (ctx->compute_stream) (void)hipStreamSynchronize(ctx->compute_stream);
    if (ctx->copy_stream2) (void)hipStreamSynchronize(ctx->copy_stream2);
    if (ctx->copy_stream2) (void)hipStreamDestroy(ctx->copy_stream2);
    if (ctx->desc_copied) (void)hipEventDestroy(ctx->desc_copied);
    if (ctx->host_done) (void)hipEventDestroy(ctx->host_done);
    (void)hipFree(ctx->d_desc);
    if (ctx->copy_stream) (void)hipStreamDestroy(ctx->copy_stream);
    if (ctx->compute_stream) (void)hipStreamDestroy(ctx->compute_stream);
    for (HostSlot& sl : ctx->slot) {
        if (sl.copied) (void)hipEventDestroy(sl.copied);
        if (sl.consumed) (void)hipEventDestroy(sl.consumed);
        if (sl.landed) (void)hipEventDestroy(sl.landed);
        (void)hipFree(sl.d_frames);
        (void)hipFree(sl.d_offsets);
        (void)hipFree(sl.d_lengths);
        (void)hipFree(sl.d_out);
        (void)hipFree(sl.d_status);
    }
    if (ctx->h_pin) (void)hipHostFree(ctx->h_pin);
    if (ctx->h_report) (void)hipHostFree(const_cast<uint32_t*>(ctx->h_report));
    (void)hipFree(ctx->d_tables);
    delete ctx;
    return FS_SUCCESS;
}

const char* fs_last_error(const fs_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_err.c_str(); }

fs_status fs_digest_batch(fs_ctx* ctx, const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths,
                          uint32_t n, uint32_t mtu, fs_digest* out, uint8_t* status, void* stream) {
    if (!ctx) return FS_E_INVALID;
    ctx->err.clear();
    if (n == 0) return FS_SUCCESS;
    if (n > kMaxFrames) return set_err(ctx, FS_E_INVALID, "fs_digest_batch: n too large (at most 2^31 frames per call)");
    if (!frames || !offsets || !lengths || !out) return set_err(ctx, FS_E_INVALID, "fs_digest_batch: null pointer");
    if (reinterpret_cast<uintptr_t>(frames) & 3u)
        return set_err(ctx, FS_E_INVALID, "fs_digest_batch: frames must be 4-byte aligned");
    FS_HIP(ctx, hipSetDevice(ctx->device));
    FS_HIP(ctx, launch(ctx, frames, offsets, lengths, n, mtu, out, status, reinterpret_cast<hipStream_t>(stream), framesum::FsOp::kDigest, nullptr, 0));
    return FS_SUCCESS;
}

fs_status fs_fill_batch(fs_ctx* ctx, uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths, uint32_t n,
                        uint32_t mtu, uint32_t flags, fs_digest* out, uint8_t* status, void* stream) {
    if (!ctx) return FS_E_INVALID;
    ctx->err.clear();
    if (flags & ~(uint32_t)(FS_FILL_CSUM | FS_FCS_APPEND)) return set_err(ctx, FS_E_INVALID, "fs_fill_batch: unknown flags");
    if (n == 0) return FS_SUCCESS;
    if (n > kMaxFrames) return set_err(ctx, FS_E_INVALID, "fs_fill_batch: n too large (at most 2^31 frames per call)");
    if (!frames || !offsets || !lengths || !out) return set_err(ctx, FS_E_INVALID, "fs_fill_batch: null pointer");
    if (reinterpret_cast<uintptr_t>(frames) & 3u)
        return set_err(ctx, FS_E_INVALID, "fs_fill_batch: frames must be 4-byte aligned");
    FS_HIP(ctx, hipSetDevice(ctx->device));
    FS_HIP(ctx, launch(ctx, frames, offsets, lengths, n, mtu, out, status, reinterpret_cast<hipStream_t>(stream), framesum::FsOp::kFill, frames, flags));
    return FS_SUCCESS;
}

fs_status fs_digest_batch_fcs(fs_ctx* ctx, const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths,
                              uint32_t n, uint32_t mtu, fs_digest* out, uint8_t* status, void* stream) {
    if (!ctx) return FS_E_INVALID;
    ctx->err.clear();
    if (n == 0) return FS_SUCCESS;
    if (n > kMaxFrames) return set_err(ctx, FS_E_INVALID, "fs_digest_batch_fcs: n too large (at most 2^31 frames per call)");
    if (!frames || !offsets || !lengths || !out) return set_err(ctx, FS_E_INVALID, "fs_digest_batch_fcs: null pointer");
    if (reinterpret_cast<uintptr_t>(frames) & 3u)
        return set_err(ctx, FS_E_INVALID, "fs_digest_batch_fcs: frames must be 4-byte aligned");
    FS_HIP(ctx, hipSetDevice(ctx->device));
    FS_HIP(ctx, launch(ctx, frames, offsets, lengths, n, mtu, out, status, reinterpret_cast<hipStream_t>(stream), framesum::FsOp::kFcs, nullptr, 0));
    return FS_SUCCESS;
}

// The descriptor scan of a host-staged call, compiled for AVX-512 and AVX2 beside the baseline
// and picked at load time (its four min/max reductions vectorize: 65,536 descriptors in ~20 us
// instead of ~150 us on the baseline SSE2 build).
// (host code: hipcc also parses this file for the device, where multiversioning does not exist)
#if defined(__HIP_DEVICE_COMPILE__)
#define FS_HOST_CLONES
#else
#define FS_HOST_CLONES __attribute__((target_clones("arch=x86-64-v4", "arch=x86-64-v3", "default")))
#endif
FS_HOST_CLONES static framesum::plan::ScanCore scan_descriptors(const uint64_t* offsets, const uint32_t* lengths, uint32_t n) {
    return framesum::plan::scan_core(offsets, lengths, n);
}

// The device address of pinned host memory [p, p + bytes) the kernel can read or write directly, or
// null.
static void* mapped(void* p, size_t bytes) {
    if (!p || !is_pinned(p, bytes)) return nullptr;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return d;
}

// A host-staged batch that fits one staging chunk (path 1). Everything runs on the compute stream,
// in its order: the descriptor copy (queued by the caller before its scan, straight from the
// caller's arrays when they are pinned), the frames' H2D copy into slot 0, one launch that writes the
// digests and verdicts into host memory through a mapped pointer (the caller's arrays when pinned,
// else the context's mirror, copied out after the wait; no D2H copy), then a polled wait.
static fs_status host_single(fs_ctx* ctx, const uint8_t* frames, uint64_t frames_bytes, const uint64_t* offsets,
                             const uint32_t* lengths, uint32_t n, uint32_t mtu, fs_digest* out, uint8_t* status,
                             const framesum::plan::Scan& sc, int force) {
    ctx->last_host_path = 1;
    uint64_t cpy_lo, cpy_hi;
    framesum::plan::copy_span(sc.lo, sc.hi, frames_bytes, cpy_lo, cpy_hi);
    HostSlot& sl = ctx->slot[0];
    fs_status st = ensure_slot(ctx, sl, cpy_hi - cpy_lo + 64, n);
    if (st != FS_SUCCESS) {
        // the descriptor copy already queued may still read the caller's arrays
        drain_host_streams(ctx);
        return st;
    }
    // The kernel writes the digests and verdicts straight to host memory (mapped pinned memory: no
    // D2H copy, no gap before it): into the caller's arrays when they are pinned, else into the
    // context's pinned mirror, copied out after the wait.
    void* d_out = mapped(out, (size_t)n * sizeof(fs_digest));
    void* d_st = status ? mapped(status, n) : nullptr;
    const bool direct = d_out && (!status || d_st);
    if (!direct) {
        d_out = ctx->d_pin + (size_t)n * 12;
        d_st = status ? ctx->d_pin + (size_t)n * 20 : nullptr;
    }
    const hipStream_t ks = ctx->compute_stream;
    // the frames behind the descriptors (issued by the caller before the scan), then the kernel, in
    // the compute stream's order: no cross-stream event between them
    FS_HIP_DRAIN(ctx, hipMemcpyAsync(sl.d_frames, frames + cpy_lo, cpy_hi - cpy_lo, hipMemcpyHostToDevice, ks));
    if (ctx->fault_chunk == 0) {
        drain_host_streams(ctx);
        return set_err(ctx, FS_E_NOMEM, "fs_digest_batch_host: injected failure (test hook)");
    }
    const uint8_t* base = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(sl.d_frames) - cpy_lo);
    const uint64_t* d_off = reinterpret_cast<const uint64_t*>(ctx->d_desc);
    const uint32_t* d_len = reinterpret_cast<const uint32_t*>(ctx->d_desc + (size_t)n * 8);
    FS_HIP_DRAIN(ctx, launch(ctx, base, d_off, d_len, n, mtu, reinterpret_cast<fs_digest*>(d_out),
                       reinterpret_cast<uint8_t*>(d_st), ks, framesum::FsOp::kDigest, nullptr, 0, force));
    FS_HIP_DRAIN(ctx, hipEventRecord(sl.consumed, ks));
    sl.used = true;
    FS_HIP_DRAIN(ctx, hipEventRecord(ctx->host_done, ks));
    FS_HIP_DRAIN(ctx, host_wait(ctx->host_done));
    if (!direct) {
        std::memcpy(out, ctx->h_pin + (size_t)n * 12, (size_t)n * sizeof(fs_digest));
        if (status) std::memcpy(status, ctx->h_pin + (size_t)n * 20, n);
    }
    ctx->host_dirty = false;
    return FS_SUCCESS;
}

// A host-staged batch read in place: frames, offsets and lengths in pinned host memory the device
// addresses directly (mapped), results written to host memory by the kernel (the caller's arrays when
// pinned, else the mirror). The small-frame kernel only: its lanes read whole 16-B chunks of adjacent
// frames, which the memory system turns into full-line PCIe reads.
static fs_status host_inplace(fs_ctx* ctx, const uint8_t* d_frames, const uint64_t* d_off, const uint32_t* d_len,
                              uint32_t n, uint32_t mtu, fs_digest* out, uint8_t* status) {
    ctx->last_host_path = 2;
    fs_status st = ensure_pinned(ctx, n);
    if (st != FS_SUCCESS) return st;
    void* d_out = mapped(out, (size_t)n * sizeof(fs_digest));
    void* d_st = status ? mapped(status, n) : nullptr;
    const bool direct = d_out && (!status || d_st);
    if (!direct) {
        d_out = ctx->d_pin + (size_t)n * 12;
        d_st = status ? ctx->d_pin + (size_t)n * 20 : nullptr;
    }
    ctx->host_dirty = true;
    const hipStream_t ks = ctx->compute_stream;
    FS_HIP_DRAIN(ctx, launch(ctx, d_frames, d_off, d_len, n, mtu, reinterpret_cast<fs_digest*>(d_out),
                       reinterpret_cast<uint8_t*>(d_st), ks, framesum::FsOp::kDigest, nullptr, 0,
                       framesum::kForceSmallExact));
    FS_HIP_DRAIN(ctx, hipEventRecord(ctx->host_done, ks));
    FS_HIP_DRAIN(ctx, host_wait(ctx->host_done));
    if (!direct) {
        std::memcpy(out, ctx->h_pin + (size_t)n * 12, (size_t)n * sizeof(fs_digest));
        if (status) std::memcpy(status, ctx->h_pin + (size_t)n * 20, n);
    }
    ctx->host_dirty = false;
    return FS_SUCCESS;
}

fs_status fs_digest_batch_host(fs_ctx* ctx, const uint8_t* frames, uint64_t frames_bytes, const uint64_t* offsets,
                               const uint32_t* lengths, uint32_t n, uint32_t mtu, fs_digest* out, uint8_t* status) {
    if (!ctx) return FS_E_INVALID;
    ctx->err.clear();
    if (n == 0) return FS_SUCCESS;
    if (n > kMaxFrames) return set_err(ctx, FS_E_INVALID, "fs_digest_batch_host: n too large (at most 2^31 frames per call)");
    if (!frames || !offsets || !lengths || !out)
        return set_err(ctx, FS_E_INVALID, "fs_digest_batch_host: null pointer");
    FS_HIP(ctx, hipSetDevice(ctx->device));
    fs_status pst = quiesce_host_streams(ctx);
    if (pst != FS_SUCCESS) return pst;
    if (n <= kChunkFrames && ctx->force_kernel != 2 && ctx->force_kernel != 3 && ctx->force_kernel != 4) {
        // A batch of short frames whose frames, offsets and lengths are all in pinned host memory:
        // the small-frame kernel reads them in place over PCIe and writes its results to host
        // memory, so the call is one launch -- no copies, no gaps between DMA commands.
        // (the frames' span is checked once the scan has found it: the 16-B chunks the kernel reads
        // stay in the pages that hold frame bytes, and pinned allocations are whole pages)
        const void* dof = mapped(const_cast<uint64_t*>(offsets), (size_t)n * 8);
        const void* dln = dof ? mapped(const_cast<uint32_t*>(lengths), (size_t)n * 4) : nullptr;
        if (dln && is_pinned(frames, 1)) {
            const framesum::plan::Scan sc =
                framesum::plan::scan_from(scan_descriptors(offsets, lengths, n), offsets, lengths, n, frames_bytes);
            if (sc.bad < n)
                return set_err(ctx, FS_E_INVALID, "fs_digest_batch_host: frame " + std::to_string(sc.bad) + " ends past frames_bytes");
            const void* df = sc.hi > sc.lo ? mapped(const_cast<uint8_t*>(frames + sc.lo), sc.hi - sc.lo) : nullptr;
            if (df && host_force(ctx, sc.max_len, sc.min_len) == framesum::kForceSmallExact &&
                (reinterpret_cast<uintptr_t>(frames) & 3u) == 0u)
                return host_inplace(ctx, static_cast<const uint8_t*>(df) - sc.lo, static_cast<const uint64_t*>(dof),
                                    static_cast<const uint32_t*>(dln), n, mtu, out, status);
        }
    }
    if (n <= kChunkFrames) {
        // The descriptors go to the device first, while the host scans them (they are n elements
        // of the caller's arrays whatever the scan finds; a frame out of range fails the call before
        // any frame byte is copied): straight from the caller's arrays when they are pinned (one
        // copy when the lengths follow the offsets, as the Go binding stages them), else through
        // the pinned mirror.
        pst = ensure_desc(ctx, n);
        if (pst == FS_SUCCESS) pst = ensure_pinned(ctx, n);
        if (pst != FS_SUCCESS) return pst;
        ctx->host_dirty = true;  // until this call has waited for all of its work
        const bool pin_desc = is_pinned(offsets, (size_t)n * 8) && is_pinned(lengths, (size_t)n * 4);
        const uint64_t* src_off = offsets;
        const uint32_t* src_len = lengths;
        if (!pin_desc) {
            src_off = reinterpret_cast<const uint64_t*>(ctx->h_pin);
            src_len = reinterpret_cast<const uint32_t*>(ctx->h_pin + (size_t)n * 8);
            std::memcpy(ctx->h_pin, offsets, (size_t)n * 8);
            std::memcpy(ctx->h_pin + (size_t)n * 8, lengths, (size_t)n * 4);
        }
        const hipStream_t ks = ctx->compute_stream;
        if (reinterpret_cast<const uint8_t*>(src_off) + (size_t)n * 8 == reinterpret_cast<const uint8_t*>(src_len)) {
            FS_HIP_DRAIN(ctx, hipMemcpyAsync(ctx->d_desc, src_off, (size_t)n * 12, hipMemcpyHostToDevice, ks));
        } else {
            FS_HIP_DRAIN(ctx, hipMemcpyAsync(ctx->d_desc, src_off, (size_t)n * 8, hipMemcpyHostToDevice, ks));
            FS_HIP_DRAIN(ctx, hipMemcpyAsync(ctx->d_desc + (size_t)n * 8, src_len, (size_t)n * 4, hipMemcpyHostToDevice, ks));
        }
        const framesum::plan::Scan sc =
            framesum::plan::scan_from(scan_descriptors(offsets, lengths, n), offsets, lengths, n, frames_bytes);
        if (sc.bad < n) {
            drain_host_streams(ctx);  // the descriptor copy reads the caller's arrays: done before returning
            return set_err(ctx, FS_E_INVALID, "fs_digest_batch_host: frame " + std::to_string(sc.bad) + " ends past frames_bytes");
        }
        const int force = host_force(ctx, sc.max_len, sc.min_len);
        if (sc.hi - sc.lo <= kChunkBytes)
            return host_single(ctx, frames, frames_bytes, offsets, lengths, n, mtu, out, status, sc, force);
        FS_HIP(ctx, hipStreamSynchronize(ks));  // (the chunked path below stages the descriptors itself)
    }
    const framesum::plan::Scan sc =
        framesum::plan::scan_from(scan_descriptors(offsets, lengths, n), offsets, lengths, n, frames_bytes);
    if (sc.bad < n)
        return set_err(ctx, FS_E_INVALID, "fs_digest_batch_host: frame " + std::to_string(sc.bad) + " ends past frames_bytes");
    const int force = host_force(ctx, sc.max_len, sc.min_len);
    ctx->host_dirty = true;  // until this call has waited for all of its work
    ctx->last_host_path = 3;
    pst = ensure_pinned(ctx, n);
    if (pst != FS_SUCCESS) return pst;
    pst = ensure_desc(ctx, n);
    if (pst != FS_SUCCESS) return pst;
    uint64_t* h_off = reinterpret_cast<uint64_t*>(ctx->h_pin);
    uint32_t* h_len = reinterpret_cast<uint32_t*>(ctx->h_pin + (size_t)n * 8);
    fs_digest* h_out = reinterpret_cast<fs_digest*>(ctx->h_pin + (size_t)n * 12);
    uint8_t* h_st = ctx->h_pin + (size_t)n * 20;
    std::vector<framesum::plan::Chunk> chunks;
    try {
        framesum::plan::host_chunks(offsets, lengths, n, frames_bytes, kChunkBytes, kChunkFrames, chunks);
    } catch (const std::bad_alloc&) {
        return set_err(ctx, FS_E_NOMEM, "fs_digest_batch_host: out of host memory");
    }
    const hipStream_t ks = ctx->compute_stream;
    // chunk k's frame bytes into its slot, on copy stream k & 1 (once the slot's previous chunk
    // has been consumed by its kernel)
    auto copy_chunk = [&](size_t k) -> fs_status {
        const framesum::plan::Chunk& c = chunks[k];
        HostSlot& sl = ctx->slot[k % kHostSlots];
        fs_status st = ensure_slot(ctx, sl, c.cpy_hi - c.cpy_lo + 64, c.c1 - c.c0);
        if (st != FS_SUCCESS) return st;
        const hipStream_t cs = (k & 1u) ? ctx->copy_stream2 : ctx->copy_stream;
        if (sl.used) FS_HIP(ctx, hipStreamWaitEvent(cs, sl.consumed, 0));  // chunk k - kHostSlots done with it
        FS_HIP(ctx, hipMemcpyAsync(sl.d_frames, frames + c.cpy_lo, c.cpy_hi - c.cpy_lo, hipMemcpyHostToDevice, cs));
        FS_HIP(ctx, hipEventRecord(sl.copied, cs));
        return FS_SUCCESS;
    };
    // chunk k's results from the pinned mirror into the caller's arrays, once they have landed
    auto deliver = [&](size_t k) -> fs_status {
        const framesum::plan::Chunk& c = chunks[k];
        FS_HIP(ctx, host_wait(ctx->slot[k % kHostSlots].landed));
        std::memcpy(out + c.c0, h_out + c.c0, (size_t)(c.c1 - c.c0) * sizeof(fs_digest));
        if (status) std::memcpy(status + c.c0, h_st + c.c0, c.c1 - c.c0);
        return FS_SUCCESS;
    };
    // the first chunk's frames stream while the descriptors are mirrored (pinned) and then
    // copied, all of them in one copy (h_off and h_len are contiguous in the mirror)
    fs_status st = copy_chunk(0);
    if (st != FS_SUCCESS) return st;
    std::memcpy(h_off, offsets, (size_t)n * 8);
    std::memcpy(h_len, lengths, (size_t)n * 4);
    const uint64_t* d_off = reinterpret_cast<const uint64_t*>(ctx->d_desc);
    const uint32_t* d_len = reinterpret_cast<const uint32_t*>(ctx->d_desc + (size_t)n * 8);
    FS_HIP(ctx, hipMemcpyAsync(ctx->d_desc, h_off, (size_t)n * 12, hipMemcpyHostToDevice, ctx->copy_stream2));
    FS_HIP(ctx, hipEventRecord(ctx->desc_copied, ctx->copy_stream2));
    FS_HIP(ctx, hipStreamWaitEvent(ks, ctx->desc_copied, 0));
    for (size_t chunk = 0; chunk < chunks.size(); ++chunk) {
        const uint32_t c0 = chunks[chunk].c0, c1 = chunks[chunk].c1;
        const uint64_t cpy_lo = chunks[chunk].cpy_lo;
        HostSlot& sl = ctx->slot[chunk % kHostSlots];
        const uint32_t cnt = c1 - c0;
        if (chunk > 0) {
            st = copy_chunk(chunk);
            if (st != FS_SUCCESS) return st;
        }
        if ((long)chunk == ctx->fault_chunk)
            return set_err(ctx, FS_E_NOMEM, "fs_digest_batch_host: injected failure (test hook)");
        FS_HIP(ctx, hipStreamWaitEvent(ks, sl.copied, 0));
        // the kernel addresses frame i at base + offsets[i]: base = staging - cpy_lo (4-B aligned)
        const uint8_t* base = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(sl.d_frames) - cpy_lo);
        FS_HIP(ctx, launch(ctx, base, d_off + c0, d_len + c0, cnt, mtu, sl.d_out, status ? sl.d_status : nullptr, ks,
                           framesum::FsOp::kDigest, nullptr, 0, force));
        FS_HIP(ctx, hipEventRecord(sl.consumed, ks));
        sl.used = true;
        FS_HIP(ctx, hipMemcpyAsync(h_out + c0, sl.d_out, (size_t)cnt * sizeof(fs_digest), hipMemcpyDeviceToHost, ks));
        if (status) FS_HIP(ctx, hipMemcpyAsync(h_st + c0, sl.d_status, cnt, hipMemcpyDeviceToHost, ks));
        FS_HIP(ctx, hipEventRecord(sl.landed, ks));
        // chunk - 2's results while this one streams (its slot's `landed` is re-recorded by chunk + 1)
        if (chunk >= 2) {
            st = deliver(chunk - 2);
            if (st != FS_SUCCESS) return st;
        }
    }
    for (size_t k = chunks.size() >= 2 ? chunks.size() - 2 : 0; k < chunks.size(); ++k) {
        st = deliver(k);
        if (st != FS_SUCCESS) return st;
    }
    FS_HIP(ctx, hipStreamSynchronize(ks));
    ctx->host_dirty = false;
    return FS_SUCCESS;
}

fs_status fs_fill_batch_host(fs_ctx* ctx, uint8_t* frames, uint64_t frames_bytes, const uint64_t* offsets,
                             const uint32_t* lengths, uint32_t n, uint32_t mtu, uint32_t flags, fs_digest* out,
                             uint8_t* status) {
    if (!ctx) return FS_E_INVALID;
    ctx->err.clear();
    if (flags & ~(uint32_t)(FS_FILL_CSUM | FS_FCS_APPEND))
        return set_err(ctx, FS_E_INVALID, "fs_fill_batch_host: unknown flags");
    if (n == 0) return FS_SUCCESS;
    if (n > kMaxFrames) return set_err(ctx, FS_E_INVALID, "fs_fill_batch_host: n too large (at most 2^31 frames per call)");
    if (!frames || !offsets || !lengths || !out) return set_err(ctx, FS_E_INVALID, "fs_fill_batch_host: null pointer");
    // One staged span [lo, hi) (the frames and, with FS_FCS_APPEND, their FCS bytes), copied in,
    // filled, copied back. Not chunk-pipelined: written spans of unordered batches may interleave.
    const uint32_t extra = (flags & FS_FCS_APPEND) ? 4u : 0u;
    const uint32_t bad = framesum::plan::first_frame_out_of_range(offsets, lengths, n, frames_bytes, extra);
    if (bad < n)
        return set_err(ctx, FS_E_INVALID, "fs_fill_batch_host: frame " + std::to_string(bad) + " ends past frames_bytes");
    uint64_t lo = UINT64_MAX, hi = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t o = offsets[i], e = o + lengths[i] + extra;
        lo = o < lo ? o : lo;
        hi = e > hi ? e : hi;
    }
    FS_HIP(ctx, hipSetDevice(ctx->device));
    fs_status pst = quiesce_host_streams(ctx);
    if (pst != FS_SUCCESS) return pst;
    ctx->host_dirty = true;  // until this call has waited for all of its work
    pst = ensure_pinned(ctx, n);
    if (pst != FS_SUCCESS) return pst;
    uint64_t* h_off = reinterpret_cast<uint64_t*>(ctx->h_pin);
    uint32_t* h_len = reinterpret_cast<uint32_t*>(ctx->h_pin + (size_t)n * 8);
    fs_digest* h_out = reinterpret_cast<fs_digest*>(ctx->h_pin + (size_t)n * 12);
    uint8_t* h_st = ctx->h_pin + (size_t)n * 20;
    std::memcpy(h_off, offsets, (size_t)n * 8);
    std::memcpy(h_len, lengths, (size_t)n * 4);
    uint64_t cpy_lo, cpy_hi;
    framesum::plan::copy_span(lo, hi, frames_bytes, cpy_lo, cpy_hi);
    HostSlot& sl = ctx->slot[0];
    fs_status st = ensure_slot(ctx, sl, cpy_hi - cpy_lo + 64, n);
    if (st != FS_SUCCESS) return st;
    hipStream_t ks = ctx->compute_stream;
    if (sl.used) FS_HIP(ctx, hipStreamWaitEvent(ks, sl.consumed, 0));
    FS_HIP(ctx, hipMemcpyAsync(sl.d_frames, frames + cpy_lo, cpy_hi - cpy_lo, hipMemcpyHostToDevice, ks));
    FS_HIP(ctx, hipMemcpyAsync(sl.d_offsets, h_off, (size_t)n * 8, hipMemcpyHostToDevice, ks));
    FS_HIP(ctx, hipMemcpyAsync(sl.d_lengths, h_len, (size_t)n * 4, hipMemcpyHostToDevice, ks));
    uint8_t* base = reinterpret_cast<uint8_t*>(reinterpret_cast<uintptr_t>(sl.d_frames) - cpy_lo);
    FS_HIP(ctx, launch(ctx, base, sl.d_offsets, sl.d_lengths, n, mtu, sl.d_out, status ? sl.d_status : nullptr, ks,
                       framesum::FsOp::kFill, base, flags));
    FS_HIP(ctx, hipMemcpyAsync(frames + lo, sl.d_frames + (lo - cpy_lo), hi - lo, hipMemcpyDeviceToHost, ks));
    FS_HIP(ctx, hipMemcpyAsync(h_out, sl.d_out, (size_t)n * sizeof(fs_digest), hipMemcpyDeviceToHost, ks));
    if (status) FS_HIP(ctx, hipMemcpyAsync(h_st, sl.d_status, n, hipMemcpyDeviceToHost, ks));
    FS_HIP(ctx, hipEventRecord(sl.consumed, ks));
    sl.used = true;
    FS_HIP(ctx, hipStreamSynchronize(ks));
    ctx->host_dirty = false;
    std::memcpy(out, h_out, (size_t)n * sizeof(fs_digest));
    if (status) std::memcpy(status, h_st, n);
    return FS_SUCCESS;
}

fs_status fs_digest_batch_multi(fs_ctx* const* ctxs, int nctx, const uint8_t* frames, uint64_t frames_bytes,
                                const uint64_t* offsets, const uint32_t* lengths, uint32_t n, uint32_t mtu,
                                fs_digest* out, uint8_t* status) {
    if (!ctxs || nctx <= 0) return FS_E_INVALID;
    for (int k = 0; k < nctx; ++k) {
        if (!ctxs[k]) return FS_E_INVALID;
        ctxs[k]->err.clear();
        for (int j = 0; j < k; ++j)
            if (ctxs[j] == ctxs[k])
                return set_err(ctxs[k], FS_E_INVALID, "fs_digest_batch_multi: a context appears twice in ctxs");
    }
    if (n == 0) return FS_SUCCESS;
    if (n > kMaxFrames)
        return set_err(ctxs[0], FS_E_INVALID, "fs_digest_batch_multi: n too large (at most 2^31 frames per call)");
    if (!frames || !offsets || !lengths || !out)
        return set_err(ctxs[0], FS_E_INVALID, "fs_digest_batch_multi: null pointer");
    const uint32_t bad = framesum::plan::first_frame_out_of_range(offsets, lengths, n, frames_bytes);
    if (bad < n)
        return set_err(ctxs[0], FS_E_INVALID, "fs_digest_batch_multi: frame " + std::to_string(bad) + " ends past frames_bytes");
    // block k = a run of frames in buffer order holding about 1/nctx of the bytes (one H2D
    // stream per GPU over its own bytes); unordered batches are ordered by offset first and
    // their results scattered back to batch order
    framesum::plan::MultiPlan plan;
    struct Block {
        std::vector<uint64_t> off;
        std::vector<uint32_t> len;
        std::vector<fs_digest> dig;
        std::vector<uint8_t> st;
    };
    std::vector<Block> blk;
    std::vector<fs_status> st;
    try {
        framesum::plan::multi_blocks(offsets, lengths, n, nctx, plan);
        blk.resize(nctx);
        st.assign(nctx, FS_SUCCESS);
        if (!plan.order.empty()) {
            for (int k = 0; k < nctx; ++k) {
                Block& b = blk[k];
                const uint32_t p0 = plan.cut[k], p1 = plan.cut[k + 1];
                b.off.resize(p1 - p0);
                b.len.resize(p1 - p0);
                b.dig.resize(p1 - p0);
                b.st.resize(status ? p1 - p0 : 0);
                for (uint32_t p = p0; p < p1; ++p) {
                    b.off[p - p0] = offsets[plan.order[p]];
                    b.len[p - p0] = lengths[plan.order[p]];
                }
            }
        }
    } catch (const std::bad_alloc&) {
        return set_err(ctxs[0], FS_E_NOMEM, "fs_digest_batch_multi: out of host memory");
    }
    auto run_block = [&](int k) {
        const uint32_t p0 = plan.cut[k], p1 = plan.cut[k + 1];
        if (p1 <= p0) return;
        if (plan.order.empty()) {
            st[k] = fs_digest_batch_host(ctxs[k], frames, frames_bytes, offsets + p0, lengths + p0, p1 - p0, mtu,
                                         out + p0, status ? status + p0 : nullptr);
            return;
        }
        Block& b = blk[k];
        st[k] = fs_digest_batch_host(ctxs[k], frames, frames_bytes, b.off.data(), b.len.data(), p1 - p0, mtu,
                                     b.dig.data(), status ? b.st.data() : nullptr);
        if (st[k] != FS_SUCCESS) return;
        for (uint32_t p = p0; p < p1; ++p) {
            out[plan.order[p]] = b.dig[p - p0];
            if (status) status[plan.order[p]] = b.st[p - p0];
        }
    };
    // One host thread per block beyond the first; if a thread cannot be started, its block runs
    // on the calling thread instead (never an exception across the ABI, no joinable thread left).
    std::vector<std::thread> workers;
    std::vector<int> inline_blocks;
    try {
        workers.reserve(nctx - 1);
        inline_blocks.reserve(nctx);
    } catch (const std::bad_alloc&) {
        return set_err(ctxs[0], FS_E_NOMEM, "fs_digest_batch_multi: out of host memory");
    }
    for (int k = 1; k < nctx; ++k) {
        try {
            workers.emplace_back(run_block, k);
        } catch (const std::system_error&) {
            inline_blocks.push_back(k);
        }
    }
    run_block(0);
    for (int k : inline_blocks) run_block(k);
    for (auto& w : workers) w.join();
    for (int k = 0; k < nctx; ++k)
        if (st[k] != FS_SUCCESS) return st[k];
    return FS_SUCCESS;
}

fs_status fs_deinterleave(fs_ctx* ctx, const uint8_t* gathered, uint32_t nshards, uint64_t n, fs_digest* out,
                          uint8_t* status, void* stream) {
    if (!ctx) return FS_E_INVALID;
    ctx->err.clear();
    if (n == 0) return FS_SUCCESS;
    if (!gathered || !out || nshards == 0) return set_err(ctx, FS_E_INVALID, "fs_deinterleave: null pointer or no shards");
    FS_HIP(ctx, hipSetDevice(ctx->device));
    FS_HIP(ctx, framesum::launch_deinterleave(gathered, nshards, n, out, status, reinterpret_cast<hipStream_t>(stream)));
    return FS_SUCCESS;
}

fs_status fs_ctx_set_workgroups(fs_ctx* ctx, int workgroups) {
    if (!ctx) return FS_E_INVALID;
    ctx->err.clear();
    if (workgroups < 0) return set_err(ctx, FS_E_INVALID, "fs_ctx_set_workgroups: workgroups must be >= 0");
    ctx->workgroups = workgroups;
    return FS_SUCCESS;
}

fs_status fs_ctx_set_kernel(fs_ctx* ctx, int variant) {
    if (!ctx) return FS_E_INVALID;
    ctx->err.clear();
    if (variant != 0 && variant != 2 && variant != 3 && variant != 4 && variant != 8)
        return set_err(ctx, FS_E_INVALID, "fs_ctx_set_kernel: variant must be 0 (automatic), 2, 3, 4 or 8");
    ctx->force_kernel = variant;
    return FS_SUCCESS;
}

int fs_ctx_last_kernel(const fs_ctx* ctx) {
    if (!ctx || !ctx->h_report) return FS_E_INVALID;
    return (int)ctx->h_report[framesum::kReportChosen];
}

#ifdef FS_TEST_HOOKS
// Test library only (-DFS_TEST_HOOKS): fs_digest_batch_host on ctx fails at chunk `chunk` (-1: never).
fs_status fs_test_set_fault(fs_ctx* ctx, long chunk) {
    if (!ctx) return FS_E_INVALID;
    ctx->fault_chunk = chunk;
    return FS_SUCCESS;
}
// ... and the context's kernel choice set to any launch_digest force value, e.g. kForceSmallExact (16):
// the small-frame kernel for every launch, whatever the reports say (the parity suite's
// "small_exact" column runs every case through that kernel's own long-frame path).
fs_status fs_test_set_kernel_exact(fs_ctx* ctx, int force) {
    if (!ctx) return FS_E_INVALID;
    ctx->force_kernel = force;
    return FS_SUCCESS;
}
// ... and which path the latest fs_digest_batch_host took: 1 staged in one chunk, 2 read in place,
// 3 chunked (0 before the first call).
int fs_test_last_host_path(const fs_ctx* ctx) { return ctx ? ctx->last_host_path : -1; }
#endif

fs_status fs_host_alloc(fs_ctx* ctx, uint64_t bytes, void** out) {
    if (!ctx || !out) return FS_E_INVALID;
    *out = nullptr;
    // Mapped (the in-place read and the direct result writes take its device address) and portable
    // (fs_digest_batch_multi's other contexts address it too). Coarse-grained: a kernel may cache its
    // lines in L2, but every launch begins with a system-scope acquire (HIP's dispatch packets), which
    // invalidates them, so a buffer the caller refills between calls is read anew
    // (test_host_inplace_refilled_buffer runs 200 refills of one buffer through the in-place path).
    if (hipHostMalloc(out, bytes, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess)
        return set_err(ctx, FS_E_NOMEM, "hipHostMalloc failed");
    return FS_SUCCESS;
}

fs_status fs_host_free(fs_ctx* ctx, void* p) {
    if (!ctx) return FS_E_INVALID;
    ctx->err.clear();
    if (p) FS_HIP(ctx, hipHostFree(p));
    return FS_SUCCESS;
}

}  // extern "C"
