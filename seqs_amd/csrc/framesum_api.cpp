// framesum C ABI (include/framesum.h) — context management, device-resident and
// host-staged batch entry points. No CPU fallback: every digest is computed by
// the gfx950 kernel (framesum_kernel.hip); a missing/unsupported device is an error.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "../../include/framesum.h"
#include "framesum_internal.h"

using framesum::FsTables;

struct fs_ctx {
    int device = 0;
    int num_cus = 0;
    FsTables* d_tables = nullptr;
    hipStream_t stream = nullptr;
    // host-staged path: grow-only device buffers
    uint8_t* d_frames = nullptr;
    uint64_t cap_frames = 0;
    uint64_t* d_offsets = nullptr;
    uint32_t* d_lengths = nullptr;
    fs_digest* d_out = nullptr;
    uint8_t* d_status = nullptr;
    uint32_t cap_n = 0;
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

fs_status ensure_staging(fs_ctx* ctx, uint64_t frames_bytes, uint32_t n) {
    if (frames_bytes > ctx->cap_frames) {
        if (ctx->d_frames) (void)hipFree(ctx->d_frames);
        ctx->d_frames = nullptr;
        ctx->cap_frames = 0;
        uint64_t cap = frames_bytes + 256;
        if (hipMalloc(&ctx->d_frames, cap) != hipSuccess) return set_err(ctx, FS_E_NOMEM, "hipMalloc frames staging");
        ctx->cap_frames = cap;
    }
    if (n > ctx->cap_n) {
        (void)hipFree(ctx->d_offsets);
        (void)hipFree(ctx->d_lengths);
        (void)hipFree(ctx->d_out);
        (void)hipFree(ctx->d_status);
        ctx->d_offsets = nullptr;
        ctx->d_lengths = nullptr;
        ctx->d_out = nullptr;
        ctx->d_status = nullptr;
        ctx->cap_n = 0;
        if (hipMalloc(&ctx->d_offsets, (size_t)n * 8) != hipSuccess ||
            hipMalloc(&ctx->d_lengths, (size_t)n * 4) != hipSuccess ||
            hipMalloc(&ctx->d_out, (size_t)n * sizeof(fs_digest)) != hipSuccess ||
            hipMalloc(&ctx->d_status, (size_t)n) != hipSuccess)
            return set_err(ctx, FS_E_NOMEM, "hipMalloc descriptor staging");
        ctx->cap_n = n;
    }
    return FS_SUCCESS;
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
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
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
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    (void)hipFree(ctx->d_tables);
    (void)hipFree(ctx->d_frames);
    (void)hipFree(ctx->d_offsets);
    (void)hipFree(ctx->d_lengths);
    (void)hipFree(ctx->d_out);
    (void)hipFree(ctx->d_status);
    delete ctx;
    return FS_SUCCESS;
}

const char* fs_last_error(const fs_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_err.c_str(); }

fs_status fs_digest_batch(fs_ctx* ctx, const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths,
                          uint32_t n, uint32_t mtu, fs_digest* out, uint8_t* status, void* stream) {
    if (!ctx) return FS_E_INVALID;
    if (n == 0) return FS_SUCCESS;
    if (!frames || !offsets || !lengths || !out) return set_err(ctx, FS_E_INVALID, "fs_digest_batch: null pointer");
    if (reinterpret_cast<uintptr_t>(frames) & 3u)
        return set_err(ctx, FS_E_INVALID, "fs_digest_batch: frames must be 4-byte aligned");
    FS_HIP(ctx, hipSetDevice(ctx->device));
    FS_HIP(ctx, framesum::launch_digest(frames, offsets, lengths, n, mtu, ctx->d_tables, out, status,
                                        reinterpret_cast<hipStream_t>(stream), ctx->num_cus));
    return FS_SUCCESS;
}

fs_status fs_digest_batch_host(fs_ctx* ctx, const uint8_t* frames, uint64_t frames_bytes, const uint64_t* offsets,
                               const uint32_t* lengths, uint32_t n, uint32_t mtu, fs_digest* out, uint8_t* status) {
    if (!ctx) return FS_E_INVALID;
    if (n == 0) return FS_SUCCESS;
    if (!frames || !offsets || !lengths || !out)
        return set_err(ctx, FS_E_INVALID, "fs_digest_batch_host: null pointer");
    FS_HIP(ctx, hipSetDevice(ctx->device));
    fs_status st = ensure_staging(ctx, frames_bytes, n);
    if (st != FS_SUCCESS) return st;
    hipStream_t s = ctx->stream;
    FS_HIP(ctx, hipMemcpyAsync(ctx->d_frames, frames, frames_bytes, hipMemcpyHostToDevice, s));
    FS_HIP(ctx, hipMemcpyAsync(ctx->d_offsets, offsets, (size_t)n * 8, hipMemcpyHostToDevice, s));
    FS_HIP(ctx, hipMemcpyAsync(ctx->d_lengths, lengths, (size_t)n * 4, hipMemcpyHostToDevice, s));
    FS_HIP(ctx, framesum::launch_digest(ctx->d_frames, ctx->d_offsets, ctx->d_lengths, n, mtu, ctx->d_tables,
                                        ctx->d_out, status ? ctx->d_status : nullptr, s, ctx->num_cus));
    FS_HIP(ctx, hipMemcpyAsync(out, ctx->d_out, (size_t)n * sizeof(fs_digest), hipMemcpyDeviceToHost, s));
    if (status) FS_HIP(ctx, hipMemcpyAsync(status, ctx->d_status, n, hipMemcpyDeviceToHost, s));
    FS_HIP(ctx, hipStreamSynchronize(s));
    return FS_SUCCESS;
}

fs_status fs_host_alloc(fs_ctx* ctx, uint64_t bytes, void** out) {
    if (!ctx || !out) return FS_E_INVALID;
    *out = nullptr;
    if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess)
        return set_err(ctx, FS_E_NOMEM, "hipHostMalloc failed");
    return FS_SUCCESS;
}

fs_status fs_host_free(fs_ctx* ctx, void* p) {
    if (!ctx) return FS_E_INVALID;
    if (p) FS_HIP(ctx, hipHostFree(p));
    return FS_SUCCESS;
}

}  // extern "C"
