// framesum multi-GPU group (include/framesum.h: fs_group_*, fs_digest_batch_sharded): one host
// process drives every GPU of a node. Each device digests its round-robin shard with the
// gfx950 kernel (through fs_digest_batch on its own context and stream); grouped point-to-point
// RCCL transfers (ncclSend / ncclRecv over xGMI) bring the 8-byte digests and 1-byte verdicts to
// the first device, where the de-interleave kernel (framesum_shard.hip) restores global frame
// order. Frames are independent (eth/crc.go:12-17), so this transfer is the only exchange. The
// batch goes in chunks (framesum_plan.h chunk_plan): chunk c's transfer and de-interleave run on
// a second stream per device while the devices digest chunk c+1. N > 1 devices is unverified on
// hardware (one GPU per build box); tests/csrc/test_plan.cpp replays the chunk plan on the host.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <new>
#include <string>
#include <vector>

#include "../../include/framesum.h"
#include "framesum_internal.h"
#include "framesum_plan.h"

struct fs_group {
    int n = 0;
    std::vector<int> dev;
    std::vector<fs_ctx*> ctx;
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> stream;
    std::vector<hipStream_t> xfer;  // per device: the gather (and on the first device the de-interleave)
    std::vector<hipEvent_t> done;   // per device and chunk: that chunk's shard kernel has finished
    std::vector<uint8_t*> send;  // per device k >= 1: its slab; device 0 sends in place from recv
    uint8_t* recv = nullptr;     // first device: n slabs back to back
    uint64_t cap_slab = 0;       // bytes per slab currently allocated
    long fault_chunk = -1;       // test library only (fs_test_group_set_fault): fail at this chunk
    long fault_gather = -1;      // test library only (fs_test_group_set_fault_gather): an RCCL error here
    bool aborted = false;        // an RCCL error aborted the communicators: the group is unusable
    std::string err;
};

namespace {

thread_local std::string g_group_create_err;

// chunks per call: about 32K rows each (a digest launch of ~50 MB of 1500-B frames, long enough to
// run at full rate), at most kMaxChunks
constexpr uint32_t kMaxChunks = 8;
constexpr uint64_t kChunkRows = 32768;

fs_status gset(fs_group* g, fs_status code, const std::string& msg) {
    if (g) g->err = msg;
    else g_group_create_err = msg;
    return code;
}

void free_slabs(fs_group* g) {
    for (int k = 0; k < g->n; ++k) {
        if (k > 0 && g->send[k]) {
            (void)hipSetDevice(g->dev[k]);
            (void)hipFree(g->send[k]);
        }
        g->send[k] = nullptr;
    }
    if (g->recv) {
        (void)hipSetDevice(g->dev[0]);
        (void)hipFree(g->recv);
    }
    g->recv = nullptr;
    g->cap_slab = 0;
}

fs_status ensure_slabs(fs_group* g, uint64_t sb) {
    if (sb <= g->cap_slab) return FS_SUCCESS;
    for (int k = 0; k < g->n; ++k) {
        (void)hipSetDevice(g->dev[k]);
        (void)hipStreamSynchronize(g->stream[k]);
        (void)hipStreamSynchronize(g->xfer[k]);
    }
    free_slabs(g);
    if (hipSetDevice(g->dev[0]) != hipSuccess || hipMalloc(&g->recv, sb * (uint64_t)g->n) != hipSuccess)
        return gset(g, FS_E_NOMEM, "fs_digest_batch_sharded: hipMalloc of the gather buffer failed");
    g->send[0] = g->recv;
    for (int k = 1; k < g->n; ++k)
        if (hipSetDevice(g->dev[k]) != hipSuccess || hipMalloc(&g->send[k], sb) != hipSuccess)
            return gset(g, FS_E_NOMEM, "fs_digest_batch_sharded: hipMalloc of a shard slab failed");
    g->cap_slab = sb;
    return FS_SUCCESS;
}

// Best-effort drain of every stream of the group (compute and transfer), so that an error exit
// leaves no kernel, transfer or de-interleave of the failed call in flight: the next call's
// kernels then never overwrite a slab an earlier ncclSend still reads, and nothing writes the
// caller's out/status after the error return.
void quiesce_group(fs_group* g) {
    for (int k = 0; k < g->n; ++k) {
        (void)hipSetDevice(g->dev[k]);
        if (g->stream[k]) (void)hipStreamSynchronize(g->stream[k]);
        if (g->xfer[k]) (void)hipStreamSynchronize(g->xfer[k]);
    }
}

fs_status fail_group(fs_group* g, fs_status code, const std::string& msg) {
    quiesce_group(g);
    return gset(g, code, msg);
}

// An RCCL error after part of a chunk's grouped sends and receives may have been enqueued: a send
// whose receive never comes would keep its transfer stream busy forever, so synchronizing that
// stream could hang. The communicators are aborted first (ncclCommAbort ends their pending
// operations and frees them), then the streams are drained. The group stays unusable: every later
// call fails until it is destroyed and created again.
fs_status fail_group_comm(fs_group* g, const std::string& msg) {
    for (int k = 0; k < g->n; ++k) {
        if (!g->comm[k]) continue;
        (void)hipSetDevice(g->dev[k]);
        (void)ncclCommAbort(g->comm[k]);
        g->comm[k] = nullptr;
    }
    g->aborted = true;
    quiesce_group(g);
    return gset(g, FS_E_HIP, msg + " (the group's RCCL communicators were aborted: destroy the group and create it again)");
}

}  // namespace

extern "C" {

uint64_t fs_shard_count(uint64_t n, uint32_t nshards, uint32_t shard) {
    return nshards == 0 ? 0 : framesum::plan::shard_count(n, nshards, shard);
}

uint64_t fs_shard_slab_bytes(uint64_t n, uint32_t nshards) {
    return nshards == 0 ? 0 : framesum::plan::slab_bytes(framesum::plan::shard_rows(n, nshards));
}

fs_status fs_group_create(const int* devices, int ndev, fs_group** out) {
    if (!out) return gset(nullptr, FS_E_INVALID, "fs_group_create: out is NULL");
    *out = nullptr;
    if (!devices || ndev <= 0) return gset(nullptr, FS_E_INVALID, "fs_group_create: no devices");
    for (int k = 0; k < ndev; ++k)
        for (int j = 0; j < k; ++j)
            if (devices[j] == devices[k]) return gset(nullptr, FS_E_INVALID, "fs_group_create: a device appears twice");
    fs_group* g = new (std::nothrow) fs_group();
    if (!g) return gset(nullptr, FS_E_NOMEM, "fs_group_create: out of host memory");
    try {
        g->n = ndev;
        g->dev.assign(devices, devices + ndev);
        g->ctx.assign(ndev, nullptr);
        g->comm.assign(ndev, nullptr);
        g->stream.assign(ndev, nullptr);
        g->xfer.assign(ndev, nullptr);
        g->done.assign((size_t)ndev * kMaxChunks, nullptr);
        g->send.assign(ndev, nullptr);
    } catch (const std::bad_alloc&) {
        delete g;
        return gset(nullptr, FS_E_NOMEM, "fs_group_create: out of host memory");
    }
    for (int k = 0; k < ndev; ++k) {
        const fs_status st = fs_ctx_create(devices[k], &g->ctx[k]);
        if (st != FS_SUCCESS) {
            const std::string msg = std::string("fs_group_create: ") + fs_last_error(nullptr);
            fs_group_destroy(g);
            return gset(nullptr, st, msg);
        }
        hipError_t e = hipSetDevice(devices[k]);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&g->stream[k], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&g->xfer[k], hipStreamNonBlocking);
        for (uint32_t c = 0; c < kMaxChunks && e == hipSuccess; ++c)
            e = hipEventCreateWithFlags(&g->done[(size_t)k * kMaxChunks + c], hipEventDisableTiming);
        if (e != hipSuccess) {
            const std::string msg = std::string("fs_group_create: stream: ") + hipGetErrorString(e);
            fs_group_destroy(g);
            return gset(nullptr, FS_E_HIP, msg);
        }
    }
    const ncclResult_t r = ncclCommInitAll(g->comm.data(), ndev, devices);
    if (r != ncclSuccess) {
        for (auto& c : g->comm) c = nullptr;  // not created
        const std::string msg = std::string("fs_group_create: ncclCommInitAll: ") + ncclGetErrorString(r);
        fs_group_destroy(g);
        return gset(nullptr, FS_E_HIP, msg);
    }
    *out = g;
    return FS_SUCCESS;
}

fs_status fs_group_destroy(fs_group* g) {
    if (!g) return FS_E_INVALID;
    for (int k = 0; k < g->n; ++k) {
        (void)hipSetDevice(g->dev[k]);
        if (g->stream[k]) (void)hipStreamSynchronize(g->stream[k]);
        if (g->xfer[k]) (void)hipStreamSynchronize(g->xfer[k]);
    }
    free_slabs(g);
    for (int k = 0; k < g->n; ++k) {
        if (g->comm[k]) (void)ncclCommDestroy(g->comm[k]);
        (void)hipSetDevice(g->dev[k]);
        if (g->stream[k]) (void)hipStreamDestroy(g->stream[k]);
        if (g->xfer[k]) (void)hipStreamDestroy(g->xfer[k]);
        for (uint32_t c = 0; c < kMaxChunks; ++c)
            if (g->done[(size_t)k * kMaxChunks + c]) (void)hipEventDestroy(g->done[(size_t)k * kMaxChunks + c]);
        if (g->ctx[k]) fs_ctx_destroy(g->ctx[k]);
    }
    delete g;
    return FS_SUCCESS;
}

const char* fs_group_last_error(const fs_group* g) { return g ? g->err.c_str() : g_group_create_err.c_str(); }

#ifdef FS_TEST_HOOKS
// Test library only (seqs_amd/lib/test/libframesum_test.so, -DFS_TEST_HOOKS): the next
// fs_digest_batch_sharded calls on g fail at chunk `chunk` (-1: never), after the earlier chunks'
// kernels, transfers and de-interleaves are queued.
fs_status fs_test_group_set_fault(fs_group* g, long chunk) {
    if (!g) return FS_E_INVALID;
    g->fault_chunk = chunk;
    return FS_SUCCESS;
}
// ... and at chunk `chunk`'s gather, after its grouped sends and receives are enqueued, as if RCCL
// had failed there (the communicator-abort path).
fs_status fs_test_group_set_fault_gather(fs_group* g, long chunk) {
    if (!g) return FS_E_INVALID;
    g->fault_gather = chunk;
    return FS_SUCCESS;
}
#endif



fs_status fs_digest_batch_sharded(fs_group* g, const uint8_t* const* frames, const uint64_t* const* offsets,
                                  const uint32_t* const* lengths, uint64_t n, uint32_t mtu, fs_digest* out,
                                  uint8_t* status) {
    if (!g) return FS_E_INVALID;
    g->err.clear();
    if (g->aborted)
        return gset(g, FS_E_HIP, "fs_digest_batch_sharded: the group's RCCL communicators were aborted by an earlier "
                                 "error: destroy the group and create it again");
    if (n == 0) return FS_SUCCESS;
    if (!frames || !offsets || !lengths || !out) return gset(g, FS_E_INVALID, "fs_digest_batch_sharded: null pointer");
    const uint32_t N = (uint32_t)g->n;
    const uint64_t m = framesum::plan::shard_rows(n, N);
    if (m > (1ull << 31)) return gset(g, FS_E_INVALID, "fs_digest_batch_sharded: more than 2^31 frames per shard");
    const uint64_t sb = framesum::plan::slab_bytes(m);
    fs_status st = ensure_slabs(g, sb);
    if (st != FS_SUCCESS) return st;
    for (uint32_t k = 0; k < N; ++k)
        if (framesum::plan::shard_count(n, N, k) > 0 && (!frames[k] || !offsets[k] || !lengths[k]))
            return gset(g, FS_E_INVALID, "fs_digest_batch_sharded: null shard pointer");
    std::vector<framesum::plan::ChunkXfer> plan;
    try {
        framesum::plan::chunk_plan(n, N, kMaxChunks, kChunkRows, plan);
    } catch (const std::bad_alloc&) {
        return gset(g, FS_E_NOMEM, "fs_digest_batch_sharded: out of host memory");
    }
    hipError_t e = hipSuccess;
    for (uint32_t c = 0; c < (uint32_t)plan.size(); ++c) {
        const framesum::plan::ChunkXfer& x = plan[c];
        if ((long)c == g->fault_chunk)  // test library only: earlier chunks are in flight here
            return fail_group(g, FS_E_HIP, "fs_digest_batch_sharded: injected fault at chunk " + std::to_string(c));
        // chunk c of every shard on its own device's compute stream, into its slab (the first
        // device: in place in the gather buffer)
        for (uint32_t k = 0; k < N; ++k) {
            const uint64_t r = framesum::plan::shard_rows_in(n, N, k, x.lo, x.hi);
            if (r == 0) continue;
            st = fs_digest_batch(g->ctx[k], frames[k], offsets[k] + x.lo, lengths[k] + x.lo, (uint32_t)r, mtu,
                                 reinterpret_cast<fs_digest*>(g->send[k] + 8 * x.lo), g->send[k] + 8 * m + x.lo,
                                 g->stream[k]);
            if (st != FS_SUCCESS)
                return fail_group(g, st, "fs_digest_batch_sharded: shard " + std::to_string(k) + ": " +
                                             fs_last_error(g->ctx[k]));
        }
        // its transfer waits for those kernels only: the compute streams go on with chunk c+1
        for (uint32_t k = 0; k < N && e == hipSuccess; ++k) {
            hipEvent_t ev = g->done[(size_t)k * kMaxChunks + c];
            e = hipSetDevice(g->dev[k]);
            if (e == hipSuccess) e = hipEventRecord(ev, g->stream[k]);
            if (e == hipSuccess) e = hipStreamWaitEvent(g->xfer[k], ev, 0);
        }
        if (e != hipSuccess) break;
        // the chunk's digest and verdict pieces of every other shard to the first device, into
        // their places in the slabs (point-to-point pairs in one group: the gather of this chunk)
        ncclResult_t r = ncclGroupStart();
        for (const framesum::plan::Piece& p : x.pieces) {
            if (r != ncclSuccess) break;
            const uint32_t k = p.shard;
            r = ncclSend(g->send[k] + p.send_dig, 8 * p.rows, ncclUint8, 0, g->comm[k], g->xfer[k]);
            if (r == ncclSuccess) r = ncclSend(g->send[k] + p.send_st, p.rows, ncclUint8, 0, g->comm[k], g->xfer[k]);
            if (r == ncclSuccess) r = ncclRecv(g->recv + p.recv_dig, 8 * p.rows, ncclUint8, (int)k, g->comm[0], g->xfer[0]);
            if (r == ncclSuccess) r = ncclRecv(g->recv + p.recv_st, p.rows, ncclUint8, (int)k, g->comm[0], g->xfer[0]);
        }
        ncclResult_t r2 = ncclGroupEnd();
        if ((long)c == g->fault_gather && r == ncclSuccess && r2 == ncclSuccess)
            r2 = ncclInternalError;  // test library only: the chunk's transfers are enqueued here
        if (r != ncclSuccess || r2 != ncclSuccess)
            return fail_group_comm(g, std::string("fs_digest_batch_sharded: chunk gather: ") +
                                          ncclGetErrorString(r != ncclSuccess ? r : r2));
        e = hipSetDevice(g->dev[0]);
        if (e == hipSuccess) e = framesum::launch_deinterleave(g->recv, N, n, out, status, g->xfer[0], x.g0, x.g1);
        if (e != hipSuccess) break;
    }
    if (e != hipSuccess)
        return fail_group(g, FS_E_HIP, std::string("fs_digest_batch_sharded: ") + hipGetErrorString(e));
    for (uint32_t k = 0; k < N && e == hipSuccess; ++k) {
        e = hipSetDevice(g->dev[k]);
        if (e == hipSuccess) e = hipStreamSynchronize(g->stream[k]);
        if (e == hipSuccess) e = hipStreamSynchronize(g->xfer[k]);
    }
    if (e != hipSuccess)
        return fail_group(g, FS_E_HIP, std::string("fs_digest_batch_sharded: ") + hipGetErrorString(e));
    return FS_SUCCESS;
}

}  // extern "C"
