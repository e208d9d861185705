/* A C replay of go/eth/digest_gpu.go (the cgo binding a seqs maintainer adds) through the
 * framesum C ABI: the same packing of a [][]byte batch -- each frame at a 4-byte aligned
 * offset, 4 spare bytes per frame for FillBatch with appendFCS, 16 spare bytes after the last
 * frame, all in pinned memory from fs_host_alloc grown on demand -- and the same calls:
 *   digest  GPU.DigestBatch   -> fs_digest_batch_host
 *   fill    GPU.FillBatch     -> fs_fill_batch_host, then the filled bytes copied back out
 *   multi   GPUs.DigestBatch  -> fs_digest_batch_multi over nctx contexts (all on device 0 here)
 *   sharded Group.DigestSharded -> fs_group_create over every visible device, the batch sharded
 *           round-robin into device memory (what the Go caller's NIC rings would hold; here
 *           hipMalloc + hipMemcpy stand in), fs_digest_batch_sharded, results read back from the
 *           first device
 * Input: a frame list file (u32 n, then n x {u32 len, len bytes}). Output: n fs_digest, n
 * verdict bytes, and for fill the filled frames as a frame list (len + 4 bytes with FCS).
 * tests/test_go_binding.py compares everything with the CPU oracle.
 * usage: go_binding_replay digest|fill|fill_fcs|multi|sharded <in.lst> <mtu> <out.bin> [nctx] */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "framesum.h"

#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

typedef struct {
    uint32_t n;
    uint32_t* len;
    uint8_t** data;
} frame_list;

static int read_list(const char* path, frame_list* fl) {
    FILE* f = fopen(path, "rb");
    if (!f || fread(&fl->n, 4, 1, f) != 1) return -1;
    fl->len = calloc(fl->n + 1, 4);
    fl->data = calloc(fl->n + 1, sizeof(uint8_t*));
    for (uint32_t i = 0; i < fl->n; ++i) {
        if (fread(&fl->len[i], 4, 1, f) != 1) return -1;
        fl->data[i] = malloc(fl->len[i] + 4); /* Go: cap >= len + 4 for appendFCS */
        if (fl->len[i] && fread(fl->data[i], 1, fl->len[i], f) != fl->len[i]) return -1;
    }
    fclose(f);
    return 0;
}

/* GPU.stage: pack into grow-on-demand pinned memory */
typedef struct {
    fs_ctx* ctx;
    uint8_t* pin;
    uint64_t pcap;
    uint64_t* offs;
    uint32_t* lens;
} gpu;

static uint8_t* stage(gpu* g, const frame_list* fl, uint32_t spare, uint64_t* total_out) {
    uint64_t total = 0;
    for (uint32_t i = 0; i < fl->n; ++i) total += ((uint64_t)fl->len[i] + spare + 3) & ~(uint64_t)3;
    total += 16;
    const uint64_t desc = (total + 7) & ~(uint64_t)7; /* the descriptors after the frames, pinned too */
    const uint64_t need = desc + 12 * (uint64_t)fl->n;
    if (need > g->pcap) {
        if (g->pin) fs_host_free(g->ctx, g->pin);
        g->pin = NULL;
        g->pcap = 0;
        void* p = NULL;
        if (fs_host_alloc(g->ctx, need, &p) != FS_SUCCESS) return NULL;
        g->pin = p;
        g->pcap = need;
    }
    g->offs = (uint64_t*)(g->pin + desc);
    g->lens = (uint32_t*)(g->pin + desc + 8 * (uint64_t)fl->n);
    uint64_t pos = 0;
    for (uint32_t i = 0; i < fl->n; ++i) {
        g->offs[i] = pos;
        g->lens[i] = fl->len[i];
        memcpy(g->pin + pos, fl->data[i], fl->len[i]);
        pos += ((uint64_t)fl->len[i] + spare + 3) & ~(uint64_t)3;
    }
    *total_out = total;
    return g->pin;
}

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s digest|fill|fill_fcs|multi in.lst mtu out.bin [nctx]\n", argv[0]);
        return 2;
    }
    const char* mode = argv[1];
    const uint32_t mtu = (uint32_t)strtoul(argv[3], NULL, 10);
    frame_list fl;
    if (read_list(argv[2], &fl) != 0) {
        fprintf(stderr, "cannot read %s\n", argv[2]);
        return 2;
    }
    gpu g = {0};
    if (fs_ctx_create(0, &g.ctx) != FS_SUCCESS) {
        fprintf(stderr, "fs_ctx_create: %s\n", fs_last_error(NULL));
        return 1;
    }
    fs_digest* out = calloc(fl.n + 1, sizeof(fs_digest));
    uint8_t* ver = calloc(fl.n + 1, 1);
    const int fill = !strcmp(mode, "fill") || !strcmp(mode, "fill_fcs");
    const uint32_t spare = !strcmp(mode, "fill_fcs") ? 4u : 0u;
    uint64_t total = 0;
    uint8_t* buf = fl.n ? stage(&g, &fl, spare, &total) : NULL;
    if (fl.n && !buf) {
        fprintf(stderr, "fs_host_alloc: %s\n", fs_last_error(g.ctx));
        return 1;
    }
    fs_status st = FS_SUCCESS;
    if (fl.n && !strcmp(mode, "digest")) {
        st = fs_digest_batch_host(g.ctx, buf, total, g.offs, g.lens, fl.n, mtu, out, ver);
    } else if (fl.n && fill) {
        st = fs_fill_batch_host(g.ctx, buf, total, g.offs, g.lens, fl.n, mtu,
                                FS_FILL_CSUM | (spare ? FS_FCS_APPEND : 0u), out, ver);
        for (uint32_t i = 0; st == FS_SUCCESS && i < fl.n; ++i)
            memcpy(fl.data[i], buf + g.offs[i], fl.len[i] + spare);
    } else if (fl.n && !strcmp(mode, "multi")) {
        const int nctx = argc > 5 ? atoi(argv[5]) : 2;
        fs_ctx** ctxs = calloc((size_t)nctx, sizeof(fs_ctx*));
        ctxs[0] = g.ctx;
        for (int k = 1; k < nctx; ++k)
            if (fs_ctx_create(0, &ctxs[k]) != FS_SUCCESS) {
                fprintf(stderr, "fs_ctx_create: %s\n", fs_last_error(NULL));
                return 1;
            }
        st = fs_digest_batch_multi(ctxs, nctx, buf, total, g.offs, g.lens, fl.n, mtu, out, ver);
        for (int k = 1; k < nctx; ++k) fs_ctx_destroy(ctxs[k]);
        free(ctxs);
    } else if (fl.n && !strcmp(mode, "sharded")) {
        /* Group.DigestSharded: OpenGroup(devices), shard k = global frames k, k + N, ... packed
         * 4-byte aligned into device k's memory, then one call; out/status on device 0 */
        const int N = fs_device_count();
        int* devs = calloc((size_t)N, sizeof(int));
        for (int k = 0; k < N; ++k) devs[k] = k;
        fs_group* grp = NULL;
        if (fs_group_create(devs, N, &grp) != FS_SUCCESS) {
            fprintf(stderr, "fs_group_create: %s\n", fs_group_last_error(NULL));
            return 1;
        }
        const uint8_t** dfr = calloc((size_t)N, sizeof(void*));
        const uint64_t** doff = calloc((size_t)N, sizeof(void*));
        const uint32_t** dlen = calloc((size_t)N, sizeof(void*));
        for (int k = 0; k < N; ++k) {
            const uint64_t nk = fs_shard_count(fl.n, (uint32_t)N, (uint32_t)k);
            uint64_t bytes = 16;
            uint64_t* ho = calloc(nk + 1, 8);
            uint32_t* hl = calloc(nk + 1, 4);
            for (uint64_t j = 0; j < nk; ++j) {
                const uint32_t i = (uint32_t)(j * (uint64_t)N + (uint64_t)k);
                ho[j] = bytes - 16;
                hl[j] = fl.len[i];
                bytes += ((uint64_t)fl.len[i] + 3) & ~(uint64_t)3;
            }
            uint8_t* hb = calloc(bytes, 1);
            for (uint64_t j = 0; j < nk; ++j) memcpy(hb + ho[j], fl.data[j * (uint64_t)N + (uint64_t)k], hl[j]);
            void *df = NULL, *dof = NULL, *dl = NULL;
            if (hipSetDevice(k) != hipSuccess || hipMalloc(&df, bytes) != hipSuccess ||
                hipMalloc(&dof, 8 * (nk + 1)) != hipSuccess || hipMalloc(&dl, 4 * (nk + 1)) != hipSuccess ||
                hipMemcpy(df, hb, bytes, hipMemcpyHostToDevice) != hipSuccess ||
                hipMemcpy(dof, ho, 8 * (nk + 1), hipMemcpyHostToDevice) != hipSuccess ||
                hipMemcpy(dl, hl, 4 * (nk + 1), hipMemcpyHostToDevice) != hipSuccess) {
                fprintf(stderr, "device staging of shard %d failed\n", k);
                return 1;
            }
            dfr[k] = df;
            doff[k] = dof;
            dlen[k] = dl;
            free(hb);
            free(ho);
            free(hl);
        }
        void *dout = NULL, *dst = NULL;
        if (hipSetDevice(0) != hipSuccess || hipMalloc(&dout, 8 * (size_t)fl.n) != hipSuccess ||
            hipMalloc(&dst, fl.n) != hipSuccess) {
            fprintf(stderr, "device output allocation failed\n");
            return 1;
        }
        st = fs_digest_batch_sharded(grp, dfr, doff, dlen, fl.n, mtu, dout, dst);
        if (st != FS_SUCCESS) {
            fprintf(stderr, "sharded failed (%d): %s\n", st, fs_group_last_error(grp));
            return 1;
        }
        if (hipMemcpy(out, dout, 8 * (size_t)fl.n, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(ver, dst, fl.n, hipMemcpyDeviceToHost) != hipSuccess) {
            fprintf(stderr, "result copy failed\n");
            return 1;
        }
        for (int k = 0; k < N; ++k) {
            (void)hipSetDevice(k);
            (void)hipFree((void*)dfr[k]);
            (void)hipFree((void*)doff[k]);
            (void)hipFree((void*)dlen[k]);
        }
        (void)hipSetDevice(0);
        (void)hipFree(dout);
        (void)hipFree(dst);
        fs_group_destroy(grp);
        free(devs);
        printf("sharded over %d device(s)\n", N);
    }
    if (st != FS_SUCCESS) {
        fprintf(stderr, "%s failed (%d): %s\n", mode, st, fs_last_error(g.ctx));
        return 1;
    }
    FILE* o = fopen(argv[4], "wb");
    fwrite(out, sizeof(fs_digest), fl.n, o);
    fwrite(ver, 1, fl.n, o);
    if (fill) {
        fwrite(&fl.n, 4, 1, o);
        for (uint32_t i = 0; i < fl.n; ++i) {
            const uint32_t l = fl.len[i] + spare;
            fwrite(&l, 4, 1, o);
            fwrite(fl.data[i], 1, l, o);
        }
    }
    fclose(o);
    if (g.pin) fs_host_free(g.ctx, g.pin);
    fs_ctx_destroy(g.ctx);
    printf("%s: %u frames\n", mode, fl.n);
    return 0;
}
