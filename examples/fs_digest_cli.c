/*
 * Minimal C client of the framesum C ABI (include/framesum.h): what a non-Python host
 * (the Go binding of INTEGRATION.md, a NIC driver loop) does, with nothing but the
 * header and libframesum.so.
 *
 *   fs_digest_cli digest <frames.bin> <offsets.u64> <lengths.u32> <out.bin> [mtu]
 *   fs_digest_cli fill   <frames.bin> <offsets.u64> <lengths.u32> <out.bin> [mtu] [flags]
 *
 * digest: fs_digest_batch_host over the frames; out.bin = n x fs_digest, then n verdict bytes.
 * fill:   fs_fill_batch_host in place; out.bin = the same, then the rewritten frames file.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "framesum.h"

static void* slurp(const char* path, size_t* bytes) {
    FILE* f = fopen(path, "rb");
    if (!f) { perror(path); exit(2); }
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    void* p = malloc(sz > 0 ? (size_t)sz : 1);
    if (sz > 0 && fread(p, 1, (size_t)sz, f) != (size_t)sz) { perror(path); exit(2); }
    fclose(f);
    *bytes = (size_t)sz;
    return p;
}

int main(int argc, char** argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: %s digest|fill frames offsets lengths out [mtu] [flags]\n", argv[0]);
        return 2;
    }
    const int fill = strcmp(argv[1], "fill") == 0;
    size_t fbytes, obytes, lbytes;
    uint8_t* frames = slurp(argv[2], &fbytes);
    uint64_t* offsets = slurp(argv[3], &obytes);
    uint32_t* lengths = slurp(argv[4], &lbytes);
    const uint32_t n = (uint32_t)(lbytes / 4);
    if (obytes != (size_t)n * 8) { fprintf(stderr, "offsets/lengths size mismatch\n"); return 2; }
    const uint32_t mtu = argc > 6 ? (uint32_t)strtoul(argv[6], NULL, 0) : 0u;
    const uint32_t flags = argc > 7 ? (uint32_t)strtoul(argv[7], NULL, 0) : FS_FILL_CSUM;

    fs_ctx* ctx = NULL;
    if (fs_ctx_create(0, &ctx) != FS_SUCCESS) {
        fprintf(stderr, "fs_ctx_create: %s\n", fs_last_error(NULL));
        return 1;
    }
    /* frames in pinned memory, as a NIC ring would be */
    void* pin = NULL;
    if (fs_host_alloc(ctx, fbytes ? fbytes : 1, &pin) != FS_SUCCESS) {
        fprintf(stderr, "fs_host_alloc: %s\n", fs_last_error(ctx));
        return 1;
    }
    memcpy(pin, frames, fbytes);
    fs_digest* out = calloc(n ? n : 1, sizeof(fs_digest));
    uint8_t* status = calloc(n ? n : 1, 1);
    fs_status st = fill ? fs_fill_batch_host(ctx, pin, fbytes, offsets, lengths, n, mtu, flags, out, status)
                        : fs_digest_batch_host(ctx, pin, fbytes, offsets, lengths, n, mtu, out, status);
    if (st != FS_SUCCESS) {
        fprintf(stderr, "%s: %s\n", fill ? "fs_fill_batch_host" : "fs_digest_batch_host", fs_last_error(ctx));
        return 1;
    }
    FILE* o = fopen(argv[5], "wb");
    if (!o) { perror(argv[5]); return 2; }
    fwrite(out, sizeof(fs_digest), n, o);
    fwrite(status, 1, n, o);
    if (fill) fwrite(pin, 1, fbytes, o);
    fclose(o);
    fs_host_free(ctx, pin);
    fs_ctx_destroy(ctx);
    printf("%u frames, ABI %u\n", n, fs_abi_version());
    return 0;
}
