/* The CPU oracle (oracle/framesum_oracle.c, TEST INFRASTRUCTURE) built with ASan + UBSan
 * (tests/csrc/Makefile) and driven over the reference's known-answer frames
 * and random frames of every shape the parity tests use: odd lengths, short frames, IP and
 * TCP options, inconsistent lengths, padding, ARP / non-IPv4, every flag of the TX fill and
 * the FCS verify. A memory or UB error aborts; the KATs must still hold. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/framesum_oracle.h"

static int fails = 0;
#define CHECK(c)                                                                      \
    do {                                                                              \
        if (!(c)) {                                                                   \
            fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c);     \
            fails++;                                                                  \
        }                                                                             \
    } while (0)

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) {
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return (uint32_t)(rng_state >> 11);
}

static int hex(char c) { return c <= '9' ? c - '0' : (c | 32) - 'a' + 10; }
static size_t unhex(const char* s, uint8_t* out) {
    size_t n = 0;
    for (; s[0] && s[1]; s += 2) out[n++] = (uint8_t)(hex(s[0]) << 4 | hex(s[1]));
    return n;
}

/* the reference's known-answer frames (tests/golden/kats.json "frames", transcribed from
 * eth/headers_test.go and stacks/stacks_test.go:591-594): kats_gen.h is generated from the
 * fixture by tests/test_host_sanitizers.py */
#include "kats_gen.h"

/* a random frame: valid-looking Eth + IPv4 (+options) + TCP/UDP (+options), then damage */
static size_t random_frame(uint8_t* f, size_t cap) {
    size_t len = rnd() % (rnd() % 4 == 0 ? 9100u : 1600u);
    if (len > cap) len = cap;
    for (size_t i = 0; i < len; ++i) f[i] = (uint8_t)rnd();
    if (len >= 14) {
        const uint32_t et = rnd() % 10;
        f[12] = et == 0 ? 0x08 : et == 1 ? 0x86 : 0x08;
        f[13] = et == 0 ? 0x06 : et == 1 ? 0xdd : 0x00;
    }
    if (len >= 34) {
        const uint32_t ihl = rnd() % 8 == 0 ? rnd() % 16 : 5 + rnd() % 3;
        f[14] = (uint8_t)((rnd() % 16 == 0 ? rnd() % 16 : 4) << 4 | ihl);
        uint32_t tl = (uint32_t)len - 14 - (rnd() % 4 == 0 ? rnd() % 40 : 0);
        if (rnd() % 16 == 0) tl = rnd() & 0xffff;
        f[16] = (uint8_t)(tl >> 8);
        f[17] = (uint8_t)tl;
        f[23] = rnd() % 8 == 0 ? (uint8_t)rnd() : rnd() % 2 ? 6 : 17;
        const size_t l4 = 14 + 4 * ihl;
        if (l4 + 14 <= len) f[l4 + 12] = (uint8_t)((5 + rnd() % 11) << 4);
    }
    return len;
}

int main(void) {
    uint8_t buf[9300];
    /* KATs */
    for (int k = 0; k < KAT_N; ++k) {
        const size_t n = unhex(kat_hex[k], buf);
        oracle_digest d;
        uint8_t st = 0xff;
        oracle_frame_digest(buf, n, 0, 1, &d, &st);
        CHECK(st == kat_verdict[k]);
        CHECK(d.l4_csum == kat_l4[k]);
        CHECK(d.ip_csum == kat_ip[k]);
    }
    CHECK(oracle_crc32_bitwise((const uint8_t*)"123456789", 9) == 0xCBF43926u);
    CHECK(oracle_crc32_zlib((const uint8_t*)"123456789", 9) == 0xCBF43926u);
    /* random frames through every entry point: digest, fill (all flags), FCS verify */
    for (int it = 0; it < 20000; ++it) {
        const size_t len = random_frame(buf, 9200);
        uint8_t* g = malloc(len + 4); /* exact-size heap copy (+ FCS room): ASan sees any overread */
        memcpy(g, buf, len);
        oracle_digest d1, d2;
        uint8_t s1, s2;
        const uint32_t mtu = rnd() % 3 == 0 ? 1514 : 0;
        oracle_frame_digest(g, len, mtu, (int)(rnd() & 1), &d1, &s1);
        CHECK(s1 <= FS_ERR_CHECKSUM);
        const uint32_t flags = rnd() % 4;
        oracle_fill_frame(g, len, mtu, flags, &d2, &s2);
        if (flags & ORACLE_FILL_CSUM) CHECK(s2 != FS_ERR_CHECKSUM);
        if (flags & ORACLE_FCS_APPEND) {
            oracle_frame_digest_fcs(g, len + 4, mtu, &d1, &s1);
            CHECK(s1 != FS_ERR_FCS);
            CHECK(d1.crc32 == d2.crc32);
        } else {
            oracle_frame_digest_fcs(g, len, mtu, &d1, &s1);
        }
        free(g);
    }
    /* batch entry points with threads over a packed batch */
    {
        enum { N = 3000 };
        uint64_t off[N];
        uint32_t ln[N];
        size_t total = 0;
        for (int i = 0; i < N; ++i) {
            ln[i] = rnd() % 1600;
            off[i] = total;
            total += (ln[i] + 3) & ~3u;
        }
        uint8_t* frames = malloc(total + 16);
        for (size_t i = 0; i < total + 16; ++i) frames[i] = (uint8_t)rnd();
        oracle_digest* out = malloc(sizeof(oracle_digest) * N);
        uint8_t* st = malloc(N);
        oracle_digest_batch(frames, off, ln, N, 0, 1, 4, out, st);
        oracle_digest_fcs_batch(frames, off, ln, N, 0, 4, out, st);
        free(frames);
        free(out);
        free(st);
    }
    if (fails) {
        fprintf(stderr, "%d check(s) failed\n", fails);
        return 1;
    }
    printf("oracle sanitizer run OK\n");
    return 0;
}
