// Host construction of the CRC-32 zero-shift operator tables (FsTables).
//
// CRC-32 (IEEE 802.3, reflected poly 0xEDB88320) is linear over GF(2): feeding
// k zero bytes to the register is the linear map Z_k = multiplication by
// x^(8k) mod P. A 32-bit register value decomposes into 4 bytes, so
// Z_k(R) = T_k[0][R&0xff] ^ T_k[1][(R>>8)&0xff] ^ T_k[2][(R>>16)&0xff] ^ T_k[3][R>>24]
// with T_k[b][v] = Z_k(v << 8b). The kernel evaluates every stream step and
// every combine step this way (framesum_kernel.hip header comment).
#include <cstring>
#include <stdexcept>

#include "framesum_internal.h"

namespace framesum {
namespace {

void byte_table(uint32_t t1[256]) {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
        t1[i] = c;
    }
}

uint32_t zero_shift(const uint32_t t1[256], uint32_t r, int nbytes) {
    for (int i = 0; i < nbytes; ++i) r = (r >> 8) ^ t1[r & 0xffu];
    return r;
}

void op_table(const uint32_t t1[256], int nbytes, uint32_t out[4][256]) {
    for (int b = 0; b < 4; ++b)
        for (uint32_t v = 0; v < 256; ++v) out[b][v] = zero_shift(t1, v << (8 * b), nbytes);
}

}  // namespace

void build_tables(FsTables* t) {
    std::memset(t, 0, sizeof(*t));
    uint32_t t1[256];
    byte_table(t1);
    static uint32_t zrow[4][256];
    op_table(t1, 64, zrow);
    for (uint32_t e = 0; e < 256; ++e)
        for (uint32_t b = 0; b < 4; ++b)
            for (uint32_t c = 0; c < 8; ++c) t->region_a[e][8 * b + c] = zrow[b][e];
    for (uint32_t b = 0; b < 4; ++b)
        for (uint32_t j = 0; j < 8; ++j) t->z64_basis[b][j] = zrow[b][1u << j];
    // region A entries are the XOR of the basis columns of their set bits (GF(2) linearity)
    for (uint32_t b = 0; b < 4; ++b)
        for (uint32_t e = 0; e < 256; ++e) {
            uint32_t v = 0;
            for (uint32_t j = 0; j < 8; ++j)
                if ((e >> j) & 1u) v ^= t->z64_basis[b][j];
            if (v != zrow[b][e]) throw std::logic_error("Z_64 basis mismatch");
        }
    op_table(t1, 32, t->z32);
    op_table(t1, 16, t->z16);
    for (int k = 0; k < 4; ++k) op_table(t1, 4 - k, t->zfin[k]);
    op_table(t1, 48, t->z48);
    op_table(t1, 12, t->z12);
    op_table(t1, 8, t->z8);
    op_table(t1, 768, t->z768);
    // the plain tables' bases (every [4][256] table is GF(2)-linear in its byte, as region A)
    const uint32_t* plain = &t->z32[0][0];
    for (uint32_t p = 0; p < 40; ++p)
        for (uint32_t j = 0; j < 8; ++j) t->plain_basis[p][j] = plain[256 * p + (1u << j)];
    for (uint32_t p = 0; p < 40; ++p)
        for (uint32_t e = 0; e < 256; ++e) {
            uint32_t v = 0;
            for (uint32_t j = 0; j < 8; ++j)
                if ((e >> j) & 1u) v ^= t->plain_basis[p][j];
            if (v != plain[256 * p + e]) throw std::logic_error("plain table basis mismatch");
        }
    // The final step Z_(4-t) replaces "Z_4 then undo t appended zero bytes"; Z_1[0] is the
    // standard byte table used for frames shorter than 4 bytes.
    if (std::memcmp(t->zfin[3][0], t1, sizeof(t1)) != 0) throw std::logic_error("Z_1 table mismatch");
}

}  // namespace framesum
