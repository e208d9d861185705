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
    byte_table(t->t1);
    op_table(t->t1, 64, t->zrow);
    op_table(t->t1, 4, t->z4);
    op_table(t->t1, 32, t->z32);
    op_table(t->t1, 16, t->z16);
    // One-byte inverse: the top byte of t1[j] identifies j (it is a permutation).
    uint8_t inv[256];
    bool seen[256] = {false};
    for (uint32_t j = 0; j < 256; ++j) {
        const uint32_t top = t->t1[j] >> 24;
        if (seen[top]) throw std::logic_error("CRC-32 table top bytes are not a permutation");
        seen[top] = true;
        inv[top] = (uint8_t)j;
    }
    std::memcpy(t->inv, inv, sizeof(inv));
}

}  // namespace framesum
