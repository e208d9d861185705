/* framesum ORACLE — TEST INFRASTRUCTURE ONLY (see framesum_oracle.c header). */
#ifndef FRAMESUM_ORACLE_H
#define FRAMESUM_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* RecvEth verdicts (stacks/portstack.go:120-142). Numeric values are the
 * contract shared with include/framesum.h (tests assert they agree). */
enum {
    FS_OK = 0,                        /* checksum verified; RecvEth continues to port lookup */
    FS_ERR_PACKET_SMOL = 1,           /* errPacketSmol          portstack.go:124 */
    FS_ERR_EXCEEDS_MTU = 2,           /* errPacketExceedsMTU    portstack.go:122 */
    FS_IGNORED_NOT_IPV4 = 3,          /* `return nil` for non-IPv4/ARP  :187-188 */
    FS_ARP = 4,                       /* handed to arpClient.recv  :191-197 */
    FS_ERR_IP_VERSION = 5,            /* errIPVersion           :135 */
    FS_ERR_INVALID_IHL = 6,           /* errInvalidIHL          :134 */
    FS_ERR_BAD_IP_TOTAL_LEN_OR_IHL = 7, /* errBadIPTotalLenOrIHL :141 */
    FS_ERR_UNKNOWN_IP_PROTO = 8,      /* errUnknownIPProto      :136 */
    FS_ERR_TOO_SHORT_TCP_OR_UDP = 9,  /* errTooShortTCPOrUDP    :125 */
    FS_ERR_ZERO_PORT = 10,            /* errZeroPort            :129 */
    FS_ERR_BAD_UDP_LENGTH = 11,       /* errBadUDPLength        :133 */
    FS_ERR_BAD_TCP_OFFSET = 12,       /* errBadTCPOffset        :130 */
    FS_ERR_CHECKSUM = 13,             /* ErrChecksumTCPorUDP    :132 */
    FS_ERR_FCS = 14                   /* FCS missing or wrong (dropped before RecvEth; not in seqs) */
};

/* fill flags (TX) */
#define ORACLE_FILL_CSUM 1u
#define ORACLE_FCS_APPEND 2u

typedef struct {
    uint32_t crc32;
    uint16_t ip_csum;
    uint16_t l4_csum;
} oracle_digest;

typedef struct {
    uint32_t sum;
    uint8_t excedent;
    uint8_t need_pad;
} oracle_crc791;

void oracle_crc791_reset(oracle_crc791* c);
size_t oracle_crc791_write(oracle_crc791* c, const uint8_t* buff, size_t len);
void oracle_crc791_add_u16(oracle_crc791* c, uint16_t value);
void oracle_crc791_add_u32(oracle_crc791* c, uint32_t value);
void oracle_crc791_add_u8(oracle_crc791* c, uint8_t value);
uint16_t oracle_crc791_sum16(const oracle_crc791* c);

uint16_t oracle_ipv4_checksum(const uint8_t* hdr20);
uint16_t oracle_udp_checksum(const uint8_t* ip, const uint8_t* udp, const uint8_t* payload, size_t n);
uint16_t oracle_tcp_checksum(const uint8_t* ip, const uint8_t* tcp, const uint8_t* opts, size_t nopts,
                             const uint8_t* payload, size_t n);
uint32_t oracle_crc32_bitwise(const uint8_t* p, size_t n);
uint32_t oracle_crc32_zlib(const uint8_t* p, size_t n);
uint8_t oracle_recv_eth(const uint8_t* f, size_t len, uint32_t mtu, uint16_t* ip_csum, uint16_t* l4_csum);
void oracle_frame_digest(const uint8_t* f, size_t len, uint32_t mtu, int use_zlib, oracle_digest* d,
                         uint8_t* status);
void oracle_fill_frame(uint8_t* f, size_t len, uint32_t mtu, uint32_t flags, oracle_digest* d, uint8_t* status);
void oracle_fill_batch(uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths, uint32_t n, uint32_t mtu,
                       uint32_t flags, oracle_digest* out, uint8_t* status);
void oracle_frame_digest_fcs(const uint8_t* f, size_t len, uint32_t mtu, oracle_digest* d, uint8_t* status);
void oracle_digest_fcs_batch(const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths, uint32_t n,
                             uint32_t mtu, int nthreads, oracle_digest* out, uint8_t* status);
void oracle_digest_batch(const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths, uint32_t n,
                         uint32_t mtu, int use_zlib, int nthreads, oracle_digest* out, uint8_t* status);

#ifdef __cplusplus
}
#endif
#endif
