/*
 * framesum ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, scalar restatement of the soypat/seqs frame-checksum path, used
 * by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * CHECKER. It is never linked into, loaded by, or called from the product
 * library (seqs_amd/lib/libframesum.so).
 *
 * Parity pinning: the reference is Go and no Go toolchain exists in this
 * image, so the reference itself cannot be built or run
 * here. This restatement is pinned by every known-answer vector the
 * reference's own tests hold for this path (tests/golden/kats.json, checked by
 * tests/test_oracle.py) and cross-checked against a second, independent
 * pure-Python restatement (oracle/pyref.py). CRC-32 has NO reference
 * implementation; it is pinned by the IEEE 802.3 check value
 * crc32("123456789") = 0xCBF43926 and by zlib's crc32().
 *
 * Every function cites the reference file:line it restates
 * (paths relative to the soypat/seqs repository root).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <pthread.h>
#include <zlib.h>

#include "framesum_oracle.h"

/* ---------------------------------------------------------------------- */
/* eth/crc.go:13-17  type CRC791 struct { sum uint32; excedent uint8; needPad bool } */

void oracle_crc791_reset(oracle_crc791* c) { /* eth/crc.go:84 */
    c->sum = 0;
    c->excedent = 0;
    c->need_pad = 0;
}

static inline uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
static inline uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* eth/crc.go:20-43  func (c *CRC791) Write(buff []byte) (n int, err error) */
size_t oracle_crc791_write(oracle_crc791* c, const uint8_t* buff, size_t len) {
    if (len == 0) return 0;                                   /* :21-23 */
    if (c->need_pad) {                                        /* :24-32 */
        c->sum += ((uint32_t)c->excedent << 8) + (uint32_t)buff[0];
        buff++;
        len--;
        c->excedent = 0;
        c->need_pad = 0;
        if (len == 0) return 1;
    }
    size_t count = len;                                       /* :33-37 hot loop */
    while (count > 1) {
        c->sum += (uint32_t)be16(buff + (len - count));
        count -= 2;
    }
    if (count != 0) {                                         /* :38-41 */
        c->excedent = buff[len - 1];
        c->need_pad = 1;
    }
    return len;
}

/* eth/crc.go:52-59  func (c *CRC791) AddUint16(value uint16) */
void oracle_crc791_add_u16(oracle_crc791* c, uint16_t value) {
    if (c->need_pad) {
        c->sum += ((uint32_t)c->excedent << 8) | (uint32_t)(value >> 8);
        c->excedent = (uint8_t)value;
    } else {
        c->sum += (uint32_t)value;
    }
}

/* eth/crc.go:46-49  func (c *CRC791) AddUint32(value uint32) */
void oracle_crc791_add_u32(oracle_crc791* c, uint32_t value) {
    oracle_crc791_add_u16(c, (uint16_t)(value >> 16));
    oracle_crc791_add_u16(c, (uint16_t)value);
}

/* eth/crc.go:62-69  func (c *CRC791) AddUint8(value uint8) */
void oracle_crc791_add_u8(oracle_crc791* c, uint8_t value) {
    if (c->need_pad) {
        c->sum += ((uint32_t)c->excedent << 8) | (uint32_t)value;
    } else {
        c->excedent = value;
    }
    c->need_pad = !c->need_pad;
}

/* eth/crc.go:72-81  func (c *CRC791) Sum16() uint16 */
uint16_t oracle_crc791_sum16(const oracle_crc791* c) {
    uint32_t sum = c->sum;
    if (c->need_pad) sum += (uint32_t)c->excedent << 8;
    while (sum >> 16 != 0) sum = (sum & 0xffff) + (sum >> 16);
    return (uint16_t)~sum;
}

/* ---------------------------------------------------------------------- */
/* eth/headers.go:333-340  func (iphdr *IPv4Header) CalculateChecksum() uint16
 * via IPv4Header.Put (eth/headers.go:289-301), which forces the version nibble
 * to 4 (`buf[0] = (4 << 4) | (iphdr.VersionAndIHL & 0xf)`), and covers the 20
 * fixed header bytes only (IP options are ignored). `hdr` = frame[14:34]. */
uint16_t oracle_ipv4_checksum(const uint8_t* hdr) {
    uint8_t buf[20];
    memcpy(buf, hdr, 20);
    buf[0] = (uint8_t)((4 << 4) | (hdr[0] & 0xf));
    buf[10] = 0;
    buf[11] = 0;
    oracle_crc791 c;
    oracle_crc791_reset(&c);
    oracle_crc791_write(&c, buf, 20);
    return oracle_crc791_sum16(&c);
}

/* eth/headers.go:382-393  func (uhdr *UDPHeader) CalculateChecksumIPv4(pseudoHeader *IPv4Header, payload []byte) uint16
 * `ip` = frame[14:34], `udp` = the 8-byte UDP header (DecodeUDPHeader, :363-370). */
uint16_t oracle_udp_checksum(const uint8_t* ip, const uint8_t* udp, const uint8_t* payload, size_t n) {
    oracle_crc791 c;
    oracle_crc791_reset(&c);
    oracle_crc791_write(&c, ip + 12, 4);        /* Source */
    oracle_crc791_write(&c, ip + 16, 4);        /* Destination */
    oracle_crc791_add_u16(&c, (uint16_t)ip[9]); /* Protocol, pads with 0 */
    oracle_crc791_add_u16(&c, be16(udp + 4));   /* Length (appears twice) */
    oracle_crc791_add_u16(&c, be16(udp + 0));   /* SourcePort */
    oracle_crc791_add_u16(&c, be16(udp + 2));   /* DestinationPort */
    oracle_crc791_add_u16(&c, be16(udp + 4));   /* Length */
    oracle_crc791_write(&c, payload, n);
    return oracle_crc791_sum16(&c);
}

/* eth/headers.go:510-527  func (thdr *TCPHeader) CalculateChecksumIPv4(pseudoHeader *IPv4Header, tcpOptions, payload []byte) uint16
 * (the `directMethod` branch; the dead PutPseudo branch :528-538 is not taken).
 * Note: UrgentPtr is NOT summed, and the TCP length is
 * TotalLength - IHL*4 in uint16 arithmetic (:516). */
uint16_t oracle_tcp_checksum(const uint8_t* ip, const uint8_t* tcp, const uint8_t* opts, size_t nopts,
                             const uint8_t* payload, size_t n) {
    oracle_crc791 c;
    oracle_crc791_reset(&c);
    uint16_t total_length = be16(ip + 2);
    uint8_t ihl = ip[0] & 0xf;                                   /* headers.go:259 IHL() */
    oracle_crc791_write(&c, ip + 12, 4);
    oracle_crc791_write(&c, ip + 16, 4);
    oracle_crc791_add_u16(&c, (uint16_t)(total_length - (uint16_t)(uint8_t)(ihl * 4)));
    oracle_crc791_add_u16(&c, (uint16_t)ip[9]);
    oracle_crc791_add_u16(&c, be16(tcp + 0));                    /* SourcePort */
    oracle_crc791_add_u16(&c, be16(tcp + 2));                    /* DestinationPort */
    oracle_crc791_add_u32(&c, be32(tcp + 4));                    /* Seq */
    oracle_crc791_add_u32(&c, be32(tcp + 8));                    /* Ack */
    oracle_crc791_add_u16(&c, be16(tcp + 12));                   /* OffsetAndFlags */
    oracle_crc791_add_u16(&c, be16(tcp + 14));                   /* WindowSizeRaw */
    oracle_crc791_write(&c, opts, nopts);
    oracle_crc791_write(&c, payload, n);
    return oracle_crc791_sum16(&c);
}

/* ---------------------------------------------------------------------- */
/* IEEE 802.3 CRC-32 (reflected poly 0xEDB88320, init/xorout 0xFFFFFFFF).
 * NOT in the reference: bit-serial definition, pinned by the
 * check value 0xCBF43926 and by zlib. */
uint32_t oracle_crc32_bitwise(const uint8_t* p, size_t n) {
    uint32_t crc = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; i++) {
        crc ^= p[i];
        for (int k = 0; k < 8; k++) crc = (crc >> 1) ^ (0xEDB88320u & (0u - (crc & 1u)));
    }
    return ~crc;
}

uint32_t oracle_crc32_zlib(const uint8_t* p, size_t n) {
    return (uint32_t)crc32(crc32(0L, Z_NULL, 0), p, (uInt)n);
}

/* ---------------------------------------------------------------------- */
/* stacks/portstack.go:163-308  func (ps *PortStack) RecvEth(ethernetFrame []byte) (err error)
 * restricted to the checksum-relevant gates, for a stack with MTU `mtu`
 * (0 = gate disabled; the reference panics for MTU > 2048, portstack.go:46-48),
 * address filters disabled (MAC :185-186, IP destination :209-210), and at least
 * one UDP and one TCP port open (:227, :285). Returns the FS_* verdict and
 * writes the IPv4 header checksum (headers.go:333, computed for any frame of
 * >= 34 bytes) and the computed L4 checksum (`gotsum`, :239 / :303; 0 when the
 * frame never reaches the compare). */
uint8_t oracle_recv_eth(const uint8_t* f, size_t len, uint32_t mtu, uint16_t* ip_csum, uint16_t* l4_csum) {
    *ip_csum = 0;
    *l4_csum = 0;
    if (len < 14 + 20) return FS_ERR_PACKET_SMOL;                         /* :167-168 */
    if (mtu != 0 && len > mtu) return FS_ERR_EXCEEDS_MTU;                 /* :169-172 */
    *ip_csum = oracle_ipv4_checksum(f + 14);
    uint16_t etype = be16(f + 12);                                        /* headers.go:209-215 */
    if (etype != 0x0800 && etype != 0x0806) return FS_IGNORED_NOT_IPV4;    /* :187-188 */
    if (etype == 0x0806) {                                                /* :191-197 */
        if (len < 14 + 28) return FS_ERR_PACKET_SMOL;
        return FS_ARP;
    }
    const uint8_t* ip = f + 14;                                           /* headers.go:273-286 */
    uint8_t ip_offset = (uint8_t)((ip[0] & 0xf) * 4);
    uint8_t offset = (uint8_t)(14 + ip_offset);                           /* :201 uint8 */
    uint16_t total_length = be16(ip + 2);
    uint16_t end = (uint16_t)(14 + total_length);                         /* :202 uint16 (wraps) */
    if ((ip[0] >> 4) != 4) return FS_ERR_IP_VERSION;                      /* :204 */
    if (ip_offset < 20) return FS_ERR_INVALID_IHL;                        /* :206 */
    if ((uint16_t)offset > end || (size_t)offset > len || (size_t)end > len)
        return FS_ERR_BAD_IP_TOTAL_LEN_OR_IHL;                            /* :211-212 */
    if (mtu != 0 && end > mtu) return FS_ERR_EXCEEDS_MTU;                 /* :213-214 */
    const uint8_t* l4 = f + offset;                                       /* :217 payload[offset:end] */
    size_t l4len = (size_t)(end - offset);
    switch (ip[9]) {
    case 17: {                                                            /* :222-244 */
        if (l4len < 8) return FS_ERR_TOO_SHORT_TCP_OR_UDP;
        uint16_t sport = be16(l4), dport = be16(l4 + 2), ulen = be16(l4 + 4), ucsum = be16(l4 + 6);
        if (dport == 0 || sport == 0) return FS_ERR_ZERO_PORT;
        if (ulen < 8) return FS_ERR_BAD_UDP_LENGTH;
        uint16_t got = oracle_udp_checksum(ip, l4, l4 + 8, l4len - 8);
        *l4_csum = got;
        return got == ucsum ? FS_OK : FS_ERR_CHECKSUM;
    }
    case 6: {                                                             /* :283-308 */
        if (l4len < 20) return FS_ERR_TOO_SHORT_TCP_OR_UDP;
        uint16_t sport = be16(l4), dport = be16(l4 + 2), tcsum = be16(l4 + 16);
        uint8_t toff = (uint8_t)((be16(l4 + 12) >> 12) * 4);              /* headers.go:477-485 */
        if (dport == 0 || sport == 0) return FS_ERR_ZERO_PORT;
        if (toff < 20 || (size_t)toff > l4len) return FS_ERR_BAD_TCP_OFFSET;
        uint16_t got = oracle_tcp_checksum(ip, l4, l4 + 20, (size_t)toff - 20, l4 + toff, l4len - toff);
        *l4_csum = got;
        return got == tcsum ? FS_OK : FS_ERR_CHECKSUM;
    }
    default:
        return FS_ERR_UNKNOWN_IP_PROTO;                                   /* :220-221 */
    }
}

void oracle_frame_digest(const uint8_t* f, size_t len, uint32_t mtu, int use_zlib, oracle_digest* d, uint8_t* status) {
    uint16_t ipc, l4c;
    uint8_t st = oracle_recv_eth(f, len, mtu, &ipc, &l4c);
    d->crc32 = use_zlib ? oracle_crc32_zlib(f, len) : oracle_crc32_bitwise(f, len);
    d->ip_csum = ipc;
    d->l4_csum = l4c;
    if (status) *status = st;
}

/* ---------------------------------------------------------------------- */
/* TX checksum fill. The reference fills a frame's checksums while
 * building it from header structs:
 *   TCP: stacks/port_tcp.go:178  pkt.IP.Checksum = pkt.IP.CalculateChecksum()
 *        stacks/port_tcp.go:193  pkt.TCP.Checksum = pkt.TCP.CalculateChecksumIPv4(&pkt.IP, nil, payload)
 *   UDP: stacks/dhcp_client.go:479 / :486 and dhcp_server.go:203 / :216 (IP, then UDP)
 * Batched over frames whose headers are already in place, the same arithmetic is the one
 * RecvEth verifies (portstack.go:239 / :303, with the frame's own TCP options, nil when
 * the data offset is 5): the IPv4 header checksum goes to frame[24:26] and the computed
 * L4 checksum to the L4 header's checksum field (TCP +16, UDP +6), both big-endian, for
 * every frame whose RecvEth evaluation reaches the checksum compare (FS_OK or
 * FS_ERR_CHECKSUM); other frames are left as they are. Neither written field enters its
 * own checksum, so after the fill RecvEth accepts the frame. The digest and verdict
 * reported are those of the frame as it is afterwards; with ORACLE_FCS_APPEND the
 * frame's IEEE CRC-32 is also written little-endian at frame[len:len+4) (FCS order on the
 * wire). */
void oracle_fill_frame(uint8_t* f, size_t len, uint32_t mtu, uint32_t flags, oracle_digest* d, uint8_t* status) {
    uint16_t ipc, l4c;
    uint8_t st = oracle_recv_eth(f, len, mtu, &ipc, &l4c);
    if ((flags & ORACLE_FILL_CSUM) && (st == FS_OK || st == FS_ERR_CHECKSUM)) {
        size_t off = 14 + (size_t)(f[14] & 0xf) * 4;
        size_t field = off + (f[14 + 9] == 6 ? 16 : 6);
        f[24] = (uint8_t)(ipc >> 8);
        f[25] = (uint8_t)ipc;
        f[field] = (uint8_t)(l4c >> 8);
        f[field + 1] = (uint8_t)l4c;
        st = oracle_recv_eth(f, len, mtu, &ipc, &l4c);
    }
    d->crc32 = oracle_crc32_zlib(f, len);
    d->ip_csum = ipc;
    d->l4_csum = l4c;
    if (flags & ORACLE_FCS_APPEND) {
        for (int b = 0; b < 4; b++) f[len + b] = (uint8_t)(d->crc32 >> (8 * b));
    }
    if (status) *status = st;
}

void oracle_fill_batch(uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths, uint32_t n, uint32_t mtu,
                       uint32_t flags, oracle_digest* out, uint8_t* status) {
    for (uint32_t i = 0; i < n; i++)
        oracle_fill_frame(frames + offsets[i], lengths[i], mtu, flags, &out[i], status ? &status[i] : NULL);
}

/* RX of a raw wire frame that still carries its 4-byte FCS (little-endian IEEE CRC-32 of the
 * bytes before it; SURVEY.md §8f rank 4, not in the reference): the digest and RecvEth
 * verdict of frame[0:len-4), the bytes a NIC that strips the FCS would hand to RecvEth,
 * with the verdict replaced by FS_ERR_FCS when the FCS is missing (len < 4) or differs. */
void oracle_frame_digest_fcs(const uint8_t* f, size_t len, uint32_t mtu, oracle_digest* d, uint8_t* status) {
    size_t inner = len >= 4 ? len - 4 : 0;
    uint8_t st;
    oracle_frame_digest(f, inner, mtu, 0, d, &st);
    if (len < 4) {
        st = FS_ERR_FCS;
    } else {
        uint32_t fcs = (uint32_t)f[inner] | ((uint32_t)f[inner + 1] << 8) | ((uint32_t)f[inner + 2] << 16) |
                       ((uint32_t)f[inner + 3] << 24);
        if (fcs != d->crc32) st = FS_ERR_FCS;
    }
    if (status) *status = st;
}

typedef struct {
    const uint8_t* frames;
    const uint64_t* offsets;
    const uint32_t* lengths;
    uint32_t begin, end, mtu;
    int use_zlib;
    int fcs;
    oracle_digest* out;
    uint8_t* status;
} batch_job;

static void* batch_worker(void* arg) {
    batch_job* j = (batch_job*)arg;
    if (j->fcs) {
        for (uint32_t i = j->begin; i < j->end; i++)
            oracle_frame_digest_fcs(j->frames + j->offsets[i], j->lengths[i], j->mtu, &j->out[i],
                                    j->status ? &j->status[i] : NULL);
        return NULL;
    }
    for (uint32_t i = j->begin; i < j->end; i++)
        oracle_frame_digest(j->frames + j->offsets[i], j->lengths[i], j->mtu, j->use_zlib, &j->out[i],
                            j->status ? &j->status[i] : NULL);
    return NULL;
}

/* Batch driver: frame i = frames[offsets[i] : offsets[i] + lengths[i]].
 * `nthreads` > 1 partitions the frames into contiguous blocks (CPU baseline). */
static void run_batch(const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths, uint32_t n,
                      uint32_t mtu, int use_zlib, int fcs, int nthreads, oracle_digest* out, uint8_t* status) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    batch_job jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t].frames = frames;
        jobs[t].offsets = offsets;
        jobs[t].lengths = lengths;
        jobs[t].begin = (uint32_t)(((uint64_t)n * t) / nthreads);
        jobs[t].end = (uint32_t)(((uint64_t)n * (t + 1)) / nthreads);
        jobs[t].mtu = mtu;
        jobs[t].use_zlib = use_zlib;
        jobs[t].fcs = fcs;
        jobs[t].out = out;
        jobs[t].status = status;
    }
    if (nthreads == 1) {
        batch_worker(&jobs[0]);
        return;
    }
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

void oracle_digest_batch(const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths, uint32_t n,
                         uint32_t mtu, int use_zlib, int nthreads, oracle_digest* out, uint8_t* status) {
    run_batch(frames, offsets, lengths, n, mtu, use_zlib, 0, nthreads, out, status);
}

void oracle_digest_fcs_batch(const uint8_t* frames, const uint64_t* offsets, const uint32_t* lengths, uint32_t n,
                             uint32_t mtu, int nthreads, oracle_digest* out, uint8_t* status) {
    run_batch(frames, offsets, lengths, n, mtu, 1, 1, nthreads, out, status);
}
