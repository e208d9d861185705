"""Pure-Python restatement of the seqs frame-checksum path — TEST INFRASTRUCTURE ONLY.

A second, independent restatement next to the C oracle (framesum_oracle.c): it
follows the Go code's *structure* (decoded header structs, CRC791 state
machine, RecvEth control flow) rather than raw byte offsets, so the two
restatements cross-check each other (tests/test_oracle.py). Small inputs only:
it is pure-Python loops. Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import anything under oracle/.

Citations are relative to the soypat/seqs repository root.
"""
from __future__ import annotations

import struct
import zlib
from dataclasses import dataclass

# Verdict codes (shared contract with include/framesum.h and framesum_oracle.h).
FS_OK = 0
FS_ERR_PACKET_SMOL = 1
FS_ERR_EXCEEDS_MTU = 2
FS_IGNORED_NOT_IPV4 = 3
FS_ARP = 4
FS_ERR_IP_VERSION = 5
FS_ERR_INVALID_IHL = 6
FS_ERR_BAD_IP_TOTAL_LEN_OR_IHL = 7
FS_ERR_UNKNOWN_IP_PROTO = 8
FS_ERR_TOO_SHORT_TCP_OR_UDP = 9
FS_ERR_ZERO_PORT = 10
FS_ERR_BAD_UDP_LENGTH = 11
FS_ERR_BAD_TCP_OFFSET = 12
FS_ERR_CHECKSUM = 13

U16 = 0xFFFF
U32 = 0xFFFFFFFF


class CRC791:
    """eth/crc.go:13-84 — RFC 791 one's-complement running sum (zero value ready)."""

    def __init__(self) -> None:
        self.sum = 0
        self.excedent = 0
        self.need_pad = False

    def write(self, buff: bytes) -> int:  # eth/crc.go:20-43
        if len(buff) == 0:
            return 0
        if self.need_pad:
            self.sum = (self.sum + (self.excedent << 8) + buff[0]) & U32
            buff = buff[1:]
            self.excedent = 0
            self.need_pad = False
            if len(buff) == 0:
                return 1
        count = len(buff)
        while count > 1:
            i = len(buff) - count
            self.sum = (self.sum + ((buff[i] << 8) | buff[i + 1])) & U32
            count -= 2
        if count != 0:
            self.excedent = buff[-1]
            self.need_pad = True
        return len(buff)

    def add_uint32(self, value: int) -> None:  # eth/crc.go:46-49
        self.add_uint16((value >> 16) & U16)
        self.add_uint16(value & U16)

    def add_uint16(self, value: int) -> None:  # eth/crc.go:52-59
        if self.need_pad:
            self.sum = (self.sum + ((self.excedent << 8) | (value >> 8))) & U32
            self.excedent = value & 0xFF
        else:
            self.sum = (self.sum + value) & U32

    def add_uint8(self, value: int) -> None:  # eth/crc.go:62-69
        if self.need_pad:
            self.sum = (self.sum + ((self.excedent << 8) | value)) & U32
        else:
            self.excedent = value
        self.need_pad = not self.need_pad

    def sum16(self) -> int:  # eth/crc.go:72-81
        s = self.sum
        if self.need_pad:
            s = (s + (self.excedent << 8)) & U32
        while s >> 16:
            s = (s & U16) + (s >> 16)
        return (~s) & U16

    def reset(self) -> None:  # eth/crc.go:84
        self.__init__()


def sum_oneshot(b: bytes) -> int:
    """eth/headers_test.go:200-216 `sum()` — the reference tests' independent helper."""
    s = 0
    count = len(b)
    while count > 1:
        i = len(b) - count
        s = (s + ((b[i] << 8) | b[i + 1])) & U32
        count -= 2
    if count > 0:
        s = (s + (b[-1] << 8)) & U32
    while s >> 16:
        s = (s & U16) + (s >> 16)
    return (~s) & U16


@dataclass
class IPv4Header:  # eth/headers.go:~240-286
    version_and_ihl: int = 0
    tos: int = 0
    total_length: int = 0
    id: int = 0
    flags: int = 0
    ttl: int = 0
    protocol: int = 0
    checksum: int = 0
    source: bytes = b"\0\0\0\0"
    destination: bytes = b"\0\0\0\0"

    def ihl(self) -> int:  # eth/headers.go:259
        return self.version_and_ihl & 0xF

    def version(self) -> int:
        return self.version_and_ihl >> 4

    def put(self) -> bytes:  # eth/headers.go:289-301 (version forced to 4)
        return struct.pack(
            ">BBHHHBBH4s4s",
            (4 << 4) | (self.version_and_ihl & 0xF),
            self.tos,
            self.total_length,
            self.id,
            self.flags,
            self.ttl,
            self.protocol,
            self.checksum,
            self.source,
            self.destination,
        )

    def calculate_checksum(self) -> int:  # eth/headers.go:333-340
        buf = bytearray(self.put())
        buf[10:12] = b"\0\0"
        c = CRC791()
        c.write(bytes(buf))
        return c.sum16()


def decode_ipv4_header(buf: bytes) -> tuple[IPv4Header, int]:  # eth/headers.go:273-286
    if len(buf) < 20:
        raise IndexError("DecodeIPv4Header: short buffer")  # `_ = buf[19]` panics
    v, tos, tl, ident, flags, ttl, proto, csum, src, dst = struct.unpack(">BBHHHBBH4s4s", buf[:20])
    h = IPv4Header(v, tos, tl, ident, flags, ttl, proto, csum, src, dst)
    return h, (h.ihl() * 4) & 0xFF


@dataclass
class UDPHeader:  # eth/headers.go:363-393
    source_port: int = 0
    destination_port: int = 0
    length: int = 0
    checksum: int = 0

    def calculate_checksum_ipv4(self, ph: IPv4Header, payload: bytes) -> int:  # :382-393
        c = CRC791()
        c.write(ph.source)
        c.write(ph.destination)
        c.add_uint16(ph.protocol)
        c.add_uint16(self.length)
        c.add_uint16(self.source_port)
        c.add_uint16(self.destination_port)
        c.add_uint16(self.length)
        c.write(payload)
        return c.sum16()


def decode_udp_header(buf: bytes) -> UDPHeader:  # eth/headers.go:363-370
    if len(buf) < 8:
        raise IndexError("DecodeUDPHeader: short buffer")
    return UDPHeader(*struct.unpack(">HHHH", buf[:8]))


@dataclass
class TCPHeader:  # eth/headers.go:429-539
    source_port: int = 0
    destination_port: int = 0
    seq: int = 0
    ack: int = 0
    offset_and_flags: int = 0
    window_size_raw: int = 0
    checksum: int = 0
    urgent_ptr: int = 0

    def offset_in_bytes(self) -> int:  # :477-485
        return ((self.offset_and_flags >> 12) * 4) & 0xFF

    def calculate_checksum_ipv4(self, ph: IPv4Header, options: bytes, payload: bytes) -> int:  # :510-527
        c = CRC791()
        c.write(ph.source)
        c.write(ph.destination)
        c.add_uint16((ph.total_length - ((ph.ihl() * 4) & 0xFF)) & U16)
        c.add_uint16(ph.protocol)
        c.add_uint16(self.source_port)
        c.add_uint16(self.destination_port)
        c.add_uint32(self.seq)
        c.add_uint32(self.ack)
        c.add_uint16(self.offset_and_flags)
        c.add_uint16(self.window_size_raw)
        c.write(options)
        c.write(payload)
        return c.sum16()


def decode_tcp_header(buf: bytes) -> tuple[TCPHeader, int]:  # eth/headers.go:429-440
    if len(buf) < 20:
        raise IndexError("DecodeTCPHeader: short buffer")
    h = TCPHeader(*struct.unpack(">HHIIHHHH", buf[:20]))
    return h, h.offset_in_bytes()


def recv_eth(frame: bytes, mtu: int = 0) -> tuple[int, int, int]:
    """stacks/portstack.go:163-308 checksum gates; returns (verdict, ip_csum, l4_csum).

    Stack model: MTU `mtu` (0 disables both MTU gates), address filters off,
    UDP and TCP ports open. ip_csum = IPv4Header.CalculateChecksum() of
    frame[14:34] for any frame >= 34 B; l4_csum = `gotsum` or 0.
    """
    if len(frame) < 14 + 20:  # :167-168
        return FS_ERR_PACKET_SMOL, 0, 0
    if mtu and len(frame) > mtu:  # :169-172
        return FS_ERR_EXCEEDS_MTU, 0, 0
    ihdr, ip_offset = decode_ipv4_header(frame[14:])
    ip_csum = ihdr.calculate_checksum()
    etype = (frame[12] << 8) | frame[13]
    if etype not in (0x0800, 0x0806):  # :187-188
        return FS_IGNORED_NOT_IPV4, ip_csum, 0
    if etype == 0x0806:  # :191-197
        if len(frame) < 14 + 28:
            return FS_ERR_PACKET_SMOL, ip_csum, 0
        return FS_ARP, ip_csum, 0
    offset = (14 + ip_offset) & 0xFF  # :201 (uint8)
    end = (14 + ihdr.total_length) & U16  # :202 (uint16, wraps)
    if ihdr.version() != 4:  # :204
        return FS_ERR_IP_VERSION, ip_csum, 0
    if ip_offset < 20:  # :206
        return FS_ERR_INVALID_IHL, ip_csum, 0
    if offset > end or offset > len(frame) or end > len(frame):  # :211
        return FS_ERR_BAD_IP_TOTAL_LEN_OR_IHL, ip_csum, 0
    if mtu and end > mtu:  # :213
        return FS_ERR_EXCEEDS_MTU, ip_csum, 0
    payload = frame[offset:end]  # :217
    if ihdr.protocol == 17:  # :222-244
        if len(payload) < 8:
            return FS_ERR_TOO_SHORT_TCP_OR_UDP, ip_csum, 0
        uhdr = decode_udp_header(payload)
        if uhdr.destination_port == 0 or uhdr.source_port == 0:
            return FS_ERR_ZERO_PORT, ip_csum, 0
        if uhdr.length < 8:
            return FS_ERR_BAD_UDP_LENGTH, ip_csum, 0
        got = uhdr.calculate_checksum_ipv4(ihdr, payload[8:])
        return (FS_OK if got == uhdr.checksum else FS_ERR_CHECKSUM), ip_csum, got
    if ihdr.protocol == 6:  # :283-308
        if len(payload) < 20:
            return FS_ERR_TOO_SHORT_TCP_OR_UDP, ip_csum, 0
        thdr, toff = decode_tcp_header(payload)
        if thdr.destination_port == 0 or thdr.source_port == 0:
            return FS_ERR_ZERO_PORT, ip_csum, 0
        if toff < 20 or toff > len(payload):
            return FS_ERR_BAD_TCP_OFFSET, ip_csum, 0
        got = thdr.calculate_checksum_ipv4(ihdr, payload[20:toff], payload[toff:])
        return (FS_OK if got == thdr.checksum else FS_ERR_CHECKSUM), ip_csum, got
    return FS_ERR_UNKNOWN_IP_PROTO, ip_csum, 0  # :220-221


def crc32_ieee(b: bytes) -> int:
    """IEEE 802.3 CRC-32 — not in the reference; zlib is the pin."""
    return zlib.crc32(b) & U32


def frame_digest(frame: bytes, mtu: int = 0) -> tuple[int, int, int, int]:
    """(crc32, ip_csum, l4_csum, verdict) for one frame."""
    verdict, ipc, l4c = recv_eth(frame, mtu)
    return crc32_ieee(frame), ipc, l4c, verdict


FS_ERR_FCS = 14  # FCS missing or wrong (dropped before RecvEth; not in the reference)
FILL_CSUM = 1
FCS_APPEND = 2


def fill_frame(frame: bytes, mtu: int = 0, flags: int = FILL_CSUM) -> tuple[bytes, tuple[int, int, int, int]]:
    """TX fill of one frame, the struct way: the header checksum fields set as
    stacks/port_tcp.go:178 + :193 (TCP) and stacks/dhcp_client.go:479 + :486 (UDP) set them,
    i.e. IPv4 CalculateChecksum() and the L4 checksum RecvEth verifies, for frames that reach
    its compare. Returns (new bytes incl. the appended FCS if asked, digest of the filled frame)."""
    f = bytearray(frame)
    verdict, ipc, got = recv_eth(bytes(f), mtu)
    if flags & FILL_CSUM and verdict in (FS_OK, FS_ERR_CHECKSUM):
        ihdr, ip_offset = decode_ipv4_header(bytes(f[14:]))
        ihdr.checksum = ipc
        f[14:34] = ihdr.put()  # eth/headers.go:289-301 (version is 4 for any frame that got here)
        l4 = 14 + ip_offset
        pos = l4 + (16 if ihdr.protocol == 6 else 6)
        f[pos : pos + 2] = got.to_bytes(2, "big")
    dig = frame_digest(bytes(f), mtu)
    if flags & FCS_APPEND:
        f += dig[0].to_bytes(4, "little")
    return bytes(f), dig


def frame_digest_fcs(wire: bytes, mtu: int = 0) -> tuple[int, int, int, int]:
    """(crc32, ip_csum, l4_csum, verdict) of a wire frame carrying its trailing FCS."""
    inner = wire[:-4] if len(wire) >= 4 else b""
    crc, ipc, l4c, verdict = frame_digest(inner, mtu)
    if len(wire) < 4 or int.from_bytes(wire[-4:], "little") != crc:
        verdict = FS_ERR_FCS
    return crc, ipc, l4c, verdict
