"""Regenerate tests/golden/dhcp_stale.json (committed fixture).

The reference's DHCP server builds its response frame in stacks/dhcp_server.go:187-216
(setResponseUDP), reusing the request's UDPPacket: it computes the IPv4 header checksum at
:203 and only then writes ToS = 192 (:209) and Flags = 0 (:210). The frame it emits therefore
carries a header checksum computed over the REQUEST's ToS and Flags: stale whenever those
differ from (192, 0). RecvEth never verifies the IPv4 checksum (stacks/portstack.go:199-215),
so such frames still pass the stack. The UDP checksum (:216) covers neither field and is valid.

This script restates that sequence step by step with the Python restatement of the header
methods (oracle/pyref.py: IPv4Header.put / calculate_checksum = eth/headers.go:289-301,
:333-340; UDPHeader.calculate_checksum_ipv4 = :382-393) and records, per request:
  pre_hex    the frame as it stands at :203 (request ToS/Flags, checksum fields zero)
  frame_hex  the frame the reference emits (ToS 192, Flags 0, the stale IPv4 checksum)
  stale_ip   the IPv4 checksum the reference writes (over the request's ToS/Flags)
  fresh_ip   the IPv4 checksum of the emitted header bytes (what fs_fill_batch writes for them)
  udp        the UDP checksum (identical either way)
The Go reference cannot run in this image, so the vectors come from the
restatement, which the reference's own KATs pin (tests/golden/kats.json).
Usage: python tests/golden/make_dhcp_stale.py
"""
import json
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import pyref  # noqa: E402

SERVER_MAC = bytes.fromhex("020000000001")
SIADDR = bytes([192, 168, 1, 1])
SERVER_PORT, CLIENT_PORT = 67, 68


def set_response_udp(req_tos: int, req_flags: int, req_id: int, payload: bytes):
    """stacks/dhcp_server.go:187-216 over a request packet with the given ToS / Flags / ID."""
    ip = pyref.IPv4Header(tos=req_tos, flags=req_flags, id=req_id)
    eth_hdr = b"\xff" * 6 + SERVER_MAC + struct.pack(">H", 0x0800)        # :189-193
    ip.destination = b"\0\0\0\0"                                          # :196
    ip.source = SIADDR                                                    # :197
    ip.protocol = 17                                                      # :198
    ip.ttl = 64                                                           # :199
    ip.id = (req_id * 25173 + 13849) & 0xFFFF                             # :200 (any ID: opaque to both sums)
    ip.version_and_ihl = 5                                                # :201
    ip.total_length = 20 + 8 + len(payload)                               # :202
    pre_ip = ip.put()                                                     # the header at :203, checksum 0
    ip.checksum = ip.calculate_checksum()                                 # :203
    stale = ip.checksum
    ip.tos = 192                                                          # :209
    ip.flags = 0                                                          # :210
    udp = pyref.UDPHeader(source_port=SERVER_PORT, destination_port=CLIENT_PORT,
                          length=ip.total_length - 20)                   # :213-215
    udp.checksum = udp.calculate_checksum_ipv4(ip, payload)              # :216
    udp_bytes = struct.pack(">HHHH", udp.source_port, udp.destination_port, udp.length, udp.checksum)
    frame = eth_hdr + ip.put() + udp_bytes + payload
    pre = eth_hdr + pre_ip + struct.pack(">HHHH", udp.source_port, udp.destination_port, udp.length, 0) + payload
    fresh = pyref.decode_ipv4_header(frame[14:])[0].calculate_checksum()
    return pre, frame, stale, fresh, udp.checksum


def main():
    rnd = random.Random(187)
    cases = []
    # request ToS / Flags as a DHCP client may send them (discover with 0/0, DF set, ToS 16),
    # and the one case where the stale checksum happens to be right (192, 0)
    for tos, flags in ((0, 0), (0, 0x4000), (16, 0), (192, 0), (0x48, 0x4000)):
        payload = bytes(rnd.randrange(256) for _ in range(300))
        pre, frame, stale, fresh, udp = set_response_udp(tos, flags, rnd.randrange(1 << 16), payload)
        cases.append({"request_tos": tos, "request_flags": flags, "pre_hex": pre.hex(), "frame_hex": frame.hex(),
                      "stale_ip": stale, "fresh_ip": fresh, "udp": udp})
    out = {"cite": "stacks/dhcp_server.go:187-216 setResponseUDP (checksum at :203, ToS/Flags written at :209-210)",
           "generator": "tests/golden/make_dhcp_stale.py (oracle/pyref.py restatement)", "cases": cases}
    with open(os.path.join(HERE, "dhcp_stale.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", len(cases), "cases")


if __name__ == "__main__":
    main()
