"""Pins the branch order of the Go RecvEthBatch (CPU only).

go/stacks/portstack_batch.go finishes each frame from the GPU verdict by walking the table
`recvEthGates`. There is no Go toolchain in this image, so this test reads that table (and the
verdict constants of go/eth/digest_gpu.go) from the Go sources as data, runs it with the
semantics of recvEthVerified's switch, and compares the outcome with a line-by-line Python
transliteration of RecvEth (/root/reference/stacks/portstack.go:163-355, restated below with
line citations), for every frame of the edge batch (every verdict class, ARP, non-IPv4) and every
stack state: destination MAC ours / broadcast / foreign, our IP unset / the frame's / another,
UDP and TCP sockets none / on the frame's port / on another port, a global handler that passes
or fails, MTU 600 / 1514 / 2048. The GPU verdict is the C oracle's (equal to the GPU's by the
parity suite)."""
import os
import re
import struct

import numpy as np
import pytest

import framegen
from oracle import coracle
from seqs_amd import pack_frames

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO_BATCH = os.path.join(ROOT, "go", "stacks", "portstack_batch.go")
GO_ETH = os.path.join(ROOT, "go", "eth", "digest_gpu.go")
OUR_MAC = bytes.fromhex("02aabbccddee")
BROADCAST = b"\xff" * 6


def go_verdicts():
    """Verdict name -> value, from the const block of go/eth/digest_gpu.go."""
    src = open(GO_ETH).read()
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"^\s*(Verdict\w+)\s+Verdict\s*=\s*(\d+)", src, re.M)}


def go_gates():
    """recvEthGates and verdictErr of go/stacks/portstack_batch.go, as data."""
    src = open(GO_BATCH).read()
    vals = go_verdicts()
    body = re.search(r"var recvEthGates = \[\.\.\.\]gate\{(.*?)\n\}", src, re.S).group(1)
    gates = []
    for line in body.strip().splitlines():
        m = re.match(r"\s*\{kind: (gate\w+)(?:, classes: \[\]eth\.Verdict\{([^}]*)\})?(?:, logged: (true|false))?\},", line)
        assert m, f"unparsed gate line: {line!r}"
        classes = [vals[c.strip().split(".")[1]] for c in m.group(2).split(",")] if m.group(2) else []
        gates.append((m.group(1), classes, m.group(3) == "true"))
    verr = {}
    eb = re.search(r"var verdictErr = \[\.\.\.\]error\{(.*?)\n\}", src, re.S).group(1)
    for m in re.finditer(r"eth\.(Verdict\w+):\s*(\w+),", eb):
        verr[vals[m.group(1)]] = None if m.group(2) == "nil" else m.group(2)
    return gates, verr


class Stack:
    def __init__(self, mac, ip, udp, tcp, glob_fails, mtu):
        self.mac, self.ip, self.udp, self.tcp, self.glob_fails, self.mtu = mac, ip, udp, tcp, glob_fails, mtu

    def find_port(self, ports, dport):
        # ports: 0 no sockets, 1 a socket on the frame's destination port, 2 one on another port
        return ports == 1


def recv_eth_reference(f: bytes, ps: Stack):
    """stacks/portstack.go:163-355, branch for branch (outcomes, no side effects beyond them)."""
    if len(f) < 14 + 20:                                            # :166-167
        return ("err", "errPacketSmol")
    if len(f) > ps.mtu:                                             # :168-171
        return ("err", "errPacketExceedsMTU")
    dst, etype = f[0:6], struct.unpack(">H", f[12:14])[0]           # :176 DecodeEthernetHeader
    if ps.glob_fails:                                               # :178-184
        return ("err", "glob")
    if dst != BROADCAST and dst != ps.mac:                          # :186-187
        return ("nil", "mac")
    if etype != 0x0800 and etype != 0x0806:                         # :187-189
        return ("nil", "etype")
    if etype == 0x0806:                                             # :191-197
        if len(f) < 14 + 28:
            return ("err", "errPacketSmol")
        return ("arp",)
    vihl = f[14]                                                    # :200 DecodeIPv4Header
    ipoff = (vihl & 0xF) * 4
    offset = 14 + ipoff                                             # :201
    tl = struct.unpack(">H", f[16:18])[0]
    end = (14 + tl) & 0xFFFF                                        # :202 (uint16)
    proto, ipdst = f[23], f[30:34]
    if (vihl >> 4) != 4:                                            # :204
        return ("err", "errIPVersion")
    if ipoff < 20:                                                  # :206
        return ("err", "errInvalidIHL")
    if ps.ip != ipdst and ps.ip != b"\0\0\0\0":                     # :209
        return ("nil", "ip")
    if offset > end or offset > len(f) or end > len(f):             # :211
        return ("err", "errBadIPTotalLenOrIHL")
    if end > ps.mtu:                                                # :213
        return ("err", "errPacketExceedsMTU")
    payload = f[offset:end]                                         # :217
    if proto == 17:                                                 # :222-244
        if ps.udp == 0:
            return ("nil", "nosock")
        if len(payload) < 8:
            return ("err", "errTooShortTCPOrUDP")
        sport, dport, ulen = struct.unpack(">HHH", payload[0:6])
        if dport == 0 or sport == 0:
            return ("err", "errZeroPort")
        if ulen < 8:
            return ("err", "errBadUDPLength")
        if not udp_checksum_ok(f, offset, end):                     # :239-242
            return ("err", "ErrChecksumTCPorUDP")
        return ("deliver", 17) if ps.find_port(ps.udp, dport) else ("nil", "noport")   # :244-246
    if proto == 6:                                                  # :283-308
        if ps.tcp == 0:
            return ("nil", "nosock")
        if len(payload) < 20:
            return ("err", "errTooShortTCPOrUDP")
        sport, dport = struct.unpack(">HH", payload[0:4])
        toff = (payload[12] >> 4) * 4
        if dport == 0 or sport == 0:
            return ("err", "errZeroPort")
        if toff < 20 or toff > len(payload):
            return ("err", "errBadTCPOffset")
        if not tcp_checksum_ok(f, offset, end):                     # :303-306
            return ("err", "ErrChecksumTCPorUDP")
        return ("deliver", 6) if ps.find_port(ps.tcp, dport) else ("nil", "noport")    # :307-312
    return ("err", "errUnknownIPProto")                             # :219-220


def _csum(words_sum):
    s = words_sum
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def _sum16(b):
    if len(b) & 1:
        b = b + b"\0"
    return sum(struct.unpack(f">{len(b) // 2}H", b))


def udp_checksum_ok(f, offset, end):
    """eth/headers.go:382-393: the pseudo-header, the UDP length counted twice, checksum excluded."""
    seg = f[offset:end]
    ulen = struct.unpack(">H", seg[4:6])[0]
    s = _sum16(f[26:34]) + 17 + ulen + _sum16(seg[0:4]) + ulen + _sum16(seg[8:])
    return _csum(s) == struct.unpack(">H", seg[6:8])[0]


def tcp_checksum_ok(f, offset, end):
    """eth/headers.go:510-527: pseudo-header with (TL - IHL*4) mod 2^16, no urgent pointer."""
    seg = f[offset:end]
    tl = struct.unpack(">H", f[16:18])[0]
    ipoff = (f[14] & 0xF) * 4
    s = _sum16(f[26:34]) + 6 + ((tl - ipoff) & 0xFFFF) + _sum16(seg[0:16]) + _sum16(seg[20:])
    return _csum(s) == struct.unpack(">H", seg[16:18])[0]


def recv_eth_batch_table(f: bytes, v: int, ps: Stack, gates, verr):
    """recvEthVerified (go/stacks/portstack_batch.go): walk recvEthGates with the verdict v."""
    names = {13: "ErrChecksumTCPorUDP"}
    ethtype = struct.unpack(">H", f[12:14])[0] if len(f) >= 14 else 0
    for kind, classes, _logged in gates:
        if kind == "gateLength":
            if len(f) < 34:
                return ("err", "errPacketSmol")
            if len(f) > ps.mtu:
                return ("err", "errPacketExceedsMTU")
        elif kind == "gateGlobal":
            if ps.glob_fails:
                return ("err", "glob")
        elif kind == "gateMAC":
            if f[0:6] != BROADCAST and f[0:6] != ps.mac:
                return ("nil", "mac")
        elif kind == "gateEtherType":
            if ethtype == 0x0806:
                return ("err", "errPacketSmol") if v == 1 else ("arp",)
            if ethtype != 0x0800:
                return ("nil", "etype")
        elif kind == "gateVerdict":
            if v in classes:
                e = verr[v]
                return ("err", names.get(v, e)) if e else ("nil", "verdict")
        elif kind == "gateIPDest":
            if ps.ip != f[30:34] and ps.ip != b"\0\0\0\0":
                return ("nil", "ip")
        elif kind == "gateSockets":
            if (f[23] == 17 and ps.udp == 0) or (f[23] == 6 and ps.tcp == 0):
                return ("nil", "nosock")
        elif kind == "gateDeliver":
            if v != 0:  # fail closed (go_deliver_fails_closed pins that the Go step does this)
                return ("err", "errUnexpectedVerdict")
            ipoff = (f[14] & 0xF) * 4
            dport = struct.unpack(">H", f[14 + ipoff + 2: 14 + ipoff + 4])[0]
            ports = ps.udp if f[23] == 17 else ps.tcp
            return ("deliver", int(f[23])) if ps.find_port(ports, dport) else ("nil", "noport")
        else:
            raise AssertionError(f"unknown gate kind {kind}")
    return ("nil", "end")


def frames_for_gates():
    frames = [bytes(f) for f in framegen.edge_batch(20250212, n_random=120)]
    out = []
    for f in frames:
        out.append(f)
        if len(f) >= 14:  # the same frame to our MAC, broadcast and a foreign MAC
            out.append(OUR_MAC + f[6:])
            out.append(BROADCAST + f[6:])
    # ARP frames around the ARP length gate (:192), to us
    for L in (34, 41, 42, 60):
        out.append(OUR_MAC + bytes(6) + b"\x08\x06" + bytes(L - 14))
    return out


def test_gate_table_parses():
    gates, verr = go_gates()
    kinds = [g[0] for g in gates]
    assert kinds[0] == "gateLength" and kinds[-1] == "gateDeliver"
    assert set(verr) == set(range(14))


@pytest.mark.parametrize("mtu", [600, 1514, 2048])
def test_recv_eth_batch_gate_order_matches_recv_eth(mtu):
    gates, verr = go_gates()
    frames = frames_for_gates()
    buf, off, ln = pack_frames(frames, align=1)
    _, verdicts = coracle.digest_batch(buf, off.astype(np.int64), ln.astype(np.int32), mtu=mtu)
    checked, outcomes = 0, set()
    for f, v in zip(frames, verdicts):
        ipdst = f[30:34] if len(f) >= 34 else b"\x0a\0\0\x01"
        for mac in (OUR_MAC, b"\x02\x11\x22\x33\x44\x55"):
            for ip in (b"\0\0\0\0", ipdst, b"\x0a\x63\x63\x63"):
                for udp in (0, 1, 2):
                    for tcp in (0, 1, 2):
                        for glob_fails in (False, True):
                            ps = Stack(mac, ip, udp, tcp, glob_fails, mtu)
                            want = recv_eth_reference(f, ps)
                            got = recv_eth_batch_table(f, int(v), ps, gates, verr)
                            assert got == want, (f"frame len {len(f)} verdict {int(v)} mac {mac.hex()} ip {ip.hex()} "
                                                 f"udp {udp} tcp {tcp} glob {glob_fails}: table {got}, RecvEth {want}")
                            checked += 1
                            outcomes.add(want)
    # the walk reached every kind of outcome
    kinds = {o[0] if o[0] != "err" else o[1] for o in outcomes}
    for k in ("deliver", "arp", "nil", "errPacketSmol", "errIPVersion", "errInvalidIHL", "errBadIPTotalLenOrIHL",
              "errUnknownIPProto", "errTooShortTCPOrUDP", "errZeroPort", "ErrChecksumTCPorUDP", "glob"):
        assert k in kinds, f"no frame reached {k}"
    assert checked > 10000


def go_deliver_fails_closed():
    """The gateDeliver case of recvEthVerified returns errUnexpectedVerdict for any verdict other
    than VerdictOK before it touches the segment (fail closed)."""
    src = open(GO_BATCH).read()
    body = re.search(r"case gateDeliver:\n(.*?)\n\t\t\}\n\t\}", src, re.S).group(1)
    first = [ln.strip() for ln in body.splitlines() if ln.strip()][:2]
    return first == ["if v != eth.VerdictOK { // fail closed: only a verified frame reaches a socket",
                     "return errUnexpectedVerdict"]


def test_deliver_step_fails_closed_in_go_source():
    assert go_deliver_fails_closed()


@pytest.mark.parametrize("v", [14, 15, 63, 255])
def test_verdicts_outside_the_table_never_deliver(v):
    """A verdict no step of the table names (VerdictFCS, an unknown value, a corrupted status
    byte) on a frame that would otherwise be delivered ends with an error, never at a socket."""
    gates, verr = go_gates()
    frames = frames_for_gates()
    buf, off, ln = pack_frames(frames, align=1)
    _, verdicts = coracle.digest_batch(buf, off.astype(np.int64), ln.astype(np.int32), mtu=1514)
    reached = 0
    for f, v0 in zip(frames, verdicts):
        if int(v0) != 0 or len(f) < 34 or f[12:14] != b"\x08\x00":
            continue
        ps = Stack(f[0:6], b"\0\0\0\0", 1, 1, False, 1514)
        if recv_eth_batch_table(f, 0, ps, gates, verr)[0] != "deliver":
            continue
        got = recv_eth_batch_table(f, v, ps, gates, verr)
        assert got[0] != "deliver", f"verdict {v} delivered"
        assert got == ("err", "errUnexpectedVerdict"), got
        reached += 1
    assert reached > 20
