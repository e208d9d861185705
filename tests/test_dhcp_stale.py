"""The DHCP server's stale IPv4 header checksum (stacks/dhcp_server.go:203 vs :209-210).

The reference computes the response's IPv4 checksum before it writes ToS = 192 and Flags = 0,
so the frame it emits carries a checksum over the request's ToS/Flags (tests/golden/
dhcp_stale.json, made by tests/golden/make_dhcp_stale.py). What the engine does with it:

* given the frame as it stands at :203 (the request's ToS/Flags), fs_fill_batch writes exactly
  the checksums the reference writes; applying the reference's two later writes (:209-210)
  then yields the reference's emitted bytes, bit for bit;
* given the emitted bytes, fs_fill_batch writes the checksum OF THOSE BYTES (RFC 791): a
  deliberate divergence from the reference's stale value whenever the request's ToS/Flags
  were not (192, 0). The reference has no TX-fill entry point over finished frames, so this is
  an extension, not a parity case;
* on RX the emitted frame passes (RecvEth never verifies the IPv4 checksum,
  stacks/portstack.go:199-215; the UDP checksum is valid): verdict OK, ip_csum = the fresh value.
"""
import json
import os

import numpy as np
import pytest

from oracle import coracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "dhcp_stale.json")


def _cases():
    return json.load(open(GOLDEN))["cases"]


def _reference_writes(frame: bytearray) -> None:
    """stacks/dhcp_server.go:209-210, applied after the fill."""
    frame[15] = 192
    frame[20:22] = b"\x00\x00"


def _pack(frames):
    from seqs_amd import pack_frames

    return pack_frames(frames, align=4)


def test_fixture_regenerates():
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_dhcp_stale as m

    for c in _cases():
        pre = bytes.fromhex(c["pre_hex"])
        payload = pre[42:]
        _, frame, stale, fresh, udp = m.set_response_udp(c["request_tos"], c["request_flags"], 0, payload)
        # the ID is opaque to both checksums' validity; compare everything the sums depend on
        assert (stale != fresh) == ((c["request_tos"], c["request_flags"]) != (192, 0))
        assert c["stale_ip"] == int.from_bytes(bytes.fromhex(c["frame_hex"])[24:26], "big")
        assert c["udp"] == int.from_bytes(bytes.fromhex(c["frame_hex"])[40:42], "big")


def test_oracle_fill_reproduces_reference_bytes():
    for c in _cases():
        buf, off, ln = _pack([bytes.fromhex(c["pre_hex"])])
        coracle.fill_batch(buf, off, ln, 0, coracle.FILL_CSUM)
        got = bytearray(buf[int(off[0]) : int(off[0]) + int(ln[0])])
        _reference_writes(got)
        assert bytes(got) == bytes.fromhex(c["frame_hex"])


def test_oracle_fill_of_emitted_bytes_diverges_deliberately():
    for c in _cases():
        frame = bytes.fromhex(c["frame_hex"])
        buf, off, ln = _pack([frame])
        coracle.fill_batch(buf, off, ln, 0, coracle.FILL_CSUM)
        got = bytes(buf[int(off[0]) : int(off[0]) + int(ln[0])])
        assert int.from_bytes(got[24:26], "big") == c["fresh_ip"]
        assert int.from_bytes(got[40:42], "big") == c["udp"]
        assert (got == frame) == (c["fresh_ip"] == c["stale_ip"])


def test_oracle_rx_of_emitted_frame():
    frames = [bytes.fromhex(c["frame_hex"]) for c in _cases()]
    buf, off, ln = _pack(frames)
    dig, st = coracle.digest_batch(buf, off.astype(np.int64), ln.astype(np.int32))
    for i, c in enumerate(_cases()):
        assert st[i] == 0 and dig["ip_csum"][i] == c["fresh_ip"] and dig["l4_csum"][i] == c["udp"]


@pytest.mark.gpu
def test_gpu_fill_and_rx_match_oracle():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from seqs_amd import Engine, split_digests

    dev = torch.device("cuda:0")
    eng = Engine(0)
    try:
        for which in ("pre_hex", "frame_hex"):
            frames = [bytes.fromhex(c[which]) for c in _cases()]
            buf, off, ln = _pack(frames)
            t = torch.from_numpy(buf.copy()).to(dev)
            out, st = eng.fill_device(t, torch.from_numpy(off.astype(np.int64)).to(dev),
                                      torch.from_numpy(ln.astype(np.int32)).to(dev), flags=1)
            torch.cuda.synchronize()
            got = t.cpu().numpy()
            exp = buf.copy()
            coracle.fill_batch(exp, off, ln, 0, coracle.FILL_CSUM)
            assert np.array_equal(got, exp)
            for i, c in enumerate(_cases()):
                f = bytearray(got[int(off[i]) : int(off[i]) + int(ln[i])])
                if which == "pre_hex":
                    _reference_writes(f)
                    assert bytes(f) == bytes.fromhex(c["frame_hex"])
                else:
                    assert int.from_bytes(f[24:26], "big") == c["fresh_ip"]
        frames = [bytes.fromhex(c["frame_hex"]) for c in _cases()]
        buf, off, ln = _pack(frames)
        out, st = eng.digest_device(torch.from_numpy(buf).to(dev), torch.from_numpy(off.astype(np.int64)).to(dev),
                                    torch.from_numpy(ln.astype(np.int32)).to(dev))
        torch.cuda.synchronize()
        crc, ipc, l4c = split_digests(out.cpu().numpy())
        st = st.cpu().numpy()
        for i, c in enumerate(_cases()):
            assert st[i] == 0 and ipc[i] == c["fresh_ip"] and l4c[i] == c["udp"]
    finally:
        eng.close()
