"""Regenerate tests/golden/*.json (committed fixtures).

kats.json   — known-answer vectors transcribed from the reference's own tests
              (data only; citations relative to the soypat/seqs root).
batch.json  — a seeded edge-case batch (tests/framegen.py) with expected
              digests from the pure-Python restatement (oracle/pyref.py),
              cross-checked here against the C oracle (and zlib for CRC-32).
              The reference (Go) cannot run in this image, so batch.json is a
              regression fixture; parity is pinned by kats.json.
Usage: python tests/golden/make_golden.py
"""
import json
import os
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

from oracle import coracle, pyref  # noqa: E402
import framegen  # noqa: E402

KATS = {
    "source": "soypat/seqs @ 2025-02-12 test files (data transcribed, not code)",
    "tcp_checksum": [{
        "cite": "eth/headers_test.go:21-26 TestTCPChecksum",
        "ip": {"VersionAndIHL": 69, "TotalLength": 60, "ID": 5534, "Flags": 16384, "TTL": 64, "Protocol": 6,
               "Checksum": 41160, "Source": [192, 168, 1, 116], "Destination": [192, 168, 1, 145]},
        "tcp": {"SourcePort": 46468, "DestinationPort": 1234, "Seq": 1104871141, "Ack": 0,
                "OffsetAndFlags": 40962, "WindowSizeRaw": 64240, "Checksum": 30430, "UrgentPtr": 0},
        "options_hex": b"\x02\x04\x05\xb4\x04\x02\x08\nFP\x10t\x00\x00\x00\x00\x01\x03\x03\x07".hex(),
        "payload_hex": "",
        "expected": 30430,
    }],
    "ip_checksum": [{
        "cite": "eth/headers_test.go:218-229 TestIPChecksum",
        "header_hex": "450000289a61000040061c14c0a80178c0a80192",
        "expected": 0x5C14,
    }],
    "crc791_oneshot": {
        "cite": "eth/headers_test.go:108-125 TestCRC791_oneshot (expected = sum() helper :200-216)",
        "inputs_hex": ["23", "23fb", "23fbde", "23fbdead", "23fbdeaddeadc0ffee", "23fbdeaddeadc0ffee00"],
    },
    "crc791_multifuzz_data_hex": b"00\x0010".hex(),  # eth/headers_test.go:128
    "crc791_fuzz_seed_hex": "23fbdeaddeadc0ffee00",   # eth/headers_test.go:147
    "frames": [
        {"cite": "stacks/stacks_test.go:591-594 TestPortStackTCPDecoding[0] (RecvEth must accept)",
         "hex": "28cdc1054d3ed85ed34303eb08004500003c76eb400040063f76c0a80192c0a80178ee1604d2a0ceb98a00000000a002faf06e800000020405b40402080a14ccf8250000000001030307",
         "verdict": 0, "l4_csum": 0x6E80, "ip_csum": 0x3F76},
        {"cite": "stacks/stacks_test.go:591-594 TestPortStackTCPDecoding[1] (stored checksum 0x0000)",
         "hex": "28cdc101137c88aedd0a709208004500002db03a4000400675590a0000be0a00007ac7ce04d22a67581700000d535018fa4b0000000068656c6c6f",
         "verdict": 0, "l4_csum": 0x0000, "ip_csum": 0x7559},
        {"cite": "eth/headers_test.go:39-51 TestUDPChecksum frame (stored UDP 0x278F, IP 0x6CDC; the reference "
                 "does not assert them — they verify under the restatement, SURVEY.md §4)",
         "hex": ("ffffffffffff784476c48db008004500" "00a24ab0000080116cdcc0a8006fc0a8" "00ff445c445c008e278f7b2276657273"
                 "696f6e223a205b322c20305d2c202270" "6f7274223a2031373530302c2022686f" "73745f696e74223a2031383132363536"
                 "30393235373432313034363733333632" "36313733323137303537363334373933" "2c2022646973706c61796e616d65223a"
                 "2022222c20226e616d65737061636573" "223a205b383135323436323030305d7d"),
         "verdict": 0, "l4_csum": 0x278F, "ip_csum": 0x6CDC},
    ],
    "crc32_check": {"cite": "IEEE 802.3 / CRC-32 catalogue check value (no reference implementation, SURVEY.md §0.1)",
                    "input_ascii": "123456789", "expected": 0xCBF43926},
}


def main():
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(KATS, f, indent=1)
    frames = framegen.edge_batch(seed=20250212, n_random=160)
    entries = []
    for fr in frames:
        v, ipc, l4c = pyref.recv_eth(fr)
        cv, cipc, cl4c = coracle.recv_eth(fr)
        assert (v, ipc, l4c) == (cv, cipc, cl4c), "pyref and C oracle disagree"
        crc = zlib.crc32(fr) & 0xFFFFFFFF
        assert crc == coracle.crc32_bitwise(fr)
        entries.append({"hex": fr.hex(), "crc32": crc, "ip_csum": ipc, "l4_csum": l4c, "verdict": v})
    mtu_entries = []
    for i, fr in enumerate(frames[:60]):
        v, ipc, l4c = pyref.recv_eth(fr, mtu=600)
        mtu_entries.append({"index": i, "ip_csum": ipc, "l4_csum": l4c, "verdict": v})
    with open(os.path.join(HERE, "batch.json"), "w") as f:
        json.dump({"generator": "tests/framegen.py edge_batch(seed=20250212, n_random=160)",
                   "frames": entries, "mtu600": mtu_entries}, f, indent=0)
    print(f"wrote {len(entries)} golden frames")


if __name__ == "__main__":
    main()
