"""The benchmark's synthetic frames are valid RecvEth input (checked by the oracle)."""
import numpy as np

from oracle import coracle
from seqs_amd import synth


def test_uniform_batch_valid():
    buf, off, ln = synth.uniform_batch(512, 1500, seed=1)
    assert buf.size >= 512 * 1500 and (ln == 1500).all()
    dig, st = coracle.digest_batch(buf, off, ln, mtu=2048)
    assert (st == 0).all()


def test_uniform_udp_and_sizes():
    for L in (64, 65, 576, 1500, 9000):
        for proto in (6, 17):
            buf, off, ln = synth.uniform_batch(64, L, seed=L, proto=proto)
            dig, st = coracle.digest_batch(buf, off, ln)
            assert (st == 0).all(), (L, proto)


def test_mixed_batch_valid():
    buf, off, ln = synth.mixed_batch(256, seed=2)
    assert list(ln[:4]) == [64, 576, 1500, 9000]
    dig, st = coracle.digest_batch(buf, off, ln)
    assert (st == 0).all()
    assert np.array_equal(off[1:], np.cumsum(ln[:-1].astype(np.int64)))


def test_hello_batch_is_the_reference_benchmark_shape():
    """stacks/benchmark_test.go:12-46, 67-98: 47-B UDP frames with the payload "hello" to
    192.168.1.1:67 from MAC 01:00:00:00:00:00's randomized peers; RecvEth accepts every one
    (the oracle's verdict 0, mtu 2048 as the benchmark's PortStack), at 48-B slots."""
    buf, off, ln = synth.hello_batch(2000, seed=0)
    assert (ln == 47).all() and np.array_equal(off, np.arange(2000) * 48)
    f = buf[:47]
    assert f[0] == 0x01 and not f[1:6].any() and bytes(f[12:14]) == b"\x08\x00" and f[14] == 0x45
    assert f[23] == 17 and bytes(f[30:34]) == bytes([192, 168, 1, 1])
    assert int.from_bytes(bytes(f[36:38]), "big") == 67 and int.from_bytes(bytes(f[38:40]), "big") == 13
    assert bytes(f[42:47]) == b"hello"
    dig, st = coracle.digest_batch(buf, off, ln, mtu=2048)
    assert (st == 0).all()
