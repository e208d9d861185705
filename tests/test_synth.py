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
