"""The C ABI from C: examples/fs_digest_cli.c links only include/framesum.h and
libframesum.so (what the cgo binding of INTEGRATION.md does) and runs the host-staged
digest and TX fill; its outputs must equal the oracle's, bit for bit."""
import os
import subprocess

import numpy as np
import pytest

from oracle import coracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "examples", "fs_digest_cli")


def write_batch(tmp_path, buf, off, ln):
    paths = [str(tmp_path / x) for x in ("frames.bin", "offsets.u64", "lengths.u32", "out.bin")]
    np.ascontiguousarray(buf, np.uint8).tofile(paths[0])
    np.ascontiguousarray(off, np.uint64).tofile(paths[1])
    np.ascontiguousarray(ln, np.uint32).tofile(paths[2])
    return paths


def test_cli_built_and_loud_without_device(tmp_path):
    assert os.path.exists(CLI), "examples/fs_digest_cli is built by __graft_entry__.build()"
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    buf = np.zeros(64, np.uint8)
    paths = write_batch(tmp_path, buf, np.zeros(1, np.uint64), np.full(1, 60, np.uint32))
    r = subprocess.run([CLI, "digest", *paths], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "fs_ctx_create" in r.stderr


@pytest.mark.gpu
def test_cli_digest_and_fill(tmp_path):
    from test_tx_fcs import pack_with_room, tx_frames

    frames = tx_frames(3, n_random=300)
    buf, off, ln = pack_with_room(frames, align=4)
    n = len(ln)
    paths = write_batch(tmp_path, buf, off, ln)
    r = subprocess.run([CLI, "digest", *paths, "1514"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    raw = np.fromfile(paths[3], np.uint8)
    dig = raw[: 8 * n].view(coracle.DIGEST_DTYPE)
    st = raw[8 * n : 9 * n]
    edig, est = coracle.digest_batch(buf, off, ln, mtu=1514)
    assert np.array_equal(dig, edig) and np.array_equal(st, est)

    r = subprocess.run([CLI, "fill", *paths, "0", "3"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    raw = np.fromfile(paths[3], np.uint8)
    dig, st, filled = raw[: 8 * n].view(coracle.DIGEST_DTYPE), raw[8 * n : 9 * n], raw[9 * n :]
    ebuf = buf.copy()
    edig, est = coracle.fill_batch(ebuf, off, ln, 0, 3)
    assert np.array_equal(filled, ebuf) and np.array_equal(dig, edig) and np.array_equal(st, est)
