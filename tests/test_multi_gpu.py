"""Multi-GPU paths on the real gfx950 engine, checked bit for bit against the CPU oracle.

- C4 (BASELINE configs[3]): 1,048,576 x 1500-B frames sharded round-robin.
  * fs_digest_batch_sharded (one process, chunked RCCL ncclSend/ncclRecv + de-interleave kernel) on the
    box's devices (a 1-device communicator on a one-GPU box);
  * seqs_amd.shard.ShardedDigest with Engine.digest_device, world 2 and 4 over gloo, each
    rank a fresh child process on cuda:0.
- C5 (BASELINE configs[4]): fs_digest_batch_multi with 8 contexts over a pinned batch of
  9000-byte jumbo frames; unordered offsets (blocks cut in buffer order).
- fs_deinterleave on random gathered slabs, N = 1..8.
- One context per distinct device (skipped below 2 devices).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from oracle import coracle  # noqa: E402
from seqs_amd import Engine, Group, digest_host_multi, shard, shard_count, shard_slab_bytes, split_digests, synth  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C4_FRAMES = 1 << 20


def ndev():
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


@pytest.fixture(scope="module")
def c4():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    buf, off, ln = synth.uniform_batch(C4_FRAMES, 1500, seed=4)
    dig, st = coracle.digest_batch(buf, off, ln, mtu=0, nthreads=16)
    return buf, off, ln, dig, st


def assert_equal_words(words, status, dig, est, label):
    crc, ipc, l4c = split_digests(words)
    bad = np.nonzero((crc != dig["crc32"]) | (ipc != dig["ip_csum"]) | (l4c != dig["l4_csum"]) | (status != est))[0]
    assert bad.size == 0, f"{label}: {bad.size} mismatches, first at {int(bad[0])}"


def shards_on(devices, buf, off, ln):
    n, N = len(ln), len(devices)
    out = []
    for k, d in enumerate(devices):
        b, o, l = shard.shard_batch(buf, off, ln, N, k)
        assert len(l) == shard_count(n, N, k)
        dev = torch.device("cuda", d)
        out.append((torch.from_numpy(b).to(dev), torch.from_numpy(o).to(dev), torch.from_numpy(l).to(dev)))
    return out


def test_group_sharded_c4(c4):
    buf, off, ln, dig, est = c4
    devices = list(range(ndev()))
    g = Group(devices)
    try:
        shards = shards_on(devices, buf, off, ln)
        words, status = g.digest_sharded(shards, len(ln))
        assert_equal_words(words.cpu().numpy(), status.cpu().numpy(), dig, est, f"group {devices}")
    finally:
        g.close()


def test_group_sharded_mixed_lengths():
    import framegen

    frames = framegen.edge_batch(9, n_random=5000)
    from seqs_amd import pack_frames

    buf, off, ln = pack_frames(frames, align=1)
    off, ln = off.astype(np.int64), ln.astype(np.int32)
    g = Group(list(range(ndev())))
    try:
        words, status = g.digest_sharded(shards_on(g.devices, buf, off, ln), len(ln), mtu=1514)
        dig, est = coracle.digest_batch(buf, off, ln, mtu=1514, nthreads=8)
        assert_equal_words(words.cpu().numpy(), status.cpu().numpy(), dig, est, "group mixed")
    finally:
        g.close()


def test_group_fault_at_chunk1_then_exact(c4):
    """an fs_digest_batch_sharded call that fails at chunk 1 (the test library's
    fs_test_group_set_fault; chunk 0's kernels, transfers and de-interleave are queued by then)
    drains every stream before returning, so the next call on the same group is bit-exact."""
    from seqs_amd import FramesumError
    from seqs_amd.framesum import TEST_LIB_PATH

    buf, off, ln, dig, est = c4
    devices = list(range(ndev()))
    g = Group(devices, lib_path=TEST_LIB_PATH)
    try:
        shards = shards_on(devices, buf, off, ln)
        assert g.lib.fs_test_group_set_fault(g._g, 1) == 0
        with pytest.raises(FramesumError, match="injected fault at chunk 1"):
            g.digest_sharded(shards, len(ln))
        assert g.lib.fs_test_group_set_fault(g._g, -1) == 0
        words, status = g.digest_sharded(shards, len(ln))
        assert_equal_words(words.cpu().numpy(), status.cpu().numpy(), dig, est, "after injected fault")
    finally:
        g.close()


def test_group_rccl_error_aborts_communicators(c4):
    """an RCCL error at chunk 1's gather (fs_test_group_set_fault_gather: its grouped
    sends and receives are already enqueued) aborts the communicators before the streams are drained,
    so the call returns instead of waiting on a transfer; the group then refuses further calls until
    it is recreated, and a new group is bit-exact."""
    from seqs_amd import FramesumError
    from seqs_amd.framesum import TEST_LIB_PATH

    buf, off, ln, dig, est = c4
    devices = list(range(ndev()))
    g = Group(devices, lib_path=TEST_LIB_PATH)
    try:
        shards = shards_on(devices, buf, off, ln)
        assert g.lib.fs_test_group_set_fault_gather(g._g, 1) == 0
        with pytest.raises(FramesumError, match="communicators were aborted"):
            g.digest_sharded(shards, len(ln))
        assert g.lib.fs_test_group_set_fault_gather(g._g, -1) == 0
        with pytest.raises(FramesumError, match="aborted by an earlier error"):
            g.digest_sharded(shards, len(ln))
    finally:
        g.close()
    g = Group(devices, lib_path=TEST_LIB_PATH)
    try:
        words, status = g.digest_sharded(shards_on(devices, buf, off, ln), len(ln))
        assert_equal_words(words.cpu().numpy(), status.cpu().numpy(), dig, est, "recreated group")
    finally:
        g.close()


def test_group_rejects_duplicate_devices():
    from seqs_amd import FramesumError

    with pytest.raises(FramesumError):
        Group([0, 0])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_gloo_c4(world, tmp_path):
    port = _free_port()
    result = str(tmp_path / "result.json")
    env = dict(os.environ, PYTHONPATH=ROOT)
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "sharded_worker.py"), str(r), str(world),
                               str(port), str(C4_FRAMES), result], env=env)
             for r in range(world)]
    try:
        codes = [p.wait(timeout=110) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert codes == [0] * world
    res = json.load(open(result))
    assert res["ok"] and res["n"] == C4_FRAMES and res["shard0"] == shard_count(C4_FRAMES, world, 0)


def test_multi_8_contexts_c5_jumbo():
    # C5's shape: 9000-B jumbo frames streamed from pinned host memory over 8 contexts
    n = 8 * 16384
    engines = [Engine(0) for _ in range(8)]
    try:
        src, off, ln = synth.uniform_batch(n, 9000, seed=5)
        pinned = engines[0].host_empty(src.shape, np.uint8)
        pinned[:] = src
        dig, est = coracle.digest_batch(src, off, ln, mtu=0, nthreads=16)
        out, st = digest_host_multi(engines, pinned, off, ln)
        assert (st == est).all()
        assert np.array_equal(out["crc32"], dig["crc32"]) and np.array_equal(out["l4_csum"], dig["l4_csum"])
        assert np.array_equal(out["ip_csum"], dig["ip_csum"])
    finally:
        for e in engines:
            e.close()


def test_multi_unordered_offsets_cut_in_buffer_order():
    # frames stored out of index order: each block still copies only its own bytes
    engines = [Engine(0) for _ in range(3)]
    try:
        buf, off, ln = synth.mixed_batch(20000, seed=6)
        perm = np.random.default_rng(1).permutation(len(ln))
        off, ln = off[perm], ln[perm]
        dig, est = coracle.digest_batch(buf, off, ln, mtu=0, nthreads=8)
        out, st = digest_host_multi(engines, buf, off, ln)
        assert (st == est).all() and np.array_equal(out["crc32"], dig["crc32"])
        assert np.array_equal(out["l4_csum"], dig["l4_csum"]) and np.array_equal(out["ip_csum"], dig["ip_csum"])
    finally:
        for e in engines:
            e.close()


@pytest.mark.parametrize("nshards", [1, 2, 3, 4, 8])
def test_deinterleave_device(nshards):
    e = Engine(0)
    try:
        rng = np.random.default_rng(nshards)
        for n in (1, nshards + 1, 1000, 65537):
            sb = shard_slab_bytes(n, nshards)
            m = (n + nshards - 1) // nshards
            g = rng.integers(0, 256, size=nshards * sb, dtype=np.uint8)
            words, status = e.deinterleave_device(torch.from_numpy(g).cuda(), nshards, n)
            torch.cuda.synchronize()
            i = np.arange(n)
            r, j = i % nshards, i // nshards
            exp_w = np.stack([g[r * sb + 8 * j + k] for k in range(8)], axis=1).view(np.int32).reshape(n, 2)
            exp_s = g[r * sb + 8 * m + j]
            assert np.array_equal(words.cpu().numpy(), exp_w)
            assert np.array_equal(status.cpu().numpy(), exp_s)
    finally:
        e.close()


@pytest.mark.skipif(ndev() < 2, reason="needs 2+ GPUs")
def test_engine_per_device_multi():
    engines = [Engine(d) for d in range(ndev())]
    try:
        buf, off, ln = synth.mixed_batch(40000, seed=8)
        dig, est = coracle.digest_batch(buf, off, ln, mtu=0, nthreads=8)
        out, st = digest_host_multi(engines, buf, off, ln)
        assert (st == est).all() and np.array_equal(out["crc32"], dig["crc32"])
        assert np.array_equal(out["l4_csum"], dig["l4_csum"])
    finally:
        for e in engines:
            e.close()
