"""The Go binding (go/eth/digest_gpu.go, go/stacks/portstack_batch.go).

There is no Go toolchain in this image, so the files are checked for the surface they must
provide, and tests/csrc/go_binding_replay.c replays DigestBatch / FillBatch / GPUs.DigestBatch
exactly (4-byte aligned packing into fs_host_alloc pinned memory, 4 spare bytes per frame for
the FCS, 16 spare bytes at the end) through the same C ABI calls, and Group.DigestSharded (the
RCCL group over every visible device, round-robin shards in device memory); on the GPU its
outputs must equal the oracle's bit for bit."""
import os
import re
import struct
import subprocess

import numpy as np
import pytest

from oracle import coracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPLAY = os.path.join(ROOT, "tests", "csrc", "build", "go_binding_replay")
GO_ETH = os.path.join(ROOT, "go", "eth", "digest_gpu.go")
GO_STACKS = os.path.join(ROOT, "go", "stacks", "portstack_batch.go")


def build_replay():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "csrc"), "build/go_binding_replay"], check=True)
    return REPLAY


def test_go_files_declare_the_binding():
    eth = open(GO_ETH).read()
    stacks = open(GO_STACKS).read()
    for sym in ("func OpenGPU(", "func (g *GPU) DigestBatch(", "func (g *GPU) FillBatch(", "func OpenGPUs(",
                "func (m *GPUs) DigestBatch(", "C.fs_digest_batch_host(", "C.fs_fill_batch_host(",
                "C.fs_digest_batch_multi(", "C.fs_host_alloc(", "func OpenGroup(", "func (g *Group) DigestSharded(",
                "func ShardCount(", "C.fs_group_create(", "C.fs_digest_batch_sharded(", "C.fs_shard_count(",
                "func (g *GPU) SetKernel(", "C.fs_ctx_set_kernel("):
        assert sym in eth, sym
    for sym in ("func (ps *PortStack) RecvEthBatch(", "func (ps *PortStack) recvEthVerified(", "deliverUDP", "deliverTCP"):
        assert sym in stacks, sym
    assert eth.startswith("//go:build framesum") and stacks.startswith("//go:build framesum")
    # the Go verdict constants are the C ABI's enum fs_verdict
    hdr = open(os.path.join(ROOT, "include", "framesum.h")).read()
    c = {int(v) for _, v in re.findall(r"(FS_[A-Z0-9_]+)\s*=\s*(\d+)", hdr)}
    go = {int(v) for v in re.findall(r"Verdict[A-Za-z0-9]+\s+Verdict = (\d+)", eth)}
    assert go == c
    # the Go kernel-variant constants are the values fs_ctx_set_kernel accepts
    kv = {int(v) for v in re.findall(r"Kernel[A-Za-z]+\s+= (\d+)", eth)}
    assert kv == {0, 2, 3, 4, 8}


def write_list(path, frames):
    with open(path, "wb") as f:
        f.write(struct.pack("<I", len(frames)))
        for fr in frames:
            f.write(struct.pack("<I", len(fr)))
            f.write(bytes(fr))


def read_out(path, n, fill=False):
    raw = open(path, "rb").read()
    dig = np.frombuffer(raw[: 8 * n], dtype=coracle.DIGEST_DTYPE)
    st = np.frombuffer(raw[8 * n : 9 * n], dtype=np.uint8)
    frames = []
    if fill:
        p = 9 * n
        (cnt,) = struct.unpack_from("<I", raw, p)
        p += 4
        for _ in range(cnt):
            (L,) = struct.unpack_from("<I", raw, p)
            frames.append(raw[p + 4 : p + 4 + L])
            p += 4 + L
    return dig, st, frames


def test_replay_built_and_loud_without_device(tmp_path):
    import torch

    exe = build_replay()
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    write_list(tmp_path / "in.lst", [bytes(60)])
    r = subprocess.run([exe, "digest", str(tmp_path / "in.lst"), "0", str(tmp_path / "o.bin")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "fs_ctx_create" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("mode,mtu", [("digest", 0), ("digest", 1514), ("multi", 0), ("sharded", 0), ("sharded", 1514)])
def test_replay_digest_matches_oracle(tmp_path, mode, mtu):
    import framegen

    frames = framegen.edge_batch(11, n_random=4000)
    exe = build_replay()
    write_list(tmp_path / "in.lst", frames)
    args = [exe, mode, str(tmp_path / "in.lst"), str(mtu), str(tmp_path / "o.bin")] + (["3"] if mode == "multi" else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    dig, st, _ = read_out(tmp_path / "o.bin", len(frames))
    from seqs_amd import pack_frames

    buf, off, ln = pack_frames(frames)
    odig, ost = coracle.digest_batch(buf, off, ln, mtu=mtu)
    assert np.array_equal(dig, odig) and np.array_equal(st, ost)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["fill", "fill_fcs"])
def test_replay_fill_matches_oracle(tmp_path, mode):
    from test_tx_fcs import tx_frames

    frames = tx_frames(12, n_random=2000)
    exe = build_replay()
    write_list(tmp_path / "in.lst", frames)
    r = subprocess.run([exe, mode, str(tmp_path / "in.lst"), "0", str(tmp_path / "o.bin")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    dig, st, filled = read_out(tmp_path / "o.bin", len(frames), fill=True)
    room = 4 if mode == "fill_fcs" else 0
    from seqs_amd import pack_frames

    buf, off, ln = pack_frames([bytes(f) + bytes(room) for f in frames])
    ln = ln - np.uint32(room)
    odig, ost = coracle.fill_batch(buf, off, ln, mtu=0, flags=1 | (2 if room else 0))
    assert np.array_equal(dig, odig) and np.array_equal(st, ost)
    for i, (o, L) in enumerate(zip(off, ln)):
        assert filled[i] == bytes(buf[int(o) : int(o) + int(L) + room]), i
