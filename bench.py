#!/usr/bin/env python3
"""framesum benchmark — BASELINE.json metric on MI355X.

A "step" = one pass of the hot path (fused CRC-32 + IPv4 + TCP/UDP checksum +
RecvEth verdict) over one batch of synthetic frames already resident in HBM.
Default workload (BASELINE configs[1], C2): 65,536 x 1500-byte TCP frames per
GPU; --config c3 runs the mixed 64/576/1500/9000 batch. NB >= 4 distinct
batches (> 256 MiB in total) are rotated so the 256 MiB Infinity Cache cannot
serve them. Multi-GPU (torchrun, one process per GPU, RCCL = torch "nccl"):
every rank digests its own shard (weak scaling, frame i of the global batch
on rank i mod N) and the per-frame digests + verdicts are gathered to rank 0
over RCCL, one gather per group of --gather-every steps, overlapped with the next
group's kernels; no other collective. Rank 0 receives the shards as they are (global
frame j*N + r is local frame j of rank r: seqs_amd.shard.gather_digests shows the
interleave; the bench does not spend a rank-0 kernel on it).

Prints ONE JSON line on rank 0 (see the contract in DESIGN.md §5).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md (8.0 TB/s)
GIB = float(1 << 30)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--warmup", type=int, default=1000,
                   help="untimed launches first: throughput reaches its steady state only after several hundred "
                        "back-to-back launches (with 20 the timed steps measured 5-10%% lower)")
    p.add_argument("--config", choices=["c2", "c3"], default="c2")
    p.add_argument("--frames", type=int, default=65536, help="frames per GPU per step")
    p.add_argument("--batches", type=int, default=4, help="distinct resident batches rotated")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline time budget (0 = skip)")
    p.add_argument("--cpu-threads", type=int, default=1)
    p.add_argument("--no-gather", action="store_true", help="skip the RCCL digest gather (N>1 diagnostics)")
    p.add_argument("--gather-every", type=int, default=64,
                   help="N>1: each stream sends the digests + verdicts of this many of its steps to rank 0 in "
                        "one RCCL gather (one collective per group, not two per step)")
    p.add_argument("--force-gather", action="store_true",
                   help="run the gather path on a single GPU too (a 1-rank process group; a test of the N>1 loop)")
    p.add_argument("--op", choices=["digest", "fill", "fcs"], default="digest",
                   help="digest: RX digest + verdict (the BASELINE metric); fill: TX checksum fill + FCS "
                        "append in place (fs_fill_batch); fcs: RX of wire frames carrying an FCS")
    p.add_argument("--min-warm", type=int, default=500,
                   help="device pre-warm: when --warmup is below this, (min-warm - warmup) extra untimed "
                        "launches run first, on the main stream, without the gather (reported as prewarm_launches)")
    p.add_argument("--streams", type=int, default=4,
                   help="HIP streams the steps rotate over: step i+1's kernel starts on the CUs step i's "
                        "tail frees (every batch is still fully digested)")
    return p.parse_args()


def make_batch(cfg: str, n: int, seed: int):
    from seqs_amd import synth

    if cfg == "c2":
        return synth.uniform_batch(n, 1500, seed=seed)
    return synth.mixed_batch(n, seed=seed)


def with_room(buf, off, ln, room: int = 4):
    """Repack a batch with `room` spare bytes after every frame (FCS space), 4-byte aligned."""
    step = (ln.astype(np.int64) + room + 3) // 4 * 4
    noff = np.zeros_like(off)
    noff[1:] = np.cumsum(step[:-1])
    nbuf = np.zeros(int(noff[-1] + step[-1]) + 16, np.uint8)
    for o, no, l in zip(off, noff, ln):
        nbuf[no : no + l] = buf[o : o + l]
    return nbuf, noff, ln


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(cfg: str, seconds: float, threads: int):
    """The C oracle (scalar restatement of eth/crc.go + headers.go + RecvEth gates, zlib
    CRC-32) timed on a bounded C1-style sample: 4,096 frames of the same workload."""
    from oracle import coracle

    coracle.load()
    buf, off, ln = make_batch(cfg, 4096, seed=101)
    nbytes = int(ln.astype(np.int64).sum())
    coracle.digest_batch(buf, off, ln, mtu=0, nthreads=threads)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        coracle.digest_batch(buf, off, ln, mtu=0, nthreads=threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds and reps >= 3:
            break
    gibs = nbytes * reps / el / GIB
    return {
        "value": round(gibs, 4),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{reps} x C1-style batch of 4096 {'1500-B TCP' if cfg == 'c2' else 'mixed'} frames "
                  f"({nbytes} B) through oracle/framesum_oracle.c (CRC791 loop -O2 -fno-tree-vectorize + zlib "
                  f"crc32), {el:.1f} s on {cpu_model()}",
    }


def load_pmc_traffic(cfg: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/), if present:
    (doubled FETCH_SIZE + WRITE_SIZE, the guide's gfx950 correction; the same divided by the
    access pattern's own calibration factor)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{cfg}.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("hbm_bytes_per_launch"), d.get("hbm_bytes_per_launch_calibrated")
    except (OSError, ValueError):
        return None, None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world == 1:
        # started without torchrun: run ourselves under it as a child process
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", os.environ.get("MASTER_PORT", "29511"),
               os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.run(cmd).returncode)

    import torch
    import torch.distributed as dist

    from seqs_amd import Engine

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)
    elif args.force_gather and not args.no_gather:
        dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1,
                                init_method=f"tcp://127.0.0.1:{os.environ.get('MASTER_PORT', '29513')}")

    n = args.frames
    engine = Engine(local)
    batches = []
    for b in range(max(1, args.batches)):
        buf, off, ln = make_batch(args.config, n, seed=1 + 1000 * rank + b)
        if args.op != "digest":
            buf, off, ln = with_room(buf, off, ln)
        tb, to, tl = torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)
        if args.op == "fcs":  # wire frames: the FCS appended once on the GPU, lengths include it
            engine.fill_device(tb, to, tl, flags=2)
            tl = tl + 4
        batches.append((tb, to, tl))
    run_op = {"digest": engine.digest_device, "fcs": engine.digest_fcs_device,
              "fill": lambda *a, **k: engine.fill_device(*a, flags=3, **k)}[args.op]
    bytes_per_batch = int(batches[-1][2].cpu().numpy().astype(np.int64).sum())
    resident = sum(int(x[0].numel()) for x in batches)
    nb = len(batches)
    ns = max(1, args.streams)
    gather = dist.is_initialized() and not args.no_gather
    main_stream = torch.cuda.current_stream(dev)
    streams = [main_stream] + [torch.cuda.Stream(dev) for _ in range(ns - 1)]
    # Output slots (digest words, then verdicts, in one 256-B-aligned slab per slot). Without a
    # gather, step i writes slot i % nslot and slot k is only ever written by stream k (nslot ==
    # ns for ns >= 2; one stream for ns == 1): stream order alone keeps a slot's launches apart.
    # With the gather, each stream owns 2 groups of G slots for its own consecutive steps; when
    # a group is full, that stream hands its slabs to rank 0 in one RCCL gather (issued on that
    # stream, so it waits for that stream's kernels only) while it fills the other group.
    G = max(1, args.gather_every) if gather else 1
    nslot = max(2, ns)
    slab = (9 * n + 255) // 256 * 256

    def views(buf, k):
        base = k * slab
        return buf[base : base + 8 * n].view(torch.int32).view(n, 2), buf[base + 8 * n : base + 9 * n]

    if gather:
        gbuf = [[torch.empty(G * slab, dtype=torch.uint8, device=dev) for _ in range(2)] for _ in range(ns)]
        gviews = [[[views(gbuf[st][g], j) for j in range(G)] for g in range(2)] for st in range(ns)]
        recv = [[[torch.empty_like(gbuf[st][g]) for _ in range(world)] if rank == 0 else None for g in range(2)]
                for st in range(ns)]
        pend = [[None, None] for _ in range(ns)]  # per stream and group: the RCCL work of its latest gather
    flat = torch.empty(nslot * slab, dtype=torch.uint8, device=dev)
    outs, stats = zip(*[views(flat, k) for k in range(nslot)])

    def step(i: int):
        fb, fo, fl = batches[i % nb]
        si = i % ns
        s = streams[si]
        if not gather:
            run_op(fb, fo, fl, mtu=0, out=outs[i % nslot], status=stats[i % nslot], stream=s)
            return
        q = i // ns
        g, j = (q // G) % 2, q % G
        with torch.cuda.stream(s):
            if j == 0 and pend[si][g] is not None:
                pend[si][g].wait()  # this stream waits until the gather has read group g's slabs
                pend[si][g] = None
            o, st = gviews[si][g][j]
            run_op(fb, fo, fl, mtu=0, out=o, status=st, stream=s)
            if j == G - 1:
                pend[si][g] = dist.gather(gbuf[si][g], recv[si][g], dst=0, async_op=True)

    def drain(i_end: int):
        if not gather:
            return
        # partly filled groups still go to rank 0 (same calls on every rank: i_end is common)
        for si in range(ns):
            q_end = (i_end - si + ns - 1) // ns  # steps this stream ran
            g = (q_end // G) % 2
            if q_end % G != 0 and pend[si][g] is None:
                with torch.cuda.stream(streams[si]):
                    pend[si][g] = dist.gather(gbuf[si][g], recv[si][g], dst=0, async_op=True)
        for si in range(ns):
            for g in range(2):
                if pend[si][g] is not None:
                    with torch.cuda.stream(streams[si]):
                        pend[si][g].wait()
                    pend[si][g] = None

    # device pre-warm (setup, not steps): throughput settles only after several hundred launches
    prewarm = max(0, args.min_warm - args.warmup)
    for i in range(prewarm):
        fb, fo, fl = batches[i % nb]
        run_op(fb, fo, fl, mtu=0, out=outs[i % nslot], status=stats[i % nslot], stream=main_stream)
    torch.cuda.synchronize()
    for i in range(args.warmup):
        step(i)
    drain(args.warmup)
    torch.cuda.synchronize()

    # ---- timed region: K steps, barrier + synchronize on both sides, max over ranks
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    drain(args.warmup + args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if gather and rank == 0:
        # every group's latest gather delivered rank 0's own slabs intact (a check of the loop)
        torch.cuda.synchronize()
        for si in range(ns):
            for g in range(2):
                assert torch.equal(recv[si][g][0], gbuf[si][g]), "gathered digests differ from rank 0's own"

    # ---- kernel-only timing with HIP events on the launch stream (roofline.achieved): one event
    # pair around K back-to-back launches on one stream (no overlap with another launch), so the
    # average is the kernel's duration plus the stream's dispatch gap; an event pair around every
    # launch would add each record's own latency to every launch.
    k0, k1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(main_stream):
        k0.record(main_stream)
        for i in range(args.steps):  # same stream, in order: no slot events needed
            fb, fo, fl = batches[i % nb]
            run_op(fb, fo, fl, mtu=0, out=outs[i % nslot], status=stats[i % nslot], stream=main_stream)
        k1.record(main_stream)
    torch.cuda.synchronize()
    k_avg_ms = k0.elapsed_time(k1) / args.steps

    total_bytes = bytes_per_batch * args.steps * world
    value = total_bytes / elapsed / GIB
    achieved_gbs = bytes_per_batch / (k_avg_ms * 1e-3) / 1e9
    traffic, traffic_cal = load_pmc_traffic(args.config) if args.op == "digest" else (None, None)

    result = None
    if rank == 0:
        cpu = None
        if world == 1 and args.cpu_seconds > 0 and args.op == "digest":
            cpu = cpu_baseline(args.config, args.cpu_seconds, args.cpu_threads)
        result = {
            "metric": "GiB/s device-resident CRC-32+Internet-csum over batched MTU frames; % HBM peak",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic: {nb} distinct resident batches ({resident / 1e6:.0f} MB) of valid frames, rotated",
            "config": {
                "workload": ("C2: 65536 x 1500-B TCP frames per GPU (BASELINE configs[1])" if args.config == "c2"
                             else "C3: 65536 mixed 64/576/1500/9000-B TCP/UDP frames per GPU (BASELINE configs[2])")
                if n == 65536 else f"{args.config} with {n} frames per GPU",
                "frames_per_gpu": n,
                "bytes_per_gpu_step": bytes_per_batch,
                "global_batch_frames": n * world,
                "parallelism": f"frames sharded round-robin over {world} GPU(s); RCCL gather of digests to rank 0"
                if world > 1 else "single GPU",
                "streams": ns,
                "prewarm_launches": prewarm,
                "op": {"digest": "RX digest + verdict (fs_digest_batch)",
                       "fill": "TX checksum fill + FCS append in place (fs_fill_batch, 4 spare bytes per frame)",
                       "fcs": "RX of wire frames with FCS (fs_digest_batch_fcs; bytes = frames incl. FCS)"}[args.op],
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved_gbs, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_calibrated": traffic_cal,
                "kernel": "digest_kernel",
                "kernel_avg_us": round(k_avg_ms * 1e3, 3),
                "kernel_timing": "HIP events around K back-to-back launches on the launch stream",
                "algorithmic_bytes_per_launch": bytes_per_batch,
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    engine.close()
    if dist.is_initialized():
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
