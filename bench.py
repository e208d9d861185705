#!/usr/bin/env python3
"""framesum benchmark — BASELINE.json metric on MI355X.

A "step" = one pass of the hot path (fused CRC-32 + IPv4 + TCP/UDP checksum +
RecvEth verdict) over one batch of synthetic frames already resident in HBM.
Default workload (BASELINE configs[1], C2): 65,536 x 1500-byte TCP frames per
GPU; --config c3 runs the mixed 64/576/1500/9000 batch; --config c4 the 1,048,576-frame
global batch sharded round-robin over the ranks (strong scaling: RCCL gather of every
step's digests to rank 0 and the de-interleave kernel there, both inside the step);
--config c5 streams 9000-byte jumbo frames from pinned host memory through
fs_digest_batch_multi, one context per GPU from ONE process (PCIe-inclusive, not HBM). NB >= 4 distinct
batches (> 256 MiB in total) are rotated so the 256 MiB Infinity Cache cannot
serve them. Multi-GPU (torchrun, one process per GPU, RCCL = torch "nccl"):
every rank digests its own shard (weak scaling, frame i of the global batch
on rank i mod N) and the per-frame digests + verdicts go to rank 0 over RCCL in rounds
(gather_plan: each round half of the steps still to come, at most --gather-every; one
batch of point-to-point transfers per round), overlapped with the later rounds' kernels; no other
collective. Rank 0 receives the shards as they are (global frame j*N + r is local frame j
of rank r: seqs_amd.shard.gather_digests shows the interleave; the bench does not spend a
rank-0 kernel on it). With N > 1 the same line also carries "c4_strong": the C4 strong-scaled
measurement (BASELINE configs[3], the config the >= 3.5x-at-4-GPUs target is quoted on).

Prints ONE JSON line on rank 0 (see the contract in DESIGN.md §5).
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np

# Kernel arguments in device memory (read by the dispatch from HBM, not across PCIe from pinned
# host memory): a HIP runtime setting read when the runtime initializes, so it is set before torch
# loads it; a caller's own setting wins. The driver's command ran 4,604-4,686 GiB/s with it against
# 4,466-4,598 without, interleaved on one box (profiles/round4/session2/env_sweep_driver_cmd.jsonl).
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md (8.0 TB/s)
GIB = float(1 << 30)


class GpuOps:
    """Every device call the bench makes: HIP streams, events and synchronization through
    torch.cuda, the engine (seqs_amd.Engine over libframesum.so), the process group over RCCL.
    tests/test_bench_dist.py swaps in CPU stand-ins (and a stand-in engine) to run the bench's
    own N > 1 loop -- rounds, point-to-point transfers, the C4 record -- over gloo on CPU."""

    backend = "nccl"

    def device(self, local: int):
        import torch

        torch.cuda.set_device(local)
        return torch.device("cuda", local)

    def init_group(self, dist, dev, **kw):
        dist.init_process_group(self.backend, device_id=dev, **kw)

    def stream(self, dev):
        import torch

        return torch.cuda.Stream(dev)

    def use(self, s):
        import torch

        return torch.cuda.stream(s)

    def sync(self):
        import torch

        torch.cuda.synchronize()

    def event(self):
        import torch

        return torch.cuda.Event(enable_timing=True)

    def settle(self, streams):
        """Wait on the host, by polling, until the work queued so far on `streams` has completed:
        an event per stream, queried until all have passed. The synchronize that closes a timed
        region then finds nothing left to wait for. HIP's blocking wait wakes the host about
        25 us after the last kernel ends; polling sees it within a few us (tools/region_ab.py,
        profiles/round3/region_ab.log: 20-step C2 region 415 -> 391 us)."""
        import torch

        evs = []
        for s in streams:
            e = torch.cuda.Event()
            e.record(s)
            evs.append(e)
        # one event at a time, the last-launched stream's last: once the last kernel ends the loop
        # sees it within one query (a sweep over every event per iteration took ~5 queries to notice)
        for e in evs:
            while not e.query():
                pass

    def mark(self, s):
        """an event recorded on stream s now (a dependency marker, no timing)"""
        import torch

        e = torch.cuda.Event()
        e.record(s)
        return e

    def wait_event(self, s, e):
        s.wait_event(e)

    def empty_cache(self):
        import torch

        torch.cuda.empty_cache()

    def engine(self, local: int):
        from seqs_amd import Engine

        return Engine(local)


GPU = GpuOps()


KERNEL_NAMES = {2: "digest_kernel_ab", 3: "digest_kernel_g", 4: "digest_kernel_a", 8: "digest_kernel_s"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--warmup", type=int, default=1000,
                   help="untimed launches first: throughput reaches its steady state only after several hundred "
                        "back-to-back launches (with 20 the timed steps measured 5-10%% lower)")
    p.add_argument("--config", choices=["c2", "c3", "c4", "c5", "small"], default="c2",
                   help="small: the reference's own benchmark shape (stacks/benchmark_test.go), 47-B UDP "
                        "'hello' frames in 48-B slots")
    p.add_argument("--frames", type=int, default=None,
                   help="frames per GPU per step (c2/c3/c5; default 65,536, c5 16,384) or of the global batch (c4; "
                        "default 1,048,576)")
    p.add_argument("--batches", type=int, default=4, help="distinct resident batches rotated")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline time budget (0 = skip)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="threads of the all-cores CPU baseline (0 = the box's CPU share: OMP_NUM_THREADS or the "
                        "affinity mask); the 1-thread figure is measured beside it")
    p.add_argument("--no-gather", action="store_true", help="skip the RCCL digest gather (N>1 diagnostics)")
    p.add_argument("--gather-every", type=int, default=64,
                   help="N>1: at most this many steps per gather round (gather_plan: rounds of half the steps "
                        "still to come, so the region ends with one step's slabs in flight)")
    p.add_argument("--no-c4", action="store_true", help="N>1: skip the C4 strong-scaled record in the line")
    p.add_argument("--c4-frames", type=int, default=1 << 20,
                   help="N>1: global frames of the C4 record (BASELINE configs[3]: 1,048,576)")
    p.add_argument("--force-gather", action="store_true",
                   help="run the gather path on a single GPU too (a 1-rank process group; a test of the N>1 loop)")
    p.add_argument("--op", choices=["digest", "fill", "fcs"], default="digest",
                   help="digest: RX digest + verdict (the BASELINE metric); fill: TX checksum fill + FCS "
                        "append in place (fs_fill_batch); fcs: RX of wire frames carrying an FCS")
    p.add_argument("--min-warm", type=int, default=500,
                   help="device pre-warm: when --warmup is below this, (min-warm - warmup) extra untimed "
                        "launches run first, over the streams, without the gather (reported as prewarm_launches)")
    p.add_argument("--kernel", type=int, default=None,
                   help="fs_ctx_set_kernel variant: 0 automatic (default; short-frame traffic moves it to the "
                        "small-frame kernel), 2 mixed-length, 3 segment, 4 one-pass, 8 small-frame preferred")
    p.add_argument("--workgroups", type=int, default=0,
                   help="fs_ctx_set_workgroups: workgroups per launch (0: one per CU; fewer give each wave several "
                        "tiles and let consecutive launches run side by side)")
    p.add_argument("--region-clocks", default=None, metavar="PATH",
                   help="measurement aid: write the timed region's CLOCK_MONOTONIC / CLOCK_BOOTTIME stamps (t0, "
                        "each step's return, t1) to PATH as JSON, to line them up with a rocprofv3 trace "
                        "(tools/region_attr.py)")
    p.add_argument("--no-sub", action="store_true",
                   help="N=1 C2: skip the C3 and C5 sub-records of the line (BASELINE configs[2], [4])")
    p.add_argument("--streams", type=int, default=5,
                   help="HIP streams the steps rotate over: step i+1's kernel starts on the CUs step i's "
                        "tail frees (every batch is still fully digested). 5 measured best on the 4 hardware "
                        "queues of the box (DESIGN.md §5.1)")
    return p.parse_args()


def make_batch(cfg: str, n: int, seed: int):
    from seqs_amd import synth

    if cfg in ("c2", "c4"):
        return synth.uniform_batch(n, 1500, seed=seed)
    if cfg == "c5":
        return synth.uniform_batch(n, 9000, seed=seed)
    if cfg == "small":
        return synth.hello_batch(n, seed=seed)
    return synth.mixed_batch(n, seed=seed)


WORKLOADS = {
    "c2": "C2: 65536 x 1500-B TCP frames per GPU (BASELINE configs[1])",
    "c3": "C3: 65536 mixed 64/576/1500/9000-B TCP/UDP frames per GPU (BASELINE configs[2])",
    "small": "the reference's benchmark shape (stacks/benchmark_test.go:12-46): 65536 x 47-B UDP 'hello' frames "
             "per GPU in 48-B slots",
}


def box_cores() -> int:
    """The CPU share of this process: OMP_NUM_THREADS when set (16 per GPU on the box), else
    the affinity mask."""
    try:
        v = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        v = 0
    return max(1, v or len(os.sched_getaffinity(0)))


def with_room(buf, off, ln, room: int = 4):
    """Repack a batch with `room` spare bytes after every frame (FCS space), 4-byte aligned."""
    step = (ln.astype(np.int64) + room + 3) // 4 * 4
    noff = np.zeros_like(off)
    noff[1:] = np.cumsum(step[:-1])
    nbuf = np.zeros(int(noff[-1] + step[-1]) + 16, np.uint8)
    for o, no, l in zip(off, noff, ln):
        nbuf[no : no + l] = buf[o : o + l]
    return nbuf, noff, ln


def gather_plan(steps: int, every: int, streams: int = 1) -> list:
    """The gather ROUNDS of a region of `steps` steps: each round takes half of the steps still
    to come (at most `every`, at least `streams`), so the rounds shrink toward the end (20 steps
    over 5 streams: 10, 5, 5). Every round's transfer overlaps the kernels of the rounds after
    it, and the region ends with at most a round of `streams` steps in flight. (Each round costs
    the host one event per stream it used: rounds of one step measured 25-30% slower at 20 steps.)"""
    out, left = [], max(0, steps)
    lo = max(1, min(streams, every))
    while left > 0:
        r = min(max(1, every), max(lo, (left + 1) // 2))
        if left - r < lo:
            r = left if left <= every else r  # no round below the floor at the end
        out.append(r)
        left -= r
    return out


def gather_schedule(rounds: list):
    """The gathers a region issues, in issue order: (after_step, buffer, slabs). Round k writes
    round buffer k % 2 (slab j = its j-th step) and is sent after its last step; a buffer is
    written again only after its previous round's transfer has been waited for. (The step loop
    below follows exactly this schedule; bench asserts it and tests/test_bench_plan.py checks it.)"""
    out, r0 = [], 0
    for k, n in enumerate(rounds):
        out.append((r0 + n - 1, k % 2, n))
        r0 += n
    return out


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_rate(cfg: str, seconds: float, threads: int):
    """The C oracle (scalar restatement of eth/crc.go + headers.go + RecvEth gates, zlib
    CRC-32) timed on a bounded C1-style sample: batches of 4,096 frames of the same workload
    (frames split over `threads` threads per batch)."""
    from oracle import coracle

    coracle.load()
    # 47-B frames: 262,144 per batch (12 MB), so the per-batch start of `threads` threads is not
    # what is timed (4,096 of them are 192 KB: 16 threads ran them slower than one)
    buf, off, ln = make_batch(cfg, 262144 if cfg == "small" else 4096, seed=101)
    nbytes = int(ln.astype(np.int64).sum())
    coracle.digest_batch(buf, off, ln, mtu=0, nthreads=threads)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        coracle.digest_batch(buf, off, ln, mtu=0, nthreads=threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds and reps >= 3:
            break
    return nbytes * reps / el / GIB, reps, nbytes, el


def cpu_baseline(cfg: str, seconds: float, threads: int):
    """All-cores figure (the box's CPU share) with the 1-thread figure beside it."""
    threads = threads or box_cores()
    what = {"c2": "1500-B TCP", "c4": "1500-B TCP", "c5": "9000-B TCP", "small": "47-B UDP 'hello'"}.get(cfg, "mixed")
    nfr = 262144 if cfg == "small" else 4096
    v1, r1, nbytes, e1 = cpu_rate(cfg, seconds / 2, 1)
    vn, rn, _, en = cpu_rate(cfg, seconds / 2, threads)
    return {
        "value": round(vn, 4),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "single_core": {"value": round(v1, 4), "unit": "GiB/s", "cores": 1},
        "sample": f"C1-style batches of {nfr} {what} frames ({nbytes} B) through oracle/framesum_oracle.c "
                  f"(CRC791 loop -O2 -fno-tree-vectorize + zlib crc32): {rn} batches in {en:.1f} s on {threads} "
                  f"threads, {r1} in {e1:.1f} s on 1 thread; {cpu_model()}",
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
    if args.config == "c5":
        return main_c5(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world == 1:
        # started without torchrun: run ourselves under it as a child process
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", os.environ.get("MASTER_PORT", "29511"),
               os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.run(cmd).returncode)

    import torch
    import torch.distributed as dist


    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = GPU.device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        GPU.init_group(dist, dev)
    elif args.force_gather and not args.no_gather:
        GPU.init_group(dist, dev, rank=0, world_size=1,
                       init_method=f"tcp://127.0.0.1:{os.environ.get('MASTER_PORT', '29513')}")

    if args.config == "c4":
        return main_c4(args, world, rank, local, dev)
    n = args.frames or 65536
    engine = GPU.engine(local)
    if args.kernel is None:
        args.kernel = 0
    engine.set_kernel(args.kernel)
    if args.workgroups:
        engine.set_workgroups(args.workgroups)
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
    # prepared calls (Engine.prepare_digest): each (batch, result slot, stream) the bench uses is
    # checked and marshalled once, so a step costs the host the C call alone (the first launch of
    # a short region comes that much sooner)
    prepared = {}
    can_prepare = hasattr(engine, "prepare_digest")

    def launch(bi, o, st, s):
        if not can_prepare:
            fb, fo, fl = batches[bi]
            return run_op(fb, fo, fl, mtu=0, out=o, status=st, stream=s)
        key = (bi, id(o), id(s))
        f = prepared.get(key)
        if f is None:
            fb, fo, fl = batches[bi]
            f = prepared[key] = engine.prepare_digest(fb, fo, fl, mtu=0, out=o, status=st, stream=s, op=args.op,
                                                      flags=3)
        return f()

    bytes_per_batch = int(batches[-1][2].cpu().numpy().astype(np.int64).sum())
    resident = sum(int(x[0].numel()) for x in batches)
    nb = len(batches)
    ns = max(1, args.streams)
    gather = dist.is_initialized() and not args.no_gather
    # every launch goes to created (non-blocking) streams, never the legacy default stream: a
    # launch there costs about 5 us more, and a short timed region (the driver's 20 steps) pays
    # it on every stream's first launch (tools/sync_overhead.py: 20.5-20.8 against 22.0-22.4 us
    # per step at K = 20; no difference at K = 200)
    main_stream = GPU.stream(dev)
    streams = [main_stream] + [GPU.stream(dev) for _ in range(ns - 1)]
    # Output slots (digest words, then verdicts, in one 256-B-aligned slab per slot). Without a
    # gather, step i writes slot i % nslot and slot k is only ever written by stream k (nslot ==
    # ns for ns >= 2; one stream for ns == 1): stream order alone keeps a slot's launches apart.
    # With the gather, the region's steps go in ROUNDS of consecutive steps (over all streams;
    # gather_plan: they shrink toward the region's end): round k's slabs are one contiguous
    # buffer (2 alternate); after its last step a transfer stream waits for every compute stream
    # and rank 0 receives every other rank's round buffer by one batch of point-to-point
    # receives (rank r sends its buffer), overlapped with the later rounds' kernels. Rank 0's
    # own slabs stay where its kernels wrote them.
    nslot = max(2, ns)
    slab = (9 * n + 255) // 256 * 256

    def views(buf, k):
        base = k * slab
        return buf[base : base + 8 * n].view(torch.int32).view(n, 2), buf[base + 8 * n : base + 9 * n]

    def round_map(K):
        """step r of a K-step region -> (round, slab); the region's rounds (gather_plan)"""
        rounds = gather_plan(K, args.gather_every, ns)
        m = [(k, j) for k, c in enumerate(rounds) for j in range(c)]
        return rounds, m

    if gather:
        plans = {K: round_map(K) for K in {args.steps, args.warmup} if K > 0}
        R = max(max(p[0]) for p in plans.values())  # slabs per round buffer
        rbuf = [torch.empty(R * slab, dtype=torch.uint8, device=dev) for _ in range(2)]
        rviews = [[views(rbuf[b], j) for j in range(R)] for b in range(2)]
        # rank 0: rank r's round-b slabs at recv[b][r]; 0xFF until received (checked at the end)
        recv = [[torch.full((R * slab,), 0xFF, dtype=torch.uint8, device=dev) for _ in range(world)]
                for _ in range(2)] if rank == 0 else None
        pend = [None, None]  # per buffer: the event marking its latest round's transfer done
        xfer = GPU.stream(dev)  # the rounds' transfers (no compute stream joins another)
        issued = []  # (after_step, buffer, slabs) of the region's gathers (== gather_schedule)
        last = {}  # buffer -> slabs its latest round carried
    flat = torch.empty(nslot * slab, dtype=torch.uint8, device=dev)
    outs, stats = zip(*[views(flat, k) for k in range(nslot)])

    def step(i: int, r: int, K: int):
        """step i overall, r-th of its region of K steps (the rounds restart with each region)"""
        s = streams[r % ns]
        if not gather:
            launch(i % nb, outs[i % nslot], stats[i % nslot], s)
            return
        rounds, rmap = plans[K]
        k, j = rmap[r]
        b = k % 2
        # the streams this round's steps run on (its first step is r - j)
        used = sorted({(r - j + t) % ns for t in range(min(ns, rounds[k]))})
        if j == 0 and pend[b] is not None:
            # buffer b's previous round has been sent: the streams that will write it wait for
            # that round's transfer (its own event, not the transfer stream's later work)
            for q in used:
                GPU.wait_event(streams[q], pend[b])
            pend[b] = None
        o, st = rviews[b][j]
        launch(i % nb, o, st, s)
        if j == rounds[k] - 1:
            m = j + 1
            for q in used:
                xfer.wait_stream(streams[q])
            with GPU.use(xfer):
                if rank == 0:
                    ops = [dist.P2POp(dist.irecv, recv[b][q][: m * slab], q) for q in range(1, world)]
                else:
                    ops = [dist.P2POp(dist.isend, rbuf[b][: m * slab], 0)]
                # wait ONCE per work, on the transfer stream (RCCL: a stream-side wait; a second
                # wait() on a point-to-point work never returns on some backends), and mark it
                for w in (dist.batch_isend_irecv(ops) if ops else []):
                    w.wait()
                pend[b] = GPU.mark(xfer)
            issued.append((r, b, m))
            last[b] = m

    def drain():
        if not gather:
            return
        for b in range(2):
            if pend[b] is not None:
                GPU.wait_event(main_stream, pend[b])  # (the synchronize after the region covers all)
                pend[b] = None

    # device pre-warm (setup, not steps): throughput settles only after several hundred launches
    prewarm = max(0, args.min_warm - args.warmup)
    for i in range(prewarm):
        # over every stream (slot k on stream k): a stream's first launch costs hundreds of us,
        # which must not land in the timed region when --warmup is below the stream count
        launch(i % nb, outs[i % nslot], stats[i % nslot], streams[i % ns])
    GPU.settle(streams)
    GPU.sync()
    if world > 1:
        dist.barrier()
    # the host spin first, then the warmup steps right before the region: the GPU stays busy up
    # to it (an idle GPU before a 20-step region cost ~9 us, tools/region_ab.py, round 3)
    gc.collect()
    host_warm()
    for i in range(args.warmup):
        step(i, i, args.warmup)
    drain()
    GPU.settle(streams + ([xfer] if gather else []))
    if gather:
        last.clear()  # the checks below cover the timed region's gathers
        issued.clear()

    # ---- timed region: K steps, barrier + synchronize on both sides, max over ranks (Python's
    # garbage collector off inside it, as timeit does: a collection is tens of us in a ~400-us region)
    if world > 1:
        dist.barrier()
    GPU.sync()
    gc.disable()
    rc = region_clocks_begin(args.region_clocks)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, i, args.steps)
        if rc is not None:
            rc["steps"].append(time.clock_gettime_ns(time.CLOCK_MONOTONIC))
    if rc is not None:
        rc["enqueued"] = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
    drain()
    # (in launch order: the stream of the region's last step is polled last)
    GPU.settle([streams[(args.steps + t) % ns] for t in range(ns)] + ([xfer] if gather else []))
    if rc is not None:
        rc["settled"] = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
    GPU.sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    region_clocks_end(rc, args.region_clocks, elapsed)
    gc.enable()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if gather:
        assert issued == gather_schedule(plans[args.steps][0]), "the region's gathers differ from gather_schedule"
    if gather and rank == 0 and world > 1:
        # every other rank's latest round arrived (valid frames: all verdicts 0, where 0xFF was)
        GPU.sync()
        for b, m in last.items():
            for q in range(1, world):
                got = recv[b][q][: m * slab].view(m, slab)[:, 8 * n : 9 * n]
                assert int(got.max().item()) == 0, f"rank {q}'s round-{b} slabs did not arrive"

    # ---- kernel-only timing with HIP events on the launch stream (roofline.achieved): one event
    # pair around K back-to-back launches on one stream (no overlap with another launch), so the
    # average is the kernel's duration plus the stream's dispatch gap; an event pair around every
    # launch would add each record's own latency to every launch.
    k0, k1 = GPU.event(), GPU.event()
    with GPU.use(main_stream):
        k0.record(main_stream)
        for i in range(args.steps):  # same stream, in order: no slot events needed
            launch(i % nb, outs[i % nslot], stats[i % nslot], main_stream)
        k1.record(main_stream)
    GPU.sync()
    k_avg_ms = k0.elapsed_time(k1) / args.steps
    engine_last_kernel = engine.last_kernel()

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
            "frames_per_s": round(n * args.steps * world / elapsed, 1),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic: {nb} distinct resident batches ({resident / 1e6:.0f} MB) of valid frames, rotated",
            "config": {
                "workload": WORKLOADS[args.config] if n == 65536 else f"{args.config} with {n} frames per GPU",
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
                "frac_mode": "single stream: algorithmic bytes / average kernel duration (HIP events around K "
                             "back-to-back launches on one stream, no overlap between launches)",
                "frac_whole_job": round(bytes_per_batch / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
                "frac_whole_job_mode": f"algorithmic bytes per step / ms_per_step of the timed region ({ns} streams: "
                                       "consecutive launches overlap each other's start and tail)",
                "traffic": traffic,
                "traffic_calibrated": traffic_cal,
                "traffic_note": "traffic = (2*FETCH_SIZE + WRITE_SIZE)*1024 per launch (profiles/pmc_<cfg>.json, separate "
                                "--pmc passes). Its excess over the algorithmic bytes is mostly the read pattern's own: "
                                "the line two neighbouring frames share is fetched twice (~8.4% on C2); "
                                "traffic_calibrated divides that pattern factor out (the kernel's excess beyond it)"
                if traffic is not None else None,
                "kernel": {0: "automatic: digest_kernel_a (one-pass) for uniform batches, digest_kernel_ab for mixed "
                              "(digest_kernel_g when a mixed tile holds a frame beyond its pieces), "
                              "digest_kernel_s once the launches it has seen ran had no frame over 128 B",
                           2: "digest_kernel_ab (mixed-length)", 3: "digest_kernel_g (segments)",
                           4: "digest_kernel_a (one-pass)",
                           8: "digest_kernel_s preferred (fs_ctx_set_kernel 8: until a launch meets a frame over 128 B, "
                              "then the automatic choice until short traffic resumes)"}.get(args.kernel),
                "kernel_chosen": KERNEL_NAMES.get(engine_last_kernel),
                "kernel_avg_us": round(k_avg_ms * 1e3, 3),
                "kernel_timing": "HIP events around K back-to-back launches on the launch stream",
                "algorithmic_bytes_per_launch": bytes_per_batch,
                # per frame the kernel also reads its 12-B descriptor (offset, length) and writes its
                # 9-B result (digest, verdict): not algorithmic bytes, but 45% of them at 47-B frames
                "metadata_bytes_per_launch": 21 * n,
                "achieved_incl_metadata": round((bytes_per_batch + 21 * n) / (k_avg_ms * 1e-3) / 1e9, 1),
            },
            "cpu_baseline": cpu,
        }
    engine.close()
    del batches, flat
    if gather:
        del rbuf, rviews, recv
    if rank == 0 and world == 1 and args.config == "c2" and args.op == "digest" and not args.no_sub:
        # BASELINE configs[2] and [4] beside the C2 headline: the C3
        # mixed batch device-resident (same steps and warmup) and the C5 jumbo batch end to end
        # from pinned host memory; the reference's 47-B benchmark frames device-resident and
        # host-staged; the TX fill and the FCS verify; each bounded to a
        # few seconds
        GPU.empty_cache()
        result["c3"] = sub_record_c3(args, dev)
        GPU.empty_cache()
        result["c5_host"] = sub_record_c5(args)
        GPU.empty_cache()
        result["small"] = sub_record_small(args, dev)
        GPU.empty_cache()
        result["fill"] = sub_record_op(args, dev, "fill")
        GPU.empty_cache()
        result["fcs"] = sub_record_op(args, dev, "fcs")
        GPU.empty_cache()
        result["small_host"] = sub_record_small_host(args)
    if world > 1 and args.config == "c2" and args.op == "digest" and not args.no_c4:
        # the C4 strong-scaled record beside the weak-scaled C2 value (same steps / warmup)
        GPU.empty_cache()
        c4 = run_c4(args, world, rank, local, dev, frames=args.c4_frames)
        if rank == 0:
            result["c4_strong"] = {k: c4[k] for k in ("value", "unit", "ms_per_step", "scaling", "config")}
            result["c4_strong"]["kernel_avg_us"] = c4["roofline"]["kernel_avg_us"]
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    return result


def single_gpu_region(engine, batches, steps: int, warmup: int, min_warm: int, ns: int, dev, op: str = "digest",
                      flags: int = 3):
    """The N = 1 step loop of main() without the gather: prewarm over the streams, host spin,
    warmup steps, then K timed steps (barrier-free: one rank) closed by a polled settle and a
    synchronize; then K back-to-back launches on one stream between HIP events. op: "digest"
    (fs_digest_batch), "fill" (fs_fill_batch with `flags`) or "fcs" (fs_digest_batch_fcs). Returns
    (elapsed seconds of the K steps, average kernel ms)."""
    import torch

    n = int(batches[0][2].numel())
    nslot = max(2, ns)
    slab = (9 * n + 255) // 256 * 256
    flat = torch.empty(nslot * slab, dtype=torch.uint8, device=dev)
    outs = [flat[k * slab: k * slab + 8 * n].view(torch.int32).view(n, 2) for k in range(nslot)]
    stats = [flat[k * slab + 8 * n: k * slab + 9 * n] for k in range(nslot)]
    streams = [GPU.stream(dev) for _ in range(ns)]
    nb = len(batches)

    # prepared calls per (batch, slot, stream), as the headline's steps (a step of the small-frame
    # record is ~5 us: the host's per-call marshalling would otherwise pace it)
    prepared = {}

    def launch(i, s):
        key = (i % nb, i % nslot, id(s))
        f = prepared.get(key)
        if f is None:
            fb, fo, fl = batches[i % nb]
            f = prepared[key] = engine.prepare_digest(fb, fo, fl, mtu=0, out=outs[i % nslot], status=stats[i % nslot],
                                                      stream=s, op=op, flags=flags)
        f()

    for i in range(max(0, min_warm - warmup)):
        launch(i, streams[i % ns])
    GPU.settle(streams)
    GPU.sync()
    gc.collect()
    host_warm()
    for i in range(warmup):
        launch(i, streams[i % ns])
    GPU.settle(streams)
    GPU.sync()
    gc.disable()
    t0 = time.perf_counter()
    for i in range(steps):
        launch(warmup + i, streams[i % ns])
    GPU.settle(streams)
    GPU.sync()
    elapsed = time.perf_counter() - t0
    gc.enable()
    k0, k1 = GPU.event(), GPU.event()
    with GPU.use(streams[0]):
        k0.record(streams[0])
        for i in range(steps):
            launch(i, streams[0])
        k1.record(streams[0])
    GPU.sync()
    return elapsed, k0.elapsed_time(k1) / steps


def sub_record_c3(args, dev):
    """C3 (BASELINE configs[2]) device-resident beside the C2 headline: 65,536 mixed
    64/576/1500/9000-B frames, 2 resident batches (365 MB, past the 256 MiB Infinity Cache),
    the automatic kernel choice (the mixed-length kernel for this batch), the same steps and
    warmup as the headline."""
    import torch

    engine = GPU.engine(0)
    t_start = time.perf_counter()
    batches = []
    for b in range(2):
        buf, off, ln = make_batch("c3", 65536, seed=301 + b)
        batches.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)))
    nbytes = int(batches[0][2].sum().item())
    elapsed, k_ms = single_gpu_region(engine, batches, args.steps, args.warmup, args.min_warm, max(1, args.streams), dev)
    chosen = KERNEL_NAMES.get(engine.last_kernel())
    engine.close()
    del batches
    return {
        "workload": WORKLOADS["c3"],
        "value": round(nbytes * args.steps / elapsed / GIB, 3),
        "unit": "GiB/s",
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "bytes_per_step": nbytes,
        "kernel_avg_us": round(k_ms * 1e3, 3),
        "frac": round(nbytes / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "frac_whole_job": round(nbytes / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
        "kernel_chosen": chosen,
        "note": "whole-job value over the same steps/warmup and streams as the headline; frac = algorithmic "
                "bytes / kernel_avg_us (HIP events around K back-to-back launches on one stream) / 8 TB/s",
        "wall_s": round(time.perf_counter() - t_start, 2),
    }


def sub_record_small(args, dev):
    """The reference's own benchmark shape beside the headline (stacks/benchmark_test.go:12-46: 47-B
    UDP 'hello' frames through RecvEth): 65,536 frames in 48-B slots, 4 resident batches, the
    automatic kernel choice (variant 0: after the launches it has seen run with no frame over 128 B,
    the small-frame kernel; kernel_chosen shows what the timed launches ran), the same steps and
    warmup as the headline. Frames/s is its natural unit."""
    import torch

    engine = GPU.engine(0)
    engine.set_kernel(0)  # the automatic choice: it moves to the small-frame kernel on this traffic
    t_start = time.perf_counter()
    n = 65536
    batches = []
    for b in range(4):
        buf, off, ln = make_batch("small", n, seed=401 + b)
        batches.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)))
    nbytes = int(batches[0][2].sum().item())
    elapsed, k_ms = single_gpu_region(engine, batches, args.steps, args.warmup, args.min_warm, max(1, args.streams), dev)
    chosen = KERNEL_NAMES.get(engine.last_kernel())
    engine.close()
    del batches
    return {
        "workload": WORKLOADS["small"],
        "value": round(nbytes * args.steps / elapsed / GIB, 3),
        "unit": "GiB/s",
        "frames_per_s": round(n * args.steps / elapsed, 1),
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "bytes_per_step": nbytes,
        "kernel_avg_us": round(k_ms * 1e3, 3),
        "kernel_chosen": chosen,
        "note": "whole-job value over the same steps/warmup and streams as the headline; a latency-bound shape "
                "(3 MB per step): frames/s, not the HBM fraction, is its figure",
        "wall_s": round(time.perf_counter() - t_start, 2),
    }


def sub_record_op(args, dev, op: str):
    """SURVEY.md §8f ranks 2 and 4 beside the RX headline, on C2's shape,
    the same steps and warmup: "fill" = the TX checksum fill with FCS append in place
    (fs_fill_batch FS_FILL_CSUM | FS_FCS_APPEND; stacks/port_tcp.go:162-194 fills the IPv4 and TCP
    checksums of every frame it sends), "fcs" = the RX of wire frames that still carry their FCS
    (fs_digest_batch_fcs). 4 resident batches of 65,536 x 1500-B frames, each with 4 spare bytes
    after it (the FCS). Algorithmic bytes: the frame bytes read (fill: the 1500-B frames, which it
    also rewrites in 8 bytes: the two checksum fields and the FCS; fcs: the 1504-B wire frames)."""
    import torch

    engine = GPU.engine(0)
    t_start = time.perf_counter()
    batches = []
    for b in range(4):
        buf, off, ln = with_room(*make_batch("c2", 65536, seed=501 + b))
        tb, to, tl = torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)
        if op == "fcs":  # wire frames: the FCS appended once, the lengths include it
            engine.fill_device(tb, to, tl, flags=2)
            tl = tl + 4
        batches.append((tb, to, tl))
    nbytes = int(batches[0][2].sum().item())
    elapsed, k_ms = single_gpu_region(engine, batches, args.steps, args.warmup, args.min_warm, max(1, args.streams), dev,
                                      op=op, flags=3)
    chosen = KERNEL_NAMES.get(engine.last_kernel())
    # the results of the last launches: every frame filled / verified
    GPU.sync()
    engine.close()
    del batches
    return {
        "workload": {"fill": "TX checksum fill + FCS append in place (fs_fill_batch FS_FILL_CSUM|FS_FCS_APPEND) of "
                             "65536 x 1500-B TCP frames, 4 spare bytes after each",
                     "fcs": "RX of 65536 x 1504-B wire frames (1500 B + FCS) through fs_digest_batch_fcs"}[op],
        "value": round(nbytes * args.steps / elapsed / GIB, 3),
        "unit": "GiB/s",
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "bytes_per_step": nbytes,
        "kernel_avg_us": round(k_ms * 1e3, 3),
        "frac": round(nbytes / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "frac_whole_job": round(nbytes / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
        "kernel_chosen": chosen,
        "note": "whole-job value over the same steps/warmup and streams as the headline; frac = frame bytes read / "
                "kernel_avg_us (HIP events around K back-to-back launches on one stream) / 8 TB/s"
                + ("; the fill also writes 8 B per frame (checksum fields + FCS), written back as dirty lines"
                   if op == "fill" else ""),
        "wall_s": round(time.perf_counter() - t_start, 2),
    }


def sub_record_small_host(args):
    """The reference's benchmark shape through the host-staged call the Go RecvEthBatch binding makes
    (stacks/benchmark_test.go:12-46 sends 47-B UDP frames through RecvEth,
    stacks/portstack.go:163): 65,536 x 47-B frames in pinned host memory, their offsets and lengths
    pinned beside them (go/eth/digest_gpu.go stages them so), fs_digest_batch_host with the automatic
    kernel choice (every frame <= 128 B: the small-frame kernel), results into pageable host arrays
    (the Go caller's slices). PCIe-inclusive; the C oracle on the same frames beside it, 16 threads
    and 1."""
    from seqs_amd import Engine

    t_start = time.perf_counter()
    eng = Engine(0)
    buf, off, ln = make_batch("small", 65536, seed=77)
    n, nbytes = len(ln), int(ln.astype(np.int64).sum())
    pin = eng.host_empty(buf.shape, np.uint8)
    pin[:] = buf
    # the offsets and then the lengths in one pinned block, as the Go binding stages them (one H2D copy)
    desc = eng.host_empty((12 * n,), np.uint8)
    poff = desc[: 8 * n].view(np.uint64)
    plen = desc[8 * n:].view(np.uint32)
    poff[:] = off
    plen[:] = ln
    from seqs_amd.framesum import DIGEST_DTYPE
    out = np.zeros(n, dtype=DIGEST_DTYPE)
    st = np.zeros(n, dtype=np.uint8)
    pout = eng.host_empty((n,), DIGEST_DTYPE)
    pst = eng.host_empty((n,), np.uint8)
    steps, warm = max(args.steps, 100), max(args.warmup, 20)
    res = {}
    for name, o, s in (("pageable_results", out, st), ("pinned_results", pout, pst)):
        for _ in range(warm):
            eng.digest_host(pin, poff, plen, out=o, status=s)
        gc.disable()
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.digest_host(pin, poff, plen, out=o, status=s)
        res[name] = time.perf_counter() - t0
        gc.enable()
    assert np.array_equal(out, pout) and np.array_equal(st, pst)
    chosen = KERNEL_NAMES.get(eng.last_kernel())
    eng.close()
    el = res["pageable_results"]
    cpu = cpu_baseline("small", 4.0, args.cpu_threads) if args.cpu_seconds > 0 else None
    return {
        "workload": "65536 x 47-B UDP 'hello' frames (stacks/benchmark_test.go:12-46) host-staged through "
                    "fs_digest_batch_host: frames + descriptors pinned, results into pageable arrays (the Go "
                    "RecvEthBatch binding's arrangement)",
        "value": round(nbytes * steps / el / GIB, 3),
        "unit": "GiB/s",
        "frames_per_s": round(n * steps / el, 1),
        "us_per_call": round(el / steps * 1e6, 2),
        "us_per_call_pinned_results": round(res["pinned_results"] / steps * 1e6, 2),
        "steps": steps,
        "warmup": warm,
        "bytes_per_step": nbytes,
        "transfer_bytes_per_call": {"h2d": nbytes + 12 * n, "d2h": 9 * n},
        "kernel_chosen": chosen,
        "cpu_baseline": cpu,
        "note": "PCIe-inclusive (not the HBM metric); cpu_baseline: the C oracle on the same 47-B frames",
        "wall_s": round(time.perf_counter() - t_start, 2),
    }


def sub_record_c5(args, steps: int = 10, warmup: int = 3):
    """C5 (BASELINE configs[4]) on one GPU beside the headline: 16,384 x 9000-B jumbo frames from
    pinned host memory through fs_digest_batch_multi (one context), results back in host memory;
    PCIe-inclusive, never the headline value."""
    from seqs_amd import Engine, digest_host_multi

    t_start = time.perf_counter()
    eng = Engine(0)
    src, off, ln = make_batch("c5", 16384, seed=55)
    pinned = eng.host_empty(src.shape, np.uint8)
    pinned[:] = src
    del src
    total = int(ln.astype(np.int64).sum())
    for _ in range(warmup):
        digest_host_multi([eng], pinned, off, ln)
    t0 = time.perf_counter()
    for _ in range(steps):
        _, st = digest_host_multi([eng], pinned, off, ln)
    elapsed = time.perf_counter() - t0
    assert (st == 0).all(), "valid frames must all verify"
    eng.close()
    gbs = total / (elapsed / steps) / 1e9
    return {
        "workload": "C5 shape on 1 GPU: 16384 x 9000-B jumbo frames streamed from pinned host memory "
                    "(fs_digest_batch_multi, one context), results back in host memory",
        "value": round(total * steps / elapsed / GIB, 3),
        "unit": "GiB/s",
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(elapsed / steps * 1e3, 4),
        "bytes_per_step": total,
        "roofline": {"bound": "pcie", "achieved": round(gbs, 2), "peak": 63.0, "unit": "GB/s",
                     "frac": round(gbs / 63.0, 4), "note": "PCIe Gen5 x16 spec 63 GB/s (MI355X_MICROARCH.md)"},
        "wall_s": round(time.perf_counter() - t_start, 2),
    }


def _clocks():
    return {"mono": time.clock_gettime_ns(time.CLOCK_MONOTONIC),
            "boot": time.clock_gettime_ns(getattr(time, "CLOCK_BOOTTIME", time.CLOCK_MONOTONIC))}


def region_clocks_begin(path):
    """--region-clocks: the clocks right before t0 (None when not asked for)."""
    return None if not path else {"t0": _clocks(), "steps": []}


def region_clocks_end(rc, path, elapsed):
    if rc is None:
        return
    rc["t1"] = _clocks()
    rc["elapsed_us"] = elapsed * 1e6
    with open(path, "a") as f:
        f.write(json.dumps(rc) + "\n")


def host_warm(seconds: float = 3e-3):
    """Keep the host thread busy for a few ms before the warmup steps that precede a timed region
    (no device work). A thread that has just slept in a blocking synchronize enqueues the region's
    first launches slowly: the 20-step C2 region after a 400-launch burst ran 408-461 us without
    this, 400-418 us with it; spinning before the warmup steps rather than after them (so the GPU
    is not idle right before the region) ran 398-402 us (tools/region_ab.py --fresh,
    profiles/round3/region_ab.log)."""
    t = time.perf_counter()
    while time.perf_counter() - t < seconds:
        pass


def time_region(world, dist, torch, body, dev, streams=()):
    """barrier + synchronize, body(), settle + synchronize + barrier; max over ranks."""
    if world > 1:
        dist.barrier()
    GPU.sync()
    gc.disable()
    t0 = time.perf_counter()
    body()
    GPU.settle(streams)
    GPU.sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gc.enable()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def main_c4(args, world, rank, local, dev):
    result = run_c4(args, world, rank, local, dev, frames=args.frames or (1 << 20))
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist_initialized():
        import torch.distributed as dist

        dist.destroy_process_group()
    return result


def dist_initialized() -> bool:
    import torch.distributed as dist

    return dist.is_available() and dist.is_initialized()


def run_c4(args, world, rank, local, dev, frames):
    """C4 (BASELINE configs[3]): one global batch of 1,048,576 x 1500-B frames per step,
    frame i on rank i mod N (strong scaling). A step: every rank digests its shard into a
    slab (digests + verdicts, fs_shard_slab_bytes layout), RCCL brings the slabs to rank 0 (one batch
    of point-to-point transfers into its gather buffer),
    rank 0's de-interleave kernel writes the digests in global frame order. Two slots
    alternate on two streams, so step i's gather and de-interleave overlap step i+1's kernel."""
    import torch
    import torch.distributed as dist

    from seqs_amd import shard_count, shard_slab_bytes

    n_global = frames
    engine = GPU.engine(local)
    if getattr(args, "workgroups", 0):
        engine.set_workgroups(args.workgroups)
    n = shard_count(n_global, world, rank)
    m = (n_global + world - 1) // world
    sb = shard_slab_bytes(n_global, world)
    nb = 2  # 2 x 1.57 GB resident at N=1: far past the 256 MiB Infinity Cache
    batches = []
    for b in range(nb):
        buf, off, ln = make_batch("c4", n, seed=1 + 1000 * rank + b)
        batches.append((torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev)))
    bytes_local = int(batches[0][2].cpu().numpy().astype(np.int64).sum())
    t = torch.tensor([bytes_local], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(t)
    bytes_global = int(t.item())
    gather = dist.is_initialized()
    streams = [GPU.stream(dev), GPU.stream(dev)]  # created streams (see main())
    # slot k: rank 0 gathers into recv[k] (world slabs back to back; its own slab is slab 0),
    # other ranks digest into send[k]
    recv = [torch.empty(world * sb, dtype=torch.uint8, device=dev) for _ in range(2)] if rank == 0 else None
    send = [recv[k][:sb] for k in range(2)] if rank == 0 else \
        [torch.empty(sb, dtype=torch.uint8, device=dev) for _ in range(2)]
    gout = [torch.empty((n_global, 2), dtype=torch.int32, device=dev) for _ in range(2)] if rank == 0 else None
    gst = [torch.empty(n_global, dtype=torch.uint8, device=dev) for _ in range(2)] if rank == 0 else None
    pend = [None, None]

    def views(k):
        return send[k][: 8 * m].view(torch.int32)[: 2 * n].view(n, 2), send[k][8 * m : 8 * m + n]

    def step(i):
        k = i % 2
        s = streams[k]
        fb, fo, fl = batches[i % nb]
        with GPU.use(s):
            if pend[k] is not None:
                for w in pend[k]:
                    w.wait()  # slot k's previous transfer has read send[k] (stream-side wait)
                pend[k] = None
            o, st = views(k)
            engine.digest_device(fb, fo, fl, mtu=0, out=o, status=st, stream=s)
            if gather and world > 1:
                # the gather as one batch of point-to-point transfers straight into rank 0's slab
                # views (rank 0's own slab is written in place by its kernel)
                if rank == 0:
                    ops = [dist.P2POp(dist.irecv, recv[k][r * sb : (r + 1) * sb], r) for r in range(1, world)]
                else:
                    ops = [dist.P2POp(dist.isend, send[k], 0)]
                pend[k] = dist.batch_isend_irecv(ops)
            if rank == 0:
                if pend[k] is not None:
                    for w in pend[k]:
                        w.wait()
                    pend[k] = None
                engine.deinterleave_device(recv[k], world, n_global, out=gout[k], status=gst[k], stream=s)

    def drain():
        for k in range(2):
            if pend[k] is not None:
                with GPU.use(streams[k]):
                    for w in pend[k]:
                        w.wait()
                pend[k] = None

    gc.collect()
    host_warm()
    for i in range(args.warmup):
        step(i)
    drain()
    GPU.settle(streams)

    def body():
        for i in range(args.steps):
            step(args.warmup + i)
        drain()

    elapsed = time_region(world, dist, torch, body, dev, streams)

    # check on rank 0: the last step's global-order output is the interleave of the slabs
    # gathered for it (the de-interleave and the gather layout), and rank 0's own frames
    if rank == 0:
        k = (args.warmup + args.steps - 1) % 2
        GPU.sync()
        g = recv[k].cpu().numpy()
        i = np.arange(n_global)
        r, j = i % world, i // world
        exp_w = np.stack([g[r * sb + 8 * j + b] for b in range(8)], axis=1).view(np.int32).reshape(n_global, 2)
        assert np.array_equal(gout[k].cpu().numpy(), exp_w), "de-interleave mismatch"
        assert np.array_equal(gst[k].cpu().numpy(), g[r * sb + 8 * m + j]), "de-interleave verdict mismatch"
        assert (gst[k].cpu().numpy() == 0).all(), "valid frames must all verify"

    # kernel-only: K back-to-back shard digests on one stream (events on the launch stream)
    k0, k1 = GPU.event(), GPU.event()
    ms = streams[0]
    with GPU.use(ms):
        k0.record(ms)
        for i in range(args.steps):
            fb, fo, fl = batches[i % nb]
            o, st = views(0)
            engine.digest_device(fb, fo, fl, mtu=0, out=o, status=st, stream=ms)
        k1.record(ms)
    GPU.sync()
    k_ms = k0.elapsed_time(k1) / args.steps
    t = torch.tensor([k_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    k_ms_max = float(t.item())
    value = bytes_global * args.steps / elapsed / GIB
    if rank == 0:
        result = {
            "metric": "GiB/s device-resident CRC-32+Internet-csum over batched MTU frames; % HBM peak",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic: {nb} distinct resident shard batches per rank of valid 1500-B TCP frames, rotated",
            "config": {
                "workload": f"C4: {n_global}-frame global batch of 1500-B frames sharded round-robin over {world} "
                            "GPU(s) (BASELINE configs[3])",
                "global_batch_frames": n_global,
                "bytes_per_step": bytes_global,
                "parallelism": f"frame i on rank i mod {world}; per step: shard digest, RCCL gather of the digests + "
                               "verdicts to rank 0, de-interleave kernel on rank 0 (all inside the step)"
                if world > 1 else "single GPU: shard = whole batch; de-interleave kernel inside the step",
                "kernel_only_gibs": round(bytes_global / (k_ms_max * 1e-3) / GIB, 3),
                "kernel_only_ms": round(k_ms_max, 5),
                "streams": 2,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(bytes_local / (k_ms * 1e-3) / 1e9, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(bytes_local / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "traffic": None,
                "kernel": "automatic choice (uniform 1500-B shards: digest_kernel_a, the one-pass kernel)",
                "kernel_avg_us": round(k_ms * 1e3, 3),
                "frac_mode": "rank 0's shard kernel, single stream",
            },
            "cpu_baseline": cpu_baseline("c4", args.cpu_seconds, args.cpu_threads)
            if world == 1 and args.cpu_seconds > 0 else None,
        }
    else:
        result = None
    engine.close()
    return result


def main_c5(args):
    """C5 (BASELINE configs[4]): 9000-B jumbo frames streamed from pinned host memory to
    --gpus GPUs from ONE process: fs_digest_batch_multi, one context per GPU, byte-balanced
    contiguous blocks, each on its own host thread with its own H2D / kernel / D2H pipeline.
    A step = one call over the whole host batch (results back in host memory). Bound by PCIe
    and host memory, not HBM."""
    import torch

    from seqs_amd import Engine, digest_host_multi

    ngpu = max(1, args.gpus)
    per_gpu = args.frames or 16384
    engines = [Engine(d) for d in range(ngpu)]
    n = per_gpu * ngpu
    src, off, ln = make_batch("c5", n, seed=55)
    pinned = engines[0].host_empty(src.shape, np.uint8)
    pinned[:] = src
    del src
    total = int(ln.astype(np.int64).sum())
    for _ in range(max(1, args.warmup)):
        digest_host_multi(engines, pinned, off, ln)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out, st = digest_host_multi(engines, pinned, off, ln)
    elapsed = time.perf_counter() - t0
    assert (st == 0).all(), "valid frames must all verify"
    value = total * args.steps / elapsed / GIB
    result = {
        "metric": "GiB/s end-to-end (pinned host memory -> GPU -> host) CRC-32+Internet-csum over batched jumbo frames",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": ngpu,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic: one pinned host batch of {n} valid 9000-B TCP frames ({total / 1e9:.2f} GB)",
        "config": {
            "workload": f"C5: {per_gpu} x 9000-B jumbo frames per GPU streamed from pinned host memory "
                        "(BASELINE configs[4]); PCIe-inclusive, not the HBM metric",
            "frames_per_gpu": per_gpu,
            "bytes_per_step": total,
            "parallelism": f"fs_digest_batch_multi over {ngpu} context(s), one per GPU, one host process",
        },
        "roofline": {"bound": "pcie", "peak": 63.0 * ngpu, "unit": "GB/s",
                     "achieved": round(total / (elapsed / args.steps) / 1e9, 2),
                     "frac": round(total / (elapsed / args.steps) / 1e9 / (63.0 * ngpu), 4),
                     "kernel": None, "note": "PCIe Gen5 x16 spec 63 GB/s per GPU (MI355X_MICROARCH.md)"},
        "cpu_baseline": cpu_baseline("c5", args.cpu_seconds, args.cpu_threads) if args.cpu_seconds > 0 else None,
    }
    print(json.dumps(result), flush=True)
    for e in engines:
        e.close()
    return result


if __name__ == "__main__":
    main()
