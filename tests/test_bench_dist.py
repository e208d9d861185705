"""bench.py's N > 1 path, run as the driver's scaling run would run it (two ranks, the same
rounds, transfers, run-time checks and C4 record), on CPU over gloo with an engine stand-in
(tests/bench_dist_driver.py). The GPU box has one GPU, so this is where the multi-rank loop is
exercised before the driver's N = 2..8 runs."""
import json
import os
import socket
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(args, world=2):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "bench_dist_driver.py")] + args,
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    lines = [l for l in outs[0][0].splitlines() if l.startswith("{")]
    assert len(lines) == 1, outs[0][0][-2000:]
    assert not [l for l in outs[1][0].splitlines() if l.startswith("{")]  # rank 0 prints alone
    return json.loads(lines[0])


def test_c2_weak_line_with_c4_record():
    d = _run(["--gpus", "2", "--steps", "20", "--warmup", "5", "--frames", "512", "--c4-frames", "4096",
              "--cpu-seconds", "0", "--min-warm", "0"])
    assert d["n_gpus"] == 2 and d["steps"] == 20 and d["scaling"] == "weak"
    assert d["config"]["global_batch_frames"] == 1024 and "RCCL" in d["config"]["parallelism"]
    c4 = d["c4_strong"]
    assert c4["scaling"] == "strong" and c4["config"]["global_batch_frames"] == 4096
    assert c4["value"] > 0 and c4["ms_per_step"] > 0


def test_c4_config_line():
    d = _run(["--gpus", "2", "--config", "c4", "--steps", "7", "--warmup", "3", "--frames", "3001",
              "--cpu-seconds", "0"])
    assert d["scaling"] == "strong" and d["n_gpus"] == 2 and d["config"]["global_batch_frames"] == 3001


def test_long_region_rounds():
    # 64 steps: rounds 32, 16, 8, 8 over 5 streams; the run-time schedule assert covers them
    d = _run(["--gpus", "2", "--steps", "64", "--warmup", "7", "--frames", "256", "--no-c4", "--cpu-seconds", "0",
              "--min-warm", "0"])
    assert d["steps"] == 64 and "c4_strong" not in d


def test_gpu_seam_calls_torch_cuda():
    """The real seam (bench.GpuOps) calls torch.cuda / torch.distributed / seqs_amd directly,
    never back into bench.GPU (the CPU stand-ins above override every method, so the loop
    tests cannot see that)."""
    import ast
    import inspect

    import bench

    src = inspect.getsource(bench.GpuOps)
    for node in ast.walk(ast.parse(src)):
        if isinstance(node, ast.Attribute) and isinstance(node.value, ast.Name):
            assert node.value.id != "GPU", f"GpuOps calls GPU.{node.attr}"
