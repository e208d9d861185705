"""CPU-side sanitizer builds: the host planning logic of the C ABI
(seqs_amd/csrc/framesum_plan.h: host-staged chunks, fs_digest_batch_multi blocks, round-robin
shard / gather / de-interleave maps) and the C oracle, each compiled with ASan + UBSan by
tests/csrc/Makefile and run to completion; any memory error or undefined behaviour aborts."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "tests", "csrc")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")


def build(target):
    subprocess.run(["make", "-s", "-C", CSRC, f"build/{target}"], check=True)
    return os.path.join(CSRC, "build", target)


def test_plan_under_asan_ubsan():
    r = subprocess.run([build("test_plan")], capture_output=True, text=True, timeout=300, env=ENV)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "plan checks OK" in r.stdout


def test_oracle_under_asan_ubsan():
    r = subprocess.run([build("test_oracle_san")], capture_output=True, text=True, timeout=300, env=ENV)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "oracle sanitizer run OK" in r.stdout
