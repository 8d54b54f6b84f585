"""Runs the C++ Dag Node / datanode mirror tests (tests/cpp/test_dagnode.cpp).

cpu: datanode entry framing + CRC, quorum reduction, slots, config validation.
gpu: TestDagNode's RS(2,1) "123456" round trip (node_test.go:18-65), the RS(10,4)
failure/quorum matrix, read-repair, RepairDataNode (per key and GPU-batched), PutMany --
every stored shard checked against the CPU oracle."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_dagnode")


def _binary():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")])
    return BIN


def test_dagnode_host_logic_cpu():
    out = subprocess.run([_binary(), "cpu"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 failed" in out.stdout


@pytest.mark.gpu
def test_dagnode_put_get_repair_gpu():
    out = subprocess.run([_binary(), "gpu"], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 failed" in out.stdout


def _sanitized(kind):
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp"), "sanitize"])
    return os.path.join(ROOT, "tests", "cpp", "build", f"test_dagnode_{kind}")


@pytest.mark.parametrize("kind,marker", [("tsan", "WARNING: ThreadSanitizer"), ("asan", "ERROR: AddressSanitizer")])
def test_host_mirror_under_sanitizers(kind, marker):
    """The whole Dag Node suite (quorum, datanode fan-out pool, read-repair queue and worker,
    GetMany / PutMany key concurrency, 12-thread concurrent Puts and degraded Gets through the
    group-commit queue) at 1/32 scale under ThreadSanitizer and AddressSanitizer + UBSan, on
    the test-only fake device layer (tests/cpp/fake_rsmi.cpp: the CPU oracle stands in for
    the GPU, so no device is needed).  Clean means: every check passes and the sanitizer
    reports nothing."""
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1")
    out = subprocess.run([_sanitized(kind), "sanitize"], capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, (out.stdout + out.stderr)[-4000:]
    assert "sanitize: " in out.stdout and " 0 failed" in out.stdout
    assert marker not in out.stderr and "runtime error" not in out.stderr
