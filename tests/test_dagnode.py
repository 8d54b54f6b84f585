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
