"""The completion-flag release covers every wave's stores (launch_done, rs_kernels.hip).

Compiles the table-of-bases kernels to gfx950 assembly and runs tools/check_flag_fence.py: every
workgroup barrier that precedes the system-scope flag atomic must be reached with no vector store
outstanding (an `s_waitcnt vmcnt(0)` after the wave's last store).  CPU only: hipcc cross-compiles.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_flag_release_waits_for_every_wave(tmp_path):
    asm = tmp_path / "tb.s"
    src = os.path.join(ROOT, "filedag-storage_amd", "csrc", "rs_kernels_tb.hip")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--cuda-device-only",
                    "-S", src, "-o", str(asm)], check=True, capture_output=True, timeout=600)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_flag_fence.py"), str(asm)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 unfenced" in r.stdout
