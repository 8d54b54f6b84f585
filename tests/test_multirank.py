"""world_size-2 gloo rehearsal of the multi-GPU path on CPU.

bench.py runs one process per GPU with no data-path collective: each rank codes its own
blocks and only the timing barrier / max-over-ranks reduction crosses ranks.  Here two
CPU ranks take their block ranges (rsmi.multi.partition_blocks), code them with the
oracle as a stand-in for their GPU (test-only), and rank 0 checks that the union is
byte-identical to one process coding the whole batch, and that bench.max_over_ranks
reduces the way the bench reports it."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    sys.path.insert(0, HERE)
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench
    import oracle_lib as orc
    from rsmi import multi

    w, r, _ = bench.dist_setup()
    assert (w, r) == (world, rank)
    k, m, S, nb = 4, 2, 1000, 13
    data = orc.splitmix64_bytes(0xF11EDA6, nb * k * S).reshape(nb, k, S)
    start, count = multi.partition_blocks(nb, world, rank)
    par = orc.encode_fast(k, m, np.ascontiguousarray(data[start:start + count]), threads=1)
    gathered = [None] * world
    dist.all_gather_object(gathered, (start, count, par))
    bench.barrier(world)
    el = bench.max_over_ranks(0.5 + rank, world)
    if rank == 0:
        full = np.concatenate([g[2] for g in sorted(gathered, key=lambda g: g[0])], axis=0)
        ref = orc.encode_fast(k, m, data, threads=1)
        np.save(os.path.join(out_dir, "ok.npy"), np.array([np.array_equal(full, ref), el == 0.5 + world - 1,
                                                          sum(g[1] for g in gathered) == nb]))
    dist.destroy_process_group()


def test_two_rank_gloo_partition_and_timing(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    ok = np.load(os.path.join(tmp_path, "ok.npy"))
    assert ok.all(), ok


@pytest.mark.parametrize("n", [2, 8])
def test_bench_spawns_ranks_itself_mock(n):
    """`bench.py --gpus N` with no launcher starts its N ranks itself (before any GPU call) and
    rank 0 prints one line with n_gpus N -- N = 8 is the driver's scaling run's shape.  --mock
    swaps the device step for a CPU stand-in so the launcher, gloo, the reductions and the JSON
    line run here without a GPU."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--mock", "--steps", "3"],
                         capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), out.stdout  # stdout holds the JSON line only
    j = json.loads(lines[0])
    assert j["n_gpus"] == n and j["mock"] and j["steps"] == 3
    assert sorted(r["rank"] for r in j["config"]["ranks"]) == list(range(n))
    assert sum(r["blocks"] for r in j["config"]["ranks"]) == 8 * n
    assert j["cpu_baseline"] is None  # timed at N = 1 only


def test_bench_rejects_world_size_mismatch():
    import subprocess

    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--mock"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr


def test_bench_device_generator_matches_oracle():
    """bench.py's torch splitmix64 (int64 arithmetic, logical shifts by masking) is
    byte-identical to the oracle's numpy generator for several blocks."""
    sys.path.insert(0, ROOT)
    import bench
    import oracle_lib as orc

    got = bench.splitmix_blocks([0, 1, 4095, 77777], 1000, "cpu").numpy()
    for j, b in enumerate([0, 1, 4095, 77777]):
        assert np.array_equal(got[j], orc.splitmix64_bytes(bench.SEED ^ b, 1000))


@pytest.mark.gpu
def test_bench_gpus2_share_device_no_launcher():
    """The exact command the N>1 path needs: `bench.py --gpus 2` with no launcher, both ranks
    on cuda:0 (--share-device; the 8-GPU run belongs to the driver).  Each rank codes and
    verifies its own share of the job's blocks."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "5", "--warmup", "1",
           "--blocks", "256", "--settle-ms", "0", "--sustained-steps", "0", "--share-device"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), out.stdout  # stdout holds the JSON line only
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["verify"]["verified"] and j["verify"]["ranks_verified"] == 2
    payload = 2 * 256 * 262144 * 5
    assert abs(j["value"] - payload / (j["ms_per_step"] * 5e-3) / 2**30) / j["value"] < 0.01


@pytest.mark.gpu
def test_bench_two_ranks_torchrun_on_one_gpu():
    """The N>1 bench path on real hardware: `torch.distributed.run` with 2 ranks sharing
    cuda:0 (--share-device; the 8-GPU run belongs to the driver).  Each rank codes its own
    blocks, rank 0 prints one JSON line whose value counts both ranks' payload."""
    import json
    import subprocess

    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "5", "--warmup", "1", "--blocks", "256", "--settle-ms", "0",
           "--sustained-steps", "0", "--share-device", "--cpu-seconds", "1"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), out.stdout  # stdout holds the JSON line only
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["steps"] == 5 and j["scaling"] == "weak"
    payload = 2 * 256 * 262144 * 5
    assert abs(j["value"] - payload / (j["ms_per_step"] * 5e-3) / 2**30) / j["value"] < 0.01
    assert j["cpu_baseline"] is None  # timed at N = 1 only


@pytest.mark.gpu
def test_bench_gpus_guard_refuses_missing_devices():
    """`bench.py --gpus N` with no launcher and no --share-device on a box with fewer than N
    GPUs exits non-zero before it starts any rank (torch.cuda.device_count() does not
    initialise the GPU): the message names the visible count, stdout stays empty."""
    import subprocess

    have = torch.cuda.device_count()
    if have < 1:
        pytest.skip("needs a GPU box")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(have + 1), "--steps", "1"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert out.returncode != 0
    assert f"only {have} GPU(s) visible" in out.stderr, out.stderr[-2000:]
    assert out.stdout.strip() == ""  # no rank ran, so no JSON line
    assert "RANK" not in out.stderr and "Traceback" not in out.stderr  # refused in the launcher itself


def _kfd_tree(root, gfx):
    """A fake sysfs with KFD topology nodes whose gfx_target_version values are `gfx`."""
    for i, v in enumerate(gfx):
        d = root / "class" / "kfd" / "kfd" / "topology" / "nodes" / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count {0 if v else 64}\nsimd_count {0 if not v else 1024}\n"
                                      f"gfx_target_version {v}\nmax_waves_per_simd 8\n")


def test_visible_gpu_count_from_injected_sysfs(tmp_path):
    """rsmi.multi.visible_gpu_count counts GPUs from the KFD topology (CPU nodes carry
    gfx_target_version 0) and applies ROCR_VISIBLE_DEVICES, then HIP/CUDA_VISIBLE_DEVICES,
    the way the runtime would, without loading it (verdict r3 item 2)."""
    sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
    from rsmi import multi

    assert multi.visible_gpu_count(str(tmp_path / "none"), env={}) is None
    _kfd_tree(tmp_path, [0, 0] + [90500] * 8)  # two CPU sockets, eight gfx950
    root = str(tmp_path)
    assert multi.sysfs_gpu_count(root) == 8
    assert multi.visible_gpu_count(root, env={}) == 8
    assert multi.visible_gpu_count(root, env={"HIP_VISIBLE_DEVICES": "0,1,2,3"}) == 4
    assert multi.visible_gpu_count(root, env={"CUDA_VISIBLE_DEVICES": "5"}) == 1
    assert multi.visible_gpu_count(root, env={"HIP_VISIBLE_DEVICES": ""}) == 0
    assert multi.visible_gpu_count(root, env={"HIP_VISIBLE_DEVICES": "0,9,1"}) == 1  # stops at the bad index
    assert multi.visible_gpu_count(root, env={"ROCR_VISIBLE_DEVICES": "2,3", "HIP_VISIBLE_DEVICES": "0,1,2"}) == 2
    assert multi.visible_gpu_count(root, env={"ROCR_VISIBLE_DEVICES": "GPU-1a2b,GPU-3c4d,7"}) == 3
    assert multi.visible_gpu_count(root, env={"HIP_VISIBLE_DEVICES": "0", "CUDA_VISIBLE_DEVICES": "0,1"}) == 1


def _probe_run(args, tmp_path, env_extra=None, timeout=600):
    import json
    import subprocess

    probe = tmp_path / "probe.json"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(RSMI_BENCH_LAUNCH_PROBE=str(probe), **(env_extra or {}))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                         timeout=timeout, env=env, cwd=ROOT)
    return out, json.loads(probe.read_text())


def test_launcher_maps_no_hip_before_spawn_mock(tmp_path):
    """The launcher of `bench.py --gpus N` has neither torch nor the HIP/HSA runtime libraries
    mapped, and no /dev/kfd descriptor, when it spawns its ranks (checked from /proc/self at
    that moment through the RSMI_BENCH_LAUNCH_PROBE hook); --mock runs the ranks on the CPU."""
    out, p = _probe_run(["--gpus", "2", "--mock", "--steps", "2", "--cpu-seconds", "0"], tmp_path)
    assert out.returncode == 0, out.stderr[-3000:]
    assert p["hip_libs_mapped"] == [] and p["kfd_fds"] == 0, p
    assert not p["torch_imported"] and not p["numpy_imported"], p


@pytest.mark.gpu
def test_launcher_counts_and_spawns_gpu_free(tmp_path):
    """On a GPU box: the launcher's sysfs count equals what the HIP runtime reports in a
    process that has initialised it (this one), and the spawn path -- `bench.py --gpus 2
    --share-device`, counted and spawned by the launcher -- runs with no HIP/HSA library mapped
    and no /dev/kfd open in the launcher at spawn time; both ranks then code and verify on
    cuda:0.  The driver's `--gpus 8` scaling run takes the same path with 8 devices counted."""
    import json

    sys.path.insert(0, os.path.join(ROOT, "filedag-storage_amd"))
    from rsmi import multi

    have = torch.cuda.device_count()
    assert have >= 1
    assert multi.visible_gpu_count() == have
    out, p = _probe_run(["--gpus", "2", "--share-device", "--steps", "3", "--warmup", "1", "--blocks", "128",
                         "--settle-ms", "0", "--sustained-steps", "0", "--cpu-seconds", "0"], tmp_path, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    assert p["gpus_counted"] == have and p["hip_libs_mapped"] == [] and p["kfd_fds"] == 0, p
    assert not p["torch_imported"], p
    j = json.loads([l for l in out.stdout.splitlines() if l.strip()][0])
    assert j["n_gpus"] == 2 and j["verify"]["ranks_verified"] == 2
