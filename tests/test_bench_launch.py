"""bench.py --gpus N: the parent starts N ranks (torch.distributed.run, 127.0.0.1) before any GPU call and
each rank refuses a launcher whose world size differs from --gpus (the reference's
`devices=args.gpus`, asr_train_diffm.py:1762-1769).  CPU only: the launch command is captured, not run."""
import os
import subprocess
import sys
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _args(gpus):
    return types.SimpleNamespace(gpus=gpus)


def test_single_gpu_runs_in_process(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.launch_ranks(_args(1), ["--steps", "3"], run=lambda c: pytest.fail("must not spawn")) is None


def test_n_gpus_spawns_n_ranks(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("KDFM_DIST_BACKEND", "gloo")
    seen = []
    rc = bench.launch_ranks(_args(2), ["--gpus", "2", "--steps", "3"], run=lambda c: seen.append(c) or 7)
    assert rc == 7 and len(seen) == 1
    cmd = seen[0]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert cmd[-4:] == ["--gpus", "2", "--steps", "3"] and cmd[-5].endswith("bench.py")
    port = int(next(a for a in cmd if a.startswith("--master-port=")).split("=")[1])
    assert 0 < port < 65536


def test_rank_checks_launcher_world(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.launch_ranks(_args(2), []) is None
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.launch_ranks(_args(4), [])


def test_world_mismatch_exits_nonzero_before_gpu():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_gpu_count_from_environment_and_kfd(tmp_path):
    assert bench.visible_gpu_count({"HIP_VISIBLE_DEVICES": "0,3,5"}, str(tmp_path)) == 3
    assert bench.visible_gpu_count({"ROCR_VISIBLE_DEVICES": ""}, str(tmp_path)) == 0
    for i, simds in enumerate((0, 1024, 1024)):   # node 0: the CPU
        os.makedirs(tmp_path / str(i))
        (tmp_path / str(i) / "properties").write_text(f"cpu_cores_count 64\nsimd_count {simds}\narray_count 32\n")
    assert bench.visible_gpu_count({}, str(tmp_path)) == 2
    assert bench.visible_gpu_count({}, str(tmp_path / "missing")) is None


def test_launcher_parent_never_touches_torch_cuda(monkeypatch):
    """The N-rank parent counts GPUs without torch.cuda (device_count / is_available / init would load HIP in
    a process that then forks the ranks): every torch.cuda entry point raises here, and torch.cuda stays
    uninitialised across the launch."""
    import torch
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("KDFM_DIST_BACKEND", raising=False)   # the nccl path, which checks the GPU count
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3")

    def boom(*a, **k):
        raise AssertionError("the launcher parent called torch.cuda")
    for name in ("device_count", "is_available", "init", "current_device", "set_device", "synchronize"):
        monkeypatch.setattr(torch.cuda, name, boom)
    seen = []
    assert bench.launch_ranks(_args(4), ["--gpus", "4"], run=lambda c: seen.append(c) or 0) == 0
    assert len(seen) == 1 and not torch.cuda.is_initialized()
    with pytest.raises(SystemExit, match="needs 8 visible GPUs, found 4"):
        bench.launch_ranks(_args(8), ["--gpus", "8"], run=lambda c: pytest.fail("must not spawn"))
