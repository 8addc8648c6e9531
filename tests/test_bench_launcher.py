"""bench.py's `--gpus N` contract: without a launcher it
runs N ranks under torch.distributed.run as a child process; under a launcher
WORLD_SIZE must equal --gpus.  CPU tests check the launcher command (run here
with a stand-in rank script under gloo) and the mismatch exit; the GPU test
runs the real bench as 2 gloo ranks sharing cuda:0 and reads n_gpus from the
one JSON line."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _env(**kw):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(kw)
    return env


def test_world_size_mismatch_exits_nonzero():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3"], cwd=ROOT,
                       env=_env(WORLD_SIZE="2"), capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
    assert not r.stdout.strip()  # no result line


def test_gpus_zero_rejected():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "0"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0


def test_launcher_command_runs_n_ranks(tmp_path):
    """The exact torch.distributed.run command bench.py starts, with the rank
    script swapped for a stand-in that joins a gloo group and reports."""
    cmd = bench.launcher_cmd(2, ["--gpus", "2", "--steps", "3"], bench._free_port())
    script = os.path.abspath(bench.__file__)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[cmd.index(script) + 1:] == ["--gpus", "2", "--steps", "3"]
    stand_in = tmp_path / "rank.py"
    stand_in.write_text(
        "import json, os, sys\n"
        "import torch.distributed as dist\n"
        "dist.init_process_group('gloo')\n"
        "print(json.dumps({'rank': dist.get_rank(), 'world': dist.get_world_size(), 'argv': sys.argv[1:]}), "
        "flush=True)\n"
        "dist.barrier(); dist.destroy_process_group()\n")
    cmd[cmd.index(script)] = str(stand_in)
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert sorted(l["rank"] for l in lines) == [0, 1]
    assert all(l["world"] == 2 and l["argv"] == ["--gpus", "2", "--steps", "3"] for l in lines)


@pytest.mark.gpu
def test_bench_gpus2_runs_two_ranks():
    """`python bench.py --gpus 2` with no launcher: two gloo ranks sharing
    cuda:0 (WGCS_DIST_BACKEND=gloo), one result line with n_gpus == 2."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "5",
                        "--warmup", "2", "--cpu-seconds", "0", "--no-e2e"], cwd=ROOT,
                       env=_env(WGCS_DIST_BACKEND="gloo"), capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert lines[0]["n_gpus"] == 2 and lines[0]["value"] > 0
    assert lines[0]["config"]["parallelism"] == "shard2 (no collective)"
