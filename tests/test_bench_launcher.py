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
    # each rank reports into its own file: two ranks printing to one stdout may interleave
    stand_in.write_text(
        "import json, os, sys\n"
        "import torch.distributed as dist\n"
        "dist.init_process_group('gloo')\n"
        f"open(os.path.join({str(tmp_path)!r}, 'rank%d.json' % dist.get_rank()), 'w').write(json.dumps("
        "{'rank': dist.get_rank(), 'world': dist.get_world_size(), 'argv': sys.argv[1:]}))\n"
        "dist.barrier(); dist.destroy_process_group()\n")
    cmd[cmd.index(script)] = str(stand_in)
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads((tmp_path / f"rank{k}.json").read_text()) for k in range(2)]
    assert sorted(l["rank"] for l in lines) == [0, 1]
    assert all(l["world"] == 2 and l["argv"] == ["--gpus", "2", "--steps", "3"] for l in lines)


def _line(n, with_strong=True, with_cpu=True):
    """A cfg2 line shaped as bench.main assembles it (roofline from
    bench.roofline with every rank's kernel time)."""
    ks = [0.0150 + 0.0001 * r for r in range(n)]
    line = {k: 1 for k in bench.REQUIRED_KEYS}
    line.update(n_gpus=n, value=5500.0 * n, scaling="weak",
                config={"workload": "cfg2", "dist": {"backend": "nccl", "world_size": n}} if n > 1 else {"workload": "cfg2"},
                roofline=bench.roofline("checksum_batch_kernel<VALIDATE,32,4,nt>", 98304000, 1500, 65536, ks[0], 2,
                                        0.0176, ks))
    if with_cpu:
        line["cpu_baseline"] = {"value": 8.8, "unit": "GiB/s", "cores": 1, "kind": "port", "sample": "s"}
    if with_strong:
        per = [1048576 * (r + 1) // n - 1048576 * r // n for r in range(n)]
        line["cfg5_strong"] = {"value": 5000.0 * n, "value_cold": 5000.0 * n, "value_warm": 5400.0 * n,
                               "warm": bench.warm_block(40.0, 176, 0.0045, 0.21, 20),
                               "n_gpus": n, "scaling": "strong", "packets_per_rank": per,
                               "roofline": bench.roofline("k", per[0] * 1500, 1500, per[0], 0.27 / n, 1, None,
                                                          [0.27 / n] * n)}
    return line


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_line_schema_complete(n):
    """bench.line_problems accepts a complete line at every N: cpu_baseline on
    rank 0 at every N, every rank's kernel time, the world size and the
    configs[4] strong-scaling block."""
    line = _line(n)
    assert bench.line_problems(line) == []
    if n > 1:
        assert line["roofline"]["kernel_ms_max"] >= line["roofline"]["kernel_ms_min"]
        assert len(line["roofline"]["kernel_ms_per_rank"]) == n


@pytest.mark.parametrize("n", [1, 4])
def test_line_schema_flags_gaps(n):
    assert "missing cfg5_strong" in bench.line_problems(_line(n, with_strong=False))
    # the configs[4] block's `value` is the cold region (K
    # steps behind exactly W warmups), carried again as value_cold; a warm
    # re-time only beside it
    line = _line(n)
    line["cfg5_strong"]["value"] = line["cfg5_strong"]["value_warm"]
    assert any("value_cold" in p for p in bench.line_problems(line))
    line = _line(n)
    del line["cfg5_strong"]["value_cold"]
    assert any("value_cold" in p for p in bench.line_problems(line))
    assert bench.line_problems(line, require_cold=False) == []
    assert "cpu_baseline missing or incomplete" in bench.line_problems(_line(n, with_cpu=False))
    if n > 1:
        line = _line(n)
        line["roofline"]["kernel_ms_per_rank"] = line["roofline"]["kernel_ms_per_rank"][:1]
        assert bench.line_problems(line) == ["roofline.kernel_ms_per_rank must list every rank"]
        line = _line(n)
        line["config"]["dist"]["world_size"] = 1
        assert bench.line_problems(line) == ["config.dist.world_size must equal n_gpus"]


def test_recorded_rehearsal_lines_complete():
    """The N > 1 lines recorded on the GPU box (gloo ranks sharing one GPU,
    profiles/r4_rehearse_gpus*.jsonl) are complete by the same check."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[4-9]_rehearse_gpus*_gloo.jsonl")))
    if not files:
        pytest.skip("no rehearsal lines recorded yet")
    for fn in files:
        pre6 = os.path.basename(fn)[:2] in ("r4", "r5")  # recorded before value_cold existed
        with open(fn) as f:
            for l in f:
                if l.startswith("{"):
                    line = json.loads(l)
                    assert line["n_gpus"] > 1
                    assert bench.line_problems(line, require_cold=not pre6) == [], fn


@pytest.mark.parametrize("rnd", ["r5", "r6"])
def test_recorded_eight_rank_rehearsal(rnd):
    """the driver's 8-GPU run is one-shot, so the 8-rank
    line was rehearsed once on the 1-GPU box (`WGCS_DIST_BACKEND=gloo python
    bench.py --gpus 8 --steps 20 --warmup 5`, 8 gloo ranks time-sharing
    cuda:0, profiles/r5_rehearse_gpus8_gloo.jsonl; again with round 6's
    bench, cfg5_strong.value_cold included): one complete
    line, every rank's kernel time, the 1M batch split over all 8, and rank
    0's CPU baseline inside the run the other 7 ranks waited for at the
    barrier."""
    fn = os.path.join(ROOT, "profiles", f"{rnd}_rehearse_gpus8_gloo.jsonl")
    if not os.path.exists(fn):
        pytest.skip("8-rank rehearsal not recorded yet")
    lines = [json.loads(l) for l in open(fn) if l.startswith("{")]
    assert len(lines) == 1
    line = lines[0]
    assert bench.line_problems(line, require_cold=rnd != "r5") == []
    if rnd != "r5":
        assert line["cfg5_strong"]["value_cold"] == line["cfg5_strong"]["value"]
    assert line["n_gpus"] == 8 and line["config"]["dist"]["world_size"] == 8
    assert len(line["roofline"]["kernel_ms_per_rank"]) == 8
    assert len(line["cfg5_strong"]["packets_per_rank"]) == 8
    assert line["cpu_baseline"]["value"] > 0


def test_recorded_final_driver_lines_agree_with_rocprof():
    """The round-5 close-out (scripts/r5_final3.sh): the driver's command,
    recorded twice on the final tree, gives complete lines, and their
    one-stream kernel time agrees with the committed rocprofv3 one-stream
    average at the same step count (profiles/r5_final3_cfg2_1s_20*_kernel_stats.csv)
    within 5 %."""
    import csv

    fn = os.path.join(ROOT, "profiles", "r5_final3_lines.jsonl")
    if not os.path.exists(fn):
        pytest.skip("final lines not recorded yet")
    lines = [json.loads(l) for l in open(fn) if l.startswith("{")]
    drv = [l for l in lines if l["tag"].startswith("cfg2_driver")]
    assert len(drv) == 2
    prof_us = []
    for tag in ("20a", "20b"):
        with open(os.path.join(ROOT, "profiles", f"r5_final3_cfg2_1s_{tag}_kernel_stats.csv")) as f:
            rows = [r for r in csv.DictReader(f) if "checksum_batch_kernel" in r["Name"]]
        assert len(rows) == 1 and int(rows[0]["Calls"]) == 45  # 20 + 5 launches, one stream
        prof_us.append(float(rows[0]["AverageNs"]) / 1e3)
    for line in drv:
        line = {k: v for k, v in line.items() if k != "tag"}
        assert bench.line_problems(line, require_cold=False) == []
        r = line["roofline"]
        assert r["traffic"] is not None and line["cpu_baseline"]["value"] > 0
        one_us = r["kernel_ms_one_stream"] * 1e3
        assert all(abs(one_us - p) / p < 0.05 for p in prof_us), (one_us, prof_us)


def test_numa_helpers(tmp_path):
    from wireguard_amd import shard

    assert shard.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert shard.parse_cpulist("") == set()

    class P:
        pci_domain_id, pci_bus_id, pci_device_id = 0, 0x75, 0

    d = tmp_path / "0000:75:00.0"
    d.mkdir()
    (d / "local_cpulist").write_text("0-7\n")
    cpus, where = shard.gpu_local_cpus(P, sysfs=str(tmp_path))
    assert cpus == set(range(8)) and where == "0000:75:00.0"
    assert shard.gpu_local_cpus(object())[0] is None


def test_gather_floats_gloo():
    """Every rank's kernel time reaches rank 0 (the N > 1 line's
    kernel_ms_per_rank), over gloo world 2 on the CPU."""
    import torch.multiprocessing as mp

    port = bench._free_port()
    mp.spawn(_gather_worker, args=(2, port), nprocs=2, join=True)


def _gather_worker(rank, world, port):
    import torch.distributed as dist

    from wireguard_amd import shard

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        got = shard.gather_floats(0.5 + rank, dist)
        assert got == [0.5, 1.5], got
        assert shard.max_over_ranks(0.5 + rank, dist) == 1.5
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2])
def test_bench_gpus_n_runs_n_ranks(n):
    """`python bench.py --gpus N` with no launcher: N gloo ranks sharing
    cuda:0 (WGCS_DIST_BACKEND=gloo), one complete result line (cfg5_strong,
    cpu_baseline, every rank's kernel time)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "5",
                        "--warmup", "2", "--cpu-seconds", "0.5", "--no-e2e"], cwd=ROOT,
                       env=_env(WGCS_DIST_BACKEND="gloo"), capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert lines[0]["n_gpus"] == n and lines[0]["value"] > 0
    assert lines[0]["config"]["parallelism"] == f"shard{n} (no collective)"
    assert bench.line_problems(lines[0]) == []


@pytest.mark.gpu
def test_bench_default_line_complete():
    """The driver's invocation shape at N = 1 (cfg2, doorbell-gated steps, the
    configs[4] strong block, the CPU baseline): one JSON line that
    bench.line_problems accepts, with the kernel no slower than the wall clock
    allows."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "5",
                        "--warmup", "2", "--cpu-seconds", "0.5", "--no-e2e"], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert bench.line_problems(line) == []
    assert "doorbell" in line["timing"]["enqueue"]
    assert line["roofline"]["kernel_ms"] <= line["ms_per_step"] * 1.05
    st = line["cfg5_strong"]
    assert st["packets_per_rank"] == [1048576] and st["roofline"]["frac"] > 0


def test_gate_streams_helper():
    """bench.gate_streams (the timed region's doorbell set-up): with bracket
    events only stream 0 waits on the bell (the others wait on e0 behind it);
    without events every launch stream waits on it itself."""
    class Dev:
        def __init__(self):
            self.calls = []

        def stream_wait_flag(self, s, bell, value):
            self.calls.append((s, value))

    for use_events, want in ((True, ["s0"]), (False, ["s0", "s1", "s2"])):
        d = Dev()
        got = bench.gate_streams(d, object(), ["s0", "s1", "s2"], use_events)
        assert got == want and [c[0] for c in d.calls] == want and all(c[1] == 1 for c in d.calls)
