"""bench.py's multi-GPU launch: `python bench.py --gpus N` starts N rank processes itself when no
torch.distributed env is set (bench.spawn_ranks), so the driver's own command measures N GPUs.

CPU: --launch-check runs the launch alone (gloo, no GPU) at world 2 and 3.
GPU: the real bench at world 2 on the one-GPU box (SYMHIP_BENCH_ONE_GPU=1: both ranks on device 0,
gloo for the barrier and the max), small batch, every side leg off; the line must say n_gpus 2 and
carry the aggregate and per-GPU rates and the roofline.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # exactly one JSON line, from rank 0
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_launch_check_spawns_n_ranks(n):
    line = _run(["--gpus", str(n), "--launch-check"])
    assert line["n_gpus"] == n and line["gpus_requested"] == n
    assert line["config"] == 4  # BASELINE config 4 (a 2^23-record shard per GPU) is the N >= 2 default
    ranks = sorted(tuple(r) for r in line["ranks"])
    assert [r[0] for r in ranks] == list(range(n))  # every rank joined
    assert [r[1] for r in ranks] == list(range(n))  # LOCAL_RANK = GPU index
    assert len({r[2] for r in ranks}) == n  # one process each


def test_launch_check_world1_no_spawn():
    line = _run(["--launch-check"])
    assert line["n_gpus"] == 1 and line["ranks"] == [0]
    assert line["config"] == 2  # the 1-GPU headline: BASELINE config 2's 2^20 SetRequests


def test_launch_check_explicit_config_kept():
    line = _run(["--gpus", "2", "--config", "2", "--launch-check"])
    assert line["n_gpus"] == 2 and line["config"] == 2


def test_failed_rank_ends_the_launch():
    # an unknown config makes argparse exit 2 in every rank: the parent must return non-zero, not hang
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "9"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0


@pytest.mark.gpu
def test_bench_world2_one_gpu():
    off = ["--cpu-seconds", "1", "--host-steps", "0", "--packetize-reps", "0", "--proxy-reps", "0",
           "--reassembly-reps", "0", "--crypto-reps", "0", "--flat-reps", "0", "--boutique-reps", "0",
           "--payload-reps", "0", "--mixed-reps", "0", "--config3-reps", "0", "--trace-reps", "0",
           "--per-record", "0", "--ref-reps", "0"]
    line = _run(["--gpus", "2", "--steps", "4", "--warmup", "1", "--records", "65536", "--prewarm-ms", "0", *off],
                env_extra={"SYMHIP_BENCH_ONE_GPU": "1"}, timeout=300)
    assert line["n_gpus"] == 2
    assert line["config"]["global_records"] == 2 * 65536
    assert line["value"] > 0 and line["per_gpu_gbps"] > 0
    assert 0 < line["roofline"]["frac"] < 1
    assert line["config"]["global"]["global_records"] == 2 * 65536
    assert line["config"]["workload"].startswith("config4")  # the N >= 2 default
    assert line["cpu_baseline"]["value"] > 0  # rank 0 carries the CPU baseline at N > 1 too
    assert line["summary"]["headline"]["n_gpus"] == 2 and "cpu_baseline" in line["summary"]
