"""`bench.py --gpus N` starts its N ranks itself (bench.py: launch_ranks) when
no launcher set WORLD_SIZE: child processes with RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* set, rendezvous on 127.0.0.1, the first failing rank
ends the others and gives the job its exit code.  The rank bodies here are the
hidden `--launch-probe` mode (a gloo all-reduce, no device), so the launcher
is checked on CPU; the GPU test checks that more ranks than visible GPUs is
refused promptly before any rank starts."""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _bench(args, timeout=120, env=None):
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=e)


@pytest.mark.parametrize("n", [1, 2, 3])
def test_launcher_starts_n_ranks(n):
    r = _bench(["--gpus", str(n), "--launch-probe"])
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == n
    assert line["rank_sum"] == n * (n + 1) // 2  # every rank joined the all-reduce
    assert line["master"] == "127.0.0.1"


def test_launcher_failing_rank_ends_the_job():
    """Rank 1 exits 7 while ranks 0 and 2 would sleep for minutes: the job
    must end with 7 within the launcher's grace period, not wait for them."""
    t0 = time.monotonic()
    r = _bench(["--gpus", "3", "--launch-probe", "--launch-probe-fail", "1"], timeout=90)
    assert r.returncode == 7, (r.returncode, r.stderr)
    assert time.monotonic() - t0 < 60
    assert "rank 1 of 3 exited with 7" in r.stderr


def test_gpus_mismatch_with_launcher_refused():
    r = _bench(["--gpus", "2", "--launch-probe"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "--gpus 2" in r.stderr


def test_gpus_zero_refused():
    r = _bench(["--gpus", "0"])
    assert r.returncode == 2


def _visible_devices():
    import torch

    return torch.cuda.device_count()


def test_more_ranks_than_devices_refused_on_cpu():
    n = max(2, _visible_devices() + 1)
    t0 = time.monotonic()
    r = _bench(["--gpus", str(n), "--no-cpu"], timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "visible GPUs" in r.stderr
    assert time.monotonic() - t0 < 100


@pytest.mark.gpu
def test_bench_gpus_more_than_visible_fails_fast():
    """on a 1-GPU box `bench.py --gpus 2` exits non-zero
    within a bound (no rank is started, no device is initialised)."""
    n = max(2, _visible_devices() + 1)
    t0 = time.monotonic()
    r = _bench(["--gpus", str(n), "--no-cpu", "--steps", "1", "--warmup", "0"], timeout=120)
    assert r.returncode != 0
    assert "visible GPUs" in r.stderr
    assert time.monotonic() - t0 < 100


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 4])
def test_bench_ranks_rehearsal_on_one_gpu(n):
    """The N-rank bench path end to end on the one-GPU box: `bench.py --gpus 2`
    with RTX_BENCH_REHEARSAL=1 starts two ranks on device 0 (gloo instead of
    RCCL, which cannot hold two ranks on one device), each renders its tile
    shard, rank 0 gathers them and prints one line with n_gpus 2 and the
    slowest rank's time; the line says it is a rehearsal."""
    t0 = time.monotonic()
    r = _bench(["--gpus", str(n), "--no-cpu", "--steps", "2", "--warmup", "1"], timeout=240,
               env={"RTX_BENCH_REHEARSAL": "1"})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == n and line["steps"] == 2
    assert line["frame_check"]["bad_frames"] == 0
    assert line["gather_check"]["rgb8_mismatch_pixels"] == 0
    assert line["value"] > 0 and line["ms_per_step"] > 0
    assert "REHEARSAL" in line["config"]["parallelism"]
    assert time.monotonic() - t0 < 240
