"""bench.py's rank-count contract on CPU (no GPU call is made on these paths):
under a launcher WORLD_SIZE must equal --gpus, and `--gpus N` without one
starts N rank processes and exits with the worst rank status."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env_over):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_over)
    return subprocess.run(["timeout", "-k", "10", "240", sys.executable, "bench.py"] + args,
                          cwd=ROOT, env=env, capture_output=True, text=True)


def test_world_size_mismatch_exits_nonzero():
    r = _run(["--gpus", "1"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2, (r.stdout, r.stderr[-2000:])
    err = json.loads(r.stderr.strip().splitlines()[-1])
    assert "WORLD_SIZE=2" in err["error"] and "--gpus 1" in err["error"]
    assert not r.stdout.strip()  # no measurement line


def test_gpus_beyond_visible_refused():
    r = _run(["--gpus", "64"], ECCR_BENCH_BACKEND="nccl")
    assert r.returncode == 2, (r.stdout, r.stderr[-2000:])
    assert "visible GPUs" in json.loads(r.stderr.strip().splitlines()[-1])["error"]


def test_launched_ranks_failure_propagates():
    """Without a GPU every launched rank fails at its first GPU call: the
    parent must have started the ranks (one traceback each) and exit non-zero
    (the worst rank status), never 0 with a measurement line."""
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is visible here: tests/test_multiproc_gpu.py covers the success path")
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--batch", "1", "--payload", "100",
              "--sweep", "none", "--no-cpu-baseline"], ECCR_BENCH_BACKEND="gloo")
    assert r.returncode != 0, (r.stdout, r.stderr[-2000:])
    assert r.stderr.count("Traceback") == 2, r.stderr[-3000:]
    assert not any(l.startswith("{") for l in r.stdout.splitlines())
