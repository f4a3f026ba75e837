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


def test_parent_signal_terminates_ranks(tmp_path):
    """killing only the launching parent (SIGTERM to its pid) must
    not leave its rank processes running (they would keep their GPUs).  The
    ranks here are stand-ins that record their pid and sleep."""
    import signal
    import time
    sleeper = tmp_path / "rank.py"
    sleeper.write_text("import os, time\n"
                       f"open(os.path.join({str(tmp_path)!r}, 'pid%s' % os.environ['RANK']), 'w')"
                       ".write(str(os.getpid()))\n"
                       "time.sleep(300)\n")
    driver = tmp_path / "driver.py"
    driver.write_text("import sys\n"
                      f"sys.path.insert(0, {ROOT!r})\n"
                      "import bench\n"
                      f"bench.__file__ = {str(sleeper)!r}\n"
                      "sys.exit(bench.launch_ranks(2, 'gloo'))\n")
    p = subprocess.Popen([sys.executable, str(driver)], cwd=ROOT)
    pids = []
    for _ in range(600):
        pids = [tmp_path / f"pid{r}" for r in range(2)]
        if all(f.exists() and f.read_text() for f in pids):
            break
        time.sleep(0.1)
    pids = [int(f.read_text()) for f in pids]
    p.send_signal(signal.SIGTERM)
    assert p.wait(60) == 128 + signal.SIGTERM
    for pid in pids:  # both ranks are gone (reaped by the parent)
        with pytest.raises(ProcessLookupError):
            os.kill(pid, 0)
