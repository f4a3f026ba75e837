"""The multi-process HIP path under test: bench.py and the
config-5 stream driver launched by torchrun with 2 ranks that share the one
GPU of the box (gloo carries the barrier / max timing: ECCR_BENCH_BACKEND),
each rank running the HIP library on its own payload range.  The children are
fresh processes started before they make any GPU call; their round trips must
hold and they must exit 0.  The RCCL runs on one rank per GPU are the
driver's (SCALE_rNN), which this rehearses process for process."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(script_args, timeout=300):
    env = dict(os.environ)
    env["ECCR_BENCH_BACKEND"] = "gloo"
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + script_args
    r = subprocess.run(["timeout", "-k", "10", str(timeout)] + cmd, cwd=ROOT, env=env,
                       capture_output=True, text=True)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


def test_bench_two_ranks_share_gpu():
    r, line = _torchrun(["bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
                         "--batch", "48", "--payload", "100000", "--no-cpu-baseline",
                         "--e2e-batch", "8", "--e2e-per-size", "2", "--e2e-reps", "1"])
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert line is not None and line["roundtrip_ok"], line
    assert line["config"]["parallelism"] == "dp2" and "gloo" in line["rehearsal"]
    assert line["value"] > 0 and line["steps"] == 2
    # the host-resident block ran on both ranks (max-over-ranks time)
    e = line["e2e"]
    assert e["config2"]["roundtrip_ok"] and e["config5_mixed"]["roundtrip_ok"], e
    assert e["config2"]["batch_per_gpu"] == 8 and e["config5_mixed"]["payloads"] == 12, e


def test_bench_gpus_flag_launches_ranks():
    """The driver's command form without a launcher: `python3 bench.py --gpus 2`
    must start 2 rank processes itself, not measure one
    GPU and call it two.  gloo rehearsal (both ranks on the box's one GPU)."""
    env = dict(os.environ, ECCR_BENCH_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--batch", "48", "--payload", "100000", "--no-cpu-baseline", "--sweep", "none", "--no-e2e"]
    r = subprocess.run(["timeout", "-k", "10", "300"] + cmd, cwd=ROOT, env=env,
                       capture_output=True, text=True)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0's line only
    line = lines[0]
    assert line["config"]["parallelism"] == "dp2" and line["ranks"] == 2, line
    assert line["roundtrip_ok"] and "gloo" in line["rehearsal"], line
    assert line["value"] > 0 and line["steps"] == 2
    # one entry per rank, distinct ranks, each with its own
    # step time, and the max of them is the line's ms_per_step
    det = line["ranks_detail"]
    assert line["world_size"] == 2 and [d["rank"] for d in det] == [0, 1], det
    assert all(d["step_ms"] > 0 and d["device"] == 0 for d in det), det  # (both on the box's one GPU)
    assert max(d["step_ms"] for d in det) <= line["ms_per_step"] * 1.001, (det, line["ms_per_step"])


def test_bench_stream_two_ranks_share_gpu():
    r, line = _torchrun([os.path.join("scripts", "bench_stream.py"), "--per-size", "2", "--reps", "1"])
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert line is not None and line["roundtrip_ok"], line
    assert line["my_payloads"] >= 1 and "gloo" in line["rehearsal"]


def test_bench_e2e_block_one_rank():
    """the driver-run bench line carries the host-resident
    (PCIe-inclusive) rates, config 2 shape and the config-5 size mix, each next
    to the PCIe bound from this box's measured pinned copy rates."""
    cmd = [sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--batch", "32",
           "--payload", "1000000", "--no-cpu-baseline", "--sweep", "none",
           "--e2e-batch", "16", "--e2e-per-size", "2", "--e2e-reps", "1"]
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run(["timeout", "-k", "10", "300"] + cmd, cwd=ROOT, env=env,
                       capture_output=True, text=True)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    e = line["e2e"]
    p = e["pcie_measured"]
    assert min(p["h2d_GBps"], p["d2h_GBps"], p["duplex_GBps"]) > 1, p
    for leg in ("config2", "config5_mixed"):
        assert e[leg]["roundtrip_ok"], e[leg]
        assert e[leg]["roundtrip_GiBps"] > 0
        # the bound is a bound: no measured rate above it (5% timing slack)
        assert 0 < e[leg]["frac_of_pcie_bound"] <= 1.05, e[leg]
    assert e["config2"]["batch_per_gpu"] == 16 and e["config5_mixed"]["payloads"] == 12
