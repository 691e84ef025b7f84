"""Tests of bench.py's rank launcher: on CPU with --launch-probe (every rank reports what it was given
and exits before any device call), and one end-to-end two-rank run on the GPU.

`python bench.py --gpus N` without a torch.distributed.run environment must start N ranks itself
(one process per GPU, LOCAL_RANK = device), pass every argument through, and return the ranks'
exit status; a world size that differs from --gpus is an error, not a silent 1-rank run.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, env=e, capture_output=True, text=True, timeout=timeout)


def probes(stdout):
    return sorted((json.loads(l) for l in stdout.splitlines() if l.startswith("{")), key=lambda d: d["rank"])


def test_launches_n_ranks_and_passes_arguments():
    args = ["--gpus", "2", "--workload", "heat2d", "--side", "64", "--steps", "2", "--launch-probe", "0"]
    p = run(args)
    assert p.returncode == 0, p.stderr[-2000:]
    got = probes(p.stdout)
    assert [d["rank"] for d in got] == [0, 1]
    assert all(d["world"] == 2 for d in got)
    assert sorted(d["local"] for d in got) == [0, 1]  # one device per rank
    assert all(d["argv"] == args for d in got)


def test_propagates_the_ranks_exit_status():
    p = run(["--gpus", "2", "--launch-probe", "3"])
    assert p.returncode != 0  # the last rank exits 3: the launcher (and bench.py) fail


def test_one_gpu_runs_in_process():
    p = run(["--gpus", "1", "--launch-probe", "0"])
    assert p.returncode == 0, p.stderr[-2000:]
    got = probes(p.stdout)
    assert len(got) == 1 and got[0]["world"] == 1


def test_world_size_mismatch_is_an_error():
    p = run(["--gpus", "2", "--launch-probe", "0"], env={"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2
    assert "--gpus 2" in p.stderr


@pytest.mark.gpu
def test_two_rank_bench_runs_end_to_end():
    """`bench.py --gpus 2` from one command, on the GPU: two ranks (one GPU each when the box has two,
    else sharing the one GPU over the IPC mailbox with a small slab), the whole distributed path
    (slab ghost rows, reductions across ranks), one JSON line with n_gpus 2."""
    import _nkpath  # noqa: F401
    import ariadne_hip as ah

    args = ["--gpus", "2", "--side", "512", "--steps", "1", "--warmup", "1", "--no-prof", "--no-cpu-baseline"]
    if ah.device_count() < 2:
        args += ["--transport", "mailbox"]
    p = run(args, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(line) == 1
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["matvecs_per_step"] == 309
    assert d["config"]["reductions"] in ("peer mailbox (IPC/xGMI)", "ncclAllReduce")
