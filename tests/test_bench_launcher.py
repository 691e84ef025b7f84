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


def _bench_module():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _path(rank, halo_us, red_us, waits=(160, 1240), launches=10):
    return {"rank": rank, "nranks": 8, "mailbox": 1, "halo_in_launch": 1, "mailbox_error": 0,
            "jv_halo_fused": launches, "jv_halo_separate": 0, "halo_waits": waits[0], "reduce_waits": waits[1],
            "halo_wait_us": halo_us, "reduce_wait_us": red_us, "launches": {"mgs_sweep": 300}}


def test_exchange_cost_from_the_wait_counters():
    """exchange_cost: deltas of the device's peer-wait clocks over the timed region -- launches x mean
    end-tile wait + block 0's reduction waits, as a share of the elapsed time."""
    b = _bench_module()
    p0 = _path(0, 100.0, 50.0, waits=(16, 10), launches=1)
    p1 = _path(0, 100.0 + 16 * 309 * 2.0, 50.0 + 4650 * 3.0, waits=(16 + 16 * 309, 10 + 4650), launches=1 + 309)
    e = b.exchange_cost(p0, p1, steps=1, elapsed=0.25)
    assert e["halo_waits"] == 16 * 309 and e["halo_launches"] == 309 and e["halo_wait_us_mean"] == 2.0
    assert e["reduce_waits"] == 4650 and e["reduce_wait_us_mean"] == 3.0
    assert e["exchange_us_per_step"] == round(309 * 2.0 + 4650 * 3.0, 1)
    assert e["exchange_share"] == round((309 * 2.0 + 4650 * 3.0) * 1e-6 / 0.25, 4)
    z = b.exchange_cost(p0, p0, steps=3, elapsed=1.0)  # one rank / no mailbox: no waits, no share
    assert z["exchange_us_per_step"] == 0.0 and z["exchange_share"] == 0.0


def test_eight_rank_json_assembly():
    """The N = 8 line's multi-GPU fields, assembled on CPU from eight synthetic rank reports: the per-DoF
    rate against config 2's single-GPU line, every rank's exchange cost, the worst rank's share."""
    b = _bench_module()
    paths = []
    for r in range(8):
        q = _path(r, 0.0, 0.0)
        q["exchange"] = b.exchange_cost(_path(r, 0.0, 0.0, (0, 0), 0), _path(r, 16 * 309 * (1.0 + r), 4650 * 2.0,
                                                                            (16 * 309, 4650), 309), 1, 0.3)
        paths.append(q)
    ref = {"value": 1264.664 * 4096 ** 2, "source": "BENCH_r04.json"}
    out = b.scaling_fields(8 * 1000.0, 4096 * 4096, paths, "bratu2d", 0, 8, 0, ref=ref)
    assert out["dof_rate"]["vs_config2_single_gpu"] == round(8000.0 / 1264.664, 3)
    assert out["dof_rate"]["exchange"] == "included"
    assert [q["rank"] for q in out["ranks"]] == list(range(8))
    assert out["exchange"]["max_halo_wait_us_mean"] == 8.0
    assert out["exchange"]["max_share"] == max(q["exchange"]["exchange_share"] for q in paths)
    json.dumps(out)  # serialisable as the bench line
    # config 4 (strong scaling, --global-n 16384): value counts global matvecs of the 16384^2 grid
    g = b.scaling_fields(451.6, 16384 ** 2, [], "bratu2d", 8, 1, 16384, ref=ref)
    assert g["dof_rate"]["vs_config2_single_gpu"] == round(451.6 * 16 / 1264.664, 3)  # the 5.71x ceiling
    assert g["dof_rate"]["exchange"].startswith("none") and "ranks" not in g


def test_config2_reference_reads_the_driver_record(tmp_path, monkeypatch):
    b = _bench_module()
    line = {"metric": "Krylov matvecs/sec", "n_gpus": 1, "value": 1264.664,
            "config": {"workload": "2D Bratu 4096x4096 (4096x4096 per GPU), ..."}}
    # the driver's record: the parsed line, or the JSON line among the captured output (stderr may follow)
    (tmp_path / "BENCH_r09.json").write_text(json.dumps({"run": {"stdout_tail": "noise\n" + json.dumps(line) +
                                                                  "\nbench.py: cpu/gpu agreement\n"}}))
    monkeypatch.setattr(b, "ROOT", str(tmp_path))
    ref = b.config2_reference()
    assert ref["value"] == 1264.664 * 4096 ** 2 and "BENCH_r09.json" in ref["source"]
    (tmp_path / "BENCH_r10.json").write_text(json.dumps({"parsed": dict(line, value=1300.0), "run": {}}))
    assert b.config2_reference()["value"] == 1300.0 * 4096 ** 2
    monkeypatch.setattr(b, "ROOT", os.path.dirname(BENCH))  # the repo's own driver records parse too
    assert b.config2_reference() is not None


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
    # the line judges its own exchange: every rank reports non-zero device peer waits over the timed step
    assert len(d["ranks"]) == 2 and d["dof_rate"]["dof_matvecs_per_s"] > 0
    if d["config"]["reductions"] == "peer mailbox (IPC/xGMI)":
        for q in d["ranks"]:
            e = q["exchange"]
            assert e["reduce_waits"] > 0 and e["reduce_wait_us_mean"] > 0, e
            assert e["halo_waits"] > 0 and e["halo_wait_us_mean"] > 0, e
            assert 0 < e["exchange_share"] < 1, e


def test_pgrid_factorisation():
    """--pgrid auto: the most cubic px x py x pz of N (BASELINE config 5: 2 x 2 x 2 at N = 8); an explicit
    grid must multiply to N."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert b.pgrid_of("auto", 8) == (2, 2, 2)
    assert b.pgrid_of("auto", 4) == (1, 2, 2) and b.pgrid_of("auto", 2) == (1, 1, 2)
    assert b.pgrid_of("auto", 27) == (3, 3, 3)
    assert b.pgrid_of("2,1,4", 8) == (2, 1, 4)
    with pytest.raises(SystemExit):
        b.pgrid_of("2,2,1", 8)


@pytest.mark.gpu
@pytest.mark.parametrize("fail", ["1", "rank:1"])
def test_rccl_bootstrap_failure_falls_back_to_the_mailbox(fail):
    """A multi-GPU line must not be lost to an RCCL bootstrap failure: with NK_BENCH_RCCL_FAIL=1 every
    rank's bootstrap "fails"; with rank:1 only rank 1's local pre-check does (the other rank
    must not be left alone inside the collective init).  All ranks agree over gloo, start over on fresh
    contexts with the peer mailbox alone, and the line says so (config.transport) -- two ranks on the
    box's GPU(s)."""
    args = ["--gpus", "2", "--side", "512", "--steps", "1", "--warmup", "1", "--no-prof", "--no-cpu-baseline"]
    p = run(args, env={"NK_BENCH_RCCL_FAIL": fail}, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(line) == 1
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["config"]["transport"].startswith("mailbox (RCCL bootstrap failed")
    if fail == "rank:1":
        assert "rank 1: NK_BENCH_RCCL_FAIL" in d["config"]["transport"]
    assert d["config"]["reductions"] == "peer mailbox (IPC/xGMI)"
    assert "falling back to the peer mailbox" in p.stderr


@pytest.mark.gpu
def test_eight_rank_block_bench_rehearsal():
    """BASELINE config 5's decomposition end to end through bench.py: --workload heat3d --global-n 64
    --pgrid auto on 8 ranks (2 x 2 x 2 blocks of 32^3; sharing the box's GPU over the mailbox when it has
    fewer): one JSON line naming the blocks, every rank's ghost faces exchanged (non-zero peer waits)."""
    import _nkpath  # noqa: F401
    import ariadne_hip as ah

    args = ["--gpus", "8", "--workload", "heat3d", "--global-n", "64", "--pgrid", "auto", "--steps", "1",
            "--warmup", "1", "--no-prof", "--no-cpu-baseline"]
    env = {}
    if ah.device_count() < 8:
        args += ["--transport", "mailbox"]
        env["GPU_MAX_HW_QUEUES"] = "1"  # 8 ranks x 4 queues would time-slice the one GPU
    p = run(args, env=env, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(line) == 1
    d = json.loads(line[0])
    assert d["n_gpus"] == 8 and d["value"] > 0 and d["config"]["parallelism"] == "blocks2x2x2"
    assert "32x32x32 block per GPU" in d["config"]["workload"]
    assert len(d["ranks"]) == 8
    for q in d["ranks"]:
        assert q["exchange"]["halo_waits"] > 0, q
