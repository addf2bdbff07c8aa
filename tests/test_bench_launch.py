"""bench.py's N > 1 plumbing on CPU: the self-launch (--gpus N without a launcher starts N
ranks with the torchrun environment and returns the worst exit status) and the N > 1 report
assembly (gather over gloo, the `multi_gpu` block, the communicator-size check), fed with
fake per-rank statistics by two gloo ranks."""
import importlib.util
import json
import os
import socket
import subprocess
import sys
import textwrap

import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_import_loads_no_torch():
    # the launching parent must not load torch (and so no HIP runtime) before it forks the ranks
    code = "import importlib.util,sys;s=importlib.util.spec_from_file_location('b','bench.py');" \
           "m=importlib.util.module_from_spec(s);s.loader.exec_module(m);print('torch' in sys.modules)"
    out = subprocess.run([sys.executable, "-c", code], cwd=REPO, capture_output=True, text=True, check=True)
    assert out.stdout.strip() == "False"


def test_self_launch_env_and_status(tmp_path):
    b = _bench()
    fake = tmp_path / "rank.py"
    fake.write_text(textwrap.dedent(f"""
        import json, os, sys
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
        env = {{k: os.environ.get(k) for k in keys}}
        json.dump({{"env": env, "argv": sys.argv[1:]}}, open(os.path.join({str(tmp_path)!r}, "r" + env["RANK"]), "w"))
        sys.exit(3 if env["RANK"] == "1" and "--fail" in sys.argv else 0)
    """))
    assert b.self_launch(2, ["--gpus", "2", "--steps", "7"], script=str(fake)) == 0
    seen = [json.load(open(tmp_path / f"r{r}")) for r in range(2)]
    for r, s in enumerate(seen):
        e = s["env"]
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["LOCAL_WORLD_SIZE"]) == (str(r), str(r), "2", "2")
        assert e["MASTER_ADDR"] == "127.0.0.1"
        assert s["argv"] == ["--gpus", "2", "--steps", "7"]
    assert seen[0]["env"]["MASTER_PORT"] == seen[1]["env"]["MASTER_PORT"]
    assert b.self_launch(2, ["--fail"], script=str(fake)) == 3


def test_self_launch_kills_stragglers(tmp_path):
    # one rank fails, its peer hangs (as in a halo receive): the peer is killed after the grace
    # period and the parent reports a failure instead of waiting forever
    b = _bench()
    fake = tmp_path / "hang.py"
    fake.write_text("import os, sys, time\nif os.environ['RANK'] == '0': sys.exit(2)\ntime.sleep(600)\n")
    rc = b.self_launch(2, [], grace_s=1.0, script=str(fake))
    assert rc == 137  # SIGKILL of the straggler, reported as 128 + 9


def test_bench_without_launcher_spawns_ranks():
    # the real script: `python bench.py --gpus 2` starts two ranks; without a GPU each fails
    # loudly (no CPU fallback) and the parent exits non-zero
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "1"], cwd=REPO,
                         env=env, capture_output=True, text=True, timeout=600)
    if out.returncode == 0:
        pytest.skip("a GPU is visible: the ranks ran for real")
    assert out.stderr.count("LbmError: no HIP device visible") == 2


def _worker(rank, world, port, out_dir, rccl):
    import torch.distributed as dist
    b = _bench()
    b._imports()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    # fake per-rank slab statistics: [rank, rccl_ranks, edge, interior, halo, halo_exposed, wall,
    # single-domain] ms/step
    mine = [rank, rccl[rank], 0.03 + rank, 3.4, 0.05 * (rank + 1), 0.01 * rank, 3.5 + rank, 3.3 + 0.1 * rank]
    res = {}
    try:
        b.check_rccl_ranks(rank, rccl[rank], world)
        res["check"] = "ok"
    except SystemExit as e:
        res["check"] = str(e)
    el, km, mm, nf, every = b.gather_ranks(mine, 1.0 + rank, 10.0 * (rank + 1), 5.0 + rank, 1000 + rank, world)
    res.update(elapsed=el, kern_ms=km, main_ms=mm, n_fluid=nf)
    if rank == 0:
        res["multi_gpu"] = b.multi_gpu_block(every, 4.5)
    json.dump(res, open(os.path.join(out_dir, f"w{rank}.json"), "w"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("rccl", [[2, 2], [2, 1]])
def test_multi_gpu_report_gloo(tmp_path, rccl):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), rccl), nprocs=world, join=True,
                       start_method="spawn")
    res = [json.load(open(tmp_path / f"w{r}.json")) for r in range(world)]
    for r, x in enumerate(res):
        assert x["elapsed"] == 2.0 and x["kern_ms"] == 20.0 and x["main_ms"] == 6.0  # max over ranks
        assert x["n_fluid"] == 2001                                                   # sum over ranks
        if rccl[r] == world:
            assert x["check"] == "ok"
        else:
            assert "RCCL communicator has 1 ranks, WORLD_SIZE 2" in x["check"]
    mg = res[0]["multi_gpu"]
    assert mg["rccl_ranks"] == min(rccl)
    assert [p["rank"] for p in mg["per_rank"]] == [0, 1]
    assert mg["per_rank"][1]["edge_ms"] == 1.03 and mg["per_rank"][1]["wall_ms_per_step"] == 4.5
    # exposed 0.00 + 0.01 ms of a 0.05 + 0.10 ms halo: hidden share 1 - 0.01 / 0.15
    assert mg["halo_hidden_frac"] == round(1 - 0.01 / 0.15, 4)
    # weak scaling against each rank's own slab stepped as one domain: 3.3 / 3.5 and 3.4 / 4.5
    assert [p["weak_scaling_eff"] for p in mg["per_rank"]] == [round(3.3 / 3.5, 4), round(3.4 / 4.5, 4)]
    assert mg["weak_scaling_eff_min"] == round(3.4 / 4.5, 4)
    assert mg["weak_scaling_eff_job"] == round(3.35 / 4.5, 4)


def test_cpu_baseline_assembly():
    """The CPU baseline child (oracle/cpu_baseline.py) on a small sample: one pinned core per
    sample, the bench workload's sample as `value`, C1 beside it."""
    b = _bench()
    line = b.finish_cpu_baseline(b.start_cpu_baseline(24, 3, quick=True), n=24)
    assert line["value"] > 0 and line["cores"] == 1 and line["kind"] == "port"
    assert "LDC 24^3" in line["sample"] and "3 step(s)" in line["sample"]
    assert line["c1"]["steps"] == 200 and line["c1"]["mlups"] > 0
    assert "c2" not in line and "c1_converge" not in line  # --quick


def test_cpu_baseline_group_is_stopped():
    """A bench that fails (or gives up waiting) ends the CPU baseline's whole process group: the
    child and the sample processes it started."""
    import time
    b = _bench()
    p = b.start_cpu_baseline(96, 50, quick=True)  # several seconds of oracle work per sample
    time.sleep(2.0)
    pgid = os.getpgid(p.pid)
    assert pgid == p.pid  # its own session / group
    b.stop_cpu_baseline(p)
    assert p.returncode is not None
    deadline = time.time() + 10
    while time.time() < deadline:
        try:
            os.killpg(pgid, 0)
        except ProcessLookupError:
            break
        time.sleep(0.1)
    else:
        raise AssertionError("baseline samples still running")
