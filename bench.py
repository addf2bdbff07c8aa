#!/usr/bin/env python3
"""bench.py -- MLUPS of the D3Q19 BGK hot path on MI355X (one process per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

With --gpus N > 1 and no WORLD_SIZE in the environment (no launcher), bench.py launches
itself: the parent starts N child processes of this script with RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, before it imports torch or touches a
GPU, waits for them and exits with the worst child status.  The children are the ranks.

Workload (weak scaling): the lid-driven cavity of ldc.cu on a 512 x 512 x (512*N) box split
into N z-slabs of 512^3 cells, one per GPU (N = 8 is BASELINE.json config C5, N = 1 the
north-star 512^3 single-GPU lattice).  A step is one reference time step over the whole
lattice: fused pull-stream + BGK collide with mask-driven bounce-back and lid NEE, the |u|
residual reduction, and for N > 1 the RCCL halo exchange of the +-z faces (5 populations
each) overlapped with the interior update plus the residual all-reduce.  Populations are
resident in HBM before timing starts (generated on the device).

Rank 0 prints ONE JSON line.  `value` = MLUPS over all ranks counting NX*NY*NZ box cells
(SURVEY.md 8(d)); `roofline.achieved` = 152 B x fluid cells / average k_step
duration from HIP events recorded on the kernel's own stream; `roofline.traffic` = the
HBM bytes per launch rocprofv3 counted for the same kernel (profiles/pmc_traffic.json);
`cpu_baseline` = the serial oracle (oracle/, a port of the reference algorithm) on one
host core, N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lattice-boltzmann-method-gpu_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
# torch, torch.distributed and lbm_amd are imported by _imports(): after the self-launch
# decision, so the launching parent never loads a HIP runtime
torch = dist = lbm_amd = cases = ldist = None

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
BYTES_PER_CELL = 152    # 19 fp32 loads + 19 fp32 stores per fluid cell update


def start_cpu_baseline(n: int = 512, steps: int = 1, quick: bool = False):
    """Start the serial CPU baseline (oracle/cpu_baseline.py) as a child process: the oracle (the
    reference algorithm restated in C, oracle/) on bounded samples, each pinned to ONE host core
    of its own (sched_setaffinity + OMP_NUM_THREADS=1), side by side with the GPU measurements
    (the GPU process's host threads keep the other cores): LDC n^3, the bench workload itself,
    for `steps` steps (~12 s per 512^3 step); C1 (LDC 64^3) 200 fixed steps and to convergence;
    C2 (LDC 256^3) and C3 (Poiseuille 128 x 512 x 128) fixed-step samples."""
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, os.path.join(REPO, "oracle", "cpu_baseline.py"), str(n), str(steps)]
    # its own process group: stop_cpu_baseline ends the samples (grandchildren) with it
    return subprocess.Popen(cmd + (["--quick"] if quick else []), env=env, stdout=subprocess.PIPE, text=True,
                            start_new_session=True)


def stop_cpu_baseline(p):
    """End the baseline's whole process group (its samples included) if it is still running: the
    bench failed or gave up waiting."""
    if p is not None and p.poll() is None:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except OSError:
            pass
        p.wait()


SAMPLE_CORES = 5  # oracle/cpu_baseline.py's samples take the highest-numbered allowed cores


def pin_away_from_samples():
    """Keep this process (and the HIP runtime threads it starts later) off the cores the CPU
    baseline's samples run on, so the GPU measurements' host side does not share them; only when
    at least four cores remain."""
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return None
    keep = allowed[:-SAMPLE_CORES]
    if len(keep) >= 4:
        os.sched_setaffinity(0, set(keep))
        return len(keep)
    return None


def finish_cpu_baseline(p, n: int = 512, timeout: float = 900.0):
    """The `cpu_baseline` object from start_cpu_baseline's child: `value` = the bench workload's
    sample (one core), the configs' samples beside it."""
    try:
        out, _ = p.communicate(timeout=timeout)
    finally:
        stop_cpu_baseline(p)
    if p.returncode != 0:
        raise SystemExit(f"cpu baseline failed ({p.returncode})")
    r = json.loads(out.strip().splitlines()[-1])
    b = r["bench"]
    line = {"value": round(b["mlups"], 3), "unit": "MLUPS", "cores": 1, "kind": "port",
            "sample": f"oracle/lbm_oracle.c (serial C port of the reference kernels, fp32, two-phase LDC) on LDC "
                      f"{n}^3 (the bench workload), {b['steps']} step(s) after set-up, {b['seconds']:.1f} s, pinned to "
                      f"core {r['core']} (sched_setaffinity, OMP_NUM_THREADS=1), host CPU: {r['cpu']}"}
    names = {"c1": "config C1: LDC 64^3, 200 fixed steps",
             "c1_converge": "config C1: LDC 64^3 to convergence (tol 1e-6, 50 hits; residual summed in fp64 as "
                            "liblbm does, so the stop step is liblbm's)",
             "c2": "config C2: LDC 256^3, 10 fixed steps (BASELINE.md 4: 1000 steps scaled down)",
             "c3": "config C3: Poiseuille 128x512x128 (pipe along y), 20 fixed steps, MLUPS over box cells "
                   "(mlups_nlattice: over the reference's stored cells)"}
    for k, what in names.items():
        if k in r:
            e = {"mlups": round(r[k]["mlups"], 3), "workload": what, "seconds": r[k]["seconds"],
                 "steps": r[k]["steps"], "core": r["cores"][k]}
            if "mlups_nlattice" in r[k]:
                e["mlups_nlattice"] = round(r[k]["mlups_nlattice"], 3)
            line[k] = e
    line["samples_run"] = "side by side, one core each"
    return line


def pmc_traffic(workload: str):
    """HBM bytes per k_step launch measured by rocprofv3 PMC passes (tools/gpu_profile.sh +
    tools/pmc_traffic.py, tools/pmc_lattices.sh + .py write profiles/pmc_traffic.json) -- only
    when recorded on the kernels this run uses (lbm_amd.kernel_fingerprint()); an entry from
    other kernels comes back as {"stale": tag} and is not reported as this run's traffic."""
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        e = json.load(open(p)).get(workload)
    except (OSError, ValueError):
        return None
    if e and e.get("kernel_src") != lbm_amd.kernel_fingerprint():
        return {"stale": e.get("tag")}
    return e


def ldc_line(n: int, steps: int, dev: int, name: str):
    """LDC n^3 (device-generated cavity) through timed_mlups: wall-clock MLUPS plus the step's
    roofline from HIP events and, when profiled on these kernels, rocprof's k_step time and the
    measured HBM traffic."""
    return timed_mlups(cases.ldc_device(n, n, n, device=dev), {"mlups": n ** 3}, steps, name=name)


def fresh_line(name: str, make, cells: dict, steps: int, lattices: int = 3):
    """One secondary line over `lattices` fresh lattices in turn (make() builds one), each with its
    own buffers: step times differ from allocation to allocation (C2's 1.28-GB population buffers'
    HBM write rates) and from process to process (C3's slow mode, section 3).
    The line is the median lattice's, with every lattice's step time, wall time and kept buffers'
    write rates beside it."""
    runs = [timed_mlups(make(), cells, steps, name=name) for _ in range(lattices)]
    order = sorted(range(lattices), key=lambda i: runs[i]["roofline"]["step_us"])
    out = dict(runs[order[lattices // 2]])
    us = [runs[i]["roofline"]["step_us"] for i in order]
    out["fresh_lattices"] = {
        "step_us_min_median_max": [us[0], us[lattices // 2], us[-1]],
        "frac_min_median_max": [round(runs[i]["roofline"]["frac"], 4) for i in (order[0], order[lattices // 2], order[-1])],
        "per_lattice": [{"step_us": r["roofline"]["step_us"], "ms_per_step": r["ms_per_step"],
                         "kept_write_gbs": [r["buffer_placement"]["candidate_write_gbs"][k]
                                            for k in r["buffer_placement"]["chosen"]]
                         if r["buffer_placement"]["candidate_write_gbs"] else [],
                         "best_candidate_write_gbs": max(r["buffer_placement"]["candidate_write_gbs"], default=None),
                         "setup": r["setup"]} for r in runs],
    }
    return out


def c2_line(dev: int, lattices: int = 3, steps: int = 1000):
    """Config C2 (LDC 256^3, 1000 steps) on three fresh lattices (fresh_line)."""
    return fresh_line("ldc_256^3 (C2)", lambda: cases.ldc_device(256, 256, 256, device=dev), {"mlups": 256 ** 3},
                      steps, lattices)


def c5_one_gpu(dev: int, steps: int = 500):
    """The C5 lattice (LDC 512 x 512 x 4096, 1.07 G cells, ~187 GB) as ONE domain on one GPU,
    BASELINE.md's 500 timed steps: what the 8-GPU configuration's total work costs a single
    MI355X (timed_mlups: the step's roofline from HIP events, traffic when profiled)."""
    lat = cases.ldc_device(512, 512, 4096, device=dev)
    return timed_mlups(lat, {"mlups": 512 * 512 * 4096}, steps, warm=3, name="ldc_512x512x4096 (C5 lattice)")


def timed_mlups(lat, cells: dict, steps: int, warm: int = 20, name: str = None):
    """Wall-clock MLUPS over `steps` steps, and the roofline of the same timed steps: HIP events
    around the timed lbm_step call on the kernels' stream (lbm_profile 2: no per-launch events,
    whose ~2-us launches would inflate small lattices' kernel times) give the device time per
    step of ALL its kernels (k_step, k_nee_fix where the lattice has one, the residual), which
    cannot exceed the wall time per step; frac = algorithmic bytes (152 B x fluid cells) / that
    time against 8 TB/s.  rocprofv3's per-kernel means for this lattice at these kernels
    (profiles/pmc_traffic.json, tools/pmc_lattices.sh; fingerprint-checked) split the step into
    k_step and k_nee_fix, with the HBM bytes per launch it counted."""
    lay = lat.layout()
    shape = lat.launch_shape()
    store = lat.storage()
    setup = lat.setup_cost()
    nee = lat.nee_path()
    algo = lat.counts()["algo_bytes_per_step"]
    lat.step(warm, history=False)
    lat.sync()
    lat.profile(2)
    t = time.perf_counter()
    lat.step(steps, history=False)
    lat.sync()
    dt = time.perf_counter() - t
    st = lat.stats()
    placement = lat.placement()
    lat.close()
    out = {k: round(v * steps / dt / 1e6, 1) for k, v in cells.items()}
    out["ms_per_step"] = round(dt / steps * 1e3, 5)
    out["steps"] = steps
    out["rows_along"] = "xy"[lay["row_axis"] - 1]
    out["active_chunks"] = lay["active_chunks"]
    out["cells_per_lane"] = shape["cells_per_lane"]
    out["grid_stride"] = shape["grid_stride"]
    out["lane_fill"] = shape["lane_fill"]
    out["nee_values"] = nee["path"]
    out["storage"] = {"compact_rows": store["compact"], "cell_slots": store["cells"],
                      "population_bytes": store["bytes"]}
    step_us = st["span_ms"] / max(1, st["span_launches"]) * 1e3
    gbs = algo / (step_us * 1e-6) / 1e9
    rl = {"step_us": round(step_us, 3), "algo_bytes_per_step": int(algo), "achieved": round(gbs, 1), "unit": "GB/s",
          "frac": round(gbs / HBM_PEAK_GBS, 4),
          "basis": "per step: all kernels of the timed steps between two HIP events on their stream (lbm_profile 2)",
          "traffic": None}
    pmc = pmc_traffic(name) if name else None
    if pmc and "stale" in pmc:
        rl["rocprof_stale"] = f"profiles/pmc_traffic.json ({pmc['stale']}) was measured on other kernels"
    elif pmc:
        k_us, fix_us = pmc.get("k_step_avg_us"), pmc.get("k_nee_fix_avg_us") or 0.0
        if k_us:
            rl["rocprof"] = {"k_step_us": k_us, "k_nee_fix_us": fix_us or None,
                             "frac_k_step": round(algo / (k_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                             "frac_k_step_plus_nee_fix": round(algo / ((k_us + fix_us) * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                             "source": f"profiles/pmc_traffic.json ({pmc.get('tag')}: rocprofv3 --kernel-trace, "
                                       f"tools/pmc_lattices.sh, another process)"}
        rl["traffic"] = pmc.get("bytes_per_launch")
        rl["traffic_over_algo"] = pmc.get("traffic_over_algo")
    out["roofline"] = rl
    out["buffer_placement"] = placement
    out["setup"] = setup
    return out


def config_lines(dev: int):
    """BASELINE configs C3 (Poiseuille 128 x 128 x 512, pipe along y) and C4 (the shipped
    bifurcation mask) as secondary lines: MLUPS over box cells and over the reference's
    NLATTICE (stored cells, its metric for sparse cases)."""
    out = {}
    geo = cases.geo_poiseuille(128, 512, 128)
    nl, _ = lbm_amd.index_transform(geo)
    k = "poiseuille_128x512x128 (C3)"
    out[k] = fresh_line(k, lambda: cases.poiseuille(128, 512, 128, device=dev)[0],
                        {"mlups_box": geo.size, "mlups_nlattice": nl}, 1000)
    # the same lattice on the x-row layout (lbm_desc.row_axis = 1), for comparison
    with lbm_amd.tuned(lbm_amd.TUNE_ROW_AXIS, 1):
        lat, geo = cases.poiseuille(128, 512, 128, device=dev)
    out["poiseuille_128x512x128 (C3), x rows"] = timed_mlups(lat, {"mlups_box": geo.size, "mlups_nlattice": nl}, 1000)
    lat, geo, _, _ = cases.bifurcation(1, device=dev)
    nl, _ = lbm_amd.index_transform(geo)
    k = "bifurcation_64x83x32 (C4)"
    out[k] = timed_mlups(lat, {"mlups_box": geo.size, "mlups_nlattice": nl}, 4401, name=k)
    # SURVEY 8(d) C4's bandwidth-relevant sparse number: the shipped mask upsampled 4x per axis
    lat, raw = cases.bifurcation_upsampled(4, device=dev)
    nl, _ = lbm_amd.index_transform(lat.geo())
    k = "bifurcation_x4_256x332x128 (C4 upsampled)"
    out[k] = timed_mlups(lat, {"mlups_box": raw.size, "mlups_nlattice": nl}, 200, name=k)
    # coronary.cu's 291 x 291 x 372 box with its five open ends on a synthetic vessel tree (the
    # reference's geo.txt is not shipped): a sparse lattice, 2.5 % of the box stored
    lat, geo = cases.coronary(cases.coronary_reference_vessel(), device=dev)
    nl, _ = lbm_amd.index_transform(geo)
    k = "coronary_291x291x372 (synthetic vessel)"
    out[k] = timed_mlups(lat, {"mlups_box": geo.size, "mlups_nlattice": nl}, 1000, name=k)
    return out


def perturbed_mlups(n: int, steps: int, dev: int):
    """LDC n^3 started from equilibria of a random velocity field (|u| ~ 0.01, fixed seed)
    instead of rest: populations then carry full-entropy bit patterns, which costs the
    HBM-bound kernel ~7% against the near-uniform data of a cavity started at rest."""
    import numpy as np
    geo = lbm_amd.geo_ldc(n, n, n)
    rho, ux, uy, uz = lbm_amd.initial_fields(0, geo)
    rng = np.random.default_rng(0)
    fl = geo == 3
    for a in (ux, uy, uz):
        a[fl] += rng.normal(0.0, 0.01, int(fl.sum())).astype(np.float32)
    lat = lbm_amd.Lattice(lbm_amd.LBM_CASE_LDC, (n, n, n), 0.55, geo, device=dev)
    lat.init_equilibrium(lbm_amd.LBM_INIT_LDC_WI, rho, ux, uy, uz)
    del rho, ux, uy, uz, geo
    lat.step(5, history=False)
    lat.sync()
    lat.profile(True)
    t = time.perf_counter()
    lat.step(steps, history=False)
    lat.sync()
    dt = time.perf_counter() - t
    st = lat.stats()
    lat.close()
    return {"mlups": round(n ** 3 * steps / dt / 1e6, 1),
            "avg_kernel_ms": round(st["step_kernel_ms"] / max(1, st["step_kernel_launches"]), 4)}


def _imports():
    """torch (before liblbm: one shared HIP runtime), torch.distributed and lbm_amd."""
    global torch, dist, lbm_amd, cases, ldist
    import torch as _torch
    import torch.distributed as _dist
    import lbm_amd as _lbm_amd
    from lbm_amd import cases as _cases
    from lbm_amd import dist as _ldist
    torch, dist, lbm_amd, cases, ldist = _torch, _dist, _lbm_amd, _cases, _ldist


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--n", type=int, default=512, help="per-GPU slab edge (nx = ny = nz_local)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(n: int, argv, grace_s: float = 420.0, script=None) -> int:
    """--gpus n > 1 without a launcher: start n ranks of this script as child processes (the
    torchrun environment: RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR,
    MASTER_PORT), wait, return the worst exit status.  Called before torch is imported; the
    parent never execs.  When a rank fails, the others get `grace_s` seconds to fail too
    (their RCCL waits give up after LBM_TUNE_SYNC_TIMEOUT_S = 300 s) before they are killed."""
    port = _free_port()
    script = script or os.path.abspath(__file__)
    kids = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        kids.append(subprocess.Popen([sys.executable, script, *argv], env=env))
    first_fail = None
    while True:
        codes = [p.poll() for p in kids]
        if all(c is not None for c in codes):
            break
        if first_fail is None and any(c not in (None, 0) for c in codes):
            first_fail = time.monotonic()
        if first_fail is not None and time.monotonic() - first_fail > grace_s:
            for p in kids:
                if p.poll() is None:
                    p.kill()
            for p in kids:
                p.wait()
            break
        time.sleep(0.2)
    worst = 0
    for p in kids:
        rc = p.returncode
        rc = 128 - rc if rc < 0 else rc  # killed by signal s: 128 + s, as a shell reports it
        if rc and (worst == 0 or rc > worst):
            worst = rc
    return worst


def check_rccl_ranks(rank: int, rccl_ranks: int, world: int):
    """The communicator liblbm built must span every rank (ncclCommCount)."""
    if rccl_ranks != world:
        raise SystemExit(f"rank {rank}: RCCL communicator has {rccl_ranks} ranks, WORLD_SIZE {world}")


def single_domain_ms(lat, steps: int, warm: int = 3) -> float:
    """Wall ms per step of this rank's slab stepped as a single domain (no communicator yet: one
    launch per step over all its planes, ghost planes left as initialised) -- the per-GPU work
    of the slab without the halo exchange, the reference point of `weak_scaling_eff`."""
    lat.step(warm, history=False)
    lat.sync()
    t = time.perf_counter()
    lat.step(steps, history=False)
    lat.sync()
    return (time.perf_counter() - t) / steps * 1e3


def gather_ranks(mine, elapsed: float, kern_ms: float, main_ms: float, n_fluid: int, world: int, group=None):
    """N > 1: the slowest rank's wall time and kernel times (max over ranks), the fluid cells of
    all slabs (sum) and every rank's row `mine` = [rank, rccl_ranks, edge, interior, halo,
    halo_exposed, wall, single_domain] (ms per step), gathered over torch.distributed (gloo)."""
    elapsed, kern_ms, main_ms = ldist.max_over_ranks([elapsed, kern_ms, main_ms], group)
    n_fluid_total = int(ldist.sum_over_ranks([n_fluid], group)[0])
    every = [None] * world
    dist.all_gather_object(every, list(mine), group=group)
    return elapsed, kern_ms, main_ms, n_fluid_total, every


def multi_gpu_block(every, job_ms_per_step: float = None) -> dict:
    """The N > 1 bench line's `multi_gpu` object from the gathered per-rank rows: per-rank slab
    timings (HIP events, ms per step) -- edge-plane launch, interior launch, halo exchange on the
    communication stream, and the part of the halo that outlasted the interior launch (not
    hidden) -- the smallest communicator any rank saw, and the hidden share of the halo.
    Weak scaling: each rank timed its own slab as a single domain before the communicator was
    attached (single_domain_ms_per_step); weak_scaling_eff = that / the rank's slab wall time per
    step, per rank and as the minimum, and for the job: the ranks' mean single-domain time / the
    job's time per step (max over ranks, barrier-bracketed)."""
    ranks = []
    for r in sorted(every):
        row = {"rank": int(r[0]), "rccl_ranks": int(r[1]), "edge_ms": round(r[2], 4), "interior_ms": round(r[3], 4),
               "halo_ms": round(r[4], 4), "halo_exposed_ms": round(r[5], 4), "wall_ms_per_step": round(r[6], 4)}
        if len(r) > 7 and r[7]:
            row["single_domain_ms_per_step"] = round(r[7], 4)
            row["weak_scaling_eff"] = round(r[7] / r[6], 4) if r[6] > 0 else None
        ranks.append(row)
    halo = sum(r["halo_ms"] for r in ranks)
    out = {
        "rccl_ranks": min(r["rccl_ranks"] for r in ranks),
        "halo_hidden_frac": round(1.0 - sum(r["halo_exposed_ms"] for r in ranks) / halo, 4) if halo > 0 else None,
    }
    effs = [r["weak_scaling_eff"] for r in ranks if r.get("weak_scaling_eff") is not None]
    if effs and len(effs) == len(ranks):
        out["weak_scaling_eff_min"] = min(effs)
        if job_ms_per_step:
            single = sum(r["single_domain_ms_per_step"] for r in ranks) / len(ranks)
            out["weak_scaling_eff_job"] = round(single / job_ms_per_step, 4)
        out["weak_scaling_ref"] = ("each rank's own 512^3 slab stepped as one domain (no halo, no all-reduce) "
                                   "on the same GPU in the same run, before lbm_attach_rccl")
    out["per_rank"] = ranks
    return out


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    # the CPU baseline runs on its own host cores while the GPU is measured (N = 1 only); this
    # process -- and every thread the HIP runtime starts from it -- keeps to the other cores
    cpu_proc = None
    if world == 1 and not args.no_cpu_baseline:
        cpu_proc = start_cpu_baseline()
        pin_away_from_samples()
    try:
        _imports()
        lbm_amd.require_gpu()
        torch.cuda.set_device(local)
        if world > 1:
            # host-side coordination only (gloo); the data path is liblbm's own RCCL communicator
            dist.init_process_group("gloo")
        run(args, world, rank, local, args.n, args.n * world, cpu_proc)
    finally:
        stop_cpu_baseline(cpu_proc)


def run(args, world, rank, local, n, nzg, cpu_proc):
    lat = cases.ldc_device(n, n, n, z_offset=rank * n, nz_global=nzg, device=local)
    single_ms = None
    if world > 1:
        # the weak-scaling reference: this slab's step as a single domain on this GPU, then a
        # fresh initial state for the slab run
        single_ms = single_domain_ms(lat, max(5, min(args.steps, 20)))
        lat.init_ldc()
        # a rank whose peer died fails its next wait with LBM_ERR_RCCL (async error poll, or
        # this limit) and exits non-zero, instead of hanging in a halo receive
        lbm_amd.tune(lbm_amd.TUNE_SYNC_TIMEOUT_S, 300)
        lat.attach_rccl(ldist.share_unique_id(rank, None, lbm_amd.rccl_unique_id), rank, world)
    rccl_rank, rccl_ranks = lat.comm_info()
    check_rccl_ranks(rank, rccl_ranks, world)
    counts = lat.counts()

    def barrier():
        if world > 1:
            dist.barrier()

    lat.step(args.warmup, history=False)
    lat.sync()
    lat.profile(True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lat.step(args.steps, history=False)
    lat.sync()
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    st = lat.stats()
    state = lat.state()
    elapsed = t1 - t0
    kern_ms = st["kernel_ms"]
    main_ms, main_n = st["step_kernel_ms"], max(1, st["step_kernel_launches"])
    per_step = lambda k: st[k + "_ms"] / args.steps  # noqa: E731
    mine = [rank, rccl_ranks, per_step("edge"), per_step("interior"), per_step("halo"), per_step("halo_exposed"),
            elapsed / args.steps * 1e3, single_ms or 0.0]
    if world > 1:
        elapsed, kern_ms, main_ms, n_fluid_total, every = gather_ranks(mine, elapsed, kern_ms, main_ms,
                                                                      counts["n_fluid"], world)
    else:
        n_fluid_total = counts["n_fluid"]
        every = [mine]
    parity_ms = [round(st[f"step_kernel_src{b}_ms"] / max(1, st[f"step_kernel_src{b}_launches"]), 4) for b in (0, 1)]
    placement = lat.placement()
    launch_shape = lat.launch_shape()
    setup = lat.setup_cost()
    lat.close()

    # attainable streaming bandwidth of this device, same run (context for roofline.frac:
    # the 8 TB/s spec peak is not reached by any kernel)
    probe_shapes = lbm_amd.probe_stream_shapes(local) if rank == 0 else None
    probe = max(probe_shapes.values()) if probe_shapes else None

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    box_cells = n * n * nzg
    ms_step = elapsed / args.steps * 1e3
    mlups = box_cells * args.steps / elapsed / 1e6
    # dominant kernel: k_step, timed with HIP events on its own stream; per step it moves
    # 152 B per fluid cell of the slab (19 fp32 pulls + 19 fp32 stores) -- one launch at
    # N = 1, two (both edge planes, then the interior) per step on a slab at N > 1
    main_avg_ms = main_ms / main_n
    main_step_ms = main_ms / args.steps
    algo_bytes = BYTES_PER_CELL * counts["n_fluid"]
    achieved = algo_bytes / (main_step_ms * 1e-3) / 1e9
    workload = f"ldc_{n}x{n}x{n}_per_gpu"
    pmc = pmc_traffic(workload)
    stale = pmc.get("stale") if pmc else None
    if stale:
        pmc = None
    line = {
        "metric": "MLUPS (million lattice updates/sec) + achieved HBM GB/s vs roofline",
        "value": round(mlups, 1),
        "unit": "MLUPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (ldc.cu cavity generated on device: rho=1, u=0, lid u=0.15/C_U)",
        "config": {
            "workload": f"LDC D3Q19 BGK {n}x{n}x{nzg} box, z-slabs of {n}x{n}x{n} per GPU "
                        f"(north-star 512^3 lattice at N=1; BASELINE config C5 at N=8)",
            "global_shape_xyz": [n, n, nzg],
            "box_cells": box_cells,
            "fluid_cells": n_fluid_total,
            "mlups_fluid_cells": round(n_fluid_total * args.steps / elapsed / 1e6, 1),
            "parallelism": f"z-slab x{world}" + (" (RCCL halo, 5 pops/face)" if world > 1 else ""),
            "tau": 0.55,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_step (fused pull-stream + BGK collide + half-way bounce-back + NEE cells)",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": pmc.get("bytes_per_launch") if pmc else None,
            "traffic_source": (f"profiles/pmc_traffic.json ({pmc.get('tag')}: rocprofv3 FETCH_SIZE x2 + WRITE_SIZE "
                               f"per launch, 512^3 N=1, same kernel fingerprint)") if pmc else
                              (f"stale: profiles/pmc_traffic.json ({stale}) was measured on other kernels" if stale
                               else None),
            "algo_bytes_per_launch": algo_bytes,
            "avg_kernel_ms": round(main_avg_ms, 4),
            "kernel_ms_per_step": round(main_step_ms, 4),
            "launches": main_n,
            "boundary_cells_per_gpu": counts["n_boundary"],
            "stream_probe_gbs": probe,
            "frac_of_stream_probe": round(achieved / probe, 4) if probe else None,
            "stream_probe": "lbm_probe_stream: best of 11 streaming-copy shapes (16-B vectors, grid-stride, "
                            "per-XCD regions or k_step-like 16-KB wave tiles, plain or non-temporal, the tiles also by "
                            "LDS-DMA; read + write bytes / time) between two of up to twenty 8-GiB allocations, picked by "
                            "the population buffers' placement rule (write-sweep rank, then the quickest tile-copy "
                            "pair of the four fastest) on this GPU in this run",
            "stream_probe_shapes_gbs": probe_shapes,
        },
        "reference_published": {"mlups": 391.86, "config": "LDC 64^3 on GTX 1050 Ti (thesis 4.9.1)"},
        "step_kernel_ms_by_source_buffer": parity_ms,
        "buffer_placement": placement,
        # lbm_create's cost: wall seconds (placement probe included), the device memory the context
        # holds, and the most it held while the placement candidates were allocated
        "setup": setup,
        "launch_shape": launch_shape,
        "residual_last": state["residual"],
        "kernel_src": lbm_amd.kernel_fingerprint(),
    }
    if world > 1:
        line["multi_gpu"] = multi_gpu_block(every, ms_step)
    if world == 1 and not args.no_secondary:
        line["secondary"] = {"ldc_64^3 (published config)": ldc_line(64, 2000, local, "ldc_64^3"),
                             "ldc_256^3 (C2)": c2_line(local),
                             f"ldc{n}_random_velocity_start": perturbed_mlups(n, 50, local),
                             "ldc_512x512x4096 (C5 lattice, single domain)": c5_one_gpu(local),
                             **config_lines(local)}
    if cpu_proc is not None:
        line["cpu_baseline"] = finish_cpu_baseline(cpu_proc)
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
