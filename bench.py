"""MPPI steps/s at K=65536, H=100 on the 750x750 costmap (BASELINE.json metric), 1..N GPUs.

One "step" = one full MPPI_step("3d") (thesis_master/warp_implementation/MPPI_isaac.py:505-720):
Philox sampling, wheel filter, 2.5D rollout, four critics, softmax-weighted
update, optimal filter and optimal rollout, with the outputs copied to host
memory.  Inputs (DEM, costmap, state) are resident in HBM before timing.

Configs (BASELINE.json configs[1..4]):
  c3  K=65,536   H=100, 1500^2 DEM @0.1 m, 750^2 costmap  (headline, default)
  c4  K=1,048,576 H=100, same scene
  c5  K=262,144  H=128, 8192^2 DEM @0.025 m, 1024^2 costmap
Scaling: STRONG.  The config's K is the global sample count; with N ranks each
owns a contiguous leaf-aligned shard (distributed.shard_bounds) and the ranks
exchange one (2H+2)-double softmax record per step with one RCCL all-gather.
`value` = global MPPI steps/s at the named K.  For N>1 rank 0 also times the
same config on its own GPU alone (`speedup_vs_1`), and the `c4` leg (K=1,048,576,
the north-star scaling config) is run beside the headline at every N.

Launch: python bench.py [--config c3|c4|c5] [--steps K --warmup W]  (N=1);
        python bench.py --gpus N: one process drives GPUs 0..N-1 through the C-ABI group
        (mppi_group_create: one context per GPU, ncclCommInitAll, one ncclAllGather per member
        per step, each member's launches enqueued by its own thread);
        python bench.py --group-devices 0,0,0,0,0,0,0,0: the same group code path with members
        sharing one GPU (records exchanged by device copies: a 1-GPU rehearsal of the 8-way split);
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N: one process per
        GPU (torch.distributed over RCCL, mppi_amd/distributed.ShardedMPPI).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

BYTES_PER_ROLLOUT_STEP = 28   # 6 DEM f32 gathers + 1 costmap f32 gather
HBM_PEAK_GBS = 8000.0         # MI355X HBM3E spec (MI355X_MICROARCH.md)

# name -> (K global, H, scene function name, start, goal, description)
CONFIGS = {
    "c2": (4096, 50, "scene_c3", (-60.0, -5.0), (65.0, 10.0),
           "C2: K=4096, H=50, 1500^2 DEM @0.1 m, 750^2 costmap @0.2 m"),
    "c3": (65536, 100, "scene_c3", (-60.0, -5.0), (65.0, 10.0),
           "C3: K=65536, H=100, 1500^2 DEM @0.1 m, 750^2 costmap @0.2 m"),
    "c4": (1048576, 100, "scene_c3", (-60.0, -5.0), (65.0, 10.0),
           "C4: K=1048576, H=100, 1500^2 DEM @0.1 m, 750^2 costmap @0.2 m"),
    "c5": (262144, 128, "scene_c5", (0.0, 0.0), (80.0, 20.0),
           "C5: K=262144, H=128, 8192^2 DEM @0.025 m (synthetic craters + fBm), 1024^2 costmap"),
    # diagnostic: one GPU's shard of C4 at 8 GPUs (what each rank of the north-star scaling runs)
    "c4s8": (131072, 100, "scene_c3", (-60.0, -5.0), (65.0, 10.0),
             "C4 shard at 8 GPUs: K=131072, H=100, 1500^2 DEM @0.1 m, 750^2 costmap @0.2 m"),
}
KERNEL_SOURCES = ("mppi_kernels.hip", "mppi_kernels.h", "mppi_detmath.h", "mppi_capi.cpp", "Makefile")



def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--proj", default="3d")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=20.0,
                    help="budget of the bounded oracle samples on the host (rank 0, N=1); 0 disables")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_latest.json"))
    ap.add_argument("--no-bilinear", action="store_true", help="skip the C5 tiled-lookup roofline leg")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 (K=1048576) strong-scaling leg")
    ap.add_argument("--timed-events", action="store_true",
                    help="record the rollout kernel's HIP events inside the timed region (not a separate pass)")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 full-step leg (N=1)")
    ap.add_argument("--no-shard", action="store_true", help="skip the C4 per-GPU shard leg (N=1)")
    ap.add_argument("--no-costmap", action="store_true", help="skip the obstacle-costmap builder leg")
    ap.add_argument("--no-cadence", action="store_true",
                    help="skip the production-cadence leg (one step per simulator frame, N=1)")
    ap.add_argument("--no-sync-pass", action="store_true",
                    help="skip the synchronous-mode pass (profiling runs: only the headline schedule's launches)")
    ap.add_argument("--sync", action="store_true",
                    help="report the synchronous mode (no deferred optimal rollout) as the headline")
    ap.add_argument("--prewarm-ms", type=float, default=150.0,
                    help="untimed steps run first for this long, so that the timed passes start at the GPU's "
                         "steady clock (a short --steps/--warmup run otherwise starts below it)")
    ap.add_argument("--group-devices", default=None,
                    help="comma-separated device of each group member (default with --gpus N>1 and no "
                         "torch.distributed launcher: 0,1,...,N-1)")
    return ap.parse_args()


def source_hash():
    """sha256 over the kernel sources: ties a committed PMC profile to the code it measured."""
    h = hashlib.sha256()
    csrc = os.path.join(PKG, "csrc")
    for name in KERNEL_SOURCES:
        with open(os.path.join(csrc, name), "rb") as f:
            h.update(name.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cgroup_cpus():
    """CPU quota of this process's cgroup (cgroup v2 cpu.max or v1 cfs quota), in CPUs; None if unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def host_cores():
    """CPUs this process is granted: its affinity set, bounded by its cgroup's CPU quota (the GPU
    box grants a share of a larger machine; os.cpu_count() reports the whole machine)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = cgroup_cpus()
    n = aff if quota is None else max(1, min(aff, int(quota)))
    return n, aff, quota


# ------------------------------------------------------------------ CPU baseline (oracle, numpy)
_CPU = {}


def _cpu_shard(args):
    """Worker: one contiguous leaf-aligned slice of K -> its softmax record (oracle.shard_record)."""
    from oracle import mppi_ref as R
    K, H, step, b, c = args
    p = R.Params(K=K, H=H)
    u0 = np.zeros(H, np.float32)
    rec, _ = R.shard_record(p, _CPU["sc"], _CPU["st"], u0, u0, step, b, c)
    return rec


def _cpu_step_pool(pool, nw, K, H, step):
    from oracle import mppi_ref as R
    bounds = R.shard_bounds(K, nw)
    recs = pool.map(_cpu_shard, [(K, H, step, b, c) for b, c in bounds])
    p = R.Params(K=K, H=H)
    root = R.tree_reduce(np.stack(recs), p.temperature) if len(recs) > 1 else recs[0]
    return R.finish(p, _CPU["sc"], _CPU["st"], root)  # noqa: the finish is part of the step


def cpu_baseline(Z, hw, cm, start, goal, budget_s):
    """The build's numpy restatement (oracle/mppi_ref.py) timed on this host:
    C1 (K=256, H=20), C2 (K=4096, H=50) and C3 (K=65536, H=100) on the C3 scene, each on 1 core and
    on all granted cores (K split into leaf-aligned shards over a fork pool, records combined with
    the same tree).  C1/C2: 3 warm-up steps then the median of >=10; C3: a few steps."""
    import multiprocessing as mp
    from oracle import mppi_ref as R
    _CPU["sc"] = R.Scene(Z, hw, cm)
    _CPU["st"] = R.State(x=start[0], y=start[1], goal_x=goal[0], goal_y=goal[1])
    nw, aff, quota = host_cores()
    table = {}
    t_all = time.perf_counter()
    ctx = mp.get_context("fork")
    with ctx.Pool(nw) as pool:
        for name, K, H, reps in (("c1", 256, 20, 10), ("c2", 4096, 50, 10), ("c3", 65536, 100, 3)):
            u0 = np.zeros(H, np.float32)
            p = R.Params(K=K, H=H)
            row = {}
            for mode in ("1core", "allcores"):
                warm = 3 if name != "c3" else 1
                ts = []
                for i in range(warm + reps):
                    t0 = time.perf_counter()
                    if mode == "1core":
                        R.mppi_step(p, _CPU["sc"], _CPU["st"], u0, u0, i)
                    else:
                        _cpu_step_pool(pool, min(nw, (K + 255) // 256), K, H, i)
                    if i >= warm:
                        ts.append(time.perf_counter() - t0)
                    if time.perf_counter() - t_all > budget_s and i >= warm:
                        break
                med = float(np.median(ts))
                row[mode] = {"steps_per_s": round(1.0 / med, 3), "median_ms": round(med * 1e3, 2),
                             "steps_timed": len(ts),
                             "workers": 1 if mode == "1core" else min(nw, (K + 255) // 256)}
            table[name] = row
    c3 = table["c3"]["allcores"]
    return {"value": c3["steps_per_s"], "unit": "MPPI steps/s", "cores": c3["workers"], "kind": "port",
            "sample": (f"oracle/mppi_ref.py (numpy f32), C3 K=65536 H=100 on {c3['workers']} worker "
                       f"processes (leaf-aligned K shards, same record tree), median of "
                       f"{c3['steps_timed']} steps; host {cpu_model()}, os.cpu_count()={os.cpu_count()}, "
                       f"affinity={aff}, cgroup quota={quota} CPUs -> {nw} workers"),
            "table": table, "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(), "granted_cores": nw,
            "affinity_cpus": aff, "cgroup_quota_cpus": quota}


# ------------------------------------------------------------------ side legs (N=1)
def bilinear_bench(torch, device, reps=20):
    """LDS-tiled DEM lookup at C5 size: 8192^2 DEM @0.025 m, N = 262144*128 queries.

    NOT on the MPPI step path (the rollout gathers the DEM through L1/L2): a standalone kernel
    for the north-star '>=60 % of HBM roofline on the bilinear kernel' figure.  `frac` is the
    lookup kernel alone with the queries already binned by 128x128-cell tile; `frac_incl_binning`
    times the binning (count, scan, scatter) and the lookup together on the same stream.
    Algorithmic bytes = the DEM once + 12 B per query (x, y in, h out).
    """
    from mppi_amd import _lib
    G, hw, N = 8192, 102.4, 262144 * 128
    xs = torch.linspace(-hw, hw, G, device=device)
    Z = (0.8 * torch.sin(0.37 * xs)[None, :] * torch.cos(0.23 * xs)[:, None]).contiguous()   # synthetic terrain
    stream = torch.cuda.Stream(device=device)
    eng = _lib.Engine(_lib.make_params(256, 8), device.index or 0)
    eng.set_stream(stream.cuda_stream)
    eng.set_dem_device(Z.data_ptr(), G, G, hw, keepalive=Z)
    g = torch.Generator(device=device)
    g.manual_seed(5)
    x = (torch.rand(N, device=device, generator=g) * 2 - 1) * hw
    y = (torch.rand(N, device=device, generator=g) * 2 - 1) * hw
    nt = eng.bilinear_tiles()
    xb, yb = torch.empty_like(x), torch.empty_like(y)
    perm = torch.empty(N, dtype=torch.int32, device=device)
    off = torch.empty(nt + 1, dtype=torch.int32, device=device)
    h = torch.empty_like(x)

    def binned():
        eng.bin_queries(x.data_ptr(), y.data_ptr(), N, xb.data_ptr(), yb.data_ptr(), perm.data_ptr(),
                        off.data_ptr())

    def lookup():
        eng.bilinear_tiled(xb.data_ptr(), yb.data_ptr(), off.data_ptr(), h.data_ptr())

    def timed(fn):
        with torch.cuda.stream(stream):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                fn()
            e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / reps

    binned()
    torch.cuda.synchronize()
    ms = timed(lookup)
    ms_all = timed(lambda: (binned(), lookup()))
    alg = G * G * 4 + 12 * N
    # scattered lookup (no binning, corners through L1/L2) on the same unsorted points
    hq = torch.empty_like(x)
    eng.bilinear_query(x.data_ptr(), y.data_ptr(), hq.data_ptr(), N)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.bilinear_query(x.data_ptr(), y.data_ptr(), hq.data_ptr(), N)
    torch.cuda.synchronize()
    scat_ms = (time.perf_counter() - t0) * 1e3
    eng.close()
    achieved = alg / (ms * 1e-3) / 1e9
    achieved_all = alg / (ms_all * 1e-3) / 1e9
    return {"bound": "hbm", "kernel": "mppi_bilinear_tiled_kernel", "on_step_path": False,
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "kernel_avg_ms": round(ms, 4),
            "incl_binning_ms": round(ms_all, 4), "frac_incl_binning": round(achieved_all / HBM_PEAK_GBS, 4),
            "algorithmic_bytes_per_launch": alg,
            "workload": f"C5 tile {G}^2 DEM (synthetic), N={N} uniform queries binned by 128x128 tile",
            "scattered_query_ms": round(scat_ms, 3),
            "scattered_frac": round(alg / (scat_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


COSTMAP_BYTES_PER_CELL = 23   # occ 1+1+1, g2 4+4, d2 4+4, out 4 (csrc/mppi_costmap.hip)


def costmap_bench(device_index, reps=20, cpu=True):
    """Surface.create_obstacles_costmap (MPPI_isaac.py:361-378) on the GPU: a 1024^2 costmap (the C5
    map, grid 8192 / 8) from 750 rocks, HIP-event device time per build, with the reference's metric
    (cv2.distanceTransform(DIST_L2, 5): the 5x5 chamfer as 16 line scans; "chamfer_raster" the same
    map by the two row-serial raster passes on one workgroup) and the exact EDT option; the oracle
    (numpy restatement, 1 core) on the same input once for reference."""
    from mppi_amd import _lib
    rng = np.random.RandomState(99)
    rocks = [[rng.uniform(-95, 95), rng.uniform(-95, 95), rng.uniform(0.0, 0.8)] for _ in range(750)]
    size, hw = 1024, 102.4
    b = _lib.CostmapBuilder(device_index)
    rec = {"workload": "1024^2 costmap @0.2 m from 750 rocks (power 20)"}
    for metric in ("chamfer", "chamfer_raster", "exact"):
        for _ in range(3):
            b.build(rocks, (0.0, 0.0), size, hw, 1.2, metric=metric)
        dev_ms, t0 = 0.0, time.perf_counter()
        for _ in range(reps):
            b.build(rocks, (0.0, 0.0), size, hw, 1.2, metric=metric)
            dev_ms += b.last_ms()
        call_ms = (time.perf_counter() - t0) / reps * 1e3
        rec[metric] = {"kernel_ms": round(dev_ms / reps, 4), "call_ms_incl_d2h": round(call_ms, 3)}
    rec["exact"]["achieved_GBs"] = round(COSTMAP_BYTES_PER_CELL * size * size / (rec["exact"]["kernel_ms"] * 1e-3)
                                          / 1e9, 1)
    b.close()
    if cpu:
        from oracle import costmap_ref as CR
        t0 = time.perf_counter()
        CR.create_obstacles_costmap_cv(rocks, (0.0, 0.0), size, hw, 1.2)
        rec["cpu_oracle_chamfer_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    return rec


# ------------------------------------------------------------------ the MPPI step runs
_SCENES = {}


def get_scene(fn):
    if fn not in _SCENES:
        from mppi_amd import scene
        _SCENES[fn] = getattr(scene, fn)()
    return _SCENES[fn]


class Runner:
    """One rank's controller for one config: the sharded engine (torch.distributed, N>1), a C-ABI
    group over `devices` (one process, N>1) or a single-GPU engine."""

    def __init__(self, cfg, device, world, solo=False, devices=None):
        from mppi_amd import _lib
        from mppi_amd.distributed import ShardedMPPI
        K, H, scene_fn, start, goal, desc = CONFIGS[cfg]
        self.K, self.H, self.desc = K, H, desc
        self.world = 1 if solo else world
        self.sharded = self.group = None
        Z, hw, cm = get_scene(scene_fn)
        state = _lib.make_state(start[0], start[1], (1.0, 0.0, 0.0), goal_x=goal[0], goal_y=goal[1])
        if devices is not None and not solo:
            self.group = _lib.Group(_lib.make_params(K, H), devices)
            self.engines = self.group.members
            self.eng = self.engines[0]
            self.k_local = self.group.shard(0)[1]
        elif self.world > 1:
            self.sharded = ShardedMPPI(K, H, device)
            self.eng = self.sharded.engine
            self.engines = [self.eng]
            self.k_local = self.sharded.k_count
        else:
            self.eng = _lib.Engine(_lib.make_params(K, H), device)
            self.engines = [self.eng]
            self.k_local = K
        for e in self.engines:
            e.set_dem(Z, hw)
            e.set_costmap(cm, hw)
            e.set_state(state)

    def set_async_tail(self, on):
        for e in self.engines:
            e.set_async_tail(on)

    def outputs(self):
        return self.group.outputs() if self.group is not None else self.eng.outputs()

    def step(self, proj, i):
        if self.group is not None:
            self.group.step(proj, i, copy=False)
        elif self.sharded is not None:
            self.sharded.step(proj, i, copy=False)
        else:
            self.eng.step(proj, i, copy=False)

    def close(self):
        if self.group is not None:
            self.group.close()
        elif self.sharded is not None:
            self.sharded.close()
        else:
            self.eng.close()


def group_parity(cfg, devices, proj, steps=3):
    """The C-ABI group's outputs (member 0) against one context over the whole K, synchronous mode, a
    few chained steps: bitwise equal when every member holds a power-of-two number of 256-trajectory
    leaves (the member roots are then subtrees of the one-context record tree)."""
    g = Runner(cfg, devices[0], 1, devices=devices)
    one = Runner(cfg, devices[0], 1, solo=True)
    try:
        g.set_async_tail(False)
        one.set_async_tail(False)
        same = True
        for i in range(steps):
            a = g.group.step(proj, 500 + i, copy=True)
            b = one.eng.step(proj, 500 + i, copy=True)
            same &= all(np.array_equal(a[k], b[k]) for k in a)
    finally:
        g.close()
        one.close()
    return bool(same)


def timed_run(torch, dist, run, proj, warmup, steps, step0, async_tail, kernel_timing=False):
    """`warmup` untimed + `steps` timed MPPI steps, barrier + synchronize on both sides; returns
    the max-over-ranks wall time of the timed steps.  Kernel timing (if any) on the first
    member's / rank's engine."""
    eng = run.eng
    run.set_async_tail(async_tail)
    eng.set_timing(False)
    for i in range(warmup):
        run.step(proj, step0 + i)

    def barrier():
        for e in run.engines:  # stops a resident step server (mppi_sync), then syncs
            e.sync()
        for d in sorted({e.device for e in run.engines}):
            torch.cuda.synchronize(d)
        if dist is not None and run.world > 1:
            dist.barrier()
            torch.cuda.synchronize()

    eng.set_timing(kernel_timing)
    barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        run.step(proj, step0 + warmup + i)
    run.outputs()          # the last step's deferred optimal rollout is in host memory too
    barrier()
    el = time.perf_counter() - t0
    if dist is not None and run.world > 1:
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def shard_bench(torch, device, proj, steps=200, warmup=20):
    """One GPU's share of the 8-GPU C4 step: K = 131 072 of the 1 048 576, H = 100,
    as a K-sharded member runs it: partial step (rollout + the member's record), the record
    all-gather through RCCL (a one-member C-ABI group with the exchange forced, MPPI_GROUP_RCCL=1:
    comm init, ncclAllGather on the member's stream), then the finish over the gathered record; the
    plain one-context step at the same K beside it.  With 8 real ranks the all-gather moves 8
    records instead of 1 (1.6 KB each)."""
    from mppi_amd import _lib
    K, H, scene_fn, start, goal, _ = CONFIGS["c4s8"]
    Z, hw, cm = get_scene(scene_fn)
    state = _lib.make_state(start[0], start[1], (1.0, 0.0, 0.0), goal_x=goal[0], goal_y=goal[1])
    old = os.environ.get("MPPI_GROUP_RCCL")
    os.environ["MPPI_GROUP_RCCL"] = "1"
    try:
        g = _lib.Group(_lib.make_params(K, H), [device])
    finally:
        if old is None:
            os.environ.pop("MPPI_GROUP_RCCL", None)
        else:
            os.environ["MPPI_GROUP_RCCL"] = old
    one = _lib.Engine(_lib.make_params(K, H), device)
    rec = {"workload": CONFIGS["c4s8"][5] + ": partial step -> 1-rank RCCL all-gather -> finish",
           "rccl": bool(g.info().get("rccl"))}
    try:
        for e in g.members + [one]:
            e.set_dem(Z, hw)
            e.set_costmap(cm, hw)
            e.set_state(state)
            e.set_async_tail(True)
        for name, fn in (("sharded", lambda i: g.step(proj, i, copy=False)),
                         ("plain", lambda i: one.step(proj, i, copy=False))):
            for i in range(warmup):
                fn(i)
            torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            for i in range(steps):
                fn(warmup + i)
            g.outputs() if name == "sharded" else one.outputs()
            torch.cuda.synchronize(device)
            dt = (time.perf_counter() - t0) / steps
            rec[f"{name}_ms_per_step"] = round(dt * 1e3, 4)
            rec[f"{name}_steps_per_s"] = round(1.0 / dt, 2)
    finally:
        g.close()
        one.close()
    return rec


def cadence_bench(torch, device, proj, frames=40):
    """The drop-in controller at its production caller's cadence (visual_terrain_stack_full_terrain.py:
    466-541: MPPI_step, then world.step(render=True) on the same GPU, one frame per step).  Per frame:
    one MPPI step (latency = call -> controls in host memory), then a stand-in for the simulator's
    frame on a stream of its own: a 1 GiB device copy (HBM-bound) and a bf16 4096^3 GEMM (LDS-tiled
    library kernel), each timed with events, then the host waits out the rest of the frame gap.  Gaps
    of 2 ms and 16 ms; schedules ("resident" option): "default" (1: the server for back-to-back calls
    only, so at a frame cadence every step runs as separate launches), "server_always" (2, idle limit
    200 us: the server relaunched for every frame, round 5's default), "server_idle2000" (2, idle limit
    2 ms: round 4's default, whose idle server holds every CU's LDS past the step) and "separate" (0).
    `slowdown` = the stand-in kernels' time beside the schedule / alone.  C3 (the headline K) and
    K=1000 (config.yaml's number_of_trajectories).  Rows with "sim_first" launch the frame's stand-in
    BEFORE the step (the simulator's kernels still in flight when the controller is called).  Every
    schedule runs alone on a context of its own (frame-interleaved contexts share the process's
    hardware queues, and a step then queued behind another context's idle server); "default" and
    "separate" in A B B A order ("pass" 1 / 2)."""
    from mppi_amd import _lib
    dev = torch.device("cuda", device)
    src = torch.ones(1 << 28, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    A = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    B = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    sim = torch.cuda.Stream(device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]

    def world_launch():
        with torch.cuda.stream(sim):
            ev[0].record(sim)
            dst.copy_(src)
            ev[1].record(sim)
            torch.matmul(A, B)
            ev[2].record(sim)

    def world_wait():
        ev[2].synchronize()
        return ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])

    def world_step():
        world_launch()
        return world_wait()

    for _ in range(5):
        world_step()
    alone = np.median(np.array([world_step() for _ in range(20)]), axis=0)
    out = {"workload": "MPPI_step (3d, deferred optimal rollout) and a simulator frame stand-in on its own "
                       "stream (1 GiB copy + bf16 4096^3 GEMM), host waits out the frame gap",
           "alone_copy_ms": round(float(alone[0]), 4), "alone_gemm_ms": round(float(alone[1]), 4), "rows": []}
    Z, hw, cm = get_scene("scene_c3")
    start, goal = CONFIGS["c3"][3], CONFIGS["c3"][4]
    state = _lib.make_state(start[0], start[1], (1.0, 0.0, 0.0), goal_x=goal[0], goal_y=goal[1])
    keys = ("server_launches", "server_relaunches", "server_steps", "cadence_steps", "server_fallbacks")

    def engine(K, opts):
        eng = _lib.Engine(_lib.make_params(K, 100), device)
        for k, v in opts.items():
            eng.set_option(k, v)
        eng.set_dem(Z, hw)
        eng.set_costmap(cm, hw)
        eng.set_state(state)
        eng.set_async_tail(True)
        for i in range(10):
            eng.step(proj, i, copy=False)
        return eng

    def run(K, sched, opts, gap_ms, sim_first, rep):
        """One schedule alone on a context of its own (several contexts at once share the process's
        hardware queues: a step then queues behind another context's idle server)."""
        eng = engine(K, opts)
        lat, wk = [], []
        i0 = eng.launch_info()
        for f in range(frames):
            if sim_first:
                world_launch()
            t0 = time.perf_counter()
            eng.step(proj, 10 + f, copy=False)
            t1 = time.perf_counter()
            lat.append((t1 - t0) * 1e3)
            wk.append(world_wait() if sim_first else world_step())
            while (time.perf_counter() - t1) * 1e3 < gap_ms:
                time.sleep(0.0002)
        i1 = eng.launch_info()
        eng.close()
        w = np.median(np.array(wk), axis=0)
        la = np.array(lat)
        out["rows"].append({
            "K": K, "schedule": sched, "pass": rep, "sim_first": sim_first, "gap_ms": gap_ms, "frames": frames,
            "latency_ms_p50": round(float(np.median(la)), 4),
            "latency_ms_p90": round(float(np.percentile(la, 90)), 4),
            "copy_ms": round(float(w[0]), 4), "gemm_ms": round(float(w[1]), 4),
            "copy_slowdown": round(float(w[0] / alone[0]), 3),
            "gemm_slowdown": round(float(w[1] / alone[1]), 3),
            **{k: i1[k] - i0[k] for k in keys}})

    for K in (65536, 1000):
        for gap_ms in (2.0, 16.0):
            # default and separate in A B B A order (at a frame cadence they run the same launches)
            for rep, (sched, opts) in enumerate((("default", {}), ("separate", {"resident": 0}),
                                                 ("separate", {"resident": 0}), ("default", {}))):
                run(K, sched, opts, gap_ms, False, rep // 2 + 1)
            run(K, "server_always", {"resident": 2}, gap_ms, False, 1)
            run(K, "server_idle2000", {"resident": 2, "resident_idle_us": 2000}, gap_ms, False, 1)
        for rep, (sched, opts) in enumerate((("default", {}), ("separate", {"resident": 0}))):
            run(K, sched, opts, 2.0, True, 1)
    return out


def chain_static(path=os.path.join(ROOT, "profiles", "isa", "chain_count.json")):
    """The chain step's static instruction count (profiles/isa/chain_count.py) if it was taken
    from the current kernel sources, else None."""
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None
    return rec.get("instructions_per_step") if rec.get("src_sha256") == source_hash() else None


def pmc_traffic(path, kernel, K_local, H):
    """HBM bytes per launch of `kernel` from a committed rocprofv3 PMC summary, only if it was
    measured on the current kernel sources (src_sha256) at the same K and H; else None."""
    try:
        with open(path) as f:
            pm = json.load(f)
    except (OSError, ValueError):
        return None, "no PMC summary"
    if pm.get("src_sha256") != source_hash():
        return None, f"PMC summary is for other kernel sources ({pm.get('src_sha256')})"
    if pm.get("K") != K_local or pm.get("H") != H:
        return None, f"PMC summary is for K={pm.get('K')} H={pm.get('H')}"
    k = pm.get("kernels", {}).get(kernel, {})
    return k.get("hbm_bytes_per_launch"), f"profiles PMC at git {pm.get('git_head')}, src {pm.get('src_sha256')}"


def main():
    args = parse()
    # stdout carries the one JSON line only: libraries print banners there (RCCL's version banner at
    # communicator init, from the shard leg's group), so fd 1 goes to stderr until the line is written
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    devices = None   # the in-process group (mppi_group_create) over these devices
    if args.group_devices:
        devices = [int(d) for d in args.group_devices.split(",") if d.strip()]
    elif world == 1 and args.gpus > 1:
        devices = list(range(args.gpus))
    if devices is not None and world > 1:
        raise SystemExit("--group-devices / an in-process group is for a single process (no torch.distributed)")
    n_gpus = len(set(devices)) if devices is not None else world
    members = len(devices) if devices is not None else world
    cpu = None
    if world == 1 and devices is None and args.cpu_baseline_seconds > 0:
        # before anything touches the GPU: the fork pool's workers must not inherit a HIP context
        Z, hw, cm = get_scene("scene_c3")
        cpu = cpu_baseline(Z, hw, cm, CONFIGS["c3"][3], CONFIGS["c3"][4], args.cpu_baseline_seconds)
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        # rank r on GPU r; MPPI_BENCH_BACKEND=gloo (host-memory exchange) lets a one-GPU box rehearse
        # several ranks on its one device (RCCL refuses two ranks on one GPU)
        backend = os.environ.get("MPPI_BENCH_BACKEND", "nccl")
        local_rank %= max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local_rank)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)

    run = Runner(args.config, local_rank, world, devices=devices)
    group_info = run.group.info() if run.group is not None else None
    K, H = run.K, run.H
    # untimed: bring the GPU to its steady clock before the measured passes
    prewarm_steps = 0
    t_pw = time.perf_counter()
    run.set_async_tail(True)
    # (ranks of torch.distributed take the same fixed number of steps: every step has a collective)
    fixed = int(args.prewarm_ms) if world > 1 else None
    while (prewarm_steps < fixed) if fixed is not None else ((time.perf_counter() - t_pw) * 1e3 < args.prewarm_ms):
        run.step(args.proj, 1_000_000 + prewarm_steps)
        prewarm_steps += 1
    run.outputs()
    # synchronous MPPI_step semantics first (every output in host memory when step() returns)
    el_sync = None if args.no_sync_pass else timed_run(torch, dist, run, args.proj, args.warmup, args.steps, 0, False)
    # headline: the optimal rollout of step i (it only feeds trajectories_sim) overlaps step i+1;
    # every step's outputs still reach pinned host memory inside the timed region
    s0 = args.warmup + args.steps
    # the rollout kernel's HIP events (mode 2: two event records per step on the engine stream,
    # no host wait) in a pass of their own; --timed-events records them inside the timed region
    # (same kernel time within 0.5 %, but ~6 % fewer steps/s: profiles/r02_notes.md)
    nt = max(args.steps // 4, 10)
    srv0 = run.eng.server_time()
    el = timed_run(torch, dist, run, args.proj, args.warmup, args.steps, s0, not args.sync,
                   kernel_timing=2 if args.timed_events else 0)
    head_info = run.eng.launch_info()   # the schedule the timed steps ran on
    srv1 = run.eng.server_time()
    n_srv = srv1[2] - srv0[2]   # the server's own clock over that pass (its warm-up steps included)
    srv_roll_us = (srv1[0] - srv0[0]) / n_srv if n_srv > 0 else None
    srv_step_us = (srv1[1] - srv0[1]) / n_srv if n_srv > 0 else None
    if not args.timed_events:
        timed_run(torch, dist, run, args.proj, args.warmup, nt, 2 * s0, not args.sync, kernel_timing=2)
    roll_ms, _, n_roll = run.eng.timing()
    # the finish and the tail in a pass of their own (mode 1 waits for the stream and for each tail
    # on the host, which moves the tail onto the next rollout)
    timed_run(torch, dist, run, args.proj, args.warmup, nt, 3 * s0, not args.sync, kernel_timing=1)
    _, fin_ms, n_fin = run.eng.timing()
    tail_ms, n_tail = run.eng.tail_timing()
    info = run.eng.launch_info()
    clock = run.eng.chain_clock()   # the last rollout's chain wave: shader MHz and cycles per step
    record_bytes = run.eng.record_len() * 8
    k_local = run.k_local
    run.close()

    def solo_rate(cfg, steps):
        """rank 0 / member 0 alone, the whole config on its GPU (the N=1 reference of this job)."""
        r = Runner(cfg, devices[0] if devices is not None else local_rank, 1, solo=True)
        t = timed_run(torch, None, r, args.proj, args.warmup, steps, 0, not args.sync)
        r.close()
        return steps / t

    speedup = None
    if world > 1:
        dist.barrier()
        if rank == 0:
            speedup = (args.steps / el) / solo_rate(args.config, args.steps)
        dist.barrier()
    elif members > 1:
        speedup = (args.steps / el) / solo_rate(args.config, args.steps)
    parity = group_parity(args.config, devices, args.proj) if devices is not None and members > 1 else None

    c4 = None
    if not args.no_c4 and args.config != "c4":
        r4 = Runner("c4", local_rank, world, devices=devices)
        c4_steps = max(10, args.steps // 8)
        t4 = timed_run(torch, dist, r4, args.proj, min(args.warmup, 5), c4_steps, 0, not args.sync)
        r4.eng.set_timing(False)
        kl4 = r4.k_local
        r4.close()
        if world > 1:
            dist.barrier()
        c4 = {"workload": CONFIGS["c4"][5] + f", K-sharded over {members} member(s) on {n_gpus} GPU(s)",
              "global_K": CONFIGS["c4"][0], "k_per_gpu": kl4, "steps": c4_steps,
              "steps_per_s": round(c4_steps / t4, 3), "ms_per_step": round(t4 / c4_steps * 1e3, 4)}
        if world > 1:
            sp = None
            if rank == 0:
                sp = (c4_steps / t4) / solo_rate("c4", c4_steps)
                c4["speedup_vs_1"] = round(sp, 3)
            dist.barrier()
        elif members > 1:
            c4["speedup_vs_1"] = round((c4_steps / t4) / solo_rate("c4", c4_steps), 3)

    if world > 1:
        launcher = ("torch.distributed.run: one process per GPU, ShardedMPPI, all_gather_into_tensor over RCCL"
                    if dist.get_backend() == "nccl" else
                    f"torch.distributed.run, ShardedMPPI, {dist.get_backend()} exchange (rehearsal)")
        parallelism = (f"K-sharded dp{world}, one {'RCCL' if dist.get_backend() == 'nccl' else dist.get_backend()} "
                       f"all_gather of a {record_bytes}-byte record per rank per step")
    elif devices is not None:
        launcher = ("one process, C-ABI group (mppi_group_create), member threads" +
                    (", ncclCommInitAll + ncclAllGather" if group_info and group_info["rccl"] else
                     ", device-copy record exchange (members share a GPU)"))
        parallelism = (f"K-sharded over {members} members on {n_gpus} GPU(s), one all-gather of a "
                       f"{record_bytes}-byte record per member per step")
    else:
        launcher = "single process"
        parallelism = "single GPU"
    if rank == 0:
        steps_per_s = args.steps / el
        k_avg_ms = roll_ms / max(n_roll, 1)
        alg_bytes = BYTES_PER_ROLLOUT_STEP * k_local * H
        achieved = alg_bytes / (k_avg_ms * 1e-3) / 1e9
        # the rollout kernel the plan chose: role split (1024-thread workgroups) or pair (512); the
        # headline steps run its body inside the resident step server, the kernel time comes from
        # the separate-launch timing pass (the same rollout body, HIP events around each launch)
        kernel = "mppi_rollout_roles_kernel" if info.get("block") == 1024 else "mppi_rollout_pair_kernel"
        traffic, traffic_src = pmc_traffic(args.pmc_json, kernel, k_local, H)
        rec = {
            "metric": "MPPI steps/sec at K=65536 H=100 on 750x750 costmap; 1/2/4/8-GPU scaling",
            "value": round(steps_per_s, 3),
            "unit": "MPPI steps/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (reference crater + obstacle recipes; reference .npy blobs are absent)",
            "config": {
                "workload": f"{run.desc}, proj={args.proj}, outputs in host memory each step",
                "global_K": K,
                "k_per_gpu": k_local,
                "H": H,
                "parallelism": parallelism,
                "launcher": launcher,
                "group": group_info,
                # ranks of the communicator the records travel over (torch.distributed's, or the
                # C-ABI group's ncclCommCount; 0: device copies / one GPU)
                "rccl_ranks": (dist.get_world_size() if dist is not None and world > 1 and dist.get_backend() == "nccl"
                               else (group_info or {}).get("rccl_ranks", 0)),
                "record_bytes_per_rank": record_bytes,
                "speedup_vs_1": round(speedup, 3) if speedup is not None else None,
                "group_parity_bitwise": parity,
                "rollout_kernel": info,
                "pipelined_tail": not args.sync,
                "prewarm": {"ms": args.prewarm_ms, "steps": prewarm_steps},
                "sync_steps_per_s": round(args.steps / el_sync, 3) if el_sync else None,
                "sync_ms_per_step": round(el_sync / args.steps * 1e3, 4) if el_sync else None,
                "schedule": ("resident step server (mppi_step_server_kernel)" if head_info.get("resident")
                             else "separate launches (rollout, finish, deferred tail)"),
                "server_launches": head_info.get("server_launches"),
                "server_rollout_us": round(srv_roll_us, 2) if srv_roll_us else None,
                "server_step_us": round(srv_step_us, 2) if srv_step_us else None,
                "server_clock_steps": n_srv,
                "server_clock": "s_memrealtime on the server: command seen -> last rollout ticket / -> completion word, averaged",
                "finish_kernel_avg_ms": round(fin_ms / max(n_fin, 1), 5),
                "chain": {"instructions_per_step": chain_static(),
                          "cycles_per_step": round(clock["cycles_per_step"], 1),
                          "shader_clock_mhz": round(clock["shader_mhz"], 1),
                          "chain_us": round(clock["chain_us"], 2),
                          "wg0_start_to_chain_us": round(clock["start_to_chain_us"], 2),
                          "wg0_chain_to_roles_done_us": round(clock["chain_to_roles_done_us"], 2),
                          "wg0_leaf_us": round(clock["leaf_us"], 2),
                          "wg_start_spread_us": round(clock["wg_start_spread_us"], 2),
                          "wg_end_spread_us": round(clock["wg_end_spread_us"], 2),
                          "wg_span_us": round(clock["wg_span_us"], 2),
                          "source": "s_memtime / s_memrealtime of the chain wave of trajectories 0-63, last step"},
                "tail_kernel_avg_ms": round(tail_ms / n_tail, 5) if n_tail else None,
                "src_sha256": source_hash(),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": kernel,
                "kernel_avg_ms": round(k_avg_ms, 5),
                "kernel_timing": "HIP events around each launch of a separate-launch pass (mppi_set_timing(2)): "
                                 "the launch waits for the side streams' work, so no noise or tail kernel runs beside it",
                "algorithmic_bytes_per_launch": alg_bytes,
            },
        }
        if c4 is not None:
            rec["c4"] = c4
        # (the shard leg before the bilinear one: after the C4 and bilinear legs the plain K = 131 072
        # step of this leg measured 0.28-0.29 ms instead of 0.17, an interaction not reproduced with
        # either leg alone, profiles/r04_notes.md; the sharded step was unaffected)
        if world == 1 and devices is None and not args.no_shard:
            rec["c4_shard"] = shard_bench(torch, local_rank, args.proj)
        if world == 1 and devices is None and not args.no_cadence:
            rec["cadence"] = cadence_bench(torch, local_rank, args.proj)
        if world == 1 and devices is None and not args.no_bilinear:
            rec["bilinear_roofline"] = bilinear_bench(torch, torch.device("cuda", local_rank))
        if world == 1 and devices is None and not args.no_c5 and args.config != "c2":
            # C2 (SURVEY.md §8(d) reports C2-C5): the small config, latency-bound (the H-step chain)
            r2 = Runner("c2", local_rank, 1, solo=True)
            t2 = timed_run(torch, None, r2, args.proj, 20, 200, 0, not args.sync)
            r2.close()
            rec["c2"] = {"workload": CONFIGS["c2"][5], "steps_per_s": round(200 / t2, 3),
                         "ms_per_step": round(t2 / 200 * 1e3, 4)}
        if world == 1 and devices is None and not args.no_c5 and args.config != "c5":
            r5 = Runner("c5", local_rank, 1, solo=True)
            t5 = timed_run(torch, None, r5, args.proj, 10, 50, 0, not args.sync)
            timed_run(torch, None, r5, args.proj, 2, 10, 100, not args.sync, kernel_timing=True)
            roll5, fin5, n5 = r5.eng.timing()
            r5.close()
            k5 = roll5 / max(n5, 1)
            alg5 = BYTES_PER_ROLLOUT_STEP * CONFIGS["c5"][0] * CONFIGS["c5"][1]
            rec["c5"] = {"workload": CONFIGS["c5"][5], "steps_per_s": round(50 / t5, 3),
                         "ms_per_step": round(t5 / 50 * 1e3, 4), "rollout_kernel_avg_ms": round(k5, 4),
                         "finish_kernel_avg_ms": round(fin5 / max(n5, 1), 4),
                         "rollout_achieved_GBs": round(alg5 / (k5 * 1e-3) / 1e9, 1),
                         "rollout_frac_of_hbm_peak": round(alg5 / (k5 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        if world == 1 and devices is None and not args.no_costmap:
            rec["costmap_builder"] = costmap_bench(local_rank, cpu=args.cpu_baseline_seconds > 0)
        if cpu is not None:
            rec["cpu_baseline"] = cpu
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(rec) + "\n").encode())
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
