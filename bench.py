"""MPPI steps/s at K=65536, H=100 on the 750x750 costmap (BASELINE.json metric), 1..N GPUs.

One "step" = one full MPPI_step("3d") (thesis_master/warp_implementation/MPPI_isaac.py:505-720):
Philox sampling, wheel filter, 2.5D rollout, four critics, softmax-weighted
update, optimal filter and optimal rollout, with the outputs copied to host
memory.  Inputs (DEM, costmap, state) are resident in HBM before timing.

Scaling: weak.  Each rank owns K_per_gpu = 65536 trajectories (the headline
shard); the global sample count is 65536*N, exchanged once per step by one
RCCL all-gather of the per-rank softmax records.  `value` counts
K=65536-trajectory MPPI steps per second over the whole job (= N x global
steps/s).

Launch: python bench.py [--steps K --warmup W]  (N=1), or
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
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
START = (-60.0, -5.0)
GOAL = (65.0, 10.0)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--k-per-gpu", type=int, default=65536)
    ap.add_argument("--horizon", type=int, default=100)
    ap.add_argument("--proj", default="3d")
    ap.add_argument("--dem-path", default="auto", choices=["auto", "lds", "global", "ws", "pair"])
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0,
                    help="bounded oracle sample on the host (rank 0, N=1); 0 disables")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_latest.json"))
    ap.add_argument("--no-bilinear", action="store_true", help="skip the C5 tiled-lookup roofline leg")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 full-step leg (K=262144, H=128, 8192^2 DEM)")
    ap.add_argument("--no-costmap", action="store_true", help="skip the obstacle-costmap builder leg")
    ap.add_argument("--sync", action="store_true",
                    help="report the synchronous mode (no deferred optimal rollout) as the headline")
    return ap.parse_args()


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(Z, hw, cm, H, seconds):
    """Oracle (numpy, float32, one core) on the same workload: whole C3 steps until `seconds` elapse."""
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    from oracle import mppi_ref as R
    K = 65536
    p = R.Params(K=K, H=H)
    sc = R.Scene(Z, hw, cm)
    st = R.State(x=START[0], y=START[1], goal_x=GOAL[0], goal_y=GOAL[1])
    u1 = np.zeros(H, np.float32)
    u2 = np.zeros(H, np.float32)
    n = 0
    t0 = time.perf_counter()
    while True:
        out = R.mppi_step(p, sc, st, u1, u2, n)
        u1, u2 = out["u1_opt"], out["u2_opt"]
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or n >= 20:
            break
    return {"value": n / el, "unit": "MPPI steps/s", "cores": 1, "kind": "port",
            "sample": f"{n} full C3 steps (K={K}, H={H}) of oracle/mppi_ref.py in {el:.1f} s on 1 core "
                      f"of {cpu_model()} (os.cpu_count()={os.cpu_count()})"}


def bilinear_bench(torch, device, reps=20):
    """LDS-tiled DEM lookup at C5 size: 8192^2 DEM @0.025 m, N = 262144*128 queries.

    Queries uniform over the tile, binned by 64x64-cell tile once (untimed: inputs resident);
    `reps` launches of mppi_bilinear_tiled timed with HIP events on the engine's stream.
    Algorithmic bytes = the DEM once + 12 B per query (x, y in, h out).
    """
    from mppi_amd import _lib
    G, hw, N = 8192, 102.4, 262144 * 128
    res = 2 * hw / G
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
    perm = torch.empty(N, dtype=torch.int64, device=device)
    off = torch.empty(nt + 1, dtype=torch.int32, device=device)
    eng.bin_queries(x.data_ptr(), y.data_ptr(), N, xb.data_ptr(), yb.data_ptr(), perm.data_ptr(), off.data_ptr())
    del perm
    h = torch.empty_like(x)
    with torch.cuda.stream(stream):
        for _ in range(3):
            eng.bilinear_tiled(xb.data_ptr(), yb.data_ptr(), off.data_ptr(), h.data_ptr())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            eng.bilinear_tiled(xb.data_ptr(), yb.data_ptr(), off.data_ptr(), h.data_ptr())
        e1.record(stream)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    alg = G * G * 4 + 12 * N
    # scattered lookup (no binning, corners through L1/L2) on the same unsorted points, for reference
    hq = torch.empty_like(x)
    eng.bilinear_query(x.data_ptr(), y.data_ptr(), hq.data_ptr(), N)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.bilinear_query(x.data_ptr(), y.data_ptr(), hq.data_ptr(), N)
    scat_ms = (time.perf_counter() - t0) * 1e3
    eng.close()
    achieved = alg / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "kernel": "mppi_bilinear_tiled_kernel", "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
            "kernel_avg_ms": round(ms, 4), "algorithmic_bytes_per_launch": alg,
            "workload": f"C5 tile {G}^2 DEM (synthetic), N={N} uniform queries binned by 64x64 tile",
            "scattered_query_ms": round(scat_ms, 3)}


def c5_bench(device_index, steps=50, warmup=10):
    """Config C5 (BASELINE.json configs[4]) on one GPU: K=262144, H=128 on the 8192^2 DEM @0.025 m.

    Same step and timing as the headline (inputs resident, outputs in host memory every step,
    deferred optimal rollout); reported beside the headline, not as `value`.
    """
    from mppi_amd import _lib, scene
    Z, hw, cm = scene.scene_c5()
    K, H = 262144, 128
    eng = _lib.Engine(_lib.make_params(K, H), device_index)
    eng.set_dem(Z, hw)
    eng.set_costmap(cm, hw)
    eng.set_state(_lib.make_state(0.0, 0.0, (1.0, 0.0, 0.0), goal_x=80.0, goal_y=20.0))
    eng.set_async_tail(True)
    for i in range(warmup):
        eng.step("3d", i, copy=False)
    eng.sync()
    t0 = time.perf_counter()
    for i in range(steps):
        eng.step("3d", warmup + i, copy=False)
    eng.outputs()
    eng.sync()
    el = time.perf_counter() - t0
    eng.set_timing(True)
    for i in range(10):
        eng.step("3d", warmup + steps + i, copy=False)
    eng.outputs()
    roll_ms, fin_ms, n = eng.timing()
    eng.close()
    k_ms = roll_ms / max(n, 1)
    alg = BYTES_PER_ROLLOUT_STEP * K * H
    return {"workload": "C5: K=262144, H=128, 8192^2 DEM @0.025 m (synthetic craters + fBm), 1024^2 costmap",
            "steps_per_s": round(steps / el, 3), "ms_per_step": round(el / steps * 1e3, 4),
            "rollout_kernel_avg_ms": round(k_ms, 4), "finish_kernel_avg_ms": round(fin_ms / max(n, 1), 4),
            "rollout_achieved_GBs": round(alg / (k_ms * 1e-3) / 1e9, 1),
            "rollout_frac_of_hbm_peak": round(alg / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


COSTMAP_BYTES_PER_CELL = 23   # occ 1+1+1, g2 4+4, d2 4+4, out 4 (csrc/mppi_costmap.hip)


def costmap_bench(device_index, reps=20, cpu=True):
    """Surface.create_obstacles_costmap (MPPI_isaac.py:361-378) on the GPU: a 1024^2 costmap (the C5
    map, grid 8192 / 8) from 750 rocks, HIP-event device time per build; the oracle (numpy raster +
    scipy exact EDT, 1 core) on the same input once for reference."""
    from mppi_amd import _lib
    rng = np.random.RandomState(99)
    rocks = [[rng.uniform(-95, 95), rng.uniform(-95, 95), rng.uniform(0.0, 0.8)] for _ in range(750)]
    size, hw = 1024, 102.4
    b = _lib.CostmapBuilder(device_index)
    for _ in range(3):
        b.build(rocks, (0.0, 0.0), size, hw, 1.2)
    dev_ms, t0 = 0.0, time.perf_counter()
    for _ in range(reps):
        b.build(rocks, (0.0, 0.0), size, hw, 1.2)
        dev_ms += b.last_ms()
    call_ms = (time.perf_counter() - t0) / reps * 1e3
    b.close()
    dev_ms /= reps
    rec = {"workload": "1024^2 costmap @0.2 m from 750 rocks (exact EDT, power 20)",
           "kernel_ms": round(dev_ms, 4), "call_ms_incl_d2h": round(call_ms, 3),
           "achieved_GBs": round(COSTMAP_BYTES_PER_CELL * size * size / (dev_ms * 1e-3) / 1e9, 1)}
    if cpu:
        from oracle import costmap_ref as CR
        t0 = time.perf_counter()
        CR.create_obstacles_costmap(rocks, (0.0, 0.0), size, hw, 1.2)
        rec["cpu_oracle_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    return rec


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        if "WORLD_SIZE" not in os.environ and args.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run (one rank per GPU)")
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    from mppi_amd import _lib, scene
    from mppi_amd.distributed import ShardedMPPI
    Z, hw, cm = scene.scene_c3()
    H = args.horizon
    Kl = args.k_per_gpu
    if Kl % 256:
        raise SystemExit("--k-per-gpu must be a multiple of 256 (reduction leaf)")
    # rank r owns trajectories [r*Kl, (r+1)*Kl) of the global K = Kl*world (shard_bounds)
    sharded = ShardedMPPI(Kl * world, H, local_rank) if world > 1 else None
    eng = sharded.engine if sharded is not None else _lib.Engine(_lib.make_params(Kl, H), local_rank)
    eng.set_dem_path(args.dem_path)
    eng.set_dem(Z, hw)
    eng.set_costmap(cm, hw)
    eng.set_state(_lib.make_state(START[0], START[1], (1.0, 0.0, 0.0), goal_x=GOAL[0], goal_y=GOAL[1]))

    if sharded is not None:
        def one_step(i):
            sharded.step(args.proj, i, copy=False)
    else:
        def one_step(i):
            eng.step(args.proj, i, copy=False)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def timed_run(async_tail, step0, steps, kernel_timing=False):
        """W warmup + `steps` timed MPPI steps; returns the max-over-ranks wall time."""
        eng.set_async_tail(async_tail)
        eng.set_timing(False)
        for i in range(args.warmup):
            one_step(step0 + i)
        eng.set_timing(kernel_timing)
        barrier()
        t0 = time.perf_counter()
        for i in range(steps):
            one_step(step0 + args.warmup + i)
        eng.outputs()         # the last step's deferred optimal rollout is in host memory too
        barrier()
        el = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([el], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # synchronous MPPI_step semantics first (every output in host memory when step() returns)
    el_sync = timed_run(False, 0, args.steps)
    # headline: the optimal rollout of step i (it only feeds trajectories_sim) overlaps step i+1;
    # every step's outputs still reach pinned host memory inside the timed region
    el = timed_run(not args.sync, args.warmup + args.steps, args.steps)
    # per-kernel HIP-event times in a separate pass (events add stream work of their own)
    timed_run(not args.sync, 2 * (args.warmup + args.steps), max(args.steps // 4, 10), kernel_timing=True)
    roll_ms, fin_ms, n_roll = eng.timing()
    tail_ms, n_tail = eng.tail_timing()
    info = eng.launch_info()

    if rank == 0:
        steps_per_s = args.steps / el
        value = steps_per_s * world * Kl / 65536.0
        k_avg_ms = roll_ms / max(n_roll, 1)
        alg_bytes = BYTES_PER_ROLLOUT_STEP * Kl * H
        achieved = alg_bytes / (k_avg_ms * 1e-3) / 1e9
        traffic = None
        if os.path.exists(args.pmc_json):
            try:
                with open(args.pmc_json) as f:
                    pm = json.load(f)
                if pm.get("K") == Kl and pm.get("H") == H:
                    traffic = pm.get("hbm_bytes_per_launch")
            except (OSError, ValueError):
                traffic = None
        rec = {
            "metric": "MPPI steps/sec at K=65536 H=100 on 750x750 costmap; 1/2/4/8-GPU scaling",
            "value": round(value, 3),
            "unit": "MPPI steps/s (K=65536-trajectory steps)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (reference crater + obstacle recipes; reference .npy blobs are absent)",
            "config": {
                "workload": f"C3: K={Kl} per GPU (global K={Kl * world}), H={H}, 1500^2 DEM @0.1 m, "
                            f"750^2 costmap @0.2 m, proj={args.proj}, outputs in host memory each step",
                "global_K": Kl * world,
                "H": H,
                "parallelism": f"K-sharded dp{world}, one RCCL all_gather per step" if world > 1 else "single GPU",
                "rollout_kernel": info,
                "global_steps_per_s": round(steps_per_s, 3),
                "pipelined_tail": not args.sync,
                "sync_steps_per_s": round(args.steps / el_sync, 3),
                "sync_ms_per_step": round(el_sync / args.steps * 1e3, 4),
                "finish_kernel_avg_ms": round(fin_ms / max(n_roll, 1), 5),
                "tail_kernel_avg_ms": round(tail_ms / n_tail, 5) if n_tail else None,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": {"auto": "mppi_rollout_pair_kernel", "pair": "mppi_rollout_pair_kernel",
                           "ws": "mppi_rollout_ws_kernel"}.get(args.dem_path, "mppi_rollout_kernel"),
                "kernel_avg_ms": round(k_avg_ms, 5),
                "algorithmic_bytes_per_launch": alg_bytes,
            },
        }
        if world == 1 and not args.no_bilinear:
            rec["bilinear_roofline"] = bilinear_bench(torch, torch.device("cuda", local_rank))
        if world == 1 and not args.no_c5:
            rec["c5"] = c5_bench(local_rank)
        if world == 1 and not args.no_costmap:
            rec["costmap_builder"] = costmap_bench(local_rank, cpu=args.cpu_baseline_seconds > 0)
        if world == 1 and args.cpu_baseline_seconds > 0:
            rec["cpu_baseline"] = cpu_baseline(Z, hw, cm, H, args.cpu_baseline_seconds)
        print(json.dumps(rec), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
