"""Generate the committed golden fixtures under tests/golden/.

Run in the BUILD container only (it needs /root/reference and hipcc):

    MPLBACKEND=Agg PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Outputs (data only; no reference source is stored):

ref_primitives.npz
    Inputs and outputs of the reference's numpy model
    thesis_master/python_mppi_projection/debug.py, imported from the read-only
    reference tree: normal_on_grid (:200-216), get_heading_tangent_vector
    (:218-232), update_position incl. scipy rotvec rotation (:259-290) and
    bilinear_interpolator (:234-257, sampled on x, y >= 0 where its floor equals
    the Warp kernel's trunc).  Inputs are float32-representable so the oracle
    sees the same operands; outputs are the reference's float64 results.

philox_rocrand.txt
    rocRAND Philox4x32-10 known answers (philox_kat.cpp, compiled here with
    hipcc and run on the host): seed, subsequence, block, 4 x uint32.

python25d.npz
    Whole trajectories of the reference's numpy integrator
    debug.generate_trajectory_25D (debug.py:312-364), imported from the
    read-only reference tree, on its own 400^2 scene (Z stored as float32):
    the fixture for the HIP "python25d" reference-integrator mode.

step_small.npz
    Regression vectors of the CPU restatement (oracle/mppi_ref.py) for whole
    MPPI steps on a small self-contained scene (200^2 DEM, 25^2 costmap stored
    in the file): 3D/2D, far/near goal, injected controls, ragged K and odd H.
    These are NOT reference outputs (Warp cannot run offline); they freeze the
    restatement that the primitives above pin, and the GPU tests compare the
    HIP engine with them bit for bit.
"""
from __future__ import annotations

import importlib.util
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "husky-rover-mppi-isaacsim_amd"))

REF_DEBUG = "/root/reference/thesis_master/python_mppi_projection/debug.py"


def _f32(a):
    return np.asarray(a, np.float32).astype(np.float64)


def load_debug():
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.dont_write_bytecode = True
    spec = importlib.util.spec_from_file_location("ref_debug", REF_DEBUG)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)      # module body runs its own 200-step demo (prints 3 lines)
    return mod


def make_primitives(n=512, seed=2026):
    dbg = load_debug()
    rng = np.random.default_rng(seed)
    out = {}
    # --- normal_on_grid
    q = _f32(rng.uniform(-3.0, 3.0, (n, 2, 2)))
    res = _f32(rng.choice([0.1, 0.025, 0.5], n))
    out["normal_q"] = q
    out["normal_res"] = res
    out["normal_out"] = np.stack([dbg.normal_on_grid(q[i], res[i]) for i in range(n)])
    # --- get_heading_tangent_vector
    nv = rng.normal(size=(n, 3))
    nv[:, 2] = np.abs(nv[:, 2]) + 1.0
    nv = _f32(nv / np.linalg.norm(nv, axis=1, keepdims=True))
    hv = _f32(rng.normal(size=(n, 3)))
    out["tangent_n"] = nv
    out["tangent_h"] = hv
    out["tangent_out"] = np.stack([dbg.get_heading_tangent_vector(nv[i], hv[i]) for i in range(n)])
    # --- update_position (translation + scipy rotvec rotation about the normal)
    x = _f32(rng.uniform(-50, 50, n))
    y = _f32(rng.uniform(-50, 50, n))
    v = _f32(rng.uniform(0.0, 2.0, n))
    w = _f32(rng.uniform(-1.0, 1.0, n))
    dt = _f32(rng.choice([0.045, 0.05, 0.1], n))
    out.update(rot_x=x, rot_y=y, rot_h=hv, rot_v=v, rot_w=w, rot_n=nv, rot_dt=dt)
    res_xy = np.zeros((n, 2))
    res_h = np.zeros((n, 3))
    for i in range(n):
        nx, ny, nh = dbg.update_position(x[i], y[i], hv[i].copy(), v[i], w[i], nv[i], dt[i])
        res_xy[i] = (nx, ny)
        res_h[i] = nh
    out["rot_out_xy"] = res_xy
    out["rot_out_h"] = res_h
    # --- bilinear_interpolator on x, y >= 0
    bx = _f32(rng.uniform(0.0, 40.0, n))
    by = _f32(rng.uniform(0.0, 40.0, n))
    bq = _f32(rng.uniform(-3.0, 3.0, (n, 2, 2)))
    bres = _f32(rng.choice([0.1, 0.025, 0.5], n))
    out.update(bil_x=bx, bil_y=by, bil_q=bq, bil_res=bres)
    out["bil_out"] = np.array([dbg.bilinear_interpolator(bx[i], by[i], bq[i], bres[i]) for i in range(n)])
    np.savez_compressed(os.path.join(HERE, "ref_primitives.npz"), **out)
    print("ref_primitives.npz:", n, "cases per primitive")


def make_philox():
    src = os.path.join(HERE, "philox_kat.cpp")
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "philox_kat")
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O1", src, "-o", exe])
        txt = subprocess.check_output([exe], text=True)
    with open(os.path.join(HERE, "philox_rocrand.txt"), "w") as f:
        f.write("# seed subsequence block r0 r1 r2 r3  (rocrand4 after rocrand_init(seed, k, 4*block))\n")
        f.write(txt)
    print("philox_rocrand.txt:", len(txt.splitlines()), "vectors")


SMALL_BUMPS = [((-3.0, -4.0), 2.4, 3.1), ((4.0, 2.5), 3.2, 2.6), ((-1.0, 6.0), 1.8, 2.2)]


def small_scene():
    from mppi_amd import scene
    Z = scene.crater_dem(200, 10.0, SMALL_BUMPS)
    obs = scene.random_obstacles(n=12, seed=5, extent=8.0, r_max=0.6)
    cm = scene.disc_costmap(25, 10.0, obs, inflate=0.5, power=10)
    return Z.astype(np.float32), 10.0, cm.astype(np.float32)


# name -> (K, H, proj, step, start(x,y), heading, wheels(l,r), goal, sigma, nominal seed, injected)
STEP_CASES = {
    "far3d": (256, 20, "3d", 0, (-6.0, -1.0), (1.0, 0.2, 0.0), (0.0, 0.0), (7.0, 3.0), (0.25, 0.25), None, False),
    "near3d": (512, 20, "3d", 3, (1.0, 1.0), (0.3, 1.0, 0.0), (0.4, 0.6), (1.9, 1.5), (0.4, 0.45), 11, False),
    "twod": (256, 20, "2d", 1, (-5.0, 2.0), (1.0, -0.5, 0.0), (0.2, 0.1), (6.0, -4.0), (0.25, 0.25), 12, False),
    "ragged": (300, 7, "3d", 5, (0.5, -7.0), (0.0, 1.0, 0.0), (0.0, 0.0), (0.0, 8.0), (0.3, 0.2), 13, False),
    "injected": (256, 16, "3d", 0, (-2.0, -2.0), (1.0, 1.0, 0.0), (0.1, 0.3), (8.0, 8.0), (0.25, 0.25), None, True),
}


def run_step_case(name, Z, hw, cm):
    from oracle import mppi_ref as R
    K, H, proj, step, start, heading, wheels, goal, sigma, nom_seed, inj = STEP_CASES[name]
    p = R.Params(K=K, H=H, seed=42)
    sc = R.Scene(Z, hw, cm)
    st = R.State(x=start[0], y=start[1], heading=np.asarray(heading, float), left_wheel_speed=wheels[0],
                 right_wheel_speed=wheels[1], goal_x=goal[0], goal_y=goal[1], std_dev_u1=sigma[0],
                 std_dev_u2=sigma[1])
    if nom_seed is None:
        u1n = np.zeros(H, np.float32)
        u2n = np.zeros(H, np.float32)
    else:
        r = np.random.default_rng(nom_seed)
        u1n = r.uniform(-0.8, 0.8, H).astype(np.float32)
        u2n = r.uniform(-0.8, 0.8, H).astype(np.float32)
    injected = None
    if inj:
        r = np.random.default_rng(99)
        injected = (r.uniform(-1, 1, (K, H)).astype(np.float32), r.uniform(-1, 1, (K, H)).astype(np.float32))
    out = R.mppi_step(p, sc, st, u1n, u2n, step, proj, injected)
    rec = dict(u_nom1=u1n, u_nom2=u2n, u1_opt=out["u1_opt"], u2_opt=out["u2_opt"], v_opt=out["v_opt"],
               w_opt=out["w_opt"], traj_sim=out["traj_sim"], hv_sim=out["hv_sim"], lw_sim=out["lw_sim"],
               rw_sim=out["rw_sim"], cost=out["cost"], root=out["root"])
    if inj:
        rec["inj_u1"], rec["inj_u2"] = injected
    return rec


def make_steps():
    Z, hw, cm = small_scene()
    data = dict(Z=Z, cm=cm, hw=np.float64(hw))
    for name in STEP_CASES:
        for k, v in run_step_case(name, Z, hw, cm).items():
            data[f"{name}/{k}"] = v
    np.savez_compressed(os.path.join(HERE, "step_small.npz"), **data)
    print("step_small.npz:", list(STEP_CASES))


# python25d cases: (K, H, dt, start extent, v range, w step std, seed)
P25_CASES = {
    "demo": (40, 250, 0.01, 15.0, (0.5, 2.5), 0.05, 11),
    "escape": (24, 200, 0.045, 12.0, (1.5, 2.5), 0.1, 12),
}


def make_python25d():
    """Whole trajectories of the reference's numpy integrator debug.generate_trajectory_25D
    (debug.py:312-364) on its own 400^2 / 20 m scene (module globals X, Y, Z, resolution;
    Z rounded to float32 so the GPU sees the same heights).  Velocity sequences are seeded
    random walks in the style of generate_linear/angular_velocities (:415-461).  A trajectory
    for which the reference raises IndexError (x or y in [19.9, 20): its i+1 / j+1 corner is
    past the grid) is redrawn; one it returns None for is stored with valid = False."""
    dbg = load_debug()
    Z32 = np.asarray(dbg.Z, np.float32)
    Zr = Z32.astype(np.float64)
    data = {"Z": Z32, "hw": np.float64(dbg.half_width), "res": np.float64(dbg.resolution),
            "grid": np.int64(Z32.shape[0])}
    for name, (K, H, dt, ext, vr, wstd, seed) in P25_CASES.items():
        rng = np.random.default_rng(seed)
        rows = {k: [] for k in ("x0", "y0", "heading", "v", "w", "traj", "valid")}
        while len(rows["x0"]) < K:
            x0, y0 = rng.uniform(-ext, ext, 2)
            hd = np.array([rng.normal(), rng.normal(), 0.0])
            v = np.clip(rng.uniform(*vr) + np.cumsum(rng.normal(0, 0.1, H)), vr[0], vr[1])
            w = np.clip(np.cumsum(rng.normal(0, wstd, H)), -0.5, 0.5)
            try:
                tr = dbg.generate_trajectory_25D(x0, y0, hd.copy(), v, w, dt, H, dbg.resolution, dbg.X, dbg.Y, Zr)
            except IndexError:
                continue
            rows["x0"].append(x0)
            rows["y0"].append(y0)
            rows["heading"].append(hd)
            rows["v"].append(v)
            rows["w"].append(w)
            rows["valid"].append(tr is not None)
            rows["traj"].append(np.zeros((H, 3)) if tr is None else tr)
        for k, val in rows.items():
            data[f"{name}/{k}"] = np.asarray(val)
        data[f"{name}/dt"] = np.float64(dt)
        print(f"python25d {name}: K={K} H={H} valid={int(np.sum(rows['valid']))}")
    np.savez_compressed(os.path.join(HERE, "python25d.npz"), **data)


if __name__ == "__main__":
    which = sys.argv[1:] or ["primitives", "philox", "steps", "python25d"]
    if "python25d" in which:
        make_python25d()
    if "primitives" in which:
        make_primitives()
    if "philox" in which:
        make_philox()
    if "steps" in which:
        make_steps()
