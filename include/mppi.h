/*
 * mppi.h — C-ABI of the MI355X MPPI rollout-and-cost engine (libmppi_hip.so).
 *
 * Drop-in boundary for the Warp MPPI step of
 * thesis_master/warp_implementation/MPPI_isaac.py (reference, read-only).
 * Plain C types only: host pointers + sizes, device pointers only where the
 * caller already owns device memory (zero-copy DEM binding, rank records).
 *
 * Conventions
 *   status:   every int-returning call returns MPPI_OK (0) or a negative
 *             code; mppi_last_error() (thread-local) holds the message.
 *   memory:   the caller owns host buffers (copied in/out); the library owns
 *             its device buffers and pinned staging.
 *   threads:  one context per device; calls on one context are serialised
 *             by the caller (the reference is single-threaded, driven from
 *             the Isaac main loop, visual_terrain_stack_full_terrain.py:466).
 *   sync:     mppi_step / mppi_step_finish / mppi_step_injected return with
 *             the outputs in host memory (the reference's .numpy() reads,
 *             MPPI_isaac.py:769-775 / visual_terrain_stack_full_terrain.py:471-472).
 */
#ifndef HUSKY_MPPI_H
#define HUSKY_MPPI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPPI_ABI_VERSION 1

enum mppi_status {
  MPPI_OK = 0,
  MPPI_EINVAL = -1, /* bad argument (reference: Warp raises on bad launch inputs) */
  MPPI_EHIP = -2,   /* HIP runtime error (device fault, OOM, no device) */
  MPPI_ESTATE = -3, /* call out of order (e.g. step before set_dem) */
};

enum mppi_proj {
  MPPI_PROJ_2D = 2, /* projection_warp.py:353-382 (_generate_trajectories_2D_kernel) */
  MPPI_PROJ_3D = 3, /* projection_warp.py:284-350 (_generate_trajectories_kernel)    */
};

typedef struct mppi_ctx mppi_ctx;

/* Controller parameters.  Replaces MPPI_Controller.__init__ config parsing
 * (MPPI_isaac.py:404-440, config.yaml) and the constants hard-coded at
 * MPPI_isaac.py:548-549,688-689, projection_warp.py:333,
 * critics_warp.py:251-253,325-329.  Float fields are used as float32, the
 * precision the Warp kernels receive them in. */
typedef struct mppi_params {
  int64_t num_trajectories; /* trajectories of THIS context (its shard of K)         */
  int64_t k_offset;         /* global index of this shard's first trajectory          */
  int32_t num_iterations;   /* H (config.yaml controller.number_of_iterations)        */
  int32_t reserved0;
  float dt;                 /* config.yaml controller.dt                              */
  float robot_radius;       /* r_wheels of _convert_inputs_to_velocities (frame_work.robot_radius) */
  float min_u1, max_u1, min_u2, max_u2;                    /* config.yaml inputs.*       */
  float v_min_linear, v_max_linear, v_min_angular, v_max_angular; /* velocities.*        */
  float temperature;        /* cost_evaluation.temperature                            */
  float filter_k, filter_a;         /* rollout wheel filter, MPPI_isaac.py:548-549 (3.5, 0.96) */
  float opt_filter_k, opt_filter_a; /* optimal-sequence filter, MPPI_isaac.py:688-689 (3.0, 0.92) */
  float wheel_offset;       /* projection_warp.py:333 (0.2)                           */
  float w_path, w_slope, w_speed, w_obstacle; /* critics_warp.py:325-329               */
  float collision_threshold, collision_penalty; /* critics_warp.py:251-253 (0.99, 1e5) */
  float horizon;            /* MPPI_isaac.py:440 dt*v_max*H (computed by the caller in float64) */
  uint64_t seed;            /* Philox key (replaces default_rng(42).integers, MPPI_isaac.py:409,517) */
} mppi_params;

/* Per-step robot / goal state: the values MPPI_step reads from the controller
 * (MPPI_isaac.py:489-503 reset("controller"), :538-539, :611-613, :510-511 of
 * the Isaac loop).  heading is normalised by the caller (MPPI_isaac.py:493). */
typedef struct mppi_state {
  float x, y;
  float heading[3];
  float left_wheel_speed, right_wheel_speed;
  float goal_x, goal_y;
  float std_dev_u1, std_dev_u2;
} mppi_state;

/* Host output pointers (any may be NULL).  Each replaces one Warp array the
 * caller reads with .numpy() after MPPI_step (MPPI_isaac.py:446-487). */
typedef struct mppi_outputs {
  float* u1_opt;          /* [H]   optimal_u1_wp                         */
  float* u2_opt;          /* [H]   optimal_u2_wp                         */
  float* lin_vel;         /* [H]   optimal_lin_vel_wp                    */
  float* ang_vel;         /* [H]   optimal_ang_vel_wp                    */
  float* traj_sim;        /* [H*3] trajectories_sim                      */
  float* heading_sim;     /* [H*3] heading_vectors_sim                   */
  float* left_wheel_sim;  /* [H*3] left_wheel_pos_sim                    */
  float* right_wheel_sim; /* [H*3] right_wheel_pos_sim                   */
} mppi_outputs;

int mppi_abi_version(void);
const char* mppi_last_error(void);

/* MPPI_Controller.__init__ + warp_setup (MPPI_isaac.py:404-487): allocate
 * device buffers on `device`; nominal controls start at zero (:446-447). */
int mppi_create(const mppi_params* params, int32_t device, mppi_ctx** out);
void mppi_destroy(mppi_ctx* ctx);

/* Run on the caller's HIP stream (e.g. torch.cuda.current_stream()); NULL = own stream. */
int mppi_set_stream(mppi_ctx* ctx, void* hip_stream);

/* self.Z_wp = wp.array(surface.Z.flatten()) (MPPI_isaac.py:460): copies the
 * row-major rows x cols DEM to the device.  x_min = y_min = -half_width and
 * resolution = 2*half_width/grid_size as in the launch args (:560-564).
 * rows * cols < 2^29 (MPPI_EINVAL otherwise). */
int mppi_set_dem(mppi_ctx* ctx, const float* z_host, int32_t rows, int32_t cols, float x_min,
                 float y_min, float resolution);

/* controller.Z_wp = DEM_warp rebinding (visual_terrain_stack_full_terrain.py:567):
 * binds a DEM already resident in device memory (zero copy; the caller keeps
 * it alive while steps run).  Waits for every stream of the device (the DEM may
 * have been written on any of them), then derives the per-cell normal table the
 * rollout reads from it. */
int mppi_set_dem_device(mppi_ctx* ctx, const float* z_device, int32_t rows, int32_t cols,
                        float x_min, float y_min, float resolution);

/* The bound DEM was written in place (the terrain manager's dem_wp.assign(...),
 * geometry_clipmaps.py:293): waits for every stream of the device and rebuilds
 * the per-cell normal table from the current heights.  The reference's kernels
 * read the live DEM at every step; here the table is derived, so an in-place
 * write without this call (or a rebinding) leaves the normals of the old
 * heights.  MPPI_EINVAL when no DEM is bound. */
int mppi_dem_updated(mppi_ctx* ctx);

/* self.costmap_wp (MPPI_isaac.py:461) / costmap_wp.assign(...)
 * (visual_terrain_stack_full_terrain.py:563): size x size row-major costmap;
 * half_width and costmap resolution as passed at MPPI_isaac.py:622-624. */
int mppi_set_costmap(mppi_ctx* ctx, const float* costmap_host, int32_t size, float half_width,
                     float resolution);

/* ---- on-device obstacle costmap ----
 * Surface.create_obstacles_costmap(obstacles, origin) (MPPI_isaac.py:361-378),
 * re-run by the Isaac loop on every high-resolution block change and then
 * uploaded with costmap_wp.assign (visual_terrain_stack_full_terrain.py:561-563).
 * obstacles: n rows of (x_global, y_global, r_obs) float64, host memory.  Per
 * obstacle the disc x_local = y_global - y0, y_local = x_global - x0, radius
 * r_obs/2 + r_robot + 0.1 is marked on the size x size grid
 * X, Y = meshgrid(linspace(-half_width, half_width, size)) (float64, as the
 * reference); then the distance to the nearest marked cell, min-max normalised,
 * (1 - d)^power (the reference: 20), float32.  metric MPPI_COSTMAP_CHAMFER5 (the
 * reference's cv2.distanceTransform(DIST_L2, 5), :374): OpenCV's published
 * 5x5 chamfer (distanceTransform_5x5, 16.16 fixed point; computed as 16
 * independent line scans), cv2.normalize NORM_MINMAX as
 * OpenCV 4.x's float32 path (float scale / shift, one fma), (1 - d) in
 * float32, the power correctly rounded (oracle/costmap_ref.py; parity
 * unpinned: cv2 is unavailable).  MPPI_COSTMAP_CHAMFER5_RASTER: the same map
 * by the two row-serial raster passes on one workgroup (diagnostic / A-B).
 * MPPI_COSTMAP_EXACT: exact Euclidean distance, float64 normalise + power, one
 * rounding; no obstacle at all gives an all-1 map.
 * 2 <= size <= 8192.
 *
 * mppi_build_costmap builds straight into the context's costmap (what the
 * reference's create + assign pair leaves in costmap_wp; resolution becomes
 * 2*half_width/size, MPPI_isaac.py:272) and, if out_host != NULL, also copies
 * it to out_host [size*size] (the ndarray the reference returns).  Synchronous.
 * The builder object does the same without a controller context. */
enum mppi_costmap_metric {
  MPPI_COSTMAP_CHAMFER5 = 0, /* cv2.distanceTransform(DIST_L2, 5), MPPI_isaac.py:374 (default) */
  MPPI_COSTMAP_EXACT = 1,    /* exact Euclidean distance transform */
  MPPI_COSTMAP_CHAMFER5_RASTER = 2, /* CHAMFER5 by the raster passes (same result, slower) */
};
typedef struct mppi_costmap_builder mppi_costmap_builder;
int mppi_build_costmap(mppi_ctx* ctx, const double* obstacles, int32_t n, int32_t size,
                       double half_width, double origin_x, double origin_y, double r_robot,
                       int32_t power, float* out_host, int32_t metric);
int mppi_costmap_builder_create(int32_t device, mppi_costmap_builder** out);
void mppi_costmap_builder_destroy(mppi_costmap_builder* b);
/* out_host [size*size] (host) or out_device [size*size] (device memory); either may be NULL. */
int mppi_costmap_builder_build(mppi_costmap_builder* b, const double* obstacles, int32_t n,
                               int32_t size, double half_width, double origin_x, double origin_y,
                               double r_robot, int32_t power, float* out_host, float* out_device,
                               int32_t metric);
/* Device time (HIP events) of the builder's last build, in milliseconds. */
int mppi_costmap_builder_last_ms(mppi_costmap_builder* b, double* ms);

/* reset("controller") (MPPI_isaac.py:489-497) + the robot/goal/sigma fields MPPI_step reads. */
int mppi_set_state(mppi_ctx* ctx, const mppi_state* state);

/* optimal_u1_wp / optimal_u2_wp as the next step's nominal sequence (MPPI_isaac.py:518-519). */
int mppi_set_nominal(mppi_ctx* ctx, const float* u1, const float* u2);
int mppi_get_nominal(mppi_ctx* ctx, float* u1, float* u2);

/* MPPI_step(proj) (MPPI_isaac.py:505-720) for a single-rank controller:
 * sample -> filter -> rollout -> critics -> softmax-weighted update -> optimal
 * filter -> optimal (3D) rollout; outputs copied to host.  `step` is the
 * Philox step counter (noise offset); the new nominal sequence replaces the
 * old one, as reset("sim") + _compute_weighted_sum do (:655-670). */
int mppi_step(mppi_ctx* ctx, int32_t proj, uint64_t step, mppi_outputs* out);

/* Same with caller-supplied sampled controls u1,u2 [K*H] trajectory-major
 * (the injected-input experiment of compare_3d_2d.py:324-533,668-688). */
int mppi_step_injected(mppi_ctx* ctx, int32_t proj, const float* u1_host, const float* u2_host,
                       mppi_outputs* out);

/* Deferred optimal rollout.  With enable != 0, mppi_step / mppi_step_finish /
 * mppi_step_injected return as soon as the control outputs are in host memory:
 * u1_opt, u2_opt, lin_vel, ang_vel in full and ROW 0 of traj_sim, heading_sim,
 * left_wheel_sim, right_wheel_sim (the pose MPPI_Controller.run consumes,
 * MPPI_isaac.py:769-773).  The rest of the optimal rollout
 * (MPPI_isaac.py:696-720) runs on a side stream, overlapping whatever the
 * caller enqueues next (typically the next step's rollout), and its rows are
 * copied to pinned host memory; mppi_get_outputs waits for it.  Values are
 * bitwise identical to the synchronous mode (enable = 0, the default). */
int mppi_set_async_tail(mppi_ctx* ctx, int32_t enable);
/* All outputs of the last step (waits for a deferred optimal rollout). */
int mppi_get_outputs(mppi_ctx* ctx, mppi_outputs* out);

/* ---- K-sharded multi-GPU step (no reference equivalent) ----
 * Record = [m, S, V1[H], V2[H]] float64 (mppi_record_len() doubles).
 * mppi_step_partial enqueues this rank's rollout and writes its record to
 * record_dev (device memory, async on the context stream); the caller
 * all-gathers the G records (RCCL) and mppi_step_finish combines them in rank
 * order and runs the optimal rollout, returning outputs in host memory. */
int64_t mppi_record_len(mppi_ctx* ctx);
int mppi_step_partial(mppi_ctx* ctx, int32_t proj, uint64_t step, double* record_dev);
int mppi_step_finish(mppi_ctx* ctx, const double* records_dev, int32_t n_records,
                     mppi_outputs* out);

/* ---- the same sharded step driven from ONE process ----
 * For a host that owns several GPUs in one process (the reference's
 * controller object, MPPI_isaac.py:397-470, is single-process; a caller that
 * wants one controller over n GPUs without torch.distributed).  The group
 * holds one context per member device, member i over trajectories
 * [begin_i, begin_i + count_i) of params->num_trajectories (256-trajectory
 * leaves split contiguously, as mppi_amd/distributed.shard_bounds), noise
 * keyed by the global trajectory index.  When every member's shard is a
 * power-of-two number of leaves (e.g. C4's 8 x 512) the member roots are
 * subtrees of the one-context record tree and a group step is bitwise equal
 * to one context over all K; other splits (3 members, ragged K) run the same
 * float64 combine with a different pairing (D2 in DESIGN.md).
 * mppi_group_step runs every member's rollout and record (members 1..n-1 on
 * threads of the group, member 0 on the caller's), all-gathers the records
 * (RCCL ncclAllGather, one communicator per member from ncclCommInitAll,
 * RCCL opened with dlopen, when the devices are distinct; device-to-device
 * copies when members share a device), runs every member's finish and
 * returns member 0's outputs; every member keeps the same nominal controls.
 * Scene, state, weights and warm starts are set on each member through
 * mppi_group_context with the single-context calls above (not while a
 * group step runs). */
typedef struct mppi_group mppi_group;
int mppi_group_create(const mppi_params* params, int32_t n, const int32_t* devices,
                      mppi_group** out);
void mppi_group_destroy(mppi_group* group);
int mppi_group_size(mppi_group* group);
int mppi_group_context(mppi_group* group, int32_t member, mppi_ctx** out);
int mppi_group_shard(mppi_group* group, int32_t member, int64_t* begin, int64_t* count);
int mppi_group_step(mppi_group* group, int32_t proj, uint64_t step, mppi_outputs* out);
/* Group facts, up to 7 values: info[0] = members, [1] = distinct devices, [2] = 1 if the records
 * travel by RCCL (else device copies), [3] = ranks of the RCCL communicator (ncclCommCount; 0
 * without RCCL), [4] = 1 if members 1..n-1 run on group threads, [5] = microseconds a member
 * thread spins for the next step before it sleeps (0 when the members outnumber the granted
 * CPUs), [6] = CPUs this process is granted (affinity, bounded by the cgroup quota). */
int mppi_group_info(mppi_group* group, int64_t* info, int32_t n);
/* Host-only test of the group's member threads (no device work, no GPU needed): n members whose
 * steps take ~20 us of host time, member fail_member's fail (fail_member >= n: none), `steps` group
 * steps.  Every step must return (no member thread left waiting), with the failing member named in
 * mppi_last_error.  info[5]: steps returned, steps failed, failures naming the member, worker
 * threads, spin microseconds. */
int mppi_group_selftest(int32_t n, int32_t fail_member, int32_t steps, int64_t* info);

/* ---- introspection (self.costs_wp / self.trajectories .numpy(), MPPI_isaac.py:466-470) ---- */
/* costs of the last step's trajectories of this context [n <= K] */
int mppi_get_costs(mppi_ctx* ctx, float* costs_host, int64_t n);
/* re-run the last step with per-rollout-step outputs (bitwise identical; [K*H] / [K*H*3]
 * trajectory-major like the reference arrays); any pointer may be NULL. */
int mppi_dump_rollouts(mppi_ctx* ctx, float* traj, float* heading, float* left_wheel,
                       float* right_wheel, float* lin_vel, float* ang_vel, float* u1, float* u2);

/* HIP-event timing of the rollout kernel and of the combine/optimal-rollout
 * kernel, measured on the context stream around each launch.  enable: 0 off,
 * 1 rollout, finish and deferred-tail events (the host waits for the stream and
 * for each tail to collect them), 2 rollout events only (no host wait; the finish
 * time reads 0).  In both modes each rollout launch waits for the work already on
 * the side streams, so no noise or deferred-tail kernel runs beside it: the
 * kernel's own time.  While timing is on,
 * steps run as separate launches (rollout, finish, tail), not on the resident
 * server, whose per-step kernel time no launch event brackets. */
int mppi_set_timing(mppi_ctx* ctx, int32_t enable);

/* Per-context options and test hooks, by name (MPPI_EINVAL for an unknown name):
 *   "resident"           sampled steps of the role-split plan (K <= 256 x CUs, records that fit
 *                        the in-kernel finish: C1-C3) on the resident step server, one launch that
 *                        stays on the GPU across steps and polls a command block in pinned memory
 *                        (mppi_step_server_kernel): no launch and no kernel boundary on a step's
 *                        path.  1 (default): for back-to-back calls only, i.e. a call within half
 *                        "resident_idle_us" of the last step's return keeps or starts it, and a
 *                        call after a longer gap (a simulator's frame: VERDICT r05 item 3, the
 *                        server's launch per frame cost more than the launches it saves) runs as
 *                        separate launches (launch_info[17]) and lets a running server go; 2: every
 *                        step whose plan fits; 0: never (env MPPI_RESIDENT=0/1/2 sets the default).
 *                        The server leaves after "resident_idle_us" without a step (a step posted
 *                        as it leaves is served by a relaunch, launch_info[15]), and every call on
 *                        the context other than mppi_step / mppi_set_state / mppi_get_outputs /
 *                        mppi_get_timing stops it first.  While it is resident it holds one
 *                        workgroup slot and ~154 KB of LDS on every CU: other kernels on the device
 *                        get the rest of each CU.  Results are bitwise those of separate launches.
 *   "resident_idle_us"   the server's idle limit, microseconds (default 200, [100, 1e6]).
 *   "finish_wait_ticks"  bound, in ticks of the 100 MHz s_memrealtime clock, on how long a
 *                        finish workgroup of the server waits for the step's rollout records
 *                        (default 1e5 = 1 ms: a running server's records arrive within microseconds
 *                        of each other; a fresh launch beside another stream's kernels that hold some
 *                        CUs has workgroups that cannot start).  A finish that gives up publishes
 *                        the failure; the host stops the server, waits for it to retire, re-arms
 *                        its counters and runs the step again as separate launches (same
 *                        results, launch_info[16]; 0: give up at once, the test hook).  A server
 *                        that does not retire within 10 s of its stop fails the call (MPPI_EHIP).
 *   "eps_after"          where separate launches and partial steps order the next steps' normals
 *                        (noise kernel, side stream): -1 (default) by the call's cadence, after the
 *                        finish for a call more than half "resident_idle_us" after the last step
 *                        returned (no event marker between the rollout and the finish: ~5 us less
 *                        latency per frame) and after the rollout for back-to-back calls and partial
 *                        steps (the noise then ends before the next rollout); 0 / 1: always after the
 *                        rollout / the finish.  Results are the same bits either way.
 *   "record_tree_finish" 1: the record-tree finish (mppi_finish_kernel) at every record count
 *                        (default 0: the column-split finish wherever its shape fits).
 *   "server_exit_after"  test hook: the next server launch leaves at its poll after serving this
 *                        many steps, whether or not the next step was posted (0: off, default);
 *                        that step is served by a relaunch. */
int mppi_set_option(mppi_ctx* ctx, const char* name, int64_t value);
int mppi_get_timing(mppi_ctx* ctx, double* rollout_ms, double* finish_ms, int64_t* launches);
/* HIP-event time of the deferred optimal-rollout kernels (side stream). */
int mppi_get_tail_timing(mppi_ctx* ctx, double* tail_ms, int64_t* launches);

/* Layout/launch facts for the last step (for tests and the bench):
 * info[0]=0 (reserved), [1]=rollout block threads, [2]=rollout blocks, [3]/[4]=cols/rows of
 * the DEM window the step's lanes can touch, [5]=rollout LDS bytes, [6]=finish kind (1 =
 * column-split mppi_colfin_kernel, 0 = record tree mppi_finish_kernel), [7]=records padded
 * (column-split) or records (tree), [8]=columns per finish workgroup, [9]=finish workgroups,
 * [10]=steps whose sampled controls the rollout keeps in LDS, [11]=1 if the step ran on the
 * resident step server (mppi_step_server_kernel), else 0; [12]/[13]/[14] = server launches /
 * steps served / failed steps so far (mppi_set_option "resident"); [15] = commands posted to a
 * server that was leaving on its idle limit and served by a relaunch (included in [12]); [16] =
 * failed server steps rerun as separate launches; [17] = steps the server could have run that ran as
 * separate launches because the call was not back-to-back ("resident" 1).  Up to 18 values. */
int mppi_get_launch_info(mppi_ctx* ctx, int64_t* info, int32_t n);

/* Shader clock of the last sampled 3D rollout, from the chain wave of trajectories 0..63
 * (s_memtime / s_memrealtime at the start and the end of its H steps), up to 10 values:
 * out[0] = shader clock in MHz, [1] = shader cycles per chain step, [2] = the chain's
 * microseconds, [3] = its shader cycles; role-split kernel, workgroup 0, microseconds:
 * [4] = workgroup start -> chain start, [5] = chain end -> every role done, [6] -> leaf
 * record written; over all workgroups (the first 4096): [7] = first -> last workgroup start,
 * [8] = first -> last record written, [9] = first start -> last record (0 where not measured);
 * out[10 + b] = first start -> workgroup b's record.  Waits for the context stream. */
int mppi_get_chain_clock(mppi_ctx* ctx, double* out, int32_t n);

/* The resident step server's own clock (s_memrealtime, 100 MHz), summed over the steps it has
 * served since mppi_create: roll_us = command seen -> last rollout ticket (the rollout of all
 * workgroups, on the server), step_us = command seen -> completion word; steps = the steps summed.
 * Does not stop the server. */
int mppi_get_server_time(mppi_ctx* ctx, double* roll_us, double* step_us, int64_t* steps);

/* Standalone DEM bilinear kernel: for n query points
 * (x[i], y[i]) in device memory, heights[i] = corner lookup + bilinear exactly
 * as projection_warp.py:8-100, on the context's DEM. */
int mppi_bilinear_query(mppi_ctx* ctx, const float* x_dev, const float* y_dev, float* h_dev,
                        int64_t n);

/* LDS-tiled DEM lookup (projection_warp.py:8-100 per query).
 * mppi_bin_queries reorders n < 2^31 device-resident query points by 128x128-cell
 * DEM tile: xs_out/ys_out [n] tile by tile, perm[pos] = input index (int32) of the
 * point now at pos, tile_off [ntiles+1] (ntiles from mppi_bilinear_tiles);
 * synchronous (order inside a tile is unspecified).  mppi_bilinear_tiled then
 * computes h[pos] for the binned points, each tile's window staged once in LDS; it
 * is ASYNCHRONOUS on the context stream (mppi_sync waits).  Results are bitwise
 * identical to mppi_bilinear_query. */
int mppi_bilinear_tiles(mppi_ctx* ctx, int32_t* ntiles);
int mppi_bin_queries(mppi_ctx* ctx, const float* x_dev, const float* y_dev, int64_t n, float* xs_out_dev,
                     float* ys_out_dev, int32_t* perm_dev, int32_t* tile_off_dev);
int mppi_bilinear_tiled(mppi_ctx* ctx, const float* xs_dev, const float* ys_dev,
                        const int32_t* tile_off_dev, float* h_dev);
/* Wait for all work enqueued on the context stream. */
int mppi_sync(mppi_ctx* ctx);

/* Test hook: enqueue on `stream` (a hipStream_t of `device`; NULL = its null stream) `groups`
 * workgroups that each hold lds_bytes (<= 160 KiB) of a CU's LDS for `microseconds` (<= 1 s) and do
 * nothing else: another stream's kernels occupying CUs when a step is posted (the simulator's, in
 * the reference's loop, visual_terrain_stack_full_terrain.py:466-541).  Asynchronous. */
int mppi_debug_hold(int32_t device, void* stream, int32_t groups, int32_t lds_bytes, int32_t microseconds);

/* ---- reference-integrator mode "python25d"  ----
 * generate_trajectory_25D of thesis_master/python_mppi_projection/debug.py:312-364,
 * the reference's numpy 2.5D integrator, for n trajectories at once, in float64,
 * on the context's DEM (row j at y = linspace(-half_width, half_width, rows)[j],
 * as debug.py's meshgrid; `resolution` as its `resolution` argument).  Inputs
 * (host): x0, y0 [n], heading [n*3], lin_vel, ang_vel [n*H] trajectory-major;
 * outputs (host): traj [n*H*3] (x, y, height per step), valid [n] (0 where the
 * reference returns None: the trajectory left |x|, |y| < bound, debug.py:359;
 * its rows from that step on are 0).  Synchronous.  Not on the MPPI step path:
 * it lets whole trajectories be compared with the reference's own function. */
int mppi_rollout_python25d(mppi_ctx* ctx, int64_t n, int32_t H, const double* x0, const double* y0,
                           const double* heading, const double* lin_vel, const double* ang_vel,
                           double dt, double half_width, double resolution, double bound,
                           double* traj, int32_t* valid);

/* Device self-test of the engine's exact-arithmetic fast paths: what = 0 checks
 * the shared-reciprocal division against IEEE a/b, what = 1 the sqrt path
 * against IEEE sqrtf, what = 2 / 3 the lean normalisation of the pair kernel's
 * chain (sqrt of a squared norm and three quotients; 3 with one dominant
 * component) against IEEE sqrtf and a/b, on n random operands; what = 4 the
 * chain's quotient (refined reciprocal, one residual correction) against a/b
 * for every significand of a and n / 2^23 divisor significands ((seed + 8191 k)
 * mod 2^23); what = 5 the noise radius' square root (sqrt_bm) against sqrtf
 * for -0, +0 and the n - 2 floats from 2^-24 up (n <= 2 + 0x4C000000); *mismatches receives the count of in-range results that differ in
 * any bit (0 expected). */
int mppi_selftest(mppi_ctx* ctx, int32_t what, int64_t n, uint64_t seed, int64_t* mismatches);

#ifdef __cplusplus
}
#endif

#endif /* HUSKY_MPPI_H */
