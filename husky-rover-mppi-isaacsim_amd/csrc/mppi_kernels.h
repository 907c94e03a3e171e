// Kernel argument blocks and launchers shared by mppi_kernels.hip and mppi_capi.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mppi {

// The resident step server's command block (mppi_capi.cpp "resident step server"): pinned host
// memory the host fills for every step (every field, then seq with release order); the server's
// workgroups poll seq and read the rest with system-scope loads.  stop == the launch's launch_id
// ends that launch (a later launch has another id: the host never clears the word).
struct ServerCmd {
  unsigned seq;    // the step's completion sequence number (written last)
  unsigned stop;   // (same 8-byte word as seq: one poll reads both; checked before seq)
  int eps_slot;    // normals slot of the step
  int cur;         // nominal buffer the step reads (the finish writes the other one)
  int tail_slot;   // deferred optimal rollout slot (mode 2)
  int mode;        // 1: finish with the whole optimal rollout, 2: step 0 only (the rest deferred)
  int noise_slot;  // >= 0: the rollout workgroups outside the finish generate the normals of Philox block
                   // base noise_n_base into this slot after their records (-1: none)
  unsigned noise_n_base_lo;
  float x0, y0, h0x, h0y, h0z, wl, wr, gx, gy, s1, s2, igx, igy, pf_scale;  // robot / goal state
  int pf_far, speed_on;
  unsigned noise_n_base_hi;
  unsigned pad1[7];
};
constexpr int kTailSlots = 4;  // deferred optimal rollouts in flight (mppi_capi.cpp; 8 / 16 measured
                               // within noise, profiles/r04_notes.md)
constexpr int kCmdWords = 25;                 // the words a step reads (seq .. noise_n_base_hi)
constexpr unsigned kDoneFail = 0x80000000u;   // done | kDoneFail: the step's finish gave up
struct FinishArgs {
  int H;
  int mode;  // 0: write root record, 1: finish (u_opt + optimal rollout),
             // 2: finish with the optimal rollout deferred to mppi_tail_kernel (step 0 only here)
  const double* recs;
  int n_recs;
  const float* rec_m;  // [n_recs] the records' m contiguous, or null (read from recs)
  unsigned long long* uopt;  // [2H] colfin: the u_opt handoff words {u bits, seq << 32} (zeroed once)
  double* scratch0;
  double* scratch1;
  double* record_out;  // mode 0
  float T;
  // finish
  float* u_nom_next;  // [2H]
  float* out;         // [16H] u1,u2,v,w,traj,hv,lw,rw
  const float* Z;
  const float4* ntab;  // per-cell normals (see RolloutArgs)
  int rows, grid;
  float x_min, y_min, res;
  float rinv_res;
  int cdiv_res;
  float x0, y0, h0x, h0y, h0z, wl, wr;
  float ok, oa, rwheel, vmin, vmax, wmin, wmax, dt, off;
  // deferred optimal rollout (mode 2 / mppi_tail_kernel)
  float* tail_in;   // [3H] v, sin(w dt), cos(w dt) of the optimal sequence
  float* tail_out;  // [12H] traj, hv, lw, rw (pinned host memory)
  // completion: after every output store, lane 0 stores `seq` to *done (pinned host
  // memory, system scope, release) so the host can spin on it instead of a stream sync
  unsigned* done;
  unsigned seq;
  // resident server: a finish workgroup that gave up stores the step's seq here, and the last finish
  // workgroup's u_opt poll stops on it (null: separate launches)
  unsigned* abort;
  uint64_t* clk;  // optional: the deferred tail's stamps (kClkServer ring)
  // multi-workgroup first tree level (launch_finish with groups > 1)
  double* level1;         // [groups][2H+2]
  unsigned* level1_cnt;   // zero-initialised, re-armed in-kernel
};

struct RolloutArgs {
  // sizes / ids
  int64_t K;         // trajectories in this launch (shard-local)
  int64_t k_offset;  // global index of trajectory 0 (Philox subsequence)
  int H;
  // DEM
  const float* Z;
  const float4* ntab;  // per-cell normals [(rows+1) x (grid+1)] (mppi_normal_table_kernel)
  int rows, grid;
  float x_min, y_min, res;
  // costmap
  const float* cm;
  int cm_size;
  float hw, res_c;
  // verified division-by-constant for grid indices (cdiv_f): reciprocal + enable flag
  float rinv_res, rinv_res_c;
  int cdiv_res, cdiv_res_c;
  // robot / goal state (MPPI_isaac.py:489-497, :611-613)
  float x0, y0, h0x, h0y, h0z, wl, wr, gx, gy, s1, s2;
  // sampling
  uint64_t seed, n_base;  // Philox key, block index of (step, t=0)
  const float* eps;       // pair kernel, MODE 0: this step's normals [blocks][2][H][256] (mppi_noise_kernel)
  const float* u_nom1;
  const float* u_nom2;
  float min_u1, max_u1, min_u2, max_u2;
  // filter (sampling_warp.py:96-138)
  float fk, fa, rwheel, vmin, vmax, wmin, wmax;
  // rollout
  float dt, off;
  // critics (critics_warp.py:85-329); pf_far/igx/igy/pf_scale/speed_on precomputed in f32
  int pf_far, speed_on;
  float igx, igy, pf_scale;
  float w_path, w_slope, w_speed, w_obs, thr, pen, T;
  // outputs
  float* cost_out;   // [K]
  double* nodes;     // [blocks][2H+2]
  float* rec_m;      // [blocks] or null: each record's m again, contiguous (the finish's scale table)
  float* ustore;     // [blocks][2][H][block] sampled controls kept for the weighted sum
  // injected controls (MODE 1), trajectory-major [K*H]
  const float* inj_u1;
  const float* inj_u2;
  // dump (DUMP)
  float *d_traj, *d_hv, *d_lw, *d_rw, *d_v, *d_w, *d_u1, *d_u2;
  int wave_prio;        // pair kernel: raise the waves' issue priority (s_setprio 2)
  int small_angle;      // max(|wmin|, |wmax|) * dt < 0.78: the Rodrigues angle's sin / cos by
                        // dm_sincosf_small (the same bits, no range reduction)
  int ucache_steps;     // pair kernel, MODE 0: steps [0, n) keep their sampled controls in LDS
                        // ([2][n][TB] floats after the scratch) for leaf_records
  // optional [8]: the chain wave of group 0 in workgroup 0 stores s_memtime / s_memrealtime at
  // the start and the end of its H steps ([0..3]: shader clock cycles per step and the clock
  // rate); role-split kernel, workgroup 0: s_memrealtime at its start, when every role is done,
  // and when its leaf record is written ([4..6])
  uint64_t* clk;
};
// clk layout: [0..8) the stamps above, then (role-split kernel) [kClkBase + 2 b], [.. + 1] =
// s_memrealtime when workgroup b (< kClkBlocks) starts and when its record is written
constexpr int kClkBase = 8, kClkBlocks = 4096;
// then (resident server) s_memrealtime per step, ring of 8 steps: [kClkServer + 8 (seq % 8) + k], k =
// 0 the head saw the command, 1 the last rollout ticket, 2 the completion word stored, 3 the
// latest end of a noise share (atomic max), 4 the deferred tail started, 5 the tail ended,
// 6 the head started polling for the command, 7 the latest end of any workgroup's step
// then (resident server, always on) [kClkServer + 64, + 68): the sums of (last ticket - command seen)
// and (completion word - command seen) in 100 MHz ticks, and their step counts
constexpr int kClkServer = kClkBase + 2 * kClkBlocks, kClkSums = kClkServer + 64, kClkWords = kClkSums + 8;
// The finish's phase-2 LDS (finish_phase2): uo[2][PS] v w sin cos[H] chain[12H] out[16H]
// lr[2][PS] floats, PS = the filter rows' stride (a multiple of 4 floats, >= H + 32 for the
// filter's read-ahead).
__host__ __device__ inline int fin_plane_stride(int H) { return ((H + 3) & ~3) + 32; }
__host__ __device__ inline int fin_phase2_floats(int H) { return 4 * fin_plane_stride(H) + 32 * H; }


// The rollout kernel (mppi_rollout_pair_kernel): 256 trajectories per 512-thread workgroup, a
// chain wave and a side wave per 64 trajectories, synchronised through LDS progress counters
// over PAIR_RING-deep rings.
constexpr int PAIR_TRAJ = 256;
// ring depth: round 4, 6 beats 8 at C3 by ~1.4 % (the control cache holds 48 steps instead of 40),
// C4 and the C4 shard unchanged (profiles/r04_notes.md)
constexpr int PAIR_RING = 6;  // = PAIR_D in mppi_kernels.hip
// floats per trajectory and step, side -> chain: (v, sin, cos, 1 - cos) of the Rodrigues angle,
// computed by the side wave at production, off the chain's serial path
constexpr int PAIR_RING_IN = 4;
// the role-split kernel's ring_out depth (x, y, cx, cy of each step, chain -> wheel and cost waves):
// round 6, 8 and 10 (two control-cache steps fewer each) measured within noise of 6 or below it
constexpr int ROLES_RING_OUT = 6;
hipError_t launch_rollout_pair(const RolloutArgs& a, int blocks, size_t lds, hipStream_t st, int proj,
                               int mode, bool dump, bool roles = false);
// The role-split rollout kernel (mppi_rollout_roles_kernel): the same 256 trajectories per
// workgroup over 1024 threads, one wave per role (chain, producer, wheel, cost) and 64
// trajectories; rings [D][4 + 4][TB] + cost[TB] + slope[TB] in LDS.
constexpr int ROLES_WAVES_PER_TRAJ_WAVE = 4;
// The resident step server (mppi_step_server_kernel): one workgroup per 256 trajectories of the
// role-split rollout, resident across steps.  Per step every workgroup waits for cmd->seq to reach
// the next sequence number (or cmd->stop; the head also leaves after idle_ticks of the 100 MHz
// clock without a command, and the others leave on the stop it relays), runs its rollout and writes its record through, and takes a ticket from rec_cnt;
// the workgroups holding the last fin_groups tickets run the column-split finish (each after rec_cnt
// reaches nroll, or wait_ticks: then the step publishes done | kDoneFail); the other workgroups
// generate the normals of step + 2 meanwhile (ServerCmd::noise_slot, a static share per ticket;
// workgroup 0's first wave keeps out of it).  Only workgroup
// 0 polls the pinned command (256 workgroups polling host memory cost ~30 us per step, one ~4 us:
// profiles/ubench/server.hip); it relays the command words and seq / stop through device memory.
struct ServerArgs {
  FinishArgs f;
  int nroll, fin_P, fin_ncol, fin_groups;
  unsigned* rec_cnt;          // [0] records counted; zeroed, re-armed by the finish
  const ServerCmd* cmd;       // pinned host memory (polled by workgroup 0 only)
  unsigned* relay;            // device: [0] seq, [1] stop (the launch_id of the launch that stopped) as relayed
                              // by the head, [16, 16 + kCmdWords) the command words
  unsigned launch_id;         // unique per launch of the context (never 0): the stop word that ends it
  float* eps[3];              // the normals slots
  float* u_nom[2];            // the nominal double buffer, [2H] each
  float* tail_in[kTailSlots];   // deferred optimal rollout inputs per slot (device)
  float* tail_out[kTailSlots];  // its outputs per slot (pinned)
  unsigned first_seq;
  uint64_t wait_ticks;        // a finish's record wait bound
  uint64_t idle_ticks;        // the head leaves after this long without a command (and relays the stop)
  unsigned exit_after;        // test hook (0: off): the head leaves at its poll after serving this many
                              // commands, whether or not the next one was posted
  uint64_t* clk;             // optional: the server stamps [kClkServer, kClkServer + 4) of RolloutArgs::clk
};
hipError_t launch_step_server(const RolloutArgs& a, const ServerArgs& z, size_t lds, hipStream_t st, int proj);
// record tree finish (mppi_finish_kernel): the fallback where the column-split shape does not fit
hipError_t launch_finish(const FinishArgs& f, size_t lds, hipStream_t st, int groups = 1);
// column-split finish: every workgroup builds the pair-scale table and reduces ncol columns
// over all n records; the last to arrive runs phase 2 (f.level1 holds >= 2H floats, f.level1_cnt
// a zeroed counter).  colfin_shape returns 0 when n is outside the kernel's range.
// (at most max_groups workgroups: more columns each).
int colfin_shape(int n, int H, int* P, int* ncol, int* groups, size_t* lds_tree, int max_groups = 1 << 30);
hipError_t launch_colfin(const FinishArgs& f, size_t lds, hipStream_t st, int P, int ncol, int groups);
// optimal rollout of the sequence a mode-2 finish left in f.tail_in (one workgroup)
constexpr int TAIL_THREADS = 256;
hipError_t launch_tail(const FinishArgs& f, hipStream_t st);
// per-cell surface normals of the DEM, [(rows+1) x (grid+1)] float4 (x, y, z, 0)
hipError_t launch_normal_table(const float* Z, int rows, int grid, float res, float4* out, hipStream_t st);
hipError_t launch_selftest(int what, int64_t n, uint64_t seed, unsigned long long* bad, hipStream_t st);
// test hook: `groups` workgroups each holding `lds` bytes of LDS for `ticks` (100 MHz)
hipError_t launch_hold(int groups, size_t lds, uint64_t ticks, hipStream_t st);
// counts the significands a in [1, 2) for which cdiv_f(a, b, y) != a / b (IEEE)
hipError_t launch_cdiv_verify(float b, float y, unsigned* bad, hipStream_t st);
// The sampling normals of one step (Philox block n_base + t/2 of global trajectory k_offset + k),
// laid out [blocks][2][H][256]: eps1 rows then eps2 rows, 256 trajectories per row.
hipError_t launch_noise(uint64_t seed, uint64_t n_base, int64_t k_offset, int blocks, int H, float* eps,
                        hipStream_t st, int max_groups);
hipError_t launch_bilinear(const float* Z, int rows, int grid, float x_min, float y_min, float res,
                           const float* xs, const float* ys, float* hs, int64_t n, hipStream_t st);
// LDS-tiled lookup over queries binned by BIL_TILE x BIL_TILE-cell DEM tile (tile count =
// ceil(rows/BIL_TILE) * ceil(cols/BIL_TILE); the binning keeps one LDS counter per tile, so
// mppi_bin_queries refuses DEMs with more than ~40 000 tiles, e.g. a skinny 2 x 2^24 grid).  Binning: G chunks of
// the queries, each one workgroup with an LDS histogram (hist[G][ntiles] scratch), the tile
// counts' exclusive scan, then the scatter: with <= 4096 tiles and the level-1 scratch (cx, cy, ci
// [n], bcur [tile rows]) two levels of LDS-sorted runs (by tile row into cx/cy/ci, then by tile),
// else each chunk straight from the tile cursors; perm int32 (n < 2^31).
constexpr int BIL_TILE = 128;
int bin_chunks(int64_t n, int ntiles);  // G for n queries
hipError_t launch_bin_queries(const float* xs, const float* ys, int64_t n, float x_min, float y_min, float res,
                              float rinv, int cdiv, int rows, int grid, int* hist, int* counts, int* cursor,
                              int* off, float* xs_out, float* ys_out, int32_t* perm, hipStream_t st,
                              float* cx, float* cy, int32_t* ci, int* bcur);
hipError_t launch_bilinear_tiled(const float* Z, int rows, int grid, float x_min, float y_min, float res,
                                 float rinv, int cdiv, const float* xs, const float* ys, float* hs,
                                 const int* tile_off, hipStream_t st);

}  // namespace mppi
