// C-ABI implementation (include/mppi.h): context, buffers, launch planning, host<->device copies.
//
// Host arithmetic that feeds the kernels (path-follow branch, intermediate
// goal, window bounds) is float32 in the reference's operation order; this
// file is compiled with -ffp-contract=off like the kernels.
#include <dlfcn.h>
#include <sched.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: RCCL is opened with dlopen by mppi_group_create

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "mppi.h"
#include "mppi_costmap.h"
#include "mppi_kernels.h"
#include "mppi_python25d.h"

using namespace mppi;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return fail(MPPI_EHIP, std::string(#expr) + " failed: " + hipGetErrorString(e_));    \
  } while (0)

constexpr size_t kLdsBytes = 160 * 1024;
constexpr int kEpsSlots = 3;
// (mppi::kTailSlots deferred optimal rollouts in flight: the tail of step i may run until step
// i + kTailSlots is issued; beside the next rollouts it gets only the issue slots their waves leave)

struct Plan {
  int traj_per_block = 256;
  int block = 256, blocks = 0;
  int grid = 0;  // rollout workgroups (the role-split kernel runs blocks beyond one per CU in turn)
  int W = 1, Wr = 1;  // the DEM window every lane of the step can touch (mppi_get_launch_info)
  size_t lds_bytes = 0, fin_lds_bytes = 0, fin_tree_bytes = 0;
  int ucache_steps = 0;   // pair kernel: steps whose sampled controls stay in LDS for the leaf
  bool roles = false;     // the role-split rollout kernel (mppi_rollout_roles_kernel)
};

}  // namespace

struct mppi_ctx {
  mppi_params p{};
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  // DEM
  float* Z = nullptr;
  bool Z_owned = false;
  float4* ntab = nullptr;  // per-cell normals of the DEM, (rows+1) x (cols+1) (mppi_normal_table_kernel)
  size_t ntab_cap = 0;
  size_t Z_cap = 0;
  int rows = 0, cols = 0;
  float x_min = 0, y_min = 0, res = 0;
  // costmap
  float* cm = nullptr;
  size_t cm_cap = 0;
  int cm_size = 0;
  float cm_hw = 0, cm_res = 0;
  CostmapScratch cms;  // mppi_build_costmap scratch
  // verified division-by-constant reciprocals (0 = use the IEEE division)
  float rinv_res = 0, rinv_res_c = 0;
  unsigned* cdiv_bad = nullptr;  // device counter for launch_cdiv_verify
  std::unordered_map<uint32_t, float> cdiv_cache;  // divisor bits -> verified y (0: none)
  // state
  mppi_state st{};
  bool have_state = false;
  // nominal sequence double buffer: u_nom[cur] is read by the next step
  float* u_nom[2] = {nullptr, nullptr};
  int cur = 0;
  // step buffers
  float* cost = nullptr;
  double* nodes = nullptr;
  float* rec_m = nullptr;  // [nodes_cap / E] the records' m, contiguous
  size_t nodes_cap = 0;
  double* scratch0 = nullptr;
  double* scratch1 = nullptr;
  float* ustore = nullptr;   // sampled controls of the current step [blocks][2][H][block]
  size_t ustore_cap = 0;
  float* stage = nullptr;     // pinned [16H]: the finish kernel stores the outputs here directly
  unsigned* done = nullptr;   // pinned completion word (FinishArgs::done)
  unsigned seq = 0;
  float* out_host = nullptr;  // [16H] last complete outputs (host memory)
  float* inj1 = nullptr;
  float* inj2 = nullptr;
  // sampling normals, one slot per step in flight: the rollout's, the next step's and the one
  // after (generated two steps ahead, so the noise kernel is never on the step's path)
  float* eps[kEpsSlots] = {nullptr, nullptr, nullptr};
  size_t eps_cap = 0;
  int64_t eps_step[kEpsSlots] = {-1, -1, -1};
  hipEvent_t eps_ev[kEpsSlots] = {nullptr, nullptr, nullptr};
  bool eps_pending[kEpsSlots] = {false, false, false};
  hipStream_t noise_stream = nullptr;
  int prio_least = 0, prio_greatest = 0;
  // finish: 1 = column-split kernel (mppi_colfin_kernel) where it applies, 0 = the record tree
  // (mppi_set_option "record_tree_finish")
  int colfin = 1;
  int num_cus = 256;  // compute units of the device (hipDeviceAttributeMultiprocessorCount)
  // host-side step timeline (env MPPI_HOST_TRACE=1, printed by mppi_destroy): per step the host
  // times (us) of 6 marks (trace_mark), summed as phases over the steps and kept for the last 8
  bool trace = false;
  double tr_m[6] = {}, tr_sum[6] = {}, tr_log[8][6] = {}, tr_prev = 0;
  long tr_n = 0;
  int roles = -1;     // rollout kernel: -1 auto (role split at <= 1 workgroup per CU), 0 pair, 1 roles (MPPI_ROLES)
  // Resident step server (mppi_step_server_kernel): sampled steps of the role-split plan run on one
  // resident launch that polls the command block `cmd` (pinned) instead of one launch per step
  // (mppi_set_option "resident", env MPPI_RESIDENT).  It exits after srv_idle_us without a command, on
  // cmd->stop == its launch id (every other call on the context stops it first: quiesce) or on a
  // failed step.  resident 1 (default): only back-to-back calls (within half the idle limit of the
  // last step's return) keep or start it, a step after a longer gap runs as separate launches (the
  // caller's frame cadence: a launch of the server per frame costs more than the launches it saves);
  // 2: every step whose plan fits; 0: never.
  int resident = 1;
  ServerCmd* cmd = nullptr;   // pinned
  unsigned* relay = nullptr;  // device [64]: workgroup 0's relay of the command (ServerArgs::relay)
  bool srv_running = false;
  bool srv_exiting = false;   // a stop was posted and the launch may not have retired yet
  unsigned srv_launch_id = 0;  // the running (or last) launch's id: its stop word
  double last_return_us = 0;  // host time the last step returned (0: none yet)
  int b2b_calls = 0;          // consecutive back-to-back steps (resident 1)
  int64_t srv_fallbacks = 0;  // server steps whose finish gave up, rerun as separate launches
  int64_t cadence_steps = 0;  // steps the server's plan fits that ran as separate launches (resident 1)
  int srv_proj = 0;
  double srv_last_us = 0;     // host time the server last became idle (its last step completed, or launch)
  uint64_t srv_idle_us = 200;  // (bench.py cadence leg: at 2000 a simulator kernel needing LDS waited
                               // out the idle server every frame)
  int64_t srv_launches = 0, srv_steps = 0, srv_failed = 0;
  int64_t srv_relaunches = 0;  // commands a leaving server did not take, served by a relaunch (wait_done)
  int srv_cmd_noise = -1;     // the normals slot the last command asked the server's noise phase for
  int fail_kind = 0;          // the last failed wait: 1 finish gave up, 2 launch retired, 3 timeout
  bool srv_warned = false;
  // the server launch of the command wait_done waits for (a relaunch serves the same command)
  bool srv_cmd_live = false;
  Plan srv_pl;
  int srv_P = 0, srv_ncol = 0, srv_groups = 0;
  size_t srv_lds = 0;
  unsigned srv_exit_after = 0;  // test hook mppi_set_option("server_exit_after"): the next launch's head
                                // leaves after serving this many commands (0: off)
  // a finish's record wait bound (100 MHz ticks; mppi_set_option): 1 ms, many step periods.  Every
  // workgroup of a running server is resident, so its records arrive within the rollouts' end spread
  // (~4 us at C3); a fresh launch whose workgroups cannot all get CUs (another stream's kernels hold
  // some) would wait for them, while the workgroups it has hold theirs: past the bound the step is
  // rerun as separate launches, which need no co-residency (step_impl)
  uint64_t fin_wait_ticks = 100000ull;
  // where the next steps' normals are ordered on the context stream (separate launches, partial
  // steps): after the rollout (an event marker between the rollout and the finish, ~5 us on the
  // step's path) or after the finish (the noise then runs into the next rollout of a back-to-back
  // caller).  eps_after: -1 by the call's cadence (default: after the finish for a call more than
  // half the idle limit after the last one returned, a simulator frame), 0 / 1 forced (mppi_set_option)
  int eps_after = -1;
  bool eps_late = false;  // this step's choice
  // the server's tail of the last step, launched once its completion word was seen (at the next
  // step's command, or when its outputs are wanted): no kernel waits on the GPU for its inputs
  bool tail_deferred = false;
  FinishArgs tail_def{};
  int tail_def_par = 0;
  hipEvent_t ev_prev_roll = nullptr;  // recorded after the last rollout that read an eps slot
  hipEvent_t ev_side[2] = {nullptr, nullptr};  // timing mode 2: the side streams' work so far
  // finish: column-split u_opt slice records / first tree level, arrival counter
  double* level1 = nullptr;       // finish kernel first-level records
  size_t level1_cap = 0;
  unsigned* level1_cnt = nullptr;  // [0]: finish handoff, [16]: the server's record count
  unsigned long long* uopt = nullptr;  // [2H] the column-split finish's tagged u_opt words
  unsigned wait_seq = 0;  // the completion word wait_done waits for
  uint64_t* clk = nullptr;  // [4] chain clock stamps of the last sampled rollout (RolloutArgs::clk)
  // tiled bilinear binning scratch
  int* bin_tile_of = nullptr;  // per-chunk tile histograms [chunks][tiles]
  size_t bin_n_cap = 0;
  int* bin_counts = nullptr;
  int* bin_cursor = nullptr;
  size_t bin_t_cap = 0;
  // two-level binning: the tile-row-sorted queries [n] and the tile-row cursors [rows of tiles]
  float* bin_cx = nullptr;
  float* bin_cy = nullptr;
  int32_t* bin_ci = nullptr;
  size_t bin_q_cap = 0;
  // the finish the last step ran (mppi_get_launch_info): 1 column-split, 0 record tree
  int fin_kind = -1, fin_P = 0, fin_ncol = 0, fin_groups = 0;
  bool last_resident = false;  // the last step ran on the resident server (mppi_get_launch_info info[11])
  // last step (for dump)
  bool have_last = false;
  int last_proj = 3, last_mode = 0;
  uint64_t last_step = 0;
  mppi_state last_state{};
  int last_nominal = 0;
  // deferred optimal rollout (mppi_set_async_tail): side stream + buffers
  bool async_tail = false;
  hipStream_t tail_stream = nullptr;
  hipEvent_t ev_fin_done = nullptr;
  hipEvent_t ev_tail[kTailSlots] = {};  // per slot: tail done
  bool tail_pending = false;       // the latest tail's outputs are not merged into out_host yet
  bool tail_inflight[kTailSlots] = {};  // the tail of that slot may still run
  hipStream_t tail_ts[kTailSlots] = {};  // the stream that slot's tail was launched on
  int tail_par = 0;                // slot of the latest tail
  float* tail_in[kTailSlots] = {};    // device [3H] per slot
  float* tail_host[kTailSlots] = {};  // pinned [12H] per slot (written by the kernel)
  // timing
  int timing = 0;  // 1: rollout, finish and tail events; 2: rollout only, no host wait (mppi_set_timing)
  hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  bool ev_roll_pending = false, ev_fin_pending = false, ev_tail_pending = false;
  double t_roll = 0, t_fin = 0, t_tail = 0;
  int64_t launches = 0, tail_launches = 0;
  Plan last_plan;
};

namespace {

int H_of(const mppi_ctx* c) { return c->p.num_iterations; }

// Reciprocal y for cdiv_f(a, b, y) that reproduces the IEEE quotient for every
// significand (checked exhaustively on the device, 2^23 cases); 0 if none of
// RN(1/b) and its two neighbours qualifies.  Cached per divisor.
int verified_reciprocal(mppi_ctx* c, float b, float* y_out) {
  uint32_t key;
  std::memcpy(&key, &b, 4);
  auto it = c->cdiv_cache.find(key);
  if (it != c->cdiv_cache.end()) {
    *y_out = it->second;
    return MPPI_OK;
  }
  float y = 0.0f;
  if (std::isfinite(b) && b != 0.0f) {
    const float y0 = (float)(1.0 / (double)b);
    const float cand[3] = {y0, std::nextafter(y0, 0.0f), std::nextafter(y0, 2.0f * y0)};
    for (float yc : cand) {
      unsigned bad = 1;
      HIP_TRY(hipMemsetAsync(c->cdiv_bad, 0, sizeof(unsigned), c->stream));
      HIP_TRY(launch_cdiv_verify(b, yc, c->cdiv_bad, c->stream));
      HIP_TRY(hipMemcpyAsync(&bad, c->cdiv_bad, sizeof(unsigned), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      if (bad == 0) {
        y = yc;
        break;
      }
    }
  }
  c->cdiv_cache[key] = y;
  *y_out = y;
  return MPPI_OK;
}
int E_of(const mppi_ctx* c) { return 2 * c->p.num_iterations + 2; }

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// (Re)allocate device buffer p for `bytes` when its capacity `cap` (bytes) is short.  The old
// contents are dropped; `st`, which may still read the old buffer, is synchronised first.
template <class T>
int grow(T*& p, size_t& cap, size_t bytes, hipStream_t st) {
  if (bytes <= cap) return MPPI_OK;
  HIP_TRY(hipStreamSynchronize(st));
  if (p) HIP_TRY(hipFree(p));
  p = nullptr;
  cap = 0;
  HIP_TRY(hipMalloc(&p, bytes));
  cap = bytes;
  return MPPI_OK;
}

int check_ready(mppi_ctx* c) {
  if (!c) return fail(MPPI_EINVAL, "null context");
  if (!c->Z) return fail(MPPI_ESTATE, "no DEM: call mppi_set_dem first");
  if (!c->cm) return fail(MPPI_ESTATE, "no costmap: call mppi_set_costmap first");
  if (!c->have_state) return fail(MPPI_ESTATE, "no state: call mppi_set_state first");
  HIP_TRY(hipSetDevice(c->device));
  return MPPI_OK;
}

// Launch geometry.  The rollouts of one step stay within H*dt*|v|max (+ wheel offset) of the robot:
// the square DEM window of that radius (every cell any lane can touch) is reported, not staged.
Plan make_plan(const mppi_ctx* c) {
  Plan pl;
  const int H = H_of(c);
  const double vabs = std::max(std::fabs((double)c->p.v_min_linear), std::fabs((double)c->p.v_max_linear));
  const double reach = (double)H * (double)c->p.dt * vabs + std::fabs((double)c->p.wheel_offset) * 1.01 + 0.01;
  const int Rc = (int)std::ceil(reach / (double)c->res) + 3;
  const int64_t span = 2 * (int64_t)Rc + 2;
  pl.W = (int)std::min<int64_t>(span, c->cols);
  pl.Wr = (int)std::min<int64_t>(span, c->rows);
  const int64_t K = c->p.num_trajectories;
  // rollout kernel: chain + side waves per 64 trajectories, DEM and normals through L1/L2,
  // rings [D][PAIR_RING_IN + 4][TB] + cost[TB] + flags + nominal + leaf scratch in LDS (profiles/r01_notes.md)
  const int TB = PAIR_TRAJ;
  pl.traj_per_block = TB;
  pl.blocks = (int)((K + TB - 1) / TB);
  // role split where the rollout is latency-bound (at most one workgroup per CU); the pair
  // kernel's 8 waves per workgroup pack 4 workgroups per CU at larger K (MPPI_ROLES=0/1 forces)
  pl.roles = c->roles < 0 ? pl.blocks <= c->num_cus : c->roles != 0;
  pl.block = (pl.roles ? ROLES_WAVES_PER_TRAJ_WAVE : 2) * TB;
  const size_t scratch = ((size_t)(TB + TB / 64) * 4 + 15) / 16 * 16 + (size_t)(TB / 256) * (2 * H + 2) * sizeof(double);
  const size_t ring_rows = pl.roles ? (size_t)4 * PAIR_RING + 4 * ROLES_RING_OUT + 2 : (size_t)(PAIR_RING_IN + 4) * PAIR_RING + 1;
  pl.lds_bytes = ring_rows * TB * sizeof(float) + 4 * (TB / 64) * sizeof(int) +
                 (size_t)((2 * H + 3) & ~3) * sizeof(float) + scratch;
  // only at one workgroup per CU (the role-split kernel always: beyond one block per CU its
  // workgroups run the blocks in turn; the pair kernel up to one block per CU): the cache takes
  // the CU's spare LDS, which a co-resident pair workgroup (C5: 4 per CU) would need instead
  pl.grid = pl.roles ? std::min(pl.blocks, std::max(c->num_cus, 1)) : pl.blocks;
  if (pl.roles || pl.blocks <= c->num_cus) {
    // the rest of the CU's LDS keeps the sampled controls of the first steps ([2][T][TB]
    // floats, 16-byte aligned after the scratch), so the leaf reduction re-reads only the
    // other steps' normals from HBM (all workgroups reduce at once: a bandwidth burst)
    // room is left for the deferred optimal rollout of the previous step (mppi_tail_kernel,
    // 12H + 4 floats), which runs beside a rollout workgroup on one CU
    const size_t base = (pl.lds_bytes + 15) / 16 * 16;
    const size_t row2 = (size_t)2 * (TB + 4) * sizeof(float);  // UCACHE_ROW: one float4 of bank skew
    // (1 KiB more: the server kernel's static command / ticket words and LDS allocation granularity)
    const size_t budget = kLdsBytes - ((size_t)(12 * H + 4) * sizeof(float) + 2047) / 1024 * 1024 - 1024;
    pl.ucache_steps = base < budget ? (int)std::min<size_t>((size_t)H, (budget - base) / row2) : 0;
    if (pl.ucache_steps > 0) pl.lds_bytes = base + (size_t)pl.ucache_steps * row2;
  }
  // finish kernel: tree phase [16][2H+2] doubles + 64 x (15 PairScale + 16 m); phase 2
  // uo[2][PS] v[H] w[H] sin[H] cos[H] chain[12H] out[16H] lr[2][PS] floats (fin_phase2_floats)
  pl.fin_tree_bytes = (size_t)16 * (2 * H + 2) * sizeof(double) + (size_t)64 * (15 * 16 + 16 * 4);
  pl.fin_lds_bytes = std::max(pl.fin_tree_bytes, ((size_t)fin_phase2_floats(H) * sizeof(float) + 15) / 16 * 16);
  return pl;
}

// Noise grid: 4 four-wave workgroups per CU.  The noise of step i+2 runs beside the finish of
// step i and the start of rollout i+1 (4 per CU measured best at C3: 10095 steps/s against 9920 at
// 3 and 9730 at 2, alternating runs, profiles/r02_notes.md).
int noise_groups(const mppi_ctx* c) { return std::max(c->num_cus, 1) * 4; }

int ensure_nodes(mppi_ctx* c, int blocks) {
  const size_t need = (size_t)std::max(blocks, 1) * E_of(c);
  if (need <= c->nodes_cap) return MPPI_OK;
  if (c->nodes) hipFree(c->nodes);
  if (c->rec_m) hipFree(c->rec_m);
  if (c->scratch0) hipFree(c->scratch0);
  if (c->scratch1) hipFree(c->scratch1);
  c->nodes = c->scratch0 = c->scratch1 = nullptr;
  c->rec_m = nullptr;
  HIP_TRY(hipMalloc(&c->nodes, need * sizeof(double)));
  HIP_TRY(hipMalloc(&c->rec_m, (size_t)std::max(blocks, 1) * sizeof(float)));
  const size_t half = ((size_t)std::max(blocks, 1) + 1) / 2 * E_of(c);
  HIP_TRY(hipMalloc(&c->scratch0, half * sizeof(double)));
  HIP_TRY(hipMalloc(&c->scratch1, half * sizeof(double)));
  c->nodes_cap = need;
  return MPPI_OK;
}

// The rollout / finish fields that follow from the robot state, in the server command's layout
// (fill_rollout copies them into the launch arguments).
void state_fields(const mppi_params& p, const mppi_state& st, ServerCmd& d) {
  d.x0 = st.x;
  d.y0 = st.y;
  d.h0x = st.heading[0];
  d.h0y = st.heading[1];
  d.h0z = st.heading[2];
  d.wl = st.left_wheel_speed;
  d.wr = st.right_wheel_speed;
  d.gx = st.goal_x;
  d.gy = st.goal_y;
  d.s1 = st.std_dev_u1;
  d.s2 = st.std_dev_u2;
  // _path_follow_critic / _maximise_speed scalar parts (critics_warp.py:111-123, :281-286)
  const float xd = st.goal_x - st.x;
  const float yd = st.goal_y - st.y;
  const float dist = std::sqrt(xd * xd + yd * yd);
  const float horizon = p.horizon;
  d.pf_far = dist > horizon ? 1 : 0;
  d.igx = st.x + (xd * horizon) / (dist + 1e-6f);
  d.igy = st.y + (yd * horizon) / (dist + 1e-6f);
  d.pf_scale = 1.0f + (2.0f * horizon) / dist;
  d.speed_on = (dist < 2.0f) ? 0 : 1;
}

void fill_rollout(const mppi_ctx* c, const Plan& pl, const mppi_state& st, uint64_t step,
                  const float* unom, RolloutArgs& a) {
  const mppi_params& p = c->p;
  const int H = p.num_iterations;
  std::memset(&a, 0, sizeof(a));
  a.K = p.num_trajectories;
  a.ucache_steps = pl.ucache_steps;
  a.k_offset = p.k_offset;
  a.H = H;
  a.Z = c->Z;
  a.ntab = c->ntab;
  a.rows = c->rows;
  a.grid = c->cols;
  a.x_min = c->x_min;
  a.y_min = c->y_min;
  a.res = c->res;
  a.cm = c->cm;
  a.cm_size = c->cm_size;
  a.hw = c->cm_hw;
  a.res_c = c->cm_res;
  a.rinv_res = c->rinv_res;
  a.cdiv_res = c->rinv_res != 0.0f;
  a.rinv_res_c = c->rinv_res_c;
  a.cdiv_res_c = c->rinv_res_c != 0.0f;
  ServerCmd d;
  state_fields(p, st, d);
  a.x0 = d.x0;
  a.y0 = d.y0;
  a.h0x = d.h0x;
  a.h0y = d.h0y;
  a.h0z = d.h0z;
  a.wl = d.wl;
  a.wr = d.wr;
  a.gx = d.gx;
  a.gy = d.gy;
  a.s1 = d.s1;
  a.s2 = d.s2;
  a.pf_far = d.pf_far;
  a.igx = d.igx;
  a.igy = d.igy;
  a.pf_scale = d.pf_scale;
  a.speed_on = d.speed_on;
  a.seed = p.seed;
  a.n_base = step * (uint64_t)((H + 1) / 2);
  a.u_nom1 = unom;
  a.u_nom2 = unom + H;
  a.min_u1 = p.min_u1;
  a.max_u1 = p.max_u1;
  a.min_u2 = p.min_u2;
  a.max_u2 = p.max_u2;
  a.fk = p.filter_k;
  a.fa = p.filter_a;
  a.rwheel = p.robot_radius;
  a.vmin = p.v_min_linear;
  a.vmax = p.v_max_linear;
  a.wmin = p.v_min_angular;
  a.wmax = p.v_max_angular;
  a.dt = p.dt;
  a.off = p.wheel_offset;
  a.w_path = p.w_path;
  a.w_slope = p.w_slope;
  a.w_speed = p.w_speed;
  a.w_obs = p.w_obstacle;
  a.thr = p.collision_threshold;
  a.pen = p.collision_penalty;
  a.T = p.temperature;
  a.cost_out = c->cost;
  a.clk = c->clk;
  a.nodes = c->nodes;
  a.rec_m = c->rec_m;
  a.ustore = c->ustore;
  a.inj_u1 = c->inj1;
  a.inj_u2 = c->inj2;
  a.wave_prio = 1;
  // |w dt| < pi/4 for every clamped w: sin / cos without the range reduction (same bits)
  a.small_angle = std::max(std::fabs(p.v_min_angular), std::fabs(p.v_max_angular)) * p.dt < 0.78f;
}

void fill_finish(const mppi_ctx* c, const Plan& pl, const mppi_state& st, FinishArgs& f) {
  const mppi_params& p = c->p;
  std::memset(&f, 0, sizeof(f));
  f.H = p.num_iterations;
  f.T = p.temperature;
  f.scratch0 = c->scratch0;
  f.scratch1 = c->scratch1;
  f.uopt = c->uopt;
  f.u_nom_next = c->u_nom[c->cur ^ 1];
  f.out = c->stage;
  f.Z = c->Z;
  f.ntab = c->ntab;
  f.rows = c->rows;
  f.grid = c->cols;
  f.x_min = c->x_min;
  f.y_min = c->y_min;
  f.res = c->res;
  f.rinv_res = c->rinv_res;
  f.cdiv_res = c->rinv_res != 0.0f;
  f.x0 = st.x;
  f.y0 = st.y;
  f.h0x = st.heading[0];
  f.h0y = st.heading[1];
  f.h0z = st.heading[2];
  f.wl = st.left_wheel_speed;
  f.wr = st.right_wheel_speed;
  f.ok = p.opt_filter_k;
  f.oa = p.opt_filter_a;
  f.rwheel = p.robot_radius;
  f.vmin = p.v_min_linear;
  f.vmax = p.v_max_linear;
  f.wmin = p.v_min_angular;
  f.wmax = p.v_max_angular;
  f.dt = p.dt;
  f.off = p.wheel_offset;
}

void collect_timing(mppi_ctx* c) {
  float ms = 0.f;
  // mode 2: the host spun on the completion word, which the finish (enqueued after ev[1])
  // publishes, so ev[1] has retired already
  if (c->ev_roll_pending && hipEventSynchronize(c->ev[1]) == hipSuccess &&
      hipEventElapsedTime(&ms, c->ev[0], c->ev[1]) == hipSuccess) {
    c->t_roll += ms;
    c->launches += 1;
  }
  if (c->ev_fin_pending && hipEventElapsedTime(&ms, c->ev[2], c->ev[3]) == hipSuccess) c->t_fin += ms;
  c->ev_roll_pending = c->ev_fin_pending = false;
}

// Tail timing events live on the side stream: fold them in once the tail is done.
void collect_tail_timing(mppi_ctx* c) {
  if (!c->ev_tail_pending) return;
  float ms = 0.f;
  if (hipEventSynchronize(c->ev[5]) == hipSuccess && hipEventElapsedTime(&ms, c->ev[4], c->ev[5]) == hipSuccess) {
    c->t_tail += ms;
    c->tail_launches += 1;
  }
  c->ev_tail_pending = false;
}

int enqueue_tail(mppi_ctx* c, const FinishArgs& f, int par);

// Launch the server's deferred tail of the last step (its completion word has been seen).
int flush_tail(mppi_ctx* c) {
  if (!c->tail_deferred) return MPPI_OK;
  c->tail_deferred = false;
  return enqueue_tail(c, c->tail_def, c->tail_def_par);
}

// Wait until no deferred optimal rollout can still read tail_in or the DEM, and
// merge the latest one's outputs into out_host[4H, 16H).
int sync_tail(mppi_ctx* c) {
  const int rc = flush_tail(c);
  if (rc) return rc;
  bool any = c->tail_pending;
  for (int i = 0; i < kTailSlots; ++i) any |= c->tail_inflight[i];
  if (!any) return MPPI_OK;
  // The tails' streams are drained, not only their events, the latest tail's last: a stream's first
  // synchronize after a kernel costs ~8-15 us of runtime work even when the kernel is long done
  // (profiles/ubench/devsync.hip), which the caller's next device synchronize would pay otherwise;
  // the older tails' stream is drained while the latest tail runs.
  hipStream_t last = c->tail_pending ? c->tail_ts[c->tail_par] : nullptr;
  for (int i = 0; i < kTailSlots; ++i)
    if (c->tail_inflight[i] && c->tail_ts[i] && c->tail_ts[i] != last) {
      const hipStream_t ts = c->tail_ts[i];
      HIP_TRY(hipStreamSynchronize(ts));
      for (int j = 0; j < kTailSlots; ++j)
        if (c->tail_ts[j] == ts) c->tail_inflight[j] = false;
    }
  if (last) HIP_TRY(hipStreamSynchronize(last));
  for (int i = 0; i < kTailSlots; ++i)
    if (c->tail_inflight[i] || (c->tail_pending && i == c->tail_par)) HIP_TRY(hipEventSynchronize(c->ev_tail[i]));
  collect_tail_timing(c);
  for (int i = 0; i < kTailSlots; ++i) c->tail_inflight[i] = false;
  if (c->tail_pending) {
    const int H = H_of(c);
    std::memcpy(c->out_host + 4 * H, c->tail_host[c->tail_par], (size_t)12 * H * sizeof(float));
    c->tail_pending = false;
  }
  return MPPI_OK;
}

// Tell the running server to leave (it finishes the step it runs, reads its launch id in cmd->stop
// and exits) without waiting: launches enqueued after it on the context stream run once it retired.
void post_stop(mppi_ctx* c) {
  if (!c->srv_running) return;
  __atomic_store_n(&c->cmd->stop, c->srv_launch_id, __ATOMIC_RELEASE);
  c->srv_running = false;
  c->srv_exiting = true;
}

// Stop the resident server and wait until it has retired: every call on the context but mppi_step /
// set_state / get_outputs / get_timing starts with this.  Bounded (10 s: its workgroups must get CUs
// to leave, which another process's kernels can hold): MPPI_EHIP if it did not retire.
int quiesce(mppi_ctx* c) {
  if (!c) return MPPI_OK;
  post_stop(c);
  if (!c->srv_exiting) return MPPI_OK;
  hipSetDevice(c->device);
  const double t0 = now_us();
  for (;;) {
    const hipError_t e = hipStreamQuery(c->stream);
    if (e == hipSuccess) break;
    if (e != hipErrorNotReady) {
      c->srv_exiting = false;
      return fail(MPPI_EHIP, std::string("step server: ") + hipGetErrorString(e));
    }
    if (now_us() - t0 > 10e6) return fail(MPPI_EHIP, "the step server did not retire within 10 s of its stop");
    std::this_thread::yield();
  }
  c->srv_exiting = false;
  return MPPI_OK;
}

// Zero the finish handoff counter (level1_cnt[0]) and the server's record counter ([16]) after a
// step that did not complete them; no launch of the context may be running.
void rearm_counters(mppi_ctx* c) {
  if (hipMemsetAsync(c->level1_cnt, 0, 128, c->stream) == hipSuccess) hipStreamSynchronize(c->stream);
}

// Launch the resident server for the posted command `seq` (its first), with the plan of the last
// server_step (c->srv_pl ...).  Neither the relay nor cmd->stop needs a reset: the relay's seq word is
// older than this command, and the stop words hold an earlier launch's id, never this one's (a
// relaunch for the same command included).
int launch_server(mppi_ctx* c, unsigned seq) {
  const Plan& pl = c->srv_pl;
  RolloutArgs a;
  fill_rollout(c, pl, c->st, 0, c->u_nom[c->cur], a);  // (state, nominal buffer: from each command)
  ServerArgs z;
  std::memset(&z, 0, sizeof(z));
  fill_finish(c, pl, c->st, z.f);
  z.f.recs = c->nodes;
  z.f.rec_m = c->rec_m;
  z.f.n_recs = pl.blocks;
  z.f.level1 = c->level1;
  z.f.level1_cnt = c->level1_cnt;
  z.f.abort = c->level1_cnt + 24;  // (re-armed with the counters after a failed step)
  z.f.done = c->done;
  z.nroll = pl.blocks;
  z.fin_P = c->srv_P;
  z.fin_ncol = c->srv_ncol;
  z.fin_groups = c->srv_groups;
  z.rec_cnt = c->level1_cnt + 16;
  z.cmd = c->cmd;
  z.relay = c->relay;
  z.clk = c->clk;
  for (int i = 0; i < kEpsSlots; ++i) z.eps[i] = c->eps[i];
  z.u_nom[0] = c->u_nom[0];
  z.u_nom[1] = c->u_nom[1];
  for (int i = 0; i < kTailSlots; ++i) {
    z.tail_in[i] = c->tail_in[i];
    z.tail_out[i] = c->tail_host[i];
  }
  z.first_seq = seq;
  if (++c->srv_launch_id == 0) c->srv_launch_id = 1;
  z.launch_id = c->srv_launch_id;
  z.wait_ticks = c->fin_wait_ticks;
  z.idle_ticks = c->srv_idle_us * 100;
  z.exit_after = c->srv_exit_after;
  c->srv_exit_after = 0;  // (the hook applies to one launch)
  HIP_TRY(launch_step_server(a, z, c->srv_lds, c->stream, c->srv_proj));
  c->srv_running = true;
  ++c->srv_launches;
  return MPPI_OK;
}

// Spin until the finish has published c->wait_seq (all outputs in pinned host memory).  A server
// that retired without taking the posted command (its head left on the idle limit just before the
// command was posted: an exit is all-or-nothing, so nothing of the step ran) is relaunched with the
// same command, counted in srv_relaunches; a fresh launch that retires without serving it fails the
// step.  A finish that gave up (done | kDoneFail), any other launch that retired without publishing,
// a stream error or 10 s without completion fail the step; the server is stopped and the counters
// re-armed.
int wait_done(mppi_ctx* c) {
  if (c->timing == 1) {  // the finish's timing events need the stream to retire
    HIP_TRY(hipStreamSynchronize(c->stream));
  }
  const unsigned want = c->wait_seq;
  const double t0 = now_us();
  std::string why;
  c->fail_kind = 0;
  bool relaunched = false;
  for (uint64_t i = 0;; ++i) {
    const unsigned v = __atomic_load_n(c->done, __ATOMIC_ACQUIRE);
    if (v == want) break;
    if (v == (want | kDoneFail)) {
      why = "the finish gave up waiting for the step's records";
      c->fail_kind = 1;
      break;
    }
    if ((i & 255) == 255) {
      const hipError_t e = hipStreamQuery(c->stream);
      if (e == hipSuccess) {
        if (__atomic_load_n(c->done, __ATOMIC_ACQUIRE) == want) break;
        c->srv_running = false;  // (an idle server has exited: the stream is empty)
        if (c->srv_cmd_live && !relaunched) {
          relaunched = true;
          ++c->srv_relaunches;
          const int rc = launch_server(c, want);
          if (rc) {
            c->srv_cmd_live = false;
            return rc;
          }
          continue;
        }
        why = relaunched ? "a freshly launched step server retired without serving the step"
                         : "the step's launch retired without publishing its outputs";
        c->fail_kind = 2;
        break;
      }
      if (e != hipErrorNotReady) {
        c->srv_cmd_live = false;
        return fail(MPPI_EHIP, std::string("step failed: ") + hipGetErrorString(e));
      }
      if (now_us() - t0 > 10e6) {
        why = "the step did not complete within 10 s";
        c->fail_kind = 3;
        break;
      }
    }
    __builtin_ia32_pause();
  }
  if (c->fail_kind == 0) {
    if (c->srv_cmd_live) c->srv_last_us = now_us();  // (the head polls for the next command from here)
    c->srv_cmd_live = false;
    return MPPI_OK;
  }
  c->srv_cmd_live = false;
  ++c->srv_failed;
  // (a server whose workgroups cannot all get CUs retires once they do: until then nothing may be
  // re-armed or rerun, and a server that never retires fails the call here)
  const std::string saved = why;
  if (quiesce(c)) {
    c->fail_kind = 3;
    return fail(MPPI_EHIP, saved + "; " + g_err);
  }
  rearm_counters(c);
  // the normals the failed step's server was to generate may be incomplete: regenerate them
  if (c->last_resident && c->srv_cmd_noise >= 0) c->eps_step[c->srv_cmd_noise] = -1;
  return fail(MPPI_EHIP, why);
}

// Normals of Philox step `step` in an eps slot, generated on `st` if no slot holds them (first
// step, or a step counter that did not advance by one).  sync: wait for the slot on the host (the
// server reads it without stream order) instead of ordering `st` after it.
int eps_for_step(mppi_ctx* c, const Plan& pl, uint64_t step, hipStream_t st, bool sync, int* slot_out) {
  const size_t need = (size_t)pl.blocks * 2 * H_of(c) * 256;
  if (need > c->eps_cap) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipStreamSynchronize(c->noise_stream));
    for (int i = 0; i < kEpsSlots; ++i) {
      if (c->eps[i]) HIP_TRY(hipFree(c->eps[i]));
      c->eps[i] = nullptr;
      c->eps_step[i] = -1;
      c->eps_pending[i] = false;
    }
    for (int i = 0; i < kEpsSlots; ++i) HIP_TRY(hipMalloc(&c->eps[i], need * sizeof(float)));
    c->eps_cap = need;
  }
  const uint64_t nb = (uint64_t)((H_of(c) + 1) / 2);
  int slot = -1;
  for (int i = 0; i < kEpsSlots; ++i)
    if (c->eps_step[i] == (int64_t)step) slot = i;
  if (slot < 0) {
    // not precomputed: any in-flight fill must finish before a slot is reused
    for (int i = 0; i < kEpsSlots; ++i)
      if (c->eps_pending[i]) {
        HIP_TRY(sync ? hipEventSynchronize(c->eps_ev[i]) : hipStreamWaitEvent(st, c->eps_ev[i], 0));
        c->eps_pending[i] = false;
      }
    slot = 0;
    for (int i = 0; i < kEpsSlots; ++i) c->eps_step[i] = -1;
    HIP_TRY(launch_noise(c->p.seed, step * nb, c->p.k_offset, pl.blocks, H_of(c), c->eps[slot], st, noise_groups(c)));
    c->eps_step[slot] = (int64_t)step;
    if (sync) HIP_TRY(hipStreamSynchronize(st));
  } else if (c->eps_pending[slot]) {  // generated on noise_stream: before this rollout
    const hipError_t q = hipEventQuery(c->eps_ev[slot]);
    if (q == hipErrorNotReady) HIP_TRY(sync ? hipEventSynchronize(c->eps_ev[slot]) : hipStreamWaitEvent(st, c->eps_ev[slot], 0));
    else if (q != hipSuccess) return fail(MPPI_EHIP, std::string("noise: ") + hipGetErrorString(q));
    c->eps_pending[slot] = false;
  }
  *slot_out = slot;
  return MPPI_OK;
}

// A slot other than `used` that holds none of the steps in (step, step + 2]: the stalest one (its
// last reader is a rollout enqueued before the current one).
int eps_victim(const mppi_ctx* c, int used, uint64_t step) {
  for (int i = 0; i < kEpsSlots; ++i) {
    if (i == used) continue;
    const int64_t s = c->eps_step[i];
    if (s > (int64_t)step && s <= (int64_t)step + 2) continue;
    return i;
  }
  return -1;
}

// After the rollout of `step` (which reads slot `used`) is enqueued: make sure the normals of steps
// step + 1 and step + 2 are generated or in flight, on noise_stream after the event `after` (recorded
// after this rollout, the last reader of a reused slot).  In steady state that is one launch, of step
// + 2's normals, which then has the finish, the host round trip and the whole next step to complete,
// so no rollout waits for it, and which runs beside the finish and the next rollout, not this one.
int speculate_eps(mppi_ctx* c, const Plan& pl, uint64_t step, int used, hipEvent_t after) {
  const uint64_t nb = (uint64_t)((H_of(c) + 1) / 2);
  bool waited = false;
  for (int d = 1; d <= 2; ++d) {
    const uint64_t target = step + (uint64_t)d;
    bool have = false;
    for (int i = 0; i < kEpsSlots; ++i) have |= c->eps_step[i] == (int64_t)target;
    if (have) continue;
    const int slot = eps_victim(c, used, step);
    if (slot < 0) return fail(MPPI_ESTATE, "no free noise slot");
    if (!waited) {
      HIP_TRY(hipStreamWaitEvent(c->noise_stream, after, 0));
      waited = true;
    }
    HIP_TRY(launch_noise(c->p.seed, target * nb, c->p.k_offset, pl.blocks, H_of(c), c->eps[slot], c->noise_stream,
                         noise_groups(c)));
    HIP_TRY(hipEventRecord(c->eps_ev[slot], c->noise_stream));
    c->eps_step[slot] = (int64_t)target;
    c->eps_pending[slot] = true;
  }
  return MPPI_OK;
}

// Enqueue the rollout kernel for the current state / nominal sequence.
int enqueue_rollout(mppi_ctx* c, int proj, uint64_t step, int mode, const Plan& pl,
                    const float* unom, const mppi_state& st, const RolloutArgs* dump_args,
                    int* spec_slot = nullptr) {
  if (proj != MPPI_PROJ_2D && proj != MPPI_PROJ_3D) return fail(MPPI_EINVAL, "proj must be 2 or 3");
  int rc = ensure_nodes(c, pl.blocks);
  if (rc) return rc;
  if (mode == 1) {  // injected controls: the leaf reads them back from here
    rc = grow(c->ustore, c->ustore_cap, (size_t)pl.blocks * pl.traj_per_block * 2 * H_of(c) * sizeof(float), c->stream);
    if (rc) return rc;
  }
  RolloutArgs a;
  fill_rollout(c, pl, st, step, unom, a);
  int eps_slot = -1;
  if (mode == 0 && pl.blocks > 0) {
    rc = eps_for_step(c, pl, step, c->stream, false, &eps_slot);
    if (rc) return rc;
    a.eps = c->eps[eps_slot];
  }
  if (dump_args) {
    a.d_traj = dump_args->d_traj;
    a.d_hv = dump_args->d_hv;
    a.d_lw = dump_args->d_lw;
    a.d_rw = dump_args->d_rw;
    a.d_v = dump_args->d_v;
    a.d_w = dump_args->d_w;
    a.d_u1 = dump_args->d_u1;
    a.d_u2 = dump_args->d_u2;
  }
  if (pl.blocks == 0) return MPPI_OK;
  if (c->timing && !dump_args) {
    // the rollout kernel's own time: nothing already enqueued on the side streams (the noise of a
    // later step, the previous step's deferred optimal rollout) runs beside the timed launch (both
    // modes, so that a kernel trace of the timing passes averages isolated launches only)
    HIP_TRY(hipEventRecord(c->ev_side[0], c->noise_stream));
    HIP_TRY(hipEventRecord(c->ev_side[1], c->tail_stream));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_side[0], 0));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_side[1], 0));
  }
  if (c->timing && !dump_args) HIP_TRY(hipEventRecord(c->ev[0], c->stream));
  HIP_TRY(launch_rollout_pair(a, pl.grid, pl.lds_bytes, c->stream, proj, mode, dump_args != nullptr, pl.roles));
  if (c->timing && !dump_args) {
    HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    c->ev_roll_pending = true;
  }
  if (eps_slot >= 0 && !dump_args && spec_slot && c->eps_late) {
    *spec_slot = eps_slot;  // (speculate_after: once the caller has enqueued the finish)
    return MPPI_OK;
  }
  if (eps_slot >= 0 && !dump_args) {  // the next steps' normals on the noise stream after this rollout
    HIP_TRY(hipEventRecord(c->ev_prev_roll, c->stream));
    return speculate_eps(c, pl, step, eps_slot, c->ev_prev_roll);
  }
  return MPPI_OK;
}

// The next steps' normals of a rollout enqueued with spec_slot set, ordered after what the context
// stream holds now (the finish): no event marker between the rollout and the finish.
int speculate_after(mppi_ctx* c, const Plan& pl, uint64_t step, int spec_slot) {
  if (spec_slot < 0) return MPPI_OK;
  HIP_TRY(hipEventRecord(c->ev_prev_roll, c->stream));
  return speculate_eps(c, pl, step, spec_slot, c->ev_prev_roll);
}

// Finish arguments for `mode` (0: rank record, 1: finish; 1 becomes 2 with the deferred
// optimal rollout): claims the completion sequence number and the tail buffers of the
// next slot, ordering the context stream after the tail that last used them.
int prepare_finish(mppi_ctx* c, const Plan& pl, const mppi_state& st, int mode, double* record_out,
                   FinishArgs& f, int& par) {
  // a server step's deferred tail (its completion word was seen) takes its slot first, so the slot
  // picked below is not the one it still has to read and write
  const int rc = flush_tail(c);
  if (rc) return rc;
  c->srv_cmd_live = false;
  fill_finish(c, pl, st, f);
  if (mode == 1 && c->async_tail) mode = 2;
  f.mode = mode;
  f.record_out = record_out;
  if (mode >= 1) {
    f.done = c->done;
    f.seq = ++c->seq;
    c->wait_seq = c->seq;
  }
  par = (c->tail_par + 1) % kTailSlots;
  if (mode == 2) {
    f.tail_in = c->tail_in[par];
    f.tail_out = c->tail_host[par];
    // the tail of two steps ago used these buffers; in steady state it finished long ago
    // (it is shorter than a rollout kernel), so the cross-stream wait is rarely enqueued
    if (c->tail_inflight[par]) {
      const hipError_t q = hipEventQuery(c->ev_tail[par]);
      if (q == hipErrorNotReady) HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_tail[par], 0));
      else if (q != hipSuccess) return fail(MPPI_EHIP, std::string("tail: ") + hipGetErrorString(q));
      else c->tail_inflight[par] = false;
    }
  }
  return MPPI_OK;
}

// The deferred optimal rollout on a side stream: after the context stream's finish (event), or, for
// the resident server (its finish has published: f.clk set), at once.  The server's tails alternate
// over the tail and the noise stream: beside a server workgroup a tail takes about
// two step periods (~175 us against ~52 us alone at C3), so on one stream each waited for the one
// before it and the host for the slot.  More streams than the process's hardware queues
// (GPU_MAX_HW_QUEUES, 4 by default: torch's, the context's, the tail's and the noise stream's)
// share a queue, and a tail queued behind the resident server on the context's queue waited for it
// (measured with one stream per slot: every fourth command 66-102 us late).
int enqueue_tail(mppi_ctx* c, const FinishArgs& f, int par) {
  const bool server = f.clk != nullptr;
  hipStream_t ts = (server && (par & 1)) ? c->noise_stream : c->tail_stream;
  if (!server) {
    HIP_TRY(hipEventRecord(c->ev_fin_done, c->stream));
    HIP_TRY(hipStreamWaitEvent(c->tail_stream, c->ev_fin_done, 0));
  }
  if (c->timing == 1) {  // (collecting waits for the previous tail: mode 2 leaves the tail untimed)
    collect_tail_timing(c);
    HIP_TRY(hipEventRecord(c->ev[4], ts));
  }
  HIP_TRY(launch_tail(f, ts));
  if (c->timing == 1) {
    HIP_TRY(hipEventRecord(c->ev[5], ts));
    c->ev_tail_pending = true;
  }
  HIP_TRY(hipEventRecord(c->ev_tail[par], ts));
  c->tail_ts[par] = ts;
  c->tail_inflight[par] = true;
  c->tail_par = par;
  c->tail_pending = true;
  return MPPI_OK;
}

int enqueue_finish(mppi_ctx* c, const Plan& pl, const mppi_state& st, const double* recs, int n,
                   int mode, double* record_out, bool timed) {
  FinishArgs f;
  int par = 0;
  int rc = prepare_finish(c, pl, st, mode, record_out, f, par);
  if (rc) return rc;
  f.recs = recs;
  f.n_recs = n;
  f.rec_m = recs == c->nodes ? c->rec_m : nullptr;  // this context's rollout records
  if (n > 1) {
    rc = ensure_nodes(c, n);
    if (rc) return rc;
    f.scratch0 = c->scratch0;
    f.scratch1 = c->scratch1;
  }
  // column-split finish (default): one launch, no partial-tree handoff between workgroups
  int cf_P = 0, cf_ncol = 0, cf_groups = 0;
  size_t cf_lds = 0;
  if (c->colfin && colfin_shape(n, H_of(c), &cf_P, &cf_ncol, &cf_groups, &cf_lds)) {
    f.level1 = c->level1;
    f.level1_cnt = c->level1_cnt;
    c->fin_kind = 1;
    c->fin_P = cf_P;
    c->fin_ncol = cf_ncol;
    c->fin_groups = cf_groups;
    const size_t lds = std::max(cf_lds, f.mode == 0 ? (size_t)0 : pl.fin_lds_bytes);
    if (timed && c->timing == 1) HIP_TRY(hipEventRecord(c->ev[2], c->stream));
    HIP_TRY(launch_colfin(f, lds, c->stream, cf_P, cf_ncol, cf_groups));
    if (timed && c->timing == 1) {
      HIP_TRY(hipEventRecord(c->ev[3], c->stream));
      c->ev_fin_pending = true;
    }
    if (f.mode == 2) return enqueue_tail(c, f, par);
    return MPPI_OK;
  }
  // first tree level on ceil(n/16) workgroups (one per aligned group of 16 records)
  const int groups = n > 16 ? (n + 15) / 16 : 1;
  if (groups > 1) {
    rc = grow(c->level1, c->level1_cap, (size_t)groups * E_of(c) * sizeof(double), c->stream);
    if (rc) return rc;
    f.level1 = c->level1;
    f.level1_cnt = c->level1_cnt;
  }
  c->fin_kind = 0;
  c->fin_P = n;
  c->fin_ncol = 0;
  c->fin_groups = groups;
  if (timed && c->timing == 1) HIP_TRY(hipEventRecord(c->ev[2], c->stream));
  HIP_TRY(launch_finish(f, f.mode == 0 ? pl.fin_tree_bytes : pl.fin_lds_bytes, c->stream, groups));
  if (timed && c->timing == 1) {
    HIP_TRY(hipEventRecord(c->ev[3], c->stream));
    c->ev_fin_pending = true;
  }
  if (f.mode == 2) return enqueue_tail(c, f, par);
  return MPPI_OK;
}

void fill_outputs(const float* o, int H, mppi_outputs* out) {
  if (out->u1_opt) std::memcpy(out->u1_opt, o, H * sizeof(float));
  if (out->u2_opt) std::memcpy(out->u2_opt, o + H, H * sizeof(float));
  if (out->lin_vel) std::memcpy(out->lin_vel, o + 2 * H, H * sizeof(float));
  if (out->ang_vel) std::memcpy(out->ang_vel, o + 3 * H, H * sizeof(float));
  if (out->traj_sim) std::memcpy(out->traj_sim, o + 4 * H, 3 * H * sizeof(float));
  if (out->heading_sim) std::memcpy(out->heading_sim, o + 7 * H, 3 * H * sizeof(float));
  if (out->left_wheel_sim) std::memcpy(out->left_wheel_sim, o + 10 * H, 3 * H * sizeof(float));
  if (out->right_wheel_sim) std::memcpy(out->right_wheel_sim, o + 13 * H, 3 * H * sizeof(float));
}

int copy_outputs(mppi_ctx* c, mppi_outputs* out) {
  const int H = H_of(c);
  int rc = wait_done(c);
  if (rc) {
    c->tail_pending = false;  // a failed step's tail (if any) has nothing to merge or to launch
    c->tail_deferred = false;
    return rc;
  }
  if (c->async_tail) {
    // controls + the first optimal-rollout row now; rows 1.. arrive with the tail
    const float* stage = c->stage;
    collect_timing(c);
    c->cur ^= 1;
    std::memcpy(c->out_host, stage, (size_t)4 * H * sizeof(float));
    if (out) {
      const float* o = stage;
      if (out->u1_opt) std::memcpy(out->u1_opt, o, H * sizeof(float));
      if (out->u2_opt) std::memcpy(out->u2_opt, o + H, H * sizeof(float));
      if (out->lin_vel) std::memcpy(out->lin_vel, o + 2 * H, H * sizeof(float));
      if (out->ang_vel) std::memcpy(out->ang_vel, o + 3 * H, H * sizeof(float));
      if (out->traj_sim) std::memcpy(out->traj_sim, o + 4 * H, 3 * sizeof(float));
      if (out->heading_sim) std::memcpy(out->heading_sim, o + 4 * H + 3, 3 * sizeof(float));
      if (out->left_wheel_sim) std::memcpy(out->left_wheel_sim, o + 4 * H + 6, 3 * sizeof(float));
      if (out->right_wheel_sim) std::memcpy(out->right_wheel_sim, o + 4 * H + 9, 3 * sizeof(float));
    }
    return MPPI_OK;
  }
  std::memcpy(c->out_host, c->stage, (size_t)16 * H * sizeof(float));
  collect_timing(c);
  c->cur ^= 1;  // the finish wrote the new nominal sequence into u_nom[cur^1]
  if (out) fill_outputs(c->out_host, H, out);
  return MPPI_OK;
}

void remember(mppi_ctx* c, int proj, uint64_t step, int mode, const Plan& pl) {
  c->have_last = true;
  c->last_proj = proj;
  c->last_step = step;
  c->last_mode = mode;
  c->last_state = c->st;
  c->last_nominal = c->cur;  // nominal buffer the rollout read (before the swap)
  c->last_plan = pl;
}

// ---- resident step server (mppi_step_server_kernel) ----
// Sampled steps of the role-split plan whose records fit the column-split finish in the rollout
// workgroups (C1-C3).  Per step the host waits (normally not at all) for the step's normals and the
// tail slot it reuses, writes the command (state, slots, nominal buffer, the slot for the normals of
// step + 2 that the server's noise phase generates, then seq), launches the server if it is not
// running, launches the PREVIOUS step's deferred optimal rollout (flush_tail: its completion word has
// been seen) and spins on the completion word.  This step's tail stays on the host (tail_deferred)
// until the next step, sync_tail (get_outputs and every call that quiesces before reading the DEM)
// or prepare_finish (any separate-launch finish: it takes the slot after the deferred one).  No launch and no kernel boundary on the step's path: the gap between two steps
// is the host's round trip (completion word seen -> next command) plus one poll of pinned memory.
// MPPI_HOST_TRACE marks of a step: 0 entry, 1 normals ready, 2 tail slot free (server), 3 command
// posted / launches enqueued, 4 side launches done (the previous tail), 5 completion seen + copies
void trace_mark(mppi_ctx* c, int k) {
  if (c && c->trace) c->tr_m[k] = now_us();
}

bool server_shape(const mppi_ctx* c, const Plan& pl, int mode, int* P, int* ncol, int* groups, size_t* lds) {
  // (every workgroup of the server must be resident at once: one rollout block per CU at most)
  if (!c->resident || mode != 0 || !pl.roles || !c->colfin || c->timing != 0 || pl.blocks < 1 ||
      pl.blocks > std::max(c->num_cus, 1))
    return false;
  size_t cf_lds = 0;
  // the finish runs in the workgroups holding the last `groups` tickets: at most one per rollout workgroup
  if (!colfin_shape(pl.blocks, H_of(c), P, ncol, groups, &cf_lds, pl.blocks)) return false;
  *lds = std::max({pl.lds_bytes, cf_lds, pl.fin_lds_bytes});
  return *lds + 256 <= kLdsBytes;  // + the kernel's static words (command, ticket)
}

int server_step(mppi_ctx* c, int proj, uint64_t step, const Plan& pl, int P, int ncol, int groups, size_t lds) {
  if (proj != MPPI_PROJ_2D && proj != MPPI_PROJ_3D) return fail(MPPI_EINVAL, "proj must be 2 or 3");
  if (c->srv_running && proj != c->srv_proj) post_stop(c);  // (the next launch queues behind it)
  // (first step: the buffers are allocated before the server holds pointers to them)
  int rc = MPPI_OK;
  if (c->nodes_cap < (size_t)pl.blocks * E_of(c) || c->eps_cap < (size_t)pl.blocks * 2 * H_of(c) * 256)
    rc = quiesce(c);
  if (!rc) rc = ensure_nodes(c, pl.blocks);
  if (rc) return rc;
  int slot = 0, noise_slot = -1;
  const uint64_t nb = (uint64_t)((H_of(c) + 1) / 2);  // Philox blocks per trajectory and step
  // a step whose normals no slot holds (first step, a jump of the step counter): the server may still
  // be writing normals of a later step in its last noise phase, so it is stopped before any slot is
  // regenerated
  bool have = false;
  for (int i = 0; i < kEpsSlots; ++i) have |= c->eps_step[i] == (int64_t)step;
  if (!have && (rc = quiesce(c))) return rc;
  rc = eps_for_step(c, pl, step, c->noise_stream, true, &slot);
  if (rc) return rc;
  trace_mark(c, 1);
  // normals of step + 1 (normally generated by the previous step's noise phase; else now, on the
  // noise stream beside this step) and of step + 2 (by this step's noise phase, in the server)
  // the server's noise phase runs mostly in the workgroups outside the finish: with fewer than a
  // quarter of them, or fewer than two (few records: every rollout workgroup may hold a finish
  // column) the noise kernel does it
  const bool srv_noise = pl.blocks - groups >= 2 &&
                         (int64_t)(pl.blocks - groups) * 4 >= (int64_t)pl.blocks;
  for (int d = 1; d <= 2; ++d) {
    const uint64_t target = step + (uint64_t)d;
    bool got = false;
    for (int i = 0; i < kEpsSlots; ++i) got |= c->eps_step[i] == (int64_t)target;
    if (got) continue;
    const int v = eps_victim(c, slot, step);
    if (v < 0) return fail(MPPI_ESTATE, "no free noise slot");
    if (d == 1 || !srv_noise) {
      HIP_TRY(launch_noise(c->p.seed, target * nb, c->p.k_offset, pl.blocks, H_of(c), c->eps[v], c->noise_stream,
                           noise_groups(c)));
      HIP_TRY(hipEventRecord(c->eps_ev[v], c->noise_stream));
      c->eps_pending[v] = true;
    } else {
      // complete before step + 2 can be commanded: every workgroup ends its noise phase before its
      // rollout of step + 1, whose records the completion of step + 1 needs
      noise_slot = v;
      c->eps_pending[v] = false;
    }
    c->eps_step[v] = (int64_t)target;
  }
  const int par = ((c->tail_deferred ? c->tail_def_par : c->tail_par) + 1) % kTailSlots;
  if (c->async_tail && c->tail_inflight[par]) {  // the tail of kTailSlots steps ago: long done
    HIP_TRY(hipEventSynchronize(c->ev_tail[par]));
    c->tail_inflight[par] = false;
  }
  trace_mark(c, 2);
  const unsigned seq = ++c->seq;
  c->wait_seq = seq;
  // the command: every field, then seq (release: the server reads the fields after seeing it)
  ServerCmd* cmd = c->cmd;
  ServerCmd d;
  std::memset(&d, 0, sizeof(d));
  state_fields(c->p, c->st, d);
  d.eps_slot = slot;
  d.cur = c->cur;
  d.tail_slot = par;
  d.mode = c->async_tail ? 2 : 1;
  d.noise_slot = noise_slot;
  c->srv_cmd_noise = noise_slot;
  const uint64_t nbase = (step + 2) * nb;
  d.noise_n_base_lo = (unsigned)nbase;
  d.noise_n_base_hi = (unsigned)(nbase >> 32);
  // a server idle for more than half its limit (since its last step completed) may be leaving: stop
  // it and start a fresh one behind it.  This is checked after the host's waits above, right before
  // the command is posted; a head that leaves anyway (a slower host) never relays the command, and
  // wait_done relaunches the server with it
  if (c->srv_running && now_us() - c->srv_last_us > 0.5 * (double)c->srv_idle_us) post_stop(c);
  unsigned* cw = reinterpret_cast<unsigned*>(cmd);
  const unsigned* dw = reinterpret_cast<const unsigned*>(&d);
  for (int i = 2; i < kCmdWords; ++i) __atomic_store_n(cw + i, dw[i], __ATOMIC_RELAXED);
  __atomic_store_n(&cmd->seq, seq, __ATOMIC_RELEASE);
  c->srv_pl = pl;
  c->srv_P = P;
  c->srv_ncol = ncol;
  c->srv_groups = groups;
  c->srv_lds = lds;
  c->srv_proj = proj;
  c->srv_cmd_live = true;
  if (!c->srv_running) {
    rc = launch_server(c, seq);
    if (rc) return rc;
  }
  c->srv_last_us = now_us();
  trace_mark(c, 3);
  ++c->srv_steps;
  c->fin_kind = 1;
  c->fin_P = P;
  c->fin_ncol = ncol;
  c->fin_groups = groups;
  rc = flush_tail(c);  // the previous step's tail (its outputs were published before this call)
  if (rc) return rc;
  if (c->async_tail) {  // rows 1.. of the optimal rollout: launched once this step has published
    FinishArgs& f = c->tail_def;
    fill_finish(c, pl, c->st, f);
    f.mode = 2;
    f.seq = seq;
    f.tail_in = c->tail_in[par];
    f.tail_out = c->tail_host[par];
    f.clk = c->clk;
    c->tail_deferred = true;
    c->tail_def_par = par;
  }
  trace_mark(c, 4);
  return MPPI_OK;
}

// The launches of one step (rollout + finish + tail) outside the server.
int enqueue_step(mppi_ctx* c, int proj, uint64_t step, int mode, const Plan& pl) {
  int spec = -1;
  int rc = enqueue_rollout(c, proj, step, mode, pl, c->u_nom[c->cur], c->st, nullptr, &spec);
  if (rc) return rc;
  trace_mark(c, 3);
  rc = enqueue_finish(c, pl, c->st, c->nodes, pl.blocks, 1, nullptr, true);
  if (rc) return rc;
  return speculate_after(c, pl, step, spec);
}

int step_impl(mppi_ctx* c, int proj, uint64_t step, int mode, mppi_outputs* out) {
  int rc = check_ready(c);
  if (rc) return rc;
  trace_mark(c, 0);
  const Plan pl = make_plan(c);
  int sP = 0, scol = 0, sgroups = 0;
  size_t slds = 0;
  bool resident = server_shape(c, pl, mode, &sP, &scol, &sgroups, &slds);
  const double now = now_us(), half = 0.5 * (double)c->srv_idle_us;
  const bool back_to_back = c->last_return_us > 0 && now - c->last_return_us <= half;
  c->b2b_calls = back_to_back ? c->b2b_calls + 1 : 0;
  c->eps_late = c->eps_after < 0 ? !back_to_back : c->eps_after == 1;
  if (resident && c->resident == 1) {
    // the caller's cadence: a call more than half the idle limit after the last step returned (a
    // simulator frame) runs as separate launches, and a server that has been idle that long is told
    // to leave (the launches queue behind it); back-to-back calls keep the server, and start one when
    // the last step ran on a server (stopped by another call since, e.g. a synchronize) or the call is
    // the second back-to-back one in a row (a lone back-to-back call after a frame-cadence step would
    // pay a server launch for one step: separate launches are cheaper there)
    if (c->srv_running ? now - c->srv_last_us > half : !(back_to_back && (c->last_resident || c->b2b_calls >= 2))) {
      post_stop(c);
      resident = false;
      ++c->cadence_steps;
    }
  }
  if (!resident) {
    post_stop(c);  // (stream order: these launches run after it retired)
    rc = flush_tail(c);
    if (rc) return rc;
  }
  rc = resident ? server_step(c, proj, step, pl, sP, scol, sgroups, slds) : enqueue_step(c, proj, step, mode, pl);
  if (rc) return rc;
  c->last_resident = resident;
  remember(c, proj, step, mode, pl);
  trace_mark(c, 4);
  rc = copy_outputs(c, out);
  // A server step that did not complete published nothing and changed no state (wait_done stopped
  // the server, waited for it to retire and re-armed its counters): this step again as separate
  // launches.  Its finish gave up (1: the rollout workgroups could not all get CUs within the wait
  // bound, e.g. beside another process's kernels): counted, the server stays the schedule.  A fresh
  // launch retired without serving its first command (2): it cannot run here, separate launches from
  // now on.  (A server that left on its idle limit as the command was posted is neither: wait_done
  // relaunched it.)
  if (resident && rc == MPPI_EHIP && (c->fail_kind == 1 || c->fail_kind == 2)) {
    if (c->fail_kind == 2) {
      if (!c->srv_warned)
        std::fprintf(stderr, "mppi: the resident step server could not run here; using separate launches\n");
      c->srv_warned = true;
      c->resident = 0;
    } else {
      ++c->srv_fallbacks;
    }
    c->last_resident = false;
    rc = enqueue_step(c, proj, step, mode, pl);
    if (rc) return rc;
    rc = copy_outputs(c, out);
  }
  c->last_return_us = now_us();
  if (c->trace) {  // marks a schedule does not set (separate launches: 1, 2) take the one before
    c->tr_m[5] = now_us();
    for (int k = 1; k < 6; ++k) c->tr_m[k] = std::max(c->tr_m[k], c->tr_m[k - 1]);
    if (c->tr_prev > 0) {
      c->tr_sum[0] += c->tr_m[0] - c->tr_prev;
      for (int k = 1; k < 6; ++k) c->tr_sum[k] += c->tr_m[k] - c->tr_m[k - 1];
      std::memcpy(c->tr_log[c->tr_n++ & 7], c->tr_m, sizeof(c->tr_m));
    }
    c->tr_prev = c->tr_m[5];
    std::memset(c->tr_m, 0, sizeof(c->tr_m));
  }
  return rc;
}

// ---- obstacle costmap builder (mppi_build_costmap / mppi_costmap_builder_*) ----

void costmap_free(CostmapScratch& sc) {
  if (sc.occ) hipFree(sc.occ);
  if (sc.first) hipFree(sc.first);
  if (sc.last) hipFree(sc.last);
  if (sc.g2) hipFree(sc.g2);
  if (sc.d2) hipFree(sc.d2);
  if (sc.range) hipFree(sc.range);
  if (sc.lines) hipFree(sc.lines);
  if (sc.obs) hipFree(sc.obs);
  if (sc.xs) hipFree(sc.xs);
  sc = CostmapScratch{};
}

int costmap_check(const double* obstacles, int32_t n, int32_t size, int32_t power, int32_t metric) {
  if (n < 0 || (n > 0 && !obstacles)) return fail(MPPI_EINVAL, "obstacles: null pointer or negative count");
  if (metric != MPPI_COSTMAP_CHAMFER5 && metric != MPPI_COSTMAP_EXACT && metric != MPPI_COSTMAP_CHAMFER5_RASTER)
    return fail(MPPI_EINVAL, "costmap metric must be MPPI_COSTMAP_CHAMFER5, MPPI_COSTMAP_EXACT or MPPI_COSTMAP_CHAMFER5_RASTER");
  if (size < 2 || size > COSTMAP_MAX_SIZE) return fail(MPPI_EINVAL, "costmap size must be in [2, 8192]");
  if (power < 0) return fail(MPPI_EINVAL, "costmap power must be >= 0");
  return MPPI_OK;
}

// Host staging for one build, with float64 arithmetic in the reference's order
// (MPPI_isaac.py:363-370): x_local = y_global - y0, y_local = x_global - x0,
// total_radius = r_obs/2 + r_robot + 0.1, squared with libm pow as CPython's `**`;
// grid coordinates as np.linspace(-hw, hw, size) (i*step + start, last = stop).
// The vectors must outlive the stream work (the caller synchronises).
int costmap_stage(CostmapScratch& sc, const double* obstacles, int32_t n, int32_t size, double hw, double ox,
                  double oy, double r_robot, std::vector<double>& obs, std::vector<double>& xs, hipStream_t st) {
  const size_t cells = (size_t)size * size;
  const size_t nseg = (size_t)(size + COSTMAP_SEG - 1) / COSTMAP_SEG;
  if (cells > sc.cells_cap) {
    HIP_TRY(hipStreamSynchronize(st));
    for (void* p : {(void*)sc.occ, (void*)sc.first, (void*)sc.last, (void*)sc.g2, (void*)sc.d2, (void*)sc.lines})
      if (p) HIP_TRY(hipFree(p));
    sc.occ = nullptr;
    sc.first = sc.last = sc.g2 = sc.d2 = nullptr;
    sc.lines = nullptr;
    sc.cells_cap = 0;
    HIP_TRY(hipMalloc(&sc.occ, cells));
    HIP_TRY(hipMalloc(&sc.first, nseg * size * sizeof(int32_t)));
    HIP_TRY(hipMalloc(&sc.last, nseg * size * sizeof(int32_t)));
    HIP_TRY(hipMalloc(&sc.g2, cells * sizeof(int32_t)));
    HIP_TRY(hipMalloc(&sc.d2, cells * sizeof(int32_t)));
    HIP_TRY(hipMalloc(&sc.lines, 16 * cells * sizeof(uint32_t)));
    sc.cells_cap = cells;
  }
  if (!sc.range) HIP_TRY(hipMalloc(&sc.range, (2 + 2 * COSTMAP_MAX_SIZE) * sizeof(int32_t)));
  const size_t nobs = (size_t)std::max<int32_t>(n, 1);
  int rc = grow(sc.obs, sc.obs_cap, nobs * 3 * sizeof(double), st);
  if (!rc) rc = grow(sc.xs, sc.xs_cap, (size_t)size * sizeof(double), st);
  if (rc) return rc;
  obs.assign(nobs * 3, 0.0);
  for (int32_t k = 0; k < n; ++k) {
    const double xg = obstacles[3 * k], yg = obstacles[3 * k + 1], r = obstacles[3 * k + 2];
    const double tr = r / 2 + r_robot + 0.1;
    obs[3 * k + 0] = yg - oy;
    obs[3 * k + 1] = xg - ox;
    obs[3 * k + 2] = std::pow(tr, 2.0);
  }
  xs.resize(size);
  const double start = -hw, stop = hw;
  const double step = (stop - start) / (double)(size - 1);
  for (int32_t i = 0; i < size; ++i) xs[i] = (double)i * step + start;
  xs[size - 1] = stop;
  HIP_TRY(hipMemcpyAsync(sc.obs, obs.data(), nobs * 3 * sizeof(double), hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(sc.xs, xs.data(), (size_t)size * sizeof(double), hipMemcpyHostToDevice, st));
  return MPPI_OK;
}

}  // namespace

struct mppi_costmap_builder {
  int device = 0;
  hipStream_t stream = nullptr;
  CostmapScratch sc;
  float* out = nullptr;
  size_t out_cap = 0;
  hipEvent_t ev[2] = {nullptr, nullptr};
  double last_ms = 0;
};

extern "C" {

int mppi_abi_version(void) { return MPPI_ABI_VERSION; }

const char* mppi_last_error(void) { return g_err.c_str(); }

int mppi_create(const mppi_params* params, int32_t device, mppi_ctx** out) {
  if (!params || !out) return fail(MPPI_EINVAL, "null argument");
  *out = nullptr;
  const mppi_params& p = *params;
  if (p.num_iterations < 1 || p.num_iterations > 255)
    return fail(MPPI_EINVAL, "num_iterations must be in [1, 255]");
  if (p.num_trajectories < 0 || p.num_trajectories > ((int64_t)1 << 31) * 64)
    return fail(MPPI_EINVAL, "num_trajectories out of range");
  if (p.k_offset < 0) return fail(MPPI_EINVAL, "k_offset must be >= 0");
  if (!(p.temperature > 0.0f)) return fail(MPPI_EINVAL, "temperature must be > 0");
  if (!(p.dt > 0.0f)) return fail(MPPI_EINVAL, "dt must be > 0");
  if (p.robot_radius == 0.0f) return fail(MPPI_EINVAL, "robot_radius must be non-zero");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev)
    return fail(MPPI_EHIP, "device " + std::to_string(device) + " not available (" +
                               std::to_string(ndev) + " HIP devices)");
  HIP_TRY(hipSetDevice(device));
  mppi_ctx* c = new mppi_ctx();
  c->p = p;
  c->device = device;
  {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
      c->num_cus = cus;
  }
  // runtime environment knobs: MPPI_HOST_TRACE, MPPI_ROLES, MPPI_RESIDENT (and
  // MPPI_GROUP_RCCL for groups)
  if (const char* e = std::getenv("MPPI_HOST_TRACE")) c->trace = std::atoi(e) != 0;
  if (const char* e = std::getenv("MPPI_ROLES")) c->roles = std::atoi(e) != 0;
  if (const char* e = std::getenv("MPPI_RESIDENT")) c->resident = std::min(std::max(std::atoi(e), 0), 2);
  const int H = p.num_iterations;
  auto cleanup = [&](int rc) {
    mppi_destroy(c);
    return rc;
  };
  // the rollout stream outranks the speculative noise stream at dispatch
  if (hipDeviceGetStreamPriorityRange(&c->prio_least, &c->prio_greatest) != hipSuccess)
    return cleanup(fail(MPPI_EHIP, "hipDeviceGetStreamPriorityRange failed"));
  if (hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, c->prio_greatest) != hipSuccess)
    return cleanup(fail(MPPI_EHIP, "hipStreamCreate failed"));
  c->own_stream = true;
  if (hipMalloc(&c->u_nom[0], 2 * H * sizeof(float)) != hipSuccess ||
      hipMalloc(&c->u_nom[1], 2 * H * sizeof(float)) != hipSuccess ||
      hipMalloc(&c->cost, std::max<int64_t>(p.num_trajectories, 1) * sizeof(float)) != hipSuccess ||
      hipHostMalloc(&c->stage, 16 * H * sizeof(float), hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc(&c->done, 64, hipHostMallocDefault) != hipSuccess ||
      hipMalloc(&c->cdiv_bad, sizeof(unsigned)) != hipSuccess ||
      hipMalloc(&c->level1_cnt, 128) != hipSuccess ||  // [0]: finish handoff, [16]: the server's record count
      hipMalloc(&c->uopt, (size_t)2 * H * sizeof(unsigned long long)) != hipSuccess ||
      hipHostMalloc(&c->cmd, sizeof(ServerCmd), hipHostMallocDefault) != hipSuccess ||
      hipMalloc(&c->relay, 64 * sizeof(unsigned)) != hipSuccess ||
      hipMalloc(&c->clk, kClkWords * sizeof(uint64_t)) != hipSuccess)
    return cleanup(fail(MPPI_EHIP, "device allocation failed"));
  for (int i = 0; i < kTailSlots; ++i)
    if (hipMalloc(&c->tail_in[i], 3 * H * sizeof(float)) != hipSuccess ||
        hipHostMalloc(&c->tail_host[i], 12 * H * sizeof(float), hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_tail[i], hipEventDisableTiming) != hipSuccess)
      return cleanup(fail(MPPI_EHIP, "tail slot allocation failed"));
  if (hipMemset(c->u_nom[0], 0, 2 * H * sizeof(float)) != hipSuccess ||
      hipMemset(c->u_nom[1], 0, 2 * H * sizeof(float)) != hipSuccess ||
      hipMemset(c->cost, 0, std::max<int64_t>(p.num_trajectories, 1) * sizeof(float)) != hipSuccess ||
      hipMemset(c->relay, 0, 64 * sizeof(unsigned)) != hipSuccess ||
      hipMemset(c->clk, 0, kClkWords * sizeof(uint64_t)) != hipSuccess)
    return cleanup(fail(MPPI_EHIP, "hipMemset failed"));
  for (auto& e : c->ev)
    if (hipEventCreate(&e) != hipSuccess) return cleanup(fail(MPPI_EHIP, "hipEventCreate failed"));
  if (hipEventCreateWithFlags(&c->ev_fin_done, hipEventDisableTiming) != hipSuccess ||
      hipStreamCreateWithFlags(&c->tail_stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithPriority(&c->noise_stream, hipStreamNonBlocking, c->prio_least) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_prev_roll, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_side[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_side[1], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->eps_ev[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->eps_ev[1], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->eps_ev[2], hipEventDisableTiming) != hipSuccess)
    return cleanup(fail(MPPI_EHIP, "side stream / event creation failed"));
  c->out_host = new float[16 * H]();
  std::memset(c->stage, 0, 16 * H * sizeof(float));
  *c->done = 0;
  std::memset(c->cmd, 0, sizeof(ServerCmd));
  if (hipMemset(c->level1_cnt, 0, 128) != hipSuccess ||
      hipMemset(c->uopt, 0, (size_t)2 * H * sizeof(unsigned long long)) != hipSuccess)
    return cleanup(fail(MPPI_EHIP, "hipMemset failed"));
  if (hipDeviceSynchronize() != hipSuccess) return cleanup(fail(MPPI_EHIP, "device sync failed"));
  *out = c;
  return MPPI_OK;
}

void mppi_destroy(mppi_ctx* c) {
  if (!c) return;
  (void)quiesce(c);
  if (c->trace && c->tr_n > 0) {
    static const char* ph[6] = {"caller", "normals wait", "tail slot wait", "command / launches", "side launches",
                                "completion + copies"};
    std::fprintf(stderr, "mppi host trace (us/step over %ld steps; server launches %ld, relaunches %ld):", c->tr_n,
                 (long)c->srv_launches, (long)c->srv_relaunches);
    for (int k = 0; k < 6; ++k) std::fprintf(stderr, "  %s %.1f", ph[k], c->tr_sum[k] / c->tr_n);
    std::fprintf(stderr, "\n");
    for (long r = std::max(0L, c->tr_n - 8); r < c->tr_n; ++r) {  // the last 8 steps' marks, from entry
      const double* lg = c->tr_log[r & 7];
      std::fprintf(stderr, "  host step %ld:", r);
      for (int k = 1; k < 6; ++k) std::fprintf(stderr, " %+7.1f", lg[k] - lg[0]);
      std::fprintf(stderr, "\n");
    }
  }
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->tail_stream) hipStreamSynchronize(c->tail_stream);
  if (c->noise_stream) hipStreamSynchronize(c->noise_stream);
  if (c->Z_owned && c->Z) hipFree(c->Z);
  if (c->ntab) hipFree(c->ntab);
  if (c->cm) hipFree(c->cm);
  costmap_free(c->cms);
  for (float* u : c->u_nom)
    if (u) hipFree(u);
  if (c->cost) hipFree(c->cost);
  if (c->rec_m) hipFree(c->rec_m);
  if (c->nodes) hipFree(c->nodes);
  if (c->scratch0) hipFree(c->scratch0);
  if (c->scratch1) hipFree(c->scratch1);
  if (c->ustore) hipFree(c->ustore);
  if (c->stage) hipHostFree(c->stage);
  if (c->done) hipHostFree(c->done);
  if (c->cdiv_bad) hipFree(c->cdiv_bad);
  delete[] c->out_host;
  for (int i = 0; i < kTailSlots; ++i) {
    if (c->tail_in[i]) hipFree(c->tail_in[i]);
    if (c->tail_host[i]) hipHostFree(c->tail_host[i]);
    if (c->ev_tail[i]) hipEventDestroy(c->ev_tail[i]);
  }
  if (c->ev_fin_done) hipEventDestroy(c->ev_fin_done);
  for (int i = 0; i < kEpsSlots; ++i) {
    if (c->eps[i]) hipFree(c->eps[i]);
    if (c->eps_ev[i]) hipEventDestroy(c->eps_ev[i]);
  }
  if (c->ev_prev_roll) hipEventDestroy(c->ev_prev_roll);
  for (hipEvent_t e : c->ev_side)
    if (e) hipEventDestroy(e);
  if (c->bin_tile_of) hipFree(c->bin_tile_of);
  if (c->level1) hipFree(c->level1);
  if (c->level1_cnt) hipFree(c->level1_cnt);
  if (c->uopt) hipFree(c->uopt);
  if (c->cmd) hipHostFree(c->cmd);
  if (c->relay) hipFree(c->relay);
  if (c->clk) hipFree(c->clk);
  if (c->bin_counts) hipFree(c->bin_counts);
  if (c->bin_cursor) hipFree(c->bin_cursor);
  if (c->bin_cx) hipFree(c->bin_cx);
  if (c->bin_cy) hipFree(c->bin_cy);
  if (c->bin_ci) hipFree(c->bin_ci);
  if (c->noise_stream) hipStreamDestroy(c->noise_stream);
  if (c->tail_stream) hipStreamDestroy(c->tail_stream);
  if (c->inj1) hipFree(c->inj1);
  if (c->inj2) hipFree(c->inj2);
  for (auto& e : c->ev)
    if (e) hipEventDestroy(e);
  if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
  delete c;
}

int mppi_set_stream(mppi_ctx* c, void* s) {
  if (!c) return fail(MPPI_EINVAL, "null context");
  if (int rc_q = quiesce(c)) return rc_q;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  int rc = sync_tail(c);
  if (rc) return rc;
  if (c->own_stream && c->stream) HIP_TRY(hipStreamDestroy(c->stream));
  if (s) {
    c->stream = (hipStream_t)s;
    c->own_stream = false;
  } else {
    HIP_TRY(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, c->prio_greatest));
    c->own_stream = true;
  }
  return MPPI_OK;
}

static int check_grid(int32_t rows, int32_t cols, float res) {
  if (rows < 2 || cols < 2) return fail(MPPI_EINVAL, "DEM must be at least 2x2");
  if (!(res > 0.0f)) return fail(MPPI_EINVAL, "DEM resolution must be > 0");
  if ((int64_t)rows * cols >= ((int64_t)1 << 29))  // kernels address cells with 32-bit byte offsets
    return fail(MPPI_EINVAL, "DEM larger than 2^29 cells");
  if (((int64_t)rows + 1) * ((int64_t)cols + 1) * 16 >= ((int64_t)1 << 32))  // the normal table, ditto
    return fail(MPPI_EINVAL, "DEM normal table above 4 GiB ((rows+1)*(cols+1) >= 2^28)");
  if (rows > (1 << 24) || cols > (1 << 24))  // cell bounds are clamped as exact floats
    return fail(MPPI_EINVAL, "DEM dimension above 2^24");
  return MPPI_OK;
}

// The DEM's per-cell normal table (read by the rollout chain instead of four corners +
// a normalisation per step); rebuilt whenever the DEM is set.  Ends synchronised.
static int build_normal_table(mppi_ctx* c) {
  const int rc = grow(c->ntab, c->ntab_cap, ((size_t)c->rows + 1) * ((size_t)c->cols + 1) * sizeof(float4), c->stream);
  if (rc) return rc;
  HIP_TRY(launch_normal_table(c->Z, c->rows, c->cols, c->res, c->ntab, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return MPPI_OK;
}

int mppi_set_dem(mppi_ctx* c, const float* z, int32_t rows, int32_t cols, float x_min, float y_min,
                 float resolution) {
  if (!c || !z) return fail(MPPI_EINVAL, "null argument");
  if (int rc_q = quiesce(c)) return rc_q;
  int rc = check_grid(rows, cols, resolution);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(c->device));
  rc = sync_tail(c);  // a deferred optimal rollout may still read the DEM
  if (rc) return rc;
  const size_t bytes = (size_t)rows * cols * sizeof(float);
  if (!c->Z_owned || bytes > c->Z_cap) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->Z_owned && c->Z) HIP_TRY(hipFree(c->Z));
    c->Z = nullptr;
    HIP_TRY(hipMalloc(&c->Z, bytes));
    c->Z_owned = true;
    c->Z_cap = bytes;
  }
  HIP_TRY(hipMemcpyAsync(c->Z, z, bytes, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->rows = rows;
  c->cols = cols;
  c->x_min = x_min;
  c->y_min = y_min;
  c->res = resolution;
  rc = build_normal_table(c);
  if (rc) return rc;
  return verified_reciprocal(c, resolution, &c->rinv_res);
}

int mppi_set_dem_device(mppi_ctx* c, const float* z, int32_t rows, int32_t cols, float x_min,
                        float y_min, float resolution) {
  if (!c || !z) return fail(MPPI_EINVAL, "null argument");
  if (int rc_q = quiesce(c)) return rc_q;
  int rc = check_grid(rows, cols, resolution);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());  // the DEM's writer may be on any stream of the device
  rc = sync_tail(c);
  if (rc) return rc;
  if (c->Z_owned && c->Z) HIP_TRY(hipFree(c->Z));
  c->Z = const_cast<float*>(z);
  c->Z_owned = false;
  c->Z_cap = 0;
  c->rows = rows;
  c->cols = cols;
  c->x_min = x_min;
  c->y_min = y_min;
  c->res = resolution;
  rc = build_normal_table(c);
  if (rc) return rc;
  return verified_reciprocal(c, resolution, &c->rinv_res);
}

int mppi_dem_updated(mppi_ctx* c) {
  if (!c) return fail(MPPI_EINVAL, "null argument");
  if (int rc_q = quiesce(c)) return rc_q;
  if (!c->Z || c->rows <= 0) return fail(MPPI_EINVAL, "no DEM bound");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());  // the in-place write may be on any stream of the device
  const int rc = sync_tail(c);      // a deferred optimal rollout may still read the table
  if (rc) return rc;
  return build_normal_table(c);
}

int mppi_set_costmap(mppi_ctx* c, const float* cm, int32_t size, float half_width, float resolution) {
  if (!c || !cm) return fail(MPPI_EINVAL, "null argument");
  if (int rc_q = quiesce(c)) return rc_q;
  if (size < 1) return fail(MPPI_EINVAL, "costmap size must be >= 1");
  if (!(resolution > 0.0f)) return fail(MPPI_EINVAL, "costmap resolution must be > 0");
  HIP_TRY(hipSetDevice(c->device));
  const size_t bytes = (size_t)size * size * sizeof(float);
  const int rc = grow(c->cm, c->cm_cap, bytes, c->stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->cm, cm, bytes, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->cm_size = size;
  c->cm_hw = half_width;
  c->cm_res = resolution;
  return verified_reciprocal(c, resolution, &c->rinv_res_c);
}

int mppi_set_state(mppi_ctx* c, const mppi_state* s) {
  if (!c || !s) return fail(MPPI_EINVAL, "null argument");
  c->st = *s;
  c->have_state = true;
  return MPPI_OK;
}

int mppi_set_nominal(mppi_ctx* c, const float* u1, const float* u2) {
  if (!c || !u1 || !u2) return fail(MPPI_EINVAL, "null argument");
  if (int rc_q = quiesce(c)) return rc_q;
  HIP_TRY(hipSetDevice(c->device));
  const int H = H_of(c);
  HIP_TRY(hipMemcpyAsync(c->u_nom[c->cur], u1, H * sizeof(float), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->u_nom[c->cur] + H, u2, H * sizeof(float), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return MPPI_OK;
}

int mppi_get_nominal(mppi_ctx* c, float* u1, float* u2) {
  if (!c || !u1 || !u2) return fail(MPPI_EINVAL, "null argument");
  if (int rc_q = quiesce(c)) return rc_q;
  HIP_TRY(hipSetDevice(c->device));
  const int H = H_of(c);
  HIP_TRY(hipMemcpyAsync(u1, c->u_nom[c->cur], H * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(u2, c->u_nom[c->cur] + H, H * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return MPPI_OK;
}

int mppi_step(mppi_ctx* c, int32_t proj, uint64_t step, mppi_outputs* out) {
  return step_impl(c, proj, step, 0, out);
}

int mppi_step_injected(mppi_ctx* c, int32_t proj, const float* u1, const float* u2,
                       mppi_outputs* out) {
  if (!c || !u1 || !u2) return fail(MPPI_EINVAL, "null argument");
  if (int rc_q = quiesce(c)) return rc_q;
  HIP_TRY(hipSetDevice(c->device));
  const size_t n = (size_t)std::max<int64_t>(c->p.num_trajectories, 1) * H_of(c);
  if (!c->inj1) {
    HIP_TRY(hipMalloc(&c->inj1, n * sizeof(float)));
    HIP_TRY(hipMalloc(&c->inj2, n * sizeof(float)));
  }
  const size_t bytes = (size_t)c->p.num_trajectories * H_of(c) * sizeof(float);
  HIP_TRY(hipMemcpyAsync(c->inj1, u1, bytes, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->inj2, u2, bytes, hipMemcpyHostToDevice, c->stream));
  return step_impl(c, proj, 0, 1, out);
}

int64_t mppi_record_len(mppi_ctx* c) { return c ? E_of(c) : -1; }

int mppi_step_partial(mppi_ctx* c, int32_t proj, uint64_t step, double* record_dev) {
  if (!c) return fail(MPPI_EINVAL, "null context");
  if (int rc_q = quiesce(c)) return rc_q;
  int rc = check_ready(c);
  if (rc) return rc;
  if (!record_dev) return fail(MPPI_EINVAL, "null record buffer");
  const Plan pl = make_plan(c);
  c->last_resident = false;
  int spec = -1;
  c->eps_late = c->eps_after == 1;  // (a group's or rank's partial steps: back to back)
  rc = enqueue_rollout(c, proj, step, 0, pl, c->u_nom[c->cur], c->st, nullptr, &spec);
  if (rc) return rc;
  remember(c, proj, step, 0, pl);
  rc = enqueue_finish(c, pl, c->st, c->nodes, pl.blocks, 0, record_dev, false);
  if (rc) return rc;
  return speculate_after(c, pl, step, spec);
}

int mppi_step_finish(mppi_ctx* c, const double* records_dev, int32_t n, mppi_outputs* out) {
  if (!c) return fail(MPPI_EINVAL, "null context");
  if (int rc_q = quiesce(c)) return rc_q;
  int rc = check_ready(c);
  if (rc) return rc;
  if (!records_dev || n < 1) return fail(MPPI_EINVAL, "records required");
  const Plan pl = c->have_last ? c->last_plan : make_plan(c);
  rc = enqueue_finish(c, pl, c->st, records_dev, n, 1, nullptr, true);
  if (rc) return rc;
  return copy_outputs(c, out);
}

int mppi_get_costs(mppi_ctx* c, float* costs, int64_t n) {
  if (!c || !costs) return fail(MPPI_EINVAL, "null argument");
  if (int rc_q = quiesce(c)) return rc_q;
  if (n < 0 || n > c->p.num_trajectories) return fail(MPPI_EINVAL, "n out of range");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipMemcpyAsync(costs, c->cost, n * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return MPPI_OK;
}

int mppi_dump_rollouts(mppi_ctx* c, float* traj, float* hv, float* lw, float* rw, float* v, float* w,
                       float* u1, float* u2) {
  if (!c) return fail(MPPI_EINVAL, "null context");
  if (int rc_q = quiesce(c)) return rc_q;
  int rc = check_ready(c);
  if (rc) return rc;
  if (!c->have_last) return fail(MPPI_ESTATE, "no step to dump");
  const size_t KH = (size_t)c->p.num_trajectories * H_of(c);
  if (KH == 0) return MPPI_OK;
  float* host[8] = {traj, hv, lw, rw, v, w, u1, u2};
  const size_t cnt[8] = {3 * KH, 3 * KH, 3 * KH, 3 * KH, KH, KH, KH, KH};
  float* dev[8] = {nullptr};
  int out_rc = MPPI_OK;
  for (int i = 0; i < 8 && out_rc == MPPI_OK; ++i)
    if (host[i] && hipMalloc(&dev[i], cnt[i] * sizeof(float)) != hipSuccess)
      out_rc = fail(MPPI_EHIP, "dump allocation failed");
  if (out_rc == MPPI_OK) {
    RolloutArgs d;
    std::memset(&d, 0, sizeof(d));
    d.d_traj = dev[0];
    d.d_hv = dev[1];
    d.d_lw = dev[2];
    d.d_rw = dev[3];
    d.d_v = dev[4];
    d.d_w = dev[5];
    d.d_u1 = dev[6];
    d.d_u2 = dev[7];
    // re-run the last step (deterministic: costs/records are rewritten with identical values)
    out_rc = enqueue_rollout(c, c->last_proj, c->last_step, c->last_mode, c->last_plan,
                             c->u_nom[c->last_nominal], c->last_state, &d);
    for (int i = 0; i < 8 && out_rc == MPPI_OK; ++i)
      if (host[i] && hipMemcpyAsync(host[i], dev[i], cnt[i] * sizeof(float), hipMemcpyDeviceToHost,
                                    c->stream) != hipSuccess)
        out_rc = fail(MPPI_EHIP, "dump copy failed");
    if (out_rc == MPPI_OK && hipStreamSynchronize(c->stream) != hipSuccess)
      out_rc = fail(MPPI_EHIP, "dump sync failed");
  }
  for (float* p : dev)
    if (p) hipFree(p);
  return out_rc;
}

int mppi_set_option(mppi_ctx* c, const char* name, int64_t value) {
  if (!c || !name) return fail(MPPI_EINVAL, "null argument");
  if (int rc_q = quiesce(c)) return rc_q;
  const std::string n(name);
  if (n == "resident") {  // the resident step server: 1 for back-to-back calls (default), 2 always, 0 never
    if (value < 0 || value > 2) return fail(MPPI_EINVAL, "resident must be 0, 1 or 2");
    c->resident = (int)value;
    return MPPI_OK;
  }
  if (n == "resident_idle_us") {  // how long an idle server stays resident
    if (value < 100 || value > 1000000) return fail(MPPI_EINVAL, "resident_idle_us must be in [100, 1e6]");
    c->srv_idle_us = (uint64_t)value;
    return MPPI_OK;
  }
  if (n == "record_tree_finish") {  // 1: the record-tree finish (mppi_finish_kernel) at any record count
    c->colfin = value == 0;
    return MPPI_OK;
  }
  if (n == "server_exit_after") {  // test hook: the next server launch's head leaves after this many commands
    if (value < 0 || value > 1000000) return fail(MPPI_EINVAL, "server_exit_after must be in [0, 1e6]");
    c->srv_exit_after = (unsigned)value;
    return MPPI_OK;
  }
  if (n == "eps_after") {  // the next steps' normals after the finish (1), the rollout (0), by cadence (-1)
    if (value < -1 || value > 1) return fail(MPPI_EINVAL, "eps_after must be -1, 0 or 1");
    c->eps_after = (int)value;
    return MPPI_OK;
  }
  if (n == "finish_wait_ticks") {  // the server finish's record wait bound (100 MHz ticks; 0: give up at once)
    if (value < 0) return fail(MPPI_EINVAL, "finish_wait_ticks must be >= 0");
    c->fin_wait_ticks = (uint64_t)value;
    return MPPI_OK;
  }
  return fail(MPPI_EINVAL, "unknown option '" + n + "'");
}

int mppi_set_timing(mppi_ctx* c, int32_t enable) {
  if (!c) return fail(MPPI_EINVAL, "null context");
  if (int rc_q = quiesce(c)) return rc_q;
  int rc = sync_tail(c);
  if (rc) return rc;
  if (enable < 0 || enable > 2) return fail(MPPI_EINVAL, "timing mode must be 0, 1 or 2");
  c->timing = enable;
  c->t_roll = c->t_fin = c->t_tail = 0.0;
  c->launches = c->tail_launches = 0;
  c->ev_roll_pending = c->ev_fin_pending = c->ev_tail_pending = false;
  return MPPI_OK;
}

int mppi_get_tail_timing(mppi_ctx* c, double* tail_ms, int64_t* n) {
  if (!c) return fail(MPPI_EINVAL, "null context");
  int rc = sync_tail(c);
  if (rc) return rc;
  if (tail_ms) *tail_ms = c->t_tail;
  if (n) *n = c->tail_launches;
  return MPPI_OK;
}

int mppi_set_async_tail(mppi_ctx* c, int32_t enable) {
  if (!c) return fail(MPPI_EINVAL, "null context");
  if (int rc_q = quiesce(c)) return rc_q;
  HIP_TRY(hipSetDevice(c->device));
  int rc = sync_tail(c);
  if (rc) return rc;
  c->async_tail = enable != 0;
  return MPPI_OK;
}

int mppi_get_outputs(mppi_ctx* c, mppi_outputs* out) {
  if (!c || !out) return fail(MPPI_EINVAL, "null argument");
  HIP_TRY(hipSetDevice(c->device));
  int rc = sync_tail(c);
  if (rc) return rc;
  fill_outputs(c->out_host, H_of(c), out);
  return MPPI_OK;
}

int mppi_get_timing(mppi_ctx* c, double* roll, double* fin, int64_t* n) {
  if (!c) return fail(MPPI_EINVAL, "null context");
  if (roll) *roll = c->t_roll;
  if (fin) *fin = c->t_fin;
  if (n) *n = c->launches;
  return MPPI_OK;
}

int mppi_get_server_time(mppi_ctx* c, double* roll_us, double* step_us, int64_t* steps) {
  if (!c) return fail(MPPI_EINVAL, "null context");
  HIP_TRY(hipSetDevice(c->device));
  uint64_t v[4] = {0, 0, 0, 0};
  // (a side stream: the context stream may hold the running server)
  HIP_TRY(hipMemcpyAsync(v, c->clk + kClkSums, sizeof(v), hipMemcpyDeviceToHost, c->noise_stream));
  HIP_TRY(hipStreamSynchronize(c->noise_stream));
  if (roll_us) *roll_us = (double)v[0] / 100.0;
  if (step_us) *step_us = (double)v[2] / 100.0;
  if (steps) *steps = (int64_t)std::min(v[1], v[3]);
  return MPPI_OK;
}

int mppi_get_chain_clock(mppi_ctx* c, double* out, int32_t n) {
  if (!c || !out) return fail(MPPI_EINVAL, "null argument");
  if (int rc_q = quiesce(c)) return rc_q;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  std::vector<uint64_t> all((size_t)kClkWords, 0);
  HIP_TRY(hipMemcpy(all.data(), c->clk, all.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  const uint64_t* v = all.data();
  // per-workgroup start / end of the last role-split rollout (its plan's blocks)
  const int nb = std::min(c->last_plan.roles ? c->last_plan.blocks : 0, kClkBlocks);
  uint64_t s_lo = UINT64_MAX, s_hi = 0, e_lo = UINT64_MAX, e_hi = 0;
  for (int b = 0; b < nb; ++b) {
    const uint64_t s0 = v[kClkBase + 2 * b], e0 = v[kClkBase + 2 * b + 1];
    s_lo = std::min(s_lo, s0);
    s_hi = std::max(s_hi, s0);
    e_lo = std::min(e_lo, e0);
    e_hi = std::max(e_hi, e0);
  }
  const bool wg_ok = nb > 0 && e_hi >= s_lo && e_lo >= s_lo;
  const double cyc = (double)(v[2] - v[0]), ticks = (double)(v[3] - v[1]);  // s_memrealtime: 100 MHz
  const int H = H_of(c);
  auto us = [&](int a, int b) { return v[a] && v[b] && v[b] >= v[a] ? (double)(v[b] - v[a]) / 100.0 : 0.0; };
  const double vals[10] = {ticks > 0 ? cyc * 100.0 / ticks : 0.0,  // shader clock, MHz (ticks: 100 MHz)
                           H > 0 ? cyc / H : 0.0, ticks / 100.0, cyc,
                           us(4, 1),   // workgroup start -> chain start
                           us(3, 5),   // chain end -> every role done
                           us(5, 6),   // -> leaf record written
                           wg_ok ? (double)(s_hi - s_lo) / 100.0 : 0.0,   // first -> last workgroup start
                           wg_ok ? (double)(e_hi - e_lo) / 100.0 : 0.0,   // first -> last record written
                           wg_ok ? (double)(e_hi - s_lo) / 100.0 : 0.0};  // first start -> last record
  for (int i = 0; i < n && i < 10; ++i) out[i] = vals[i];
  // then, per workgroup b, the time from the first workgroup start to b's record (microseconds)
  for (int b = 0; b < nb && 10 + b < n; ++b)
    out[10 + b] = wg_ok ? (double)(v[kClkBase + 2 * b + 1] - s_lo) / 100.0 : 0.0;
  // then (resident server) the stamps of the last 8 steps (kClkServer ring), microseconds from the
  // oldest stamp of the ring (0 = not stamped): out[10 + nb + 8 r + k], r = 0..7 in step order
  uint64_t lo = UINT64_MAX;
  for (int k = 0; k < 64; ++k)
    if (v[kClkServer + k]) lo = std::min(lo, v[kClkServer + k]);
  const int last = (int)(c->seq & 7);
  for (int r = 0; r < 8; ++r)
    for (int k = 0; k < 8; ++k) {
      const int idx = 10 + nb + 8 * r + k;
      const uint64_t x = v[kClkServer + 8 * ((last + 1 + r) & 7) + k];
      if (idx < n) out[idx] = x && lo != UINT64_MAX ? (double)(x - lo) / 100.0 : 0.0;
    }
  return MPPI_OK;
}

int mppi_get_launch_info(mppi_ctx* c, int64_t* info, int32_t n) {
  if (!c || !info) return fail(MPPI_EINVAL, "null argument");
  const Plan& pl = c->last_plan;
  const int64_t v[18] = {0, pl.block, pl.blocks, pl.W, pl.Wr, (int64_t)pl.lds_bytes, c->fin_kind,
                         c->fin_P, c->fin_ncol, c->fin_groups, pl.ucache_steps, c->last_resident ? 1 : 0,
                         c->srv_launches, c->srv_steps, c->srv_failed, c->srv_relaunches, c->srv_fallbacks,
                         c->cadence_steps};
  for (int i = 0; i < n && i < 18; ++i) info[i] = v[i];
  return MPPI_OK;
}

int mppi_bilinear_query(mppi_ctx* c, const float* x, const float* y, float* h, int64_t n) {
  if (!c || !x || !y || !h) return fail(MPPI_EINVAL, "null argument");
  if (int rc_q = quiesce(c)) return rc_q;
  if (!c->Z) return fail(MPPI_ESTATE, "no DEM");
  if (n < 0) return fail(MPPI_EINVAL, "n < 0");
  HIP_TRY(hipSetDevice(c->device));
  if (n == 0) return MPPI_OK;
  HIP_TRY(launch_bilinear(c->Z, c->rows, c->cols, c->x_min, c->y_min, c->res, x, y, h, n, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return MPPI_OK;
}

int mppi_bilinear_tiles(mppi_ctx* c, int32_t* ntiles) {
  if (!c || !ntiles) return fail(MPPI_EINVAL, "null argument");
  if (!c->Z) return fail(MPPI_ESTATE, "no DEM");
  *ntiles = ((c->rows + BIL_TILE - 1) / BIL_TILE) * ((c->cols + BIL_TILE - 1) / BIL_TILE);
  return MPPI_OK;
}

int mppi_bin_queries(mppi_ctx* c, const float* x, const float* y, int64_t n, float* xs_out, float* ys_out,
                     int32_t* perm, int32_t* tile_off) {
  if (!c || !x || !y || !xs_out || !ys_out || !perm || !tile_off) return fail(MPPI_EINVAL, "null argument");
  if (int rc_q = quiesce(c)) return rc_q;
  if (!c->Z) return fail(MPPI_ESTATE, "no DEM");
  if (n < 0 || n > INT32_MAX) return fail(MPPI_EINVAL, "n out of range [0, 2^31)");
  HIP_TRY(hipSetDevice(c->device));
  int32_t nt = 0;
  mppi_bilinear_tiles(c, &nt);
  // the histogram and scatter kernels keep one counter per tile in LDS: a skinny DEM (one side
  // under 128 cells) can have more tiles than that holds
  if ((size_t)nt * sizeof(int) > kLdsBytes - 1024)
    return fail(MPPI_EINVAL, "bin_queries: " + std::to_string(nt) + " tiles of 128 x 128 cells exceed the LDS "
                             "histogram (at most " + std::to_string((kLdsBytes - 1024) / sizeof(int)) +
                             "); use mppi_bilinear_query for this DEM");
  const size_t hist = (size_t)bin_chunks(n, nt) * nt;  // [chunks][tiles] per-chunk histograms
  const int rc = grow(c->bin_tile_of, c->bin_n_cap, std::max<size_t>(hist, 1) * sizeof(int), c->stream);
  if (rc) return rc;
  if ((size_t)nt > c->bin_t_cap) {
    if (c->bin_counts) HIP_TRY(hipFree(c->bin_counts));
    if (c->bin_cursor) HIP_TRY(hipFree(c->bin_cursor));
    c->bin_counts = c->bin_cursor = nullptr;
    // counts [nt], then the tile-row cursors of the two-level scatter [nt] (rows of tiles <= nt)
    HIP_TRY(hipMalloc(&c->bin_counts, 2 * (size_t)nt * sizeof(int)));
    HIP_TRY(hipMalloc(&c->bin_cursor, (size_t)nt * sizeof(int)));
    c->bin_t_cap = (size_t)nt;
  }
  if ((size_t)n > c->bin_q_cap) {
    for (void* p : {(void*)c->bin_cx, (void*)c->bin_cy, (void*)c->bin_ci})
      if (p) HIP_TRY(hipFree(p));
    c->bin_cx = c->bin_cy = nullptr;
    c->bin_ci = nullptr;
    HIP_TRY(hipMalloc(&c->bin_cx, (size_t)n * sizeof(float)));
    HIP_TRY(hipMalloc(&c->bin_cy, (size_t)n * sizeof(float)));
    HIP_TRY(hipMalloc(&c->bin_ci, (size_t)n * sizeof(int32_t)));
    c->bin_q_cap = (size_t)n;
  }
  HIP_TRY(launch_bin_queries(x, y, n, c->x_min, c->y_min, c->res, c->rinv_res, c->rinv_res != 0.0f, c->rows,
                             c->cols, c->bin_tile_of, c->bin_counts, c->bin_cursor, tile_off, xs_out, ys_out,
                             perm, c->stream, c->bin_cx, c->bin_cy, c->bin_ci, c->bin_counts + nt));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return MPPI_OK;
}

int mppi_bilinear_tiled(mppi_ctx* c, const float* xs, const float* ys, const int32_t* tile_off, float* h) {
  if (!c || !xs || !ys || !tile_off || !h) return fail(MPPI_EINVAL, "null argument");
  if (int rc_q = quiesce(c)) return rc_q;
  if (!c->Z) return fail(MPPI_ESTATE, "no DEM");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(launch_bilinear_tiled(c->Z, c->rows, c->cols, c->x_min, c->y_min, c->res, c->rinv_res,
                                c->rinv_res != 0.0f, xs, ys, h, tile_off, c->stream));
  return MPPI_OK;
}

int mppi_sync(mppi_ctx* c) {
  if (!c) return fail(MPPI_EINVAL, "null context");
  if (int rc_q = quiesce(c)) return rc_q;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return MPPI_OK;
}

int mppi_debug_hold(int32_t device, void* stream, int32_t groups, int32_t lds_bytes, int32_t microseconds) {
  if (groups < 1 || groups > 65536 || lds_bytes < 64 || (size_t)lds_bytes > kLdsBytes || microseconds < 0 ||
      microseconds > 1000000)
    return fail(MPPI_EINVAL, "debug_hold: groups in [1, 65536], lds_bytes in [64, 160 KiB], microseconds <= 1e6");
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(launch_hold(groups, (size_t)lds_bytes, (uint64_t)microseconds * 100, (hipStream_t)stream));
  return MPPI_OK;
}

int mppi_selftest(mppi_ctx* c, int32_t what, int64_t n, uint64_t seed, int64_t* mismatches) {
  if (!c || !mismatches) return fail(MPPI_EINVAL, "null argument");
  if (int rc_q = quiesce(c)) return rc_q;
  if (what < 0 || what > 5 || n < 0 || (what == 5 && n > 2 + 0x4C000000LL)) return fail(MPPI_EINVAL, "bad selftest arguments");
  HIP_TRY(hipSetDevice(c->device));
  unsigned long long* d = nullptr;
  HIP_TRY(hipMalloc(&d, sizeof(*d)));
  unsigned long long h = 0;
  hipError_t e = hipMemsetAsync(d, 0, sizeof(*d), c->stream);
  if (e == hipSuccess) e = launch_selftest(what, n, seed, d, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  hipFree(d);
  if (e != hipSuccess) return fail(MPPI_EHIP, std::string("selftest: ") + hipGetErrorString(e));
  *mismatches = (int64_t)h;
  return MPPI_OK;
}

int mppi_build_costmap(mppi_ctx* c, const double* obstacles, int32_t n, int32_t size, double half_width,
                       double origin_x, double origin_y, double r_robot, int32_t power, float* out_host,
                       int32_t metric) {
  if (!c) return fail(MPPI_EINVAL, "null context");
  if (int rc_q = quiesce(c)) return rc_q;
  int rc = costmap_check(obstacles, n, size, power, metric);
  if (rc) return rc;
  const float res = (float)(2 * half_width / size);  // Surface.costmap_resolution (MPPI_isaac.py:272)
  if (!(res > 0.0f)) return fail(MPPI_EINVAL, "costmap resolution must be > 0");
  HIP_TRY(hipSetDevice(c->device));
  const size_t bytes = (size_t)size * size * sizeof(float);
  rc = grow(c->cm, c->cm_cap, bytes, c->stream);
  if (rc) return rc;
  std::vector<double> obs, xs;
  rc = costmap_stage(c->cms, obstacles, n, size, half_width, origin_x, origin_y, r_robot, obs, xs, c->stream);
  if (rc) return rc;
  HIP_TRY(launch_costmap_build(c->cms, n, size, power, c->cm, c->stream, metric));
  if (out_host) HIP_TRY(hipMemcpyAsync(out_host, c->cm, bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->cm_size = size;
  c->cm_hw = (float)half_width;
  c->cm_res = res;
  return verified_reciprocal(c, res, &c->rinv_res_c);
}

int mppi_costmap_builder_create(int32_t device, mppi_costmap_builder** out) {
  if (!out) return fail(MPPI_EINVAL, "null argument");
  *out = nullptr;
  HIP_TRY(hipSetDevice(device));
  auto* b = new mppi_costmap_builder();
  b->device = device;
  if (hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&b->ev[0]) != hipSuccess || hipEventCreate(&b->ev[1]) != hipSuccess) {
    mppi_costmap_builder_destroy(b);
    return fail(MPPI_EHIP, "costmap builder: stream/event creation failed");
  }
  *out = b;
  return MPPI_OK;
}

void mppi_costmap_builder_destroy(mppi_costmap_builder* b) {
  if (!b) return;
  hipSetDevice(b->device);
  if (b->stream) hipStreamSynchronize(b->stream);
  costmap_free(b->sc);
  if (b->out) hipFree(b->out);
  for (auto& e : b->ev)
    if (e) hipEventDestroy(e);
  if (b->stream) hipStreamDestroy(b->stream);
  delete b;
}

int mppi_costmap_builder_build(mppi_costmap_builder* b, const double* obstacles, int32_t n, int32_t size,
                               double half_width, double origin_x, double origin_y, double r_robot, int32_t power,
                               float* out_host, float* out_device, int32_t metric) {
  if (!b) return fail(MPPI_EINVAL, "null builder");
  int rc = costmap_check(obstacles, n, size, power, metric);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(b->device));
  const size_t bytes = (size_t)size * size * sizeof(float);
  if (!out_device) {
    rc = grow(b->out, b->out_cap, bytes, b->stream);
    if (rc) return rc;
  }
  float* dst = out_device ? out_device : b->out;
  std::vector<double> obs, xs;
  rc = costmap_stage(b->sc, obstacles, n, size, half_width, origin_x, origin_y, r_robot, obs, xs, b->stream);
  if (rc) return rc;
  HIP_TRY(hipEventRecord(b->ev[0], b->stream));
  HIP_TRY(launch_costmap_build(b->sc, n, size, power, dst, b->stream, metric));
  HIP_TRY(hipEventRecord(b->ev[1], b->stream));
  if (out_host) HIP_TRY(hipMemcpyAsync(out_host, dst, bytes, hipMemcpyDeviceToHost, b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));
  float ms = 0;
  HIP_TRY(hipEventElapsedTime(&ms, b->ev[0], b->ev[1]));
  b->last_ms = ms;
  return MPPI_OK;
}

int mppi_costmap_builder_last_ms(mppi_costmap_builder* b, double* ms) {
  if (!b || !ms) return fail(MPPI_EINVAL, "null argument");
  *ms = b->last_ms;
  return MPPI_OK;
}

int mppi_rollout_python25d(mppi_ctx* c, int64_t n, int32_t H, const double* x0, const double* y0,
                           const double* heading, const double* lin_vel, const double* ang_vel, double dt,
                           double half_width, double resolution, double bound, double* traj, int32_t* valid) {
  if (!c) return fail(MPPI_EINVAL, "null context");
  if (int rc_q = quiesce(c)) return rc_q;
  if (n < 0 || H < 1) return fail(MPPI_EINVAL, "python25d: need n >= 0 and H >= 1");
  if (n == 0) return MPPI_OK;
  if (!x0 || !y0 || !heading || !lin_vel || !ang_vel || !traj || !valid)
    return fail(MPPI_EINVAL, "python25d: null argument");
  if (!c->Z) return fail(MPPI_ESTATE, "python25d: set a DEM first");
  if (!(resolution > 0.0) || !(half_width > 0.0)) return fail(MPPI_EINVAL, "python25d: bad grid geometry");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  const size_t nH = (size_t)n * H;
  const size_t bytes = (5 * (size_t)n + 2 * nH + 3 * nH) * sizeof(double) + (size_t)n * sizeof(int32_t);
  char* buf = nullptr;
  HIP_TRY(hipMalloc(&buf, bytes));
  double* d = (double*)buf;
  P25Args a;
  a.Z = c->Z;
  a.rows = c->rows;
  a.cols = c->cols;
  a.hw = half_width;
  a.res = resolution;
  a.xstep = (half_width - -half_width) / (double)(c->cols - 1);
  a.ystep = (half_width - -half_width) / (double)(c->rows - 1);
  a.dt = dt;
  a.bound = bound;
  a.n = n;
  a.H = H;
  a.x0 = d;
  a.y0 = d + n;
  a.hd = d + 2 * n;
  a.v = d + 5 * n;
  a.w = a.v + nH;
  a.traj = d + 5 * n + 2 * nH;
  a.valid = (int32_t*)(a.traj + 3 * nH);
  hipError_t e = hipMemcpyAsync((void*)a.x0, x0, n * sizeof(double), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync((void*)a.y0, y0, n * sizeof(double), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync((void*)a.hd, heading, 3 * n * sizeof(double), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync((void*)a.v, lin_vel, nH * sizeof(double), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync((void*)a.w, ang_vel, nH * sizeof(double), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = launch_python25d(a, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(traj, a.traj, 3 * nH * sizeof(double), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(valid, a.valid, n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  hipFree(buf);
  if (e != hipSuccess) return fail(MPPI_EHIP, std::string("python25d: ") + hipGetErrorString(e));
  return MPPI_OK;
}

// ---- multi-GPU group in one process ----
// One context per member device over a contiguous, leaf-aligned shard of the global K (as
// mppi_amd/distributed.shard_bounds), Philox keyed by the global index; per step every member
// runs its partial step (rollout + its record), the records are all-gathered (RCCL, one
// ncclAllGather per member inside one group call, on the members' streams; members sharing a
// device exchange by device copies), and every member combines them in member order and runs the
// finish (identical controls everywhere; member 0's outputs are returned).
}  // extern "C"

namespace {
struct RcclApi {
  void* h = nullptr;
  ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  ncclResult_t (*comm_count)(const ncclComm_t, int*) = nullptr;
};
// RCCL from the process (torch may already hold one) or librccl.so.1; nullptr if unavailable
const RcclApi* rccl_api(std::string& why) {
  static RcclApi api;
  static bool tried = false;
  static std::string err;
  if (!tried) {
    tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      err = std::string("RCCL not found: ") + dlerror();
    } else {
      api.h = h;
      api.comm_init_all = reinterpret_cast<decltype(api.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
      api.comm_destroy = reinterpret_cast<decltype(api.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
      api.all_gather = reinterpret_cast<decltype(api.all_gather)>(dlsym(h, "ncclAllGather"));
      api.group_start = reinterpret_cast<decltype(api.group_start)>(dlsym(h, "ncclGroupStart"));
      api.group_end = reinterpret_cast<decltype(api.group_end)>(dlsym(h, "ncclGroupEnd"));
      api.error_string = reinterpret_cast<decltype(api.error_string)>(dlsym(h, "ncclGetErrorString"));
      api.comm_count = reinterpret_cast<decltype(api.comm_count)>(dlsym(h, "ncclCommCount"));
      if (!api.comm_init_all || !api.comm_destroy || !api.all_gather || !api.group_start || !api.group_end)
        err = "RCCL lacks ncclCommInitAll / ncclAllGather / ncclGroupStart";
    }
  }
  why = err;
  return err.empty() ? &api : nullptr;
}
}  // namespace

struct mppi_group {
  int n = 0, E = 0;
  std::vector<mppi_ctx*> ctx;
  std::vector<int> dev;
  std::vector<int64_t> begin, count;
  std::vector<double*> rec;       // [E] this member's record (its device)
  std::vector<double*> gathered;  // [n * E] every member's record, member order (its device)
  std::vector<hipEvent_t> ev;     // copy exchange: this member's record is ready
  std::vector<double> empty_rec;  // the empty record (m = +inf, S = V = 0) for empty shards
  bool use_rccl = false;
  std::vector<ncclComm_t> comm;
  // Member threads (members 1..n-1; member 0 runs on the caller's thread).  Every member
  // enqueues its own partial step, exchange and finish and waits for its own completion word,
  // so the n enqueue paths (a few kernel launches + events each) run side by side instead of
  // one after another on the caller's thread (which skewed member n-1's rollout start by n
  // enqueue paths).  Handshake: the caller publishes the step (proj, step, out) and bumps `gen`;
  // each worker runs its member and decrements `pending`.  Workers spin for a short while after
  // each step (a control loop calls again within microseconds) and then sleep on the condition
  // variable.  One RCCL communicator per member, each driven only by its member's thread (the
  // one-thread-per-device use of ncclCommInitAll communicators: no group call needed).
  bool threaded = false;
  int spin_us = 0;      // how long a worker spins for the next step before it sleeps (granted_cpus)
  int cpus = 0;         // CPUs this process is granted
  bool selftest = false;  // mppi_group_selftest: host-only member steps (no GPU work at all), member
  int fail_member = -1;   // fail_member's failing
  std::vector<std::thread> workers;
  std::atomic<uint64_t> gen{0};
  std::atomic<int> pending{0};
  std::atomic<int> recorded{0};   // copy exchange: members whose record event is recorded
  std::atomic<int> sleepers{0};
  std::atomic<bool> stop{false};
  std::mutex mu;
  std::condition_variable cv;
  int cur_proj = 3;
  uint64_t cur_step = 0;
  mppi_outputs* cur_out = nullptr;
  std::vector<int> rc;
  std::vector<std::string> err;
};

namespace {

// Member i's partial step: rollout + its record (an empty member contributes the empty record).
int group_partial(mppi_group* g, int i, int proj, uint64_t step) {
  mppi_ctx* c = g->ctx[i];
  HIP_TRY(hipSetDevice(g->dev[i]));
  if (g->count[i] > 0) return mppi_step_partial(c, proj, step, g->rec[i]);
  HIP_TRY(hipMemcpyAsync(g->rec[i], g->empty_rec.data(), (size_t)g->E * sizeof(double), hipMemcpyHostToDevice,
                         c->stream));
  return MPPI_OK;
}

// Member i receives every member's record into gathered[i] (device copies, members that share
// a device or the device-copy mode): wait for each record's event, then a peer copy.
int group_copy_in(mppi_group* g, int i) {
  const size_t bytes = (size_t)g->E * sizeof(double);
  HIP_TRY(hipSetDevice(g->dev[i]));
  for (int j = 0; j < g->n; ++j) {
    HIP_TRY(hipStreamWaitEvent(g->ctx[i]->stream, g->ev[j], 0));
    HIP_TRY(hipMemcpyPeerAsync(g->gathered[i] + (size_t)j * g->E, g->dev[i], g->rec[j], g->dev[j], bytes,
                               g->ctx[i]->stream));
  }
  return MPPI_OK;
}

// Member i combines the n records in member order, runs the finish and waits for its outputs.
int group_finish(mppi_group* g, int i, mppi_outputs* out) {
  mppi_ctx* c = g->ctx[i];
  HIP_TRY(hipSetDevice(g->dev[i]));
  const Plan pl = c->have_last ? c->last_plan : make_plan(c);
  const int rc = enqueue_finish(c, pl, c->st, g->gathered[i], g->n, 1, nullptr, true);
  if (rc) return rc;
  return copy_outputs(c, out);
}

// One member's whole step on its own thread (threaded groups).
int group_member_step(mppi_group* g, int i) {
  int rc = group_partial(g, i, g->cur_proj, g->cur_step);
  if (!g->use_rccl) {  // every member's record event must be recorded before anyone waits on it
    if (rc == MPPI_OK && hipEventRecord(g->ev[i], g->ctx[i]->stream) != hipSuccess)
      rc = fail(MPPI_EHIP, "group: hipEventRecord failed");
    g->recorded.fetch_add(1, std::memory_order_acq_rel);
    while (g->recorded.load(std::memory_order_acquire) < g->n) __builtin_ia32_pause();
    if (rc) return rc;
    rc = group_copy_in(g, i);
  } else {
    // every member enqueues its all-gather, also after a failed partial step (its record buffer
    // exists): the collective needs every rank, and a missing one would leave the other members'
    // gathers, finishes and completion waits pending (the step fails on this member's error)
    std::string why;
    const RcclApi* api = rccl_api(why);
    if (!api) return fail(MPPI_EHIP, "group: " + why);
    const std::string saved = g_err;
    const ncclResult_t r = api->all_gather(g->rec[i], g->gathered[i], (size_t)g->E, ncclFloat64, g->comm[i],
                                           g->ctx[i]->stream);
    if (rc) {
      g_err = saved;
      return rc;
    }
    if (r != ncclSuccess)
      return fail(MPPI_EHIP, std::string("group: ncclAllGather: ") + (api->error_string ? api->error_string(r) : "error"));
  }
  if (rc) return rc;
  return group_finish(g, i, i == 0 ? g->cur_out : nullptr);
}

// mppi_group_selftest's member step: no GPU work, ~20 us of host time; member fail_member fails
int group_selftest_member(mppi_group* g, int i) {
  std::this_thread::sleep_for(std::chrono::microseconds(20));
  return i == g->fail_member ? fail(MPPI_EHIP, "injected failure") : MPPI_OK;
}

// CPUs this process may run on: its affinity set, bounded by its cgroup's CPU quota (cgroup v2)
int granted_cpus() {
  cpu_set_t set;
  int n = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : (int)std::thread::hardware_concurrency();
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    long q = 0, per = 0;
    if (std::fscanf(f, "%ld %ld", &q, &per) == 2 && q > 0 && per > 0) n = std::min<int>(n, std::max<long>(1, q / per));
    std::fclose(f);
  }
  return std::max(n, 1);
}

void group_worker(mppi_group* g, int i);

// Member threads: they spin (200 us, a control loop calls again within microseconds) only while the
// caller and every worker can hold a CPU of their own; on fewer granted CPUs they sleep at once.
void start_workers(mppi_group* g) {
  g->threaded = g->n > 1;
  g->rc.assign(g->n, MPPI_OK);
  g->err.assign(g->n, std::string());
  g->cpus = granted_cpus();
  g->spin_us = g->n < g->cpus ? 200 : 0;
  for (int i = 1; g->threaded && i < g->n; ++i) g->workers.emplace_back(group_worker, g, i);
}

void group_worker(mppi_group* g, int i) {
  if (!g->ctx.empty()) hipSetDevice(g->dev[i]);
  uint64_t seen = 0;  // the generation at start_workers (not a load here: a step posted before this
                      // thread ran would be taken as already seen, and the caller would wait for it)
  for (;;) {
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t now;
    for (int spin = 0; (now = g->gen.load(std::memory_order_acquire)) == seen && !g->stop.load(); ++spin) {
      if ((spin & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(g->spin_us)) {
        std::unique_lock<std::mutex> lk(g->mu);
        g->sleepers.fetch_add(1);
        g->cv.wait(lk, [&] { return g->gen.load() != seen || g->stop.load(); });
        g->sleepers.fetch_sub(1);
      } else {
        __builtin_ia32_pause();
      }
    }
    if (g->stop.load()) return;
    seen = now;
    const int rc = g->selftest ? group_selftest_member(g, i) : group_member_step(g, i);
    g->rc[i] = rc;
    if (rc) g->err[i] = g_err;
    g->pending.fetch_sub(1, std::memory_order_acq_rel);
  }
}

// The caller's thread: publish the step, run member 0, wait for the others.
int group_step_threaded(mppi_group* g, int proj, uint64_t step, mppi_outputs* out) {
  g->cur_proj = proj;
  g->cur_step = step;
  g->cur_out = out;
  for (int i = 0; i < g->n; ++i) {
    g->rc[i] = MPPI_OK;
    g->err[i].clear();
  }
  g->recorded.store(0, std::memory_order_relaxed);
  g->pending.store(g->n - 1, std::memory_order_relaxed);
  {
    std::lock_guard<std::mutex> lk(g->mu);  // a worker about to sleep sees the new generation
    g->gen.fetch_add(1, std::memory_order_acq_rel);
  }
  if (g->sleepers.load() > 0) g->cv.notify_all();
  g->rc[0] = g->selftest ? group_selftest_member(g, 0) : group_member_step(g, 0);
  if (g->rc[0]) g->err[0] = g_err;
  while (g->pending.load(std::memory_order_acquire) > 0) __builtin_ia32_pause();
  for (int i = 0; i < g->n; ++i)
    if (g->rc[i]) return fail(g->rc[i], "group member " + std::to_string(i) + ": " + g->err[i]);
  return MPPI_OK;
}

}  // namespace

extern "C" {

int mppi_group_create(const mppi_params* params, int32_t n, const int32_t* devices, mppi_group** out) {
  if (!params || !devices || !out || n < 1) return fail(MPPI_EINVAL, "group: null argument or n < 1");
  *out = nullptr;
  const int64_t K = params->num_trajectories;
  if (K < 1) return fail(MPPI_EINVAL, "group: num_trajectories must be >= 1");
  auto* g = new mppi_group();
  g->n = n;
  g->E = 2 * params->num_iterations + 2;
  const int64_t leaves = (K + 255) / 256, per = (leaves + n - 1) / n;
  bool distinct = true;
  for (int i = 0; i < n; ++i) {
    const int64_t b = std::min<int64_t>(K, (int64_t)i * per * 256), e = std::min<int64_t>(K, (int64_t)(i + 1) * per * 256);
    g->begin.push_back(b);
    g->count.push_back(e - b);
    g->dev.push_back(devices[i]);
    for (int j = 0; j < i; ++j) distinct &= devices[j] != devices[i];
  }
  auto bail = [&](int rc) {
    mppi_group_destroy(g);
    return rc;
  };
  for (int i = 0; i < n; ++i) {
    mppi_params p = *params;
    p.num_trajectories = g->count[i] > 0 ? g->count[i] : 256;  // an empty shard's context serves the finish
    p.k_offset = params->k_offset + g->begin[i];
    mppi_ctx* c = nullptr;
    int rc = mppi_create(&p, devices[i], &c);
    if (rc) return bail(rc);
    g->ctx.push_back(c);
    double *r = nullptr, *ga = nullptr;
    hipEvent_t e = nullptr;
    if (hipSetDevice(devices[i]) != hipSuccess || hipMalloc(&r, (size_t)g->E * sizeof(double)) != hipSuccess ||
        hipMalloc(&ga, (size_t)n * g->E * sizeof(double)) != hipSuccess ||
        hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      if (r) hipFree(r);
      if (ga) hipFree(ga);
      return bail(fail(MPPI_EHIP, "group: device buffers"));
    }
    g->rec.push_back(r);
    g->gathered.push_back(ga);
    g->ev.push_back(e);
  }
  g->empty_rec.assign((size_t)g->E, 0.0);
  g->empty_rec[0] = INFINITY;
  // MPPI_GROUP_RCCL: unset = RCCL between distinct devices (n > 1); 1 = also for one member
  // (exercises the RCCL exchange on a 1-GPU host); 0 = device copies only
  const char* env = std::getenv("MPPI_GROUP_RCCL");
  const int force = env ? std::atoi(env) : -1;
  if (distinct && ((n > 1 && force != 0) || force == 1)) {
    std::string why;
    const RcclApi* api = rccl_api(why);
    if (!api) return bail(fail(MPPI_EHIP, "group: " + why));
    g->comm.assign(n, nullptr);
    const ncclResult_t r = api->comm_init_all(g->comm.data(), n, g->dev.data());
    if (r != ncclSuccess) {
      g->comm.clear();
      return bail(fail(MPPI_EHIP, std::string("group: ncclCommInitAll: ") +
                                      (api->error_string ? api->error_string(r) : "error")));
    }
    g->use_rccl = true;
  }
  try {  // member threads (n > 1): every member enqueues its own step
    start_workers(g);
  } catch (const std::exception& ex) {
    return bail(fail(MPPI_EHIP, std::string("group: worker threads: ") + ex.what()));
  }
  *out = g;
  return MPPI_OK;
}

int mppi_group_selftest(int32_t n, int32_t fail_member, int32_t steps, int64_t* info) {
  if (n < 2 || steps < 1 || !info) return fail(MPPI_EINVAL, "group selftest: n >= 2, steps >= 1, info");
  auto* g = new mppi_group();
  g->n = n;
  g->selftest = true;
  g->fail_member = fail_member;
  g->dev.assign(n, 0);
  try {  // (std::thread can throw: the exception must not cross the C ABI)
    start_workers(g);
  } catch (const std::exception& ex) {
    mppi_group_destroy(g);
    return fail(MPPI_EHIP, std::string("group selftest: worker threads: ") + ex.what());
  }
  int64_t done = 0, failed = 0, named = 0;
  for (int k = 0; k < steps; ++k) {
    const int rc = group_step_threaded(g, 3, (uint64_t)k, nullptr);
    ++done;
    failed += rc != MPPI_OK;
    named += rc != MPPI_OK && g_err.find("member " + std::to_string(fail_member) + ": injected") != std::string::npos;
  }
  const int64_t v[5] = {done, failed, named, (int64_t)g->workers.size(), g->spin_us};
  for (int i = 0; i < 5; ++i) info[i] = v[i];
  mppi_group_destroy(g);
  return MPPI_OK;
}

void mppi_group_destroy(mppi_group* g) {
  if (!g) return;
  if (!g->workers.empty()) {
    {
      std::lock_guard<std::mutex> lk(g->mu);
      g->stop.store(true);
    }
    g->cv.notify_all();
    for (auto& t : g->workers)
      if (t.joinable()) t.join();
  }
  std::string why;
  const RcclApi* api = g->comm.empty() ? nullptr : rccl_api(why);
  for (size_t i = 0; i < g->comm.size(); ++i)
    if (g->comm[i] && api) api->comm_destroy(g->comm[i]);
  for (size_t i = 0; i < g->ctx.size(); ++i) {
    hipSetDevice(g->dev[i]);
    if (i < g->rec.size() && g->rec[i]) hipFree(g->rec[i]);
    if (i < g->gathered.size() && g->gathered[i]) hipFree(g->gathered[i]);
    if (i < g->ev.size() && g->ev[i]) hipEventDestroy(g->ev[i]);
    mppi_destroy(g->ctx[i]);
  }
  delete g;
}

int mppi_group_size(mppi_group* g) { return g ? g->n : -1; }

int mppi_group_context(mppi_group* g, int32_t i, mppi_ctx** out) {
  if (!g || !out || i < 0 || i >= g->n) return fail(MPPI_EINVAL, "group: bad member index");
  *out = g->ctx[i];
  return MPPI_OK;
}

int mppi_group_shard(mppi_group* g, int32_t i, int64_t* begin, int64_t* count) {
  if (!g || i < 0 || i >= g->n) return fail(MPPI_EINVAL, "group: bad member index");
  if (begin) *begin = g->begin[i];
  if (count) *count = g->count[i];
  return MPPI_OK;
}

int mppi_group_info(mppi_group* g, int64_t* info, int32_t n) {
  if (!g || !info) return fail(MPPI_EINVAL, "null argument");
  int ranks = 0;
  if (g->use_rccl && !g->comm.empty()) {
    std::string why;
    const RcclApi* api = rccl_api(why);
    if (api && api->comm_count) api->comm_count(g->comm[0], &ranks);
  }
  std::vector<int> devs(g->dev);
  std::sort(devs.begin(), devs.end());
  const int64_t distinct = std::unique(devs.begin(), devs.end()) - devs.begin();
  const int64_t v[7] = {g->n, distinct, g->use_rccl ? 1 : 0, ranks, g->threaded ? 1 : 0, g->spin_us, g->cpus};
  for (int i = 0; i < n && i < 7; ++i) info[i] = v[i];
  return MPPI_OK;
}

int mppi_group_step(mppi_group* g, int32_t proj, uint64_t step, mppi_outputs* out) {
  if (!g) return fail(MPPI_EINVAL, "null group");
  if (g->n == 1 && !g->use_rccl) return mppi_step(g->ctx[0], proj, step, out);
  if (proj != MPPI_PROJ_2D && proj != MPPI_PROJ_3D) return fail(MPPI_EINVAL, "proj must be 2 or 3");
  const int n = g->n;
  for (int i = 0; i < n; ++i) {
    const int rc = check_ready(g->ctx[i]);  // every member (an empty one runs the finish) needs its scene
    if (rc) return rc;
  }
  if (g->threaded) return group_step_threaded(g, proj, step, out);
  // one thread: every member's rollout and record, the exchange, every member's finish
  for (int i = 0; i < n; ++i) {
    const int rc = group_partial(g, i, proj, step);
    if (rc) return rc;
  }
  if (g->use_rccl) {
    std::string why;
    const RcclApi* api = rccl_api(why);
    if (!api) return fail(MPPI_EHIP, "group: " + why);
    ncclResult_t r = api->group_start();
    for (int i = 0; i < n && r == ncclSuccess; ++i)
      r = api->all_gather(g->rec[i], g->gathered[i], (size_t)g->E, ncclFloat64, g->comm[i], g->ctx[i]->stream);
    const ncclResult_t r2 = api->group_end();
    if (r != ncclSuccess || r2 != ncclSuccess)
      return fail(MPPI_EHIP, std::string("group: ncclAllGather: ") +
                                 (api->error_string ? api->error_string(r != ncclSuccess ? r : r2) : "error"));
  } else {
    for (int i = 0; i < n; ++i) {
      HIP_TRY(hipSetDevice(g->dev[i]));
      HIP_TRY(hipEventRecord(g->ev[i], g->ctx[i]->stream));
    }
    for (int i = 0; i < n; ++i) {
      const int rc = group_copy_in(g, i);
      if (rc) return rc;
    }
  }
  for (int i = 0; i < n; ++i) {
    mppi_ctx* c = g->ctx[i];
    HIP_TRY(hipSetDevice(g->dev[i]));
    const Plan pl = c->have_last ? c->last_plan : make_plan(c);
    const int rc = enqueue_finish(c, pl, c->st, g->gathered[i], n, 1, nullptr, true);
    if (rc) return rc;
  }
  for (int i = 0; i < n; ++i) {
    HIP_TRY(hipSetDevice(g->dev[i]));
    const int rc = copy_outputs(g->ctx[i], i == 0 ? out : nullptr);
    if (rc) return rc;
  }
  return MPPI_OK;
}

}  // extern "C"
