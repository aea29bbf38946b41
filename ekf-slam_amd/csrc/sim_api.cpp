// Host side of include/ekf_sim.h: device buffers of the simulator, one run = one simulator launch
// (which also writes the filter's descriptors) + the filter's launches over the run's messages.
// The simulator runs on a stream of its own with double-buffered run buffers, so run r's
// simulation overlaps run r−1's filter work; the host waits only for the simulation (it needs
// each filter's final parity for the handle's host mirror).
// A run without SURVEY messages on the HBM pipeline takes the parallel form instead: the wheels per
// filter, then every (message, filter) sensed at once into marker arrays, which ekf_replay_device
// plans on the GPU — no host round trip at all (EKF_SIM_PARALLEL=0 keeps the sequential kernel).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ekf.h"
#include "ekf_device.hpp"
#include "ekf_internal.hpp"
#include "ekf_launch.hpp"
#include "ekf_sim.h"
#include "sim_launch.hpp"

using namespace ekfslam;

struct ekf_sim {
  ekf_t h = nullptr;
  ekf_sim_config cfg{};
  HandleInfo info{};
  int L = 0, m = 0;
  long long tick = 0, msg = 0;  // global tick / message index of the next run
  double* lm = nullptr;
  unsigned* sighted = nullptr;
  SimState* st = nullptr;
  int* par = nullptr;
  hipStream_t sst = nullptr;        // the simulator's stream
  hipEvent_t ev_sim = nullptr;      // simulation of the current run done
  hipEvent_t ev_done[2] = {nullptr, nullptr};  // filter work of the run that used buffer b done
  int* host_par_pinned = nullptr;
  SimState* host_st_pinned = nullptr;  // [F] poses after the last run (the handle's t_odom_robot)
  int buf = 0;                      // run buffer of the next run
  double* cmd[2] = {nullptr, nullptr};
  int* sense[2] = {nullptr, nullptr};
  size_t cap_ticks = 0, cap_msgs = 0;
  MsgDesc* desc[2] = {nullptr, nullptr};
  PlanEntry* plan = nullptr;
  // markers and poses of a run by run buffer: the record (cfg.record) and the parallel form's
  // hand-over to ekf_replay_device
  struct Markers {
    int* ids = nullptr;       // [T][F][M]
    int* act = nullptr;       // [T][F][M]
    double* rel = nullptr;    // [T][F][M][2]
    int* cnt = nullptr;       // [T][F]
    double* truth = nullptr;  // [T][F][3]
    double* odom = nullptr;   // [T][3] (filter 0's)
    double* odomF = nullptr;  // [T][F][3] (the planner's input)
  } mk[2];
  bool mk_alloc = false;
  int last_T = 0, last_b = 0;
  std::vector<int> host_par;
  std::vector<double> host_odom;    // [F][3] t_odom_robot after the last run
};

namespace {

void free_run(ekf_sim* s) {
  for (void* p : {static_cast<void*>(s->cmd[0]), static_cast<void*>(s->sense[0]),
                  static_cast<void*>(s->desc[0]), static_cast<void*>(s->cmd[1]),
                  static_cast<void*>(s->sense[1]), static_cast<void*>(s->desc[1]),
                  static_cast<void*>(s->plan)})
    if (p) hipFree(p);
  for (auto& k : s->mk) {
    for (void* p : {static_cast<void*>(k.ids), static_cast<void*>(k.act), static_cast<void*>(k.rel),
                    static_cast<void*>(k.cnt), static_cast<void*>(k.truth),
                    static_cast<void*>(k.odom), static_cast<void*>(k.odomF)})
      if (p) hipFree(p);
    k = ekf_sim::Markers{};
  }
  for (int b = 0; b < 2; ++b) {
    s->cmd[b] = nullptr;
    s->sense[b] = nullptr;
    s->desc[b] = nullptr;
  }
  s->plan = nullptr;
  s->mk_alloc = false;
  s->cap_ticks = s->cap_msgs = 0;
}

// The parallel form (no SURVEY message, HBM pipeline, M ≤ kMaxChunk; EKF_SIM_PARALLEL=0: never).
bool parallel_ok(const ekf_sim* s, int T, const int* sense) {
  const char* e = std::getenv("EKF_SIM_PARALLEL");
  if ((e && std::atoi(e) == 0) || s->info.resident || s->cfg.marker_stride > kMaxChunk) return false;
  for (int t = 0; sense && t < T; ++t)
    if (sense[t] == EKF_SENSE_SURVEY) return false;
  return true;
}

// run buffers for T messages (grown, never shrunk)
int reserve(ekf_sim* s, int T) {
  const size_t F = static_cast<size_t>(s->info.F), M = static_cast<size_t>(s->cfg.marker_stride);
  const size_t ticks = static_cast<size_t>(T) * s->cfg.ticks_per_msg;
  if (static_cast<size_t>(T) <= s->cap_msgs && ticks <= s->cap_ticks) return EKF_OK;
  if (hipStreamSynchronize(s->info.stream) != hipSuccess ||
      hipStreamSynchronize(s->sst) != hipSuccess)
    return EKF_E_HIP;
  free_run(s);
  const size_t Tn = std::max<size_t>(T, 1);
  const size_t tk = Tn * s->cfg.ticks_per_msg;
  bool ok = hipMalloc(&s->plan, Tn * sizeof(PlanEntry)) == hipSuccess;
  for (int b = 0; b < 2 && ok; ++b)
    ok = hipMalloc(&s->cmd[b], tk * 2 * sizeof(double)) == hipSuccess &&
         hipMalloc(&s->sense[b], Tn * sizeof(int)) == hipSuccess &&
         hipMalloc(&s->desc[b], Tn * F * sizeof(MsgDesc)) == hipSuccess;
  // markers: both buffers for the parallel form (one run's planner reads them while the next run's
  // simulation writes the other), buffer 0 only for a record of the sequential form
  const bool par = !s->info.resident && s->cfg.marker_stride <= kMaxChunk;
  for (int b = 0; b < (par ? 2 : 1) && ok && (par || s->cfg.record); ++b) {
    auto& k = s->mk[b];
    ok = hipMalloc(&k.ids, Tn * F * M * sizeof(int)) == hipSuccess &&
         hipMalloc(&k.act, Tn * F * M * sizeof(int)) == hipSuccess &&
         hipMalloc(&k.rel, Tn * F * M * 2 * sizeof(double)) == hipSuccess &&
         hipMalloc(&k.cnt, Tn * F * sizeof(int)) == hipSuccess &&
         hipMalloc(&k.truth, Tn * F * 3 * sizeof(double)) == hipSuccess &&
         hipMalloc(&k.odom, Tn * 3 * sizeof(double)) == hipSuccess &&
         hipMalloc(&k.odomF, Tn * F * 3 * sizeof(double)) == hipSuccess;
    s->mk_alloc = ok;
  }
  if (!ok) {
    free_run(s);
    return EKF_E_NOMEM;
  }
  // the resident plan: one entry per message, every filter (off = t·F)
  std::vector<PlanEntry> pe(Tn);
  for (size_t t = 0; t < Tn; ++t) pe[t] = PlanEntry{static_cast<int>(t * F), 0, static_cast<int>(F), 0};
  if (hipMemcpy(s->plan, pe.data(), Tn * sizeof(PlanEntry), hipMemcpyHostToDevice) != hipSuccess) {
    free_run(s);  // no capacity is recorded for buffers whose plan never arrived
    return EKF_E_HIP;
  }
  s->cap_msgs = Tn;
  s->cap_ticks = tk;
  return EKF_OK;
}

// The parallel form of ekf_sim_run (parallel_ok): simulation on the simulator's stream, then
// ekf_replay_device over its marker arrays behind it on the handle's streams. The planning state
// stays on the device (the handle adopts it at its next host access), so the host never waits.
int run_parallel(ekf_sim* s, int T, const double* wheel_cmd, const int* sense) {
  const int b = s->buf;
  s->buf ^= 1;
  const hipStream_t st = s->sst;
  const size_t ticks = static_cast<size_t>(T) * s->cfg.ticks_per_msg;
  auto& k = s->mk[b];
  // buffer b (commands, senses, markers) was last read by the run before the previous one
  if (hipStreamWaitEvent(st, s->ev_done[b], 0) != hipSuccess ||
      hipMemcpyAsync(s->cmd[b], wheel_cmd, ticks * 2 * sizeof(double), hipMemcpyHostToDevice, st) !=
          hipSuccess ||
      (sense && hipMemcpyAsync(s->sense[b], sense, T * sizeof(int), hipMemcpyHostToDevice, st) !=
                    hipSuccess))
    return EKF_E_HIP;
  SimArgs a{};
  a.cmd = s->cmd[b];
  a.sense = sense ? s->sense[b] : nullptr;
  a.lm = s->lm;
  a.st = s->st;
  a.out_ids = k.ids;
  a.out_act = k.act;
  a.out_rel = k.rel;
  a.out_cnt = k.cnt;
  a.out_truth = k.truth;
  a.out_odom = s->cfg.record ? k.odom : nullptr;
  a.seed = s->cfg.seed;
  a.tick0 = s->tick;
  a.msg0 = s->msg;
  a.f0 = s->cfg.f0;
  a.F = s->info.F;
  a.L = s->L;
  a.T = T;
  a.tpm = s->cfg.ticks_per_msg;
  a.m = s->m;
  a.M = s->cfg.marker_stride;
  a.N = s->info.N;
  a.slip = s->cfg.slip;
  a.sigma = s->cfg.sensor_sigma;
  a.range = s->cfg.max_range;
  a.radius = s->cfg.wheel_radius;
  a.track = s->cfg.track_width;
  if (launch_sim_parallel(a, k.truth, k.odomF, st) != hipSuccess ||
      hipEventRecord(s->ev_sim, st) != hipSuccess ||
      hipStreamWaitEvent(s->info.stream, s->ev_sim, 0) != hipSuccess ||
      hipStreamWaitEvent(s->info.bulk, s->ev_sim, 0) != hipSuccess)
    return EKF_E_HIP;
  s->tick += static_cast<long long>(ticks);
  s->msg += T;
  s->last_T = T;
  s->last_b = b;
  const int rc = ekf_replay_device(s->h, T, s->cfg.marker_stride, k.cnt, k.ids, k.act, k.rel,
                                   k.odomF);
  if (rc) return rc;
  // the chain launch on the main stream polls the planner (or follows it): done there ⇒ read
  return hipEventRecord(s->ev_done[b], s->info.stream) == hipSuccess ? EKF_OK : EKF_E_HIP;
}

}  // namespace

extern "C" {

void ekf_sim_config_default(ekf_sim_config* c) {
  if (!c) return;
  std::memset(c, 0, sizeof(*c));
  c->seed = 20240317ull;
  c->ticks_per_msg = 40;
  c->slip = 0.02;
  c->sensor_sigma = 1e-3;
  c->max_range = 5.0;
  c->max_markers = 16;
  c->marker_stride = 16;
  c->wheel_radius = 0.033;
  c->track_width = 0.160;
  c->start_theta = -1.0;
}

int ekf_sim_create(ekf_sim_t* out, ekf_t filter, const ekf_sim_config* cfg, int n_map,
                   const double* landmarks) {
  if (!out || !filter || !cfg || n_map <= 0 || n_map > kSimMaxMap || !landmarks) return EKF_E_ARG;
  *out = nullptr;
  ekf_sim* s = new ekf_sim;
  s->h = filter;
  s->cfg = *cfg;
  if (int rc = handle_info(filter, &s->info)) {
    delete s;
    return rc;
  }
  s->L = n_map;
  s->m = std::min(cfg->max_markers, n_map);
  if (n_map > s->info.N || cfg->ticks_per_msg <= 0 || s->m <= 0 || s->m > kMaxChunk ||
      cfg->marker_stride < s->m || cfg->wheel_radius <= 0.0 || cfg->track_width <= 0.0 ||
      cfg->ticks_per_msg > 64) {
    delete s;
    return EKF_E_ARG;
  }
  const size_t F = static_cast<size_t>(s->info.F), words = (n_map + 31) / 32;
  hipSetDevice(s->info.device);
  bool ok = hipMalloc(&s->lm, F * n_map * 2 * sizeof(double)) == hipSuccess &&
            hipMalloc(&s->sighted, F * words * sizeof(unsigned)) == hipSuccess &&
            hipMalloc(&s->st, F * sizeof(SimState)) == hipSuccess &&
            hipMalloc(&s->par, F * sizeof(int)) == hipSuccess;
  std::vector<SimState> st(F);
  for (auto& v : st) {
    std::memset(&v, 0, sizeof(v));
    v.truth[0] = cfg->start_theta;
    v.truth[1] = cfg->start_x;
    v.truth[2] = cfg->start_y;
  }
  ok = ok && hipStreamCreateWithFlags(&s->sst, hipStreamNonBlocking) == hipSuccess &&
       hipEventCreateWithFlags(&s->ev_sim, hipEventDisableTiming) == hipSuccess &&
       hipEventCreateWithFlags(&s->ev_done[0], hipEventDisableTiming) == hipSuccess &&
       hipEventCreateWithFlags(&s->ev_done[1], hipEventDisableTiming) == hipSuccess &&
       hipHostMalloc(reinterpret_cast<void**>(&s->host_par_pinned), F * sizeof(int),
                     hipHostMallocDefault) == hipSuccess &&
       hipHostMalloc(reinterpret_cast<void**>(&s->host_st_pinned), F * sizeof(SimState),
                     hipHostMallocDefault) == hipSuccess &&
       hipEventRecord(s->ev_done[0], s->info.stream) == hipSuccess &&
       hipEventRecord(s->ev_done[1], s->info.stream) == hipSuccess &&
       hipMemcpy(s->lm, landmarks, F * n_map * 2 * sizeof(double), hipMemcpyHostToDevice) == hipSuccess &&
       hipMemset(s->sighted, 0, F * words * sizeof(unsigned)) == hipSuccess &&
       hipMemcpy(s->st, st.data(), F * sizeof(SimState), hipMemcpyHostToDevice) == hipSuccess;
  if (!ok) {
    ekf_sim_destroy(s);
    return EKF_E_NOMEM;
  }
  s->host_par.assign(F, 0);
  s->host_odom.assign(3 * F, 0.0);
  *out = s;
  return EKF_OK;
}

int ekf_sim_destroy(ekf_sim_t s) {
  if (!s) return EKF_E_ARG;
  if (s->info.stream) hipStreamSynchronize(s->info.stream);
  if (s->sst) hipStreamSynchronize(s->sst);
  free_run(s);
  for (void* p : {static_cast<void*>(s->lm), static_cast<void*>(s->sighted),
                  static_cast<void*>(s->st), static_cast<void*>(s->par)})
    if (p) hipFree(p);
  if (s->host_par_pinned) hipHostFree(s->host_par_pinned);
  if (s->host_st_pinned) hipHostFree(s->host_st_pinned);
  for (hipEvent_t e : {s->ev_sim, s->ev_done[0], s->ev_done[1]})
    if (e) hipEventDestroy(e);
  if (s->sst) hipStreamDestroy(s->sst);
  delete s;
  return EKF_OK;
}

int ekf_sim_run(ekf_sim_t s, int T, const double* wheel_cmd, const int* sense) {
  if (!s || T < 0 || (T > 0 && !wheel_cmd)) return EKF_E_ARG;
  if (T == 0) return EKF_OK;
  if (sense)
    for (int t = 0; t < T; ++t) {
      if (sense[t] < EKF_SENSE_NEAREST || sense[t] > EKF_SENSE_ALL) return EKF_E_ARG;
      if (sense[t] == EKF_SENSE_ALL && (s->L > kMaxChunk || s->cfg.marker_stride < s->L))
        return EKF_E_ARG;
    }
  if (int rc = handle_info(s->h, &s->info)) return rc;  // host-planned work first, bulk joined
  // (Joseph form on the HBM pipeline: both forms write kJoseph chunks of ≤ kMaxJoseph = kMaxChunk
  // markers; the resident path carries the form in its own kernel)
  const bool par = parallel_ok(s, T, sense);
  hipSetDevice(s->info.device);
  if (int rc = reserve(s, T)) return rc;
  if (par) return run_parallel(s, T, wheel_cmd, sense);
  const int b = s->buf;
  s->buf ^= 1;
  const hipStream_t st = s->sst;
  const size_t F = static_cast<size_t>(s->info.F);
  const size_t ticks = static_cast<size_t>(T) * s->cfg.ticks_per_msg;
  // the handle's host mirror is authoritative (host-planned calls between runs flip parities)
  if (int rc = handle_parity(s->h, s->host_par.data())) return rc;
  std::memcpy(s->host_par_pinned, s->host_par.data(), F * sizeof(int));
  if (hipMemcpyAsync(s->par, s->host_par_pinned, F * sizeof(int), hipMemcpyHostToDevice, st) !=
      hipSuccess)
    return EKF_E_HIP;
  // buffer b was last read by the filter work of the run before the previous one
  if (hipStreamWaitEvent(st, s->ev_done[b], 0) != hipSuccess) return EKF_E_HIP;
  if (hipMemcpyAsync(s->cmd[b], wheel_cmd, ticks * 2 * sizeof(double), hipMemcpyHostToDevice, st) !=
      hipSuccess)
    return EKF_E_HIP;
  if (sense && hipMemcpyAsync(s->sense[b], sense, T * sizeof(int), hipMemcpyHostToDevice, st) !=
                   hipSuccess)
    return EKF_E_HIP;
  SimArgs a{};
  a.cmd = s->cmd[b];
  a.sense = sense ? s->sense[b] : nullptr;
  a.lm = s->lm;
  a.sighted = s->sighted;
  a.st = s->st;
  a.par = s->par;
  a.desc = s->desc[b];
  if (s->cfg.record) {
    const auto& k = s->mk[0];
    a.out_ids = k.ids;
    a.out_act = k.act;
    a.out_rel = k.rel;
    a.out_cnt = k.cnt;
    a.out_truth = k.truth;
    a.out_odom = k.odom;
  }
  a.seed = s->cfg.seed;
  a.tick0 = s->tick;
  a.msg0 = s->msg;
  a.f0 = s->cfg.f0;
  a.F = s->info.F;
  a.L = s->L;
  a.T = T;
  a.tpm = s->cfg.ticks_per_msg;
  a.m = s->m;
  a.M = s->cfg.marker_stride;
  a.N = s->info.N;
  a.slip = s->cfg.slip;
  a.sigma = s->cfg.sensor_sigma;
  a.range = s->cfg.max_range;
  a.radius = s->cfg.wheel_radius;
  a.track = s->cfg.track_width;
  a.joseph = s->info.joseph && !s->info.resident;
  if (launch_sim(a, st) != hipSuccess) return EKF_E_HIP;
  // each filter's final parity (its inactive messages do not flip it) and odometry: the host mirror
  if (hipMemcpyAsync(s->host_par_pinned, s->par, F * sizeof(int), hipMemcpyDeviceToHost, st) !=
          hipSuccess ||
      hipMemcpyAsync(s->host_st_pinned, s->st, F * sizeof(SimState), hipMemcpyDeviceToHost, st) !=
          hipSuccess ||
      hipEventRecord(s->ev_sim, st) != hipSuccess || hipEventSynchronize(s->ev_sim) != hipSuccess)
    return EKF_E_HIP;
  std::memcpy(s->host_par.data(), s->host_par_pinned, F * sizeof(int));
  for (size_t f = 0; f < F; ++f)
    for (int k = 0; k < 3; ++k) s->host_odom[3 * f + k] = s->host_st_pinned[f].odom[k];
  s->tick += static_cast<long long>(ticks);
  s->msg += T;
  s->last_T = T;
  s->last_b = 0;
  // the filter's kernels behind the simulation (their descriptors), then release buffer b
  if (hipStreamWaitEvent(s->info.stream, s->ev_sim, 0) != hipSuccess) return EKF_E_HIP;
  const int rc = run_device_plan(s->h, s->desc[b], s->plan, T, s->host_par.data(),
                                 s->host_odom.data());
  if (rc) return rc;
  if (int r2 = handle_info(s->h, &s->info)) return r2;  // joins the bulk stream into main
  return hipEventRecord(s->ev_done[b], s->info.stream) == hipSuccess ? EKF_OK : EKF_E_HIP;
}

int ekf_sim_markers(ekf_sim_t s, int* counts, int* ids, int* actions, double* rel_xy) {
  if (!s || !s->cfg.record) return EKF_E_ARG;
  const size_t n = static_cast<size_t>(s->last_T) * s->info.F, M = s->cfg.marker_stride;
  const auto& k = s->mk[s->last_b];
  if (hipStreamSynchronize(s->info.stream) != hipSuccess ||
      hipStreamSynchronize(s->sst) != hipSuccess)
    return EKF_E_HIP;
  if ((counts && hipMemcpy(counts, k.cnt, n * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) ||
      (ids && hipMemcpy(ids, k.ids, n * M * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) ||
      (actions && hipMemcpy(actions, k.act, n * M * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) ||
      (rel_xy && hipMemcpy(rel_xy, k.rel, n * M * 2 * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess))
    return EKF_E_HIP;
  return EKF_OK;
}

int ekf_sim_poses(ekf_sim_t s, double* odom, double* truth) {
  if (!s || !s->cfg.record) return EKF_E_ARG;
  const size_t T = static_cast<size_t>(s->last_T);
  const auto& k = s->mk[s->last_b];
  if (hipStreamSynchronize(s->info.stream) != hipSuccess ||
      hipStreamSynchronize(s->sst) != hipSuccess)
    return EKF_E_HIP;
  if ((odom && hipMemcpy(odom, k.odom, T * 3 * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) ||
      (truth && hipMemcpy(truth, k.truth, T * s->info.F * 3 * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess))
    return EKF_E_HIP;
  return EKF_OK;
}

}  // extern "C"
