// Host runtime behind include/ekf.h: device memory, the handle's HIP stream, message staging and
// the launch sequence for the reference's two callbacks (nuslam/src/slam.cpp:180-316, :318-530).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <array>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "ekf.h"
#include "ekf_device.hpp"
#include "ekf_internal.hpp"
#include "ekf_launch.hpp"
#include "geom.hpp"

using namespace ekfslam;

namespace {

constexpr int kRing = 16;  // pinned staging slots (host may run this many uploads ahead)

struct Marker {
  int id;
  double zr, zb;
};

struct Launch {
  int kind;    // 0 = gain + Σ pass, 1 = association + gain + Σ pass (one marker), 2 = posterior
               // only, 3 = a chunk of associated markers (k_assoc_msg) + Σ pass
  size_t off;  // first descriptor
  int f0, nf, kw;
};

struct StageSlot {
  MsgDesc* p = nullptr;
  size_t cap = 0;
  hipEvent_t ev = nullptr;
  bool used = false;
};

struct ProfEvents {
  std::vector<hipEvent_t> start, stop;
};

}  // namespace

static_assert(EKF_RESIDENT_MAX_N == kResidentMaxN, "ekf.h and ekf_launch.hpp agree");

struct ekf_ctx {
  ekf_config cfg{};
  int n = 0, ld = 0, ldk = 0, F = 0;
  size_t w = 8;
  hipStream_t stream = nullptr;  // chain + factors (+ association, posterior)
  hipStream_t bulk = nullptr;    // Σ passes: chunk t's pass overlaps chunk t+1's chain
  bool serial = false;           // EKF_SERIAL=1: every kernel on one stream (per-dispatch PMC)
  bool resident = false;         // n ≤ kResidentMaxN, fp64: Σ in registers (ekf_resident.hip)
  bool defer = false;            // ekf_defer: plan now, upload and launch later
  bool joseph = false;           // ekf_set_joseph (resident: its own kernel; pipeline: kJoseph chunks)
  bool assoc_msg = true;         // unknown association by chunks (k_assoc_msg); EKF_ASSOC_MSG=0:
                                 // one association kernel + launch pair per marker
  bool main_dirty = false;       // work on the main stream since the bulk stream last joined it
  bool main_unordered = false;   // the main stream ran descriptor-reading work (k_posterior) that
                                 // nothing on the bulk stream is ordered after: a device planner
                                 // on the bulk stream must wait for it before rewriting ddesc
  bool epoch_owed = false;       // the last Σ pass published no device epoch (the flush's last
                                 // launch: the next flush joins the bulk stream on the host)
  AmArgs am{};                   // k_assoc_msg scratch (allocated at the first association chunk)
  int am_route = 0;              // unknown association: EKF_ASSOC_* (fixed at ekf_create)
  int am_route_j = 0;            // ... for the Joseph-form kernel (its larger LDS may fit fewer)
  int am_group = 1;              // filters per k_assoc_msg launch (co-resident, assoc_msg_group)
  int am_group_j = 1;            // ... Joseph form
  int bulk_cus_per_xcd = 0;      // CUs the bulk stream may use on each XCD
  int main_cus_per_xcd = 0;      // CUs the main stream may use on each XCD (0: every CU, no mask)
  unsigned* fatal_h = nullptr;   // host-mapped: a device poll timed out (EKF_E_TIMEOUT)
  unsigned* fatal_d = nullptr;   // its device address (PassArgs::fatal)
  hipEvent_t ev_chain = nullptr;          // main → bulk: the chunk's chain is done
  hipEvent_t ev_join = nullptr;           // bulk → main: everything issued so far
  bool devsync = false;                   // streams synchronise through device epochs
  unsigned* sync = nullptr;               // device epochs: Σ pass done, its ticket, chains done
  hipEvent_t ev_sig[2] = {nullptr, nullptr};  // bulk → main: Σ pass of launch s, by s & 1
  long long seq = 0;                      // launch pairs issued
  // dev only (EKF_DBG_ORDER bit mask, tools/diag_handover.py): conservative hand-off variants
  // for locating a missing ordering edge of the event schedule
  unsigned dbg_order = 0;
  std::vector<hipEvent_t> dbg_ev;         // bit 4: a fresh event per Σ pass (never re-recorded)
  unsigned long long* dlog = nullptr;     // bit 4096: PassArgs::dlog
  void* sig[2] = {nullptr, nullptr};
  double* x[2] = {nullptr, nullptr};
  void* kcat = nullptr;
  void* mcat = nullptr;
  FilterCtl* ctl = nullptr;
  ChunkRec* rec = nullptr;
  void* stage = nullptr; // StageRec<T>[2][F]: a kLook chain's rebuild operands (kStageIn)
  MsgDesc* ddesc = nullptr;
  size_t sig_stride = 0, x_stride = 0, km_stride = 0;
  // ekf_replay_device: the planning state lives on the device while dev_plan (ping-pong by
  // dstate_cur); the host mirror below adopts it (adopt_device_plan) before it is used again
  PlanState* dstate[2] = {nullptr, nullptr};
  PlanState* hstate = nullptr;  // pinned: host → device and back
  int dstate_cur = 0;
  bool dev_plan = false;
  hipStream_t plan_stream = nullptr;  // the stream the last device planner ran on
  unsigned plan_total = 0;    // kSyncPlan: descriptors device planners have counted so far
  unsigned need_plan = 0;     // the next chain launch polls kSyncPlan for this (0: none)
  // host mirror
  std::vector<Pose2> odom;
  std::vector<int> parity;
  std::vector<char> pending;
  std::vector<int> prev_m;       // ≥ 0: last chunk was a pipelined pair (its record is valid)
  std::vector<std::array<int, kMaxChunk>> prev_ids;  // that chunk's landmark ids
  std::vector<std::array<long, 2>> stg_desc;  // plan_d indices of its last two pipelined chunks
                                              // ([0] the last), −1: none (kStageOut planning)
  // launch plan: descriptors for a whole call (or a whole replay) uploaded with ONE copy
  std::vector<MsgDesc> plan_d;
  std::vector<Launch> plan_l;
  size_t ddesc_cap = 0;
  // pinned staging ring (the host may run kRing uploads ahead of the device), every slot ring_cap
  StageSlot ring[kRing];
  size_t ring_cap = 0;
  int ring_next = 0;
  // scratch
  std::vector<std::vector<Marker>> msgs;
  std::vector<char> absent;  // batch paths: counts[f] == 0, the filter gets no message this step
  // profiling
  bool prof = false;
  ProfEvents pe[5];
  std::vector<hipEvent_t> pool;
  long long prof_launches[5] = {0, 0, 0, 0, 0};
  long long prof_chunks = 0;  // chunks the timed chain launches walked
  double prof_ms[5] = {0, 0, 0, 0, 0};
};

#define HIPCHK(expr)                       \
  do {                                     \
    if ((expr) != hipSuccess) return EKF_E_HIP; \
  } while (0)

namespace {

template <typename T>
PassArgs<T> args(ekf_ctx* h, const MsgDesc* desc, int f0) {
  PassArgs<T> a{};
  a.sig[0] = static_cast<T*>(h->sig[0]);
  a.sig[1] = static_cast<T*>(h->sig[1]);
  a.sig_stride = h->sig_stride;
  a.x[0] = h->x[0];
  a.x[1] = h->x[1];
  a.x_stride = h->x_stride;
  a.kcat = static_cast<T*>(h->kcat);
  a.mcat = static_cast<T*>(h->mcat);
  a.km_stride = h->km_stride;
  a.ldk = h->ldk;
  a.ctl = h->ctl;
  a.rec = h->rec;
  a.rec_stride = static_cast<size_t>(h->F);
  a.stage = static_cast<StageRec<T>*>(h->stage);
  a.sync = h->sync;
  a.fatal = h->fatal_d;
  a.desc = desc;
  a.n = h->n;
  a.ld = h->ld;
  a.N = h->cfg.n_landmarks;
  a.f0 = f0;
  a.q = h->cfg.q_noise;
  a.r = h->cfg.r_noise;
  a.gate = h->cfg.mah_gate;
  a.joseph = h->joseph ? 1 : 0;
  a.dbg = static_cast<int>(h->dbg_order >> 8);
  a.dlog = h->dlog;
  return a;
}

hipEvent_t pool_get(ekf_ctx* h) {
  if (!h->pool.empty()) {
    hipEvent_t e = h->pool.back();
    h->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Launch `fn` bracketed by events when profiling (kind 0 = Σ pass, 1 = chain, 2 = association,
// 3 = factors, 4 = resident filter kernel).
template <typename Fn>
int timed(ekf_ctx* h, int kind, hipStream_t st, Fn fn) {
  (void)st;
  hipEvent_t a = nullptr, b = nullptr;
  if (h->prof) {
    a = pool_get(h);
    b = pool_get(h);
  }
  const hipError_t e = fn(a && b ? a : nullptr, a && b ? b : nullptr);
  if (h->prof && a && b) {
    h->pe[kind].start.push_back(a);
    h->pe[kind].stop.push_back(b);
  }
  return e == hipSuccess ? EKF_OK : EKF_E_HIP;
}

void fill_desc(MsgDesc* d, int m, int flags, int parity, const Pose2& odom) {
  std::memset(d, 0, sizeof(MsgDesc));
  d->m = m;
  d->flags = flags;
  d->parity = parity;
  d->odom[0] = odom.theta;
  d->odom[1] = odom.x;
  d->odom[2] = odom.y;
}

// The filter's next chunk has no planned predecessor in this plan (upload, association, posterior,
// reset, device plan): no staged rebuild operands.
void forget_desc(ekf_ctx* h, int f) { h->stg_desc[f] = {-1L, -1L}; }

// slam.cpp:208-210 (host, glibc, as the reference)
inline void measure(double rx, double ry, double* zr, double* zb) {
  *zr = std::sqrt(std::pow(rx, 2) + std::pow(ry, 2));
  *zb = std::atan2(ry, rx);
}

// Main waits for everything issued to the bulk stream so far.
int join_bulk(ekf_ctx* h) {
  if (hipEventRecord(h->ev_join, h->bulk) != hipSuccess ||
      hipStreamWaitEvent(h->stream, h->ev_join, 0) != hipSuccess)
    return EKF_E_HIP;
  return EKF_OK;
}

// The main stream runs the chains back to back; the bulk stream runs each chunk's factors and Σ
// pass. With disjoint CU masks (devsync) the two streams synchronise on the device only: a chain
// polls the Σ-pass epoch (it needs the pass two launches back: Σ_in and x of the chunk before the
// previous one, and this parity's ChunkRec free again), the factor kernel polls its filter's chain
// epoch. A hipStreamWaitEvent hop between the queues costs 6–12 µs, a device poll ≈ 1–2 µs.
// Without the CU split a spinning factor grid could hold every CU the chain needs, so events are
// used instead (the kernels' polls are then satisfied on arrival).
// `nchunks` consecutive chunks of filters [f0, f0+nf) (descriptors dptr[i·nf + k]): ONE chain
// launch that walks them all (rebuilding its block from the chunk before each time), then per chunk the factor
// kernel and the Σ pass on the bulk stream. More than one chunk only with devsync, where the bulk
// kernels of chunk i wait on the device for the chain's epoch of chunk i.
// hd: the host copy of the group's descriptors (nullptr: written on the device, no kStageOut).
template <typename T>
int launch_group(ekf_ctx* h, const MsgDesc* dptr, const MsgDesc* hd, int f0, int nf, int nchunks,
                 bool pipelined, bool nolook, bool publish_end, int stage_hint) {
  PassArgs<T> a = args<T>(h, dptr, f0);
  a.desc_stride = nf;
  const unsigned s0 = static_cast<unsigned>(h->seq);
  a.seq = s0;
  const bool two = pipelined && !h->serial;
  hipStream_t ms = h->stream, bs = two ? h->bulk : h->stream;
  a.polls = two && h->devsync ? 1 : 0;
  a.need_plan = a.polls ? h->need_plan : 0u;
  h->need_plan = 0;
  a.first_ready = h->epoch_owed ? 1 : 0;  // (the host joined the bulk stream since that pass)
  {  // dev A/B: stream-ordered chains gather their (complete) Σ_in instead of rebuilding
    static const bool g = [] {
      const char* e = std::getenv("EKF_SERIAL_GATHER");
      return e && std::atoi(e) != 0;
    }();
    a.gather = g && ms == bs && !a.polls ? 1 : 0;
  }
  if (pipelined && !nolook) {
    // events: a rebuilding (kLook) chain needs the Σ pass two launches back
    if (!h->devsync) {
      if (h->dbg_order & 1u) {
        if (join_bulk(h)) return EKF_E_HIP;
      } else if (h->dbg_order & 16u) {
        if (s0 >= 2 && s0 - 2 < h->dbg_ev.size())
          HIPCHK(hipStreamWaitEvent(ms, h->dbg_ev[s0 - 2], 0));
      } else {
        HIPCHK(hipStreamWaitEvent(ms, h->ev_sig[s0 & 1], 0));
      }
    }
  } else if (!a.polls) {
    // a chain that gathers its own Σ_in needs the previous pass: everything on the bulk stream
    if (join_bulk(h)) return EKF_E_HIP;
  }
  if (h->dbg_order & 8192u) HIPCHK(launch_dbg_sum<T>(a, nf, 3, ms));
  int rc = timed(h, 1, ms, [&](hipEvent_t e0, hipEvent_t e1) {
    return launch_chain<T>(a, nf, nchunks, ms, e0, e1);
  });
  if (rc) return rc;
  if (h->prof) h->prof_chunks += nchunks;
  if (two && !h->devsync) {  // nchunks == 1 here
    HIPCHK(hipEventRecord(h->ev_chain, ms));
    HIPCHK(hipStreamWaitEvent(bs, h->ev_chain, 0));
  }
  for (int i = 0; i < nchunks; ++i) {
    PassArgs<T> ai = a;
    ai.desc = dptr + static_cast<size_t>(i) * nf;
    ai.seq = s0 + static_cast<unsigned>(i);
    // Inside a device-synchronised group the factor kernel of chunk i publishes the Σ-pass epoch
    // of chunk i−1 (the kernel boundary has made that pass's output visible): one launch less per
    // chunk on the bulk stream. The group's last pass gets its own epoch kernel.
    const bool in_group = h->devsync && nchunks > 1;
    ai.pub_sigma = in_group && i > 0 ? ai.seq : 0u;
    // factors gather the materialised Σ_in (the previous Σ pass, same stream) and the record
    rc = timed(h, 3, bs, [&](hipEvent_t e0, hipEvent_t e1) {
      return launch_factors<T>(ai, nf, bs, e0, e1);
    });
    if (rc) return rc;
    if (h->dbg_order & 8192u) HIPCHK(launch_dbg_sum<T>(ai, nf, 1, bs));
    // some filter stages the rebuild operands of its chunk after next (device-written descriptors:
    // the caller's hint — the group's first stage_hint chunks may, the last two of a device replay
    // have no chunk after next in it — the staging kernel reads every descriptor's own flags)
    bool stage = !hd && i < stage_hint;
    for (int k = 0; hd && k < nf; ++k) {
      const int fl = hd[static_cast<size_t>(i) * nf + k].flags;
      stage = stage || ((fl & kActive) && (fl & kStageOut));
    }
    const bool last = i + 1 == nchunks;
    rc = timed(h, 0, bs, [&](hipEvent_t e0, hipEvent_t e1) {
      return launch_sigma_pass<T>(ai, nf, last ? publish_end : !in_group, stage, bs, e0, e1);
    });
    if (rc) return rc;
    if (h->dbg_order & 8192u) HIPCHK(launch_dbg_sum<T>(ai, nf, 2, bs));
    if (!h->devsync) HIPCHK(hipEventRecord(h->ev_sig[(s0 + i) & 1], bs));
    if (h->dbg_order & 16u) {
      while (h->dbg_ev.size() <= s0 + i) {
        hipEvent_t e = nullptr;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        h->dbg_ev.push_back(e);
      }
      HIPCHK(hipEventRecord(h->dbg_ev[s0 + i], bs));
    }
    if ((h->dbg_order & 8u) && !h->devsync) {  // every launch pair drained before the next
      HIPCHK(hipStreamSynchronize(bs));
      HIPCHK(hipStreamSynchronize(ms));
    }
  }
  h->seq += nchunks;
  h->epoch_owed = a.polls && !publish_end;
  return EKF_OK;
}

// nolook: some active filter's first chunk gathers its own Σ_in (no kLook rebuild)
// publish_end: the group's last Σ pass publishes its device epoch (false only for a flush's last
// launch, whose successor the next flush orders on the host: one kernel less on the stream's tail)
// stage_hint (device-written descriptors): the group's first stage_hint chunks may stage rebuild
// operands (kStageOut), so only they are followed by the staging kernel
int group(ekf_ctx* h, const MsgDesc* dptr, const MsgDesc* hd, int f0, int nf, int nchunks,
          bool pipelined, bool nolook = true, bool publish_end = true, int stage_hint = 0) {
  return h->cfg.dtype == EKF_F32
             ? launch_group<float>(h, dptr, hd, f0, nf, nchunks, pipelined, nolook, publish_end,
                                   stage_hint)
             : launch_group<double>(h, dptr, hd, f0, nf, nchunks, pipelined, nolook, publish_end,
                                    stage_hint);
}

// The chain → factors kernels of a message are a latency-bound critical path; the Σ pass of the
// previous chunk runs beside them on the bulk stream and, sharing their CUs, slowed the chain by
// ~35 %. With few filters the two streams get disjoint CU masks: the main stream kCuSplit CUs per
// XCD, the bulk stream the rest (a CU mask must leave every XCD at least one CU; mask bit b lands on
// XCD b mod 8). EKF_CU_SPLIT=<CUs per XCD> overrides, 0 disables.
constexpr int kCuSplit = 4;
constexpr int kCuSplitMaxFilters = 32;

int create_streams(ekf_ctx* h) {
  int split = h->F <= kCuSplitMaxFilters ? kCuSplit : 0;
  if (const char* e = std::getenv("EKF_CU_SPLIT")) split = std::atoi(e);
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->cfg.device) !=
      hipSuccess)
    cus = 0;
  constexpr int kXcd = 8;
  h->bulk_cus_per_xcd = cus / kXcd;
  if (split > 0 && cus % kXcd == 0 && split * kXcd < cus) {
    h->bulk_cus_per_xcd = cus / kXcd - split;
    h->main_cus_per_xcd = split;
    const int words = (cus + 31) / 32;
    std::vector<uint32_t> mmain(words, 0), mbulk(words, 0);
    for (int b = 0; b < cus; ++b) (b < split * kXcd ? mmain : mbulk)[b / 32] |= 1u << (b % 32);
    if (hipExtStreamCreateWithCUMask(&h->stream, words, mmain.data()) == hipSuccess &&
        hipExtStreamCreateWithCUMask(&h->bulk, words, mbulk.data()) == hipSuccess) {
      // device-epoch hand-offs by default; EKF_DEVSYNC=0 synchronises the streams with events
      // (same kernels, one chain launch per chunk: bit-identical to the single-stream order)
      // A persistent multi-chunk chain launch needs every filter's chain resident at once (a
      // chain's chunk i+2 waits for the Σ pass of chunk i over ALL filters, whose factor kernels
      // wait for every chain): with more filters than main-stream CUs it would spin into its
      // timeouts, so such a split synchronises with events.
      const char* e = std::getenv("EKF_DEVSYNC");
      h->devsync = !(e && std::atoi(e) == 0) && h->F <= split * kXcd;
      return EKF_OK;
    }
    if (h->stream) hipStreamDestroy(h->stream);
    h->stream = nullptr;
  }
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&h->bulk, hipStreamNonBlocking) != hipSuccess)
    return EKF_E_HIP;
  return EKF_OK;
}

// Both streams idle (before host reads/writes of device state).
int drain(ekf_ctx* h) {
  HIPCHK(hipStreamSynchronize(h->bulk));
  HIPCHK(hipStreamSynchronize(h->stream));
  return EKF_OK;
}

// devsync: k_assoc waits on the device for the last Σ pass (its epoch is h->seq) instead of the
// main stream joining the bulk stream first
int assoc(ekf_ctx* h, const MsgDesc* dptr, int f0, int nf, bool poll) {
  if (h->cfg.dtype == EKF_F32) {
    PassArgs<float> a = args<float>(h, dptr, f0);
    a.polls = poll ? 1 : 0;
    a.need_sigma = poll ? static_cast<unsigned>(h->seq) : 0u;
    return timed(h, 2, h->stream, [&](hipEvent_t e0, hipEvent_t e1) {
      return launch_assoc<float>(a, nf, h->stream, e0, e1);
    });
  }
  PassArgs<double> a = args<double>(h, dptr, f0);
  a.polls = poll ? 1 : 0;
  a.need_sigma = poll ? static_cast<unsigned>(h->seq) : 0u;
  return timed(h, 2, h->stream, [&](hipEvent_t e0, hipEvent_t e1) {
    return launch_assoc<double>(a, nf, h->stream, e0, e1);
  });
}

// Known association, one message per filter in [f0, f0+nf): msgs[k] holds filter f0+k's markers.
// Predict + chunks of ≤ kMaxChunk corrections + posterior (slam.cpp:180-316), appended to the plan.
// absent[k] (batch paths): filter f0+k receives no message this step — its descriptor is inactive,
// nothing of it changes (an empty MarkerArray is rejected before anything changes, EKF_E_EMPTY).
void plan_known(ekf_ctx* h, int f0, int nf, bool predict, const char* absent = nullptr) {
  // Joseph form on the pipeline: ≤ kMaxJoseph (= kMaxChunk) markers per chunk (the chain's row map
  // Z holds K's and V = ΣHᵀ − K·S's columns, 4 per marker; k_chain<T, true>)
  const bool jos = h->joseph && !h->resident;
  const int cm = jos ? kMaxJoseph : kMaxChunk;
  int chunks = 1;
  for (int k = 0; k < nf; ++k)
    chunks = std::max(chunks, static_cast<int>((h->msgs[k].size() + cm - 1) / cm));
  for (int chunk = 0; chunk < chunks; ++chunk) {
    const size_t off = h->plan_d.size();
    h->plan_d.resize(off + nf);
    int kw = 4;
    for (int k = 0; k < nf; ++k) {
      const int f = f0 + k;
      const auto& mk = h->msgs[k];
      const int nchunks = std::max(1, static_cast<int>((mk.size() + cm - 1) / cm));
      MsgDesc* d = &h->plan_d[off + k];
      if (chunk >= nchunks || (absent && absent[k])) {
        std::memset(d, 0, sizeof(MsgDesc));
        continue;
      }
      const int b = chunk * cm;
      const int m = std::max(0, std::min(cm, static_cast<int>(mk.size()) - b));
      int flags = kActive | (jos ? kJoseph : 0);
      if (chunk == 0 && (predict || h->pending[f])) flags |= kFirst;
      if (chunk == nchunks - 1 && predict) flags |= kLast;
      // rebuild from the chunk before (its Σ pass may run); the resident kernel carries Σ itself
      if (h->prev_m[f] >= 0 && !h->resident) flags |= kLook;
      fill_desc(d, m, flags, h->parity[f], h->odom[f]);
      d->prev_m = h->prev_m[f];
      for (int i = 0; i < kMaxChunk; ++i) d->prev_ids[i] = h->prev_ids[f][i];
      for (int i = 0; i < m; ++i) {
        d->ids[i] = mk[b + i].id;
        d->z[i][0] = mk[b + i].zr;
        d->z[i][1] = mk[b + i].zb;
      }
      // the k_patch_stage behind the Σ pass two chunks back gathers this chain's rebuild operands
      // (the Σ_in' it reads is that pass's output)
      if ((flags & kLook) && h->stage && h->stg_desc[f][1] >= 0) {
        MsgDesc* sd = &h->plan_d[h->stg_desc[f][1]];
        sd->flags |= kStageOut;
        sd->stg_m = m;
        sd->stg_pm = h->prev_m[f];
        for (int i = 0; i < kMaxChunk; ++i) {
          sd->stg_ids[i] = d->ids[i];
          sd->stg_pids[i] = h->prev_ids[f][i];
        }
        d->flags |= kStageIn;
      }
      h->stg_desc[f] = {static_cast<long>(off + k), h->stg_desc[f][0]};
      h->prev_m[f] = m;
      for (int i = 0; i < m; ++i) h->prev_ids[f][i] = mk[b + i].id;
      h->parity[f] ^= 1;
      kw = std::max(kw, ((2 + (jos ? 4 : 2) * m + 3) / 4) * 4);
      if (chunk == 0) h->pending[f] = 0;
    }
    h->plan_l.push_back(Launch{0, off, f0, nf, kw});
  }
}

// Unknown association (slam.cpp:318-530), markers [i0, i1) of each filter's message: per marker the
// association kernel + a single-marker launch pair. Decisions land in FilterCtl::assoc_j/new at
// slot i % kMaxAssoc.
void plan_assoc(ekf_ctx* h, int f0, int nf, bool predict, bool posterior, int i0, int i1,
                const char* absent = nullptr) {
  for (int i = i0; i < i1; ++i) {
    const size_t off = h->plan_d.size();
    h->plan_d.resize(off + nf);
    for (int k = 0; k < nf; ++k) {
      const int f = f0 + k;
      const auto& mk = h->msgs[k];
      const int mf = static_cast<int>(mk.size());
      MsgDesc* d = &h->plan_d[off + k];
      if (i >= std::max(mf, 1) || (absent && absent[k])) {
        std::memset(d, 0, sizeof(MsgDesc));
        continue;
      }
      int flags = kActive | kNoInit | (h->joseph && !h->resident ? kJoseph : 0);
      h->prev_m[f] = -1;  // association chunks run unpipelined
      forget_desc(h, f);
      if (i == 0 && (predict || h->pending[f])) flags |= kFirst;
      if (i == std::max(mf, 1) - 1 && posterior) flags |= kLast;
      const int m = mf > 0 ? 1 : 0;
      fill_desc(d, m, flags, h->parity[f], h->odom[f]);
      d->assoc_slot = i % kMaxAssoc;
      if (m) {
        d->ids[0] = -1;
        d->z[0][0] = mk[i].zr;
        d->z[0][1] = mk[i].zb;
      }
      h->parity[f] ^= 1;
      if (i == 0) h->pending[f] = 0;
    }
    h->plan_l.push_back(Launch{1, off, f0, nf, 4});
  }
}

// Which path unknown association takes (EKF_ASSOC_*). k_assoc_msg's G workgroups per filter spin
// on each other's granules, so all G must be resident at once on the CUs of the stream it runs on
// (the bulk stream; the main stream with EKF_SERIAL, whose CU mask may be narrower): G workgroups
// on one XCD (XCD-local placement) or ⌈G / 8⌉ on each (agent placement). A launch holds only as
// many filters as the CUs hold at once (assoc_msg_group: co-resident by construction). Beyond
// that the markers go one per launch (k_assoc + a launch pair).
int assoc_cus_per_xcd(const ekf_ctx* h) {
  return h->serial && h->main_cus_per_xcd > 0 ? h->main_cus_per_xcd : h->bulk_cus_per_xcd;
}
int am_route(ekf_ctx* h, bool joseph = false) {
  if (h->resident || !h->assoc_msg) return EKF_ASSOC_MARKER;
  const int G = (h->cfg.n_landmarks + kAmSlots - 1) / kAmSlots;
  const int per_xcd =
      assoc_msg_blocks_per_cu(h->cfg.dtype == EKF_F32, joseph) * assoc_cus_per_xcd(h);
  const char* e = std::getenv("EKF_AM_XCD");  // EKF_AM_XCD=0: the agent placement only
  if (G > 1 && G <= per_xcd && !(e && std::atoi(e) == 0)) return EKF_ASSOC_CHUNK_XCD;
  if ((G + 7) / 8 <= per_xcd) return EKF_ASSOC_CHUNK;
  return EKF_ASSOC_MARKER;
}

// k_assoc_msg's tables and granules for every filter (once; zeroed so no stale tag matches)
int ensure_am(ekf_ctx* h) {
  if (h->am.hist) return EKF_OK;
  const int G = (h->cfg.n_landmarks + kAmSlots - 1) / kAmSlots;
  const size_t Np = static_cast<size_t>(G) * kAmSlots, F = static_cast<size_t>(h->F);
  AmArgs b{};
  b.G = G;
  b.hist_stride = kMaxChunk * Np;
  b.cur_stride = (kMaxChunk + 1) * Np;
  b.gran_stride = static_cast<size_t>(kMaxChunk + 1) * G * 4;
  b.xcd = h->am_route == EKF_ASSOC_CHUNK_XCD ? 1 : 0;
  b.spin = 1u << 22;  // ≈ 0.1 s of polls per exchange
  if (const char* e = std::getenv("EKF_AM_SPIN_LOG2")) b.spin = 1u << std::min(std::atoi(e), 30);
  if (const char* e = std::getenv("EKF_AM_DROP")) b.drop = std::atoi(e) != 0 ? 1 : 0;
  auto release = [&]() {
    if (b.hist) hipFree(b.hist);
    if (b.cur) hipFree(b.cur);
    if (b.gran) hipFree(b.gran);
  };
  if (hipMalloc(&b.hist, sizeof(AmHist) * b.hist_stride * F) != hipSuccess ||
      hipMalloc(&b.cur, sizeof(AmCur) * b.cur_stride * F) != hipSuccess ||
      hipMalloc(&b.gran, sizeof(unsigned long long) * b.gran_stride * F) != hipSuccess) {
    release();
    return EKF_E_NOMEM;
  }
  if (hipMemset(b.gran, 0, sizeof(unsigned long long) * b.gran_stride * F) != hipSuccess) {
    release();
    return EKF_E_HIP;
  }
  h->am = b;
  for (int jv = 0; jv < 2; ++jv) {
    const int slots_x =
        assoc_msg_blocks_per_cu(h->cfg.dtype == EKF_F32, jv != 0) * assoc_cus_per_xcd(h);
    (jv ? h->am_group_j : h->am_group) =
        b.xcd ? 8 * std::max(1, slots_x / G) : std::max(1, 8 * slots_x / G);
  }
  return EKF_OK;
}

// Unknown association by chunks (k_assoc_msg): markers [i0, i1) of each filter's message in chunks
// of ≤ kMaxChunk, each chunk one association launch + one Σ pass. Decisions land in
// FilterCtl::assoc_j/new at slot i % kMaxAssoc, as plan_assoc's.
void plan_assoc_msg(ekf_ctx* h, int f0, int nf, bool predict, bool posterior, int i0, int i1,
                    const char* absent = nullptr) {
  int chunks = 1;
  for (int k = 0; k < nf; ++k) {
    const int mf = std::min(static_cast<int>(h->msgs[k].size()), i1);
    chunks = std::max(chunks, (mf - i0 + kMaxChunk - 1) / kMaxChunk);
  }
  for (int chunk = 0; chunk < chunks; ++chunk) {
    const size_t off = h->plan_d.size();
    h->plan_d.resize(off + nf);
    for (int k = 0; k < nf; ++k) {
      const int f = f0 + k;
      const auto& mk = h->msgs[k];
      const int mf = std::min(static_cast<int>(mk.size()), i1);
      const int nch = std::max(1, (mf - i0 + kMaxChunk - 1) / kMaxChunk);
      MsgDesc* d = &h->plan_d[off + k];
      if (chunk >= nch || (absent && absent[k]) || (mf <= i0 && i0 > 0)) {
        std::memset(d, 0, sizeof(MsgDesc));
        continue;
      }
      const int b = i0 + chunk * kMaxChunk;
      const int m = std::max(0, std::min(kMaxChunk, mf - b));
      int flags = kActive | kNoInit | (h->joseph ? kJoseph : 0);
      h->prev_m[f] = -1;  // association chunks run unpipelined
      forget_desc(h, f);
      if (b == 0 && (predict || h->pending[f])) flags |= kFirst;
      if (chunk == nch - 1 && posterior) flags |= kLast;
      fill_desc(d, m, flags, h->parity[f], h->odom[f]);
      d->assoc_slot = b % kMaxAssoc;
      for (int i = 0; i < m; ++i) {
        d->ids[i] = -1;
        d->z[i][0] = mk[b + i].zr;
        d->z[i][1] = mk[b + i].zb;
      }
      h->parity[f] ^= 1;
      if (b == 0) h->pending[f] = 0;
    }
    h->plan_l.push_back(Launch{3, off, f0, nf, 4});
  }
}

// Route unknown association: whole chunks through k_assoc_msg on the HBM pipeline (either form:
// k_assoc_msg<T, J>); the resident path, EKF_ASSOC_MSG=0 and maps too large for the bulk stream's
// CUs to hold a filter's workgroups at once (am_route; the Joseph kernel's own occupancy, in the
// placement fixed at creation) take one marker per launch.
void plan_unknown(ekf_ctx* h, int f0, int nf, bool predict, bool posterior, int i0, int i1,
                  const char* absent = nullptr) {
  if (h->am_route != EKF_ASSOC_MARKER && (!h->joseph || h->am_route_j == h->am_route))
    plan_assoc_msg(h, f0, nf, predict, posterior, i0, i1, absent);
  else
    plan_assoc(h, f0, nf, predict, posterior, i0, i1, absent);
}

// One association chunk per filter of [f0, f0+nf) (descriptors dptr), then its Σ pass, both on the
// bulk stream (the pass's CUs; the main stream's chains are not involved). The bulk stream joins
// the main stream first if the latter ran anything since (a chain wrote t_map_odom there).
int assoc_msg_group(ekf_ctx* h, const MsgDesc* dptr, int f0, int nf, bool publish_end) {
  if (int rc = ensure_am(h)) return rc;
  hipStream_t bs = h->serial ? h->stream : h->bulk;
  if (!h->serial && h->main_dirty) {
    HIPCHK(hipEventRecord(h->ev_chain, h->stream));
    HIPCHK(hipStreamWaitEvent(h->bulk, h->ev_chain, 0));
    h->main_dirty = false;
    h->main_unordered = false;
  }
  const unsigned seq = static_cast<unsigned>(h->seq);
  // A filter's G workgroups spin on each other, so a launch holds only as many filters as the
  // stream's CUs hold at once (workgroups are not guaranteed to be dispatched in order): XCD-local
  // placement ⌊slots per XCD / G⌋ filters on each of the 8 XCDs (filter k of a launch on XCD
  // k mod 8), agent placement ⌊slots / G⌋ filters spread over all of them. Filters are
  // independent, so any grouping gives the same bits.
  const int group_nf = h->joseph ? h->am_group_j : h->am_group;
  auto run = [&](auto tag) -> int {
    using T = decltype(tag);
    PassArgs<T> a = args<T>(h, dptr, f0);
    a.seq = seq;
    a.polls = h->devsync && !h->serial ? 1 : 0;
    for (int g0 = 0; g0 < nf; g0 += group_nf) {
      PassArgs<T> ag = args<T>(h, dptr + g0, f0 + g0);
      ag.seq = a.seq;
      ag.polls = a.polls;
      const int gn = std::min(group_nf, nf - g0);
      const int rc = timed(h, 2, bs, [&](hipEvent_t e0, hipEvent_t e1) {
        return launch_assoc_msg<T>(ag, h->am, gn, bs, e0, e1);
      });
      if (rc) return rc;
    }
    return timed(h, 0, bs, [&](hipEvent_t e0, hipEvent_t e1) {
      return launch_sigma_pass<T>(a, nf, publish_end, false, bs, e0, e1);
    });
  };
  const int rc = h->cfg.dtype == EKF_F32 ? run(float{}) : run(double{});
  if (rc) return rc;
  if (!h->devsync) HIPCHK(hipEventRecord(h->ev_sig[seq & 1], bs));
  h->seq += 1;
  h->epoch_owed = h->devsync && !h->serial && !publish_end;
  return EKF_OK;
}

void plan_posterior(ekf_ctx* h, int f) {
  h->prev_m[f] = -1;
  forget_desc(h, f);
  const size_t off = h->plan_d.size();
  h->plan_d.resize(off + 1);
  fill_desc(&h->plan_d[off], 0, kActive, h->parity[f], h->odom[f]);
  h->plan_l.push_back(Launch{2, off, f, 1, 4});
}

int posterior_launch(ekf_ctx* h, const MsgDesc* dp, int f0, int nf) {
  const hipError_t e =
      h->cfg.dtype == EKF_F32
          ? launch_posterior<float>(args<float>(h, dp, f0), nf, h->stream)
          : launch_posterior<double>(args<double>(h, dp, f0), nf, h->stream);
  return e == hipSuccess ? EKF_OK : EKF_E_HIP;
}

// Upload capacity for `need` descriptors. The device buffer grows geometrically (a re-allocation
// drains both streams). The pinned ring — host-planned uploads only, so ekf_replay_device never
// grows it — grows EVERY slot together, so an allocation happens the first time a plan this large
// is seen, never on a later same-sized call that lands on a ring slot not used before (a
// hipHostMalloc costs ≈ 120 µs, a device re-allocation a drain: round 3 measured both inside a
// 20-message bench region). Host plans are flushed every kFlushDesc descriptors (plus one
// message), which bounds the ring.
constexpr size_t kDescInit = 256;  // descriptors at creation (×F/64 for wide handles)
int reserve_device(ekf_ctx* h, size_t need) {
  if (need <= h->ddesc_cap) return EKF_OK;
  if (drain(h)) return EKF_E_HIP;  // the previous launch may still read the old buffer
  if (h->ddesc) HIPCHK(hipFree(h->ddesc));
  h->ddesc = nullptr;
  const size_t cap = std::max(need, 2 * h->ddesc_cap);
  if (hipMalloc(&h->ddesc, cap * sizeof(MsgDesc)) != hipSuccess) return EKF_E_NOMEM;
  h->ddesc_cap = cap;
  return EKF_OK;
}
int reserve_upload(ekf_ctx* h, size_t need) {
  if (int rc = reserve_device(h, need)) return rc;
  if (need > h->ring_cap || !h->ring[0].p) {
    const size_t cap = std::max(need, std::min(2 * h->ring_cap, h->ddesc_cap));
    for (StageSlot& sl : h->ring) {
      if (sl.used) HIPCHK(hipEventSynchronize(sl.ev));
      if (sl.p) HIPCHK(hipHostFree(sl.p));
      sl.p = nullptr;
      sl.used = false;
      if (hipHostMalloc(reinterpret_cast<void**>(&sl.p), cap * sizeof(MsgDesc),
                        hipHostMallocDefault) != hipSuccess)
        return EKF_E_NOMEM;
      sl.cap = cap;
    }
    h->ring_cap = cap;
  }
  return EKF_OK;
}

// The next pinned staging slot, once the device is done with its last upload.
int next_slot(ekf_ctx* h, StageSlot** out) {
  StageSlot& sl = h->ring[h->ring_next];
  h->ring_next = (h->ring_next + 1) % kRing;
  if (sl.used) HIPCHK(hipEventSynchronize(sl.ev));
  *out = &sl;
  return EKF_OK;
}

// Resident path: the plan's descriptors and its entry list (packed behind them, in MsgDesc-sized
// slots) go up with one copy, then ONE kernel launch runs the whole plan, a workgroup per filter.
int flush_resident(ekf_ctx* h) {
  const size_t nd = h->plan_d.size(), nl = h->plan_l.size();
  if (nl == 0) return EKF_OK;
  const size_t pslots = (nl * sizeof(PlanEntry) + sizeof(MsgDesc) - 1) / sizeof(MsgDesc);
  const size_t ns = nd + pslots;
  if (int rc = reserve_upload(h, ns)) return rc;
  StageSlot* slp = nullptr;
  if (int rc = next_slot(h, &slp)) return rc;
  StageSlot& sl = *slp;
  std::memcpy(sl.p, h->plan_d.data(), nd * sizeof(MsgDesc));
  PlanEntry* pe = reinterpret_cast<PlanEntry*>(sl.p + nd);
  int flo = INT_MAX, fhi = 0;
  for (size_t i = 0; i < nl; ++i) {
    const Launch& L = h->plan_l[i];
    pe[i] = PlanEntry{static_cast<int>(L.off), L.f0, L.nf, L.kind};
    flo = std::min(flo, L.f0);
    fhi = std::max(fhi, L.f0 + L.nf);
  }
  HIPCHK(hipMemcpyAsync(h->ddesc, sl.p, ns * sizeof(MsgDesc), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipEventRecord(sl.ev, h->stream));
  sl.used = true;
  const PassArgs<double> a = args<double>(h, h->ddesc, 0);
  const PlanEntry* dplan = reinterpret_cast<const PlanEntry*>(h->ddesc + nd);
  const int rc = timed(h, 4, h->stream, [&](hipEvent_t e0, hipEvent_t e1) {
    return launch_resident(a, dplan, static_cast<int>(nl), flo, fhi - flo, h->stream, e0, e1);
  });
  h->plan_d.clear();
  h->plan_l.clear();
  for (int f = 0; f < h->F; ++f) forget_desc(h, f);
  std::fill(h->prev_m.begin(), h->prev_m.end(), -1);
  return rc;
}

// Upload the whole plan with one copy, then enqueue its launches in order.
int flush(ekf_ctx* h) {
  if (h->resident) return flush_resident(h);
  const size_t nd = h->plan_d.size();
  if (nd == 0) return EKF_OK;
  if (int rc = reserve_upload(h, nd)) return rc;
  StageSlot* slp = nullptr;
  if (int rc = next_slot(h, &slp)) return rc;
  StageSlot& sl = *slp;
  std::memcpy(sl.p, h->plan_d.data(), nd * sizeof(MsgDesc));
  if (join_bulk(h)) return EKF_E_HIP;  // the bulk stream may still read descriptors
  HIPCHK(hipMemcpyAsync(h->ddesc, sl.p, nd * sizeof(MsgDesc), hipMemcpyHostToDevice, h->stream));
  // the bulk stream reads these descriptors too: one main → bulk hop per upload
  HIPCHK(hipEventRecord(h->ev_chain, h->stream));
  HIPCHK(hipStreamWaitEvent(h->bulk, h->ev_chain, 0));
  h->main_dirty = false;
  h->main_unordered = false;
  HIPCHK(hipEventRecord(sl.ev, h->stream));
  sl.used = true;
  int rc = EKF_OK;
  const size_t nl = h->plan_l.size();
  for (size_t li = 0; li < nl && !rc;) {
    const Launch& L = h->plan_l[li];
    const MsgDesc* dp = h->ddesc + L.off;
    if (L.kind == 0) {  // a run of known-association chunks → one persistent chain launch
      size_t lj = li + 1;
      if (h->devsync && !h->serial)  // the bulk kernels must run beside the chain launch
        while (lj < nl && h->plan_l[lj].kind == 0 && h->plan_l[lj].f0 == L.f0 &&
               h->plan_l[lj].nf == L.nf && h->plan_l[lj].off == h->plan_l[lj - 1].off + L.nf)
          ++lj;
      bool nolook = false;
      for (int k = 0; k < L.nf; ++k) {
        const int fl = h->plan_d[L.off + k].flags;
        nolook = nolook || ((fl & kActive) && !(fl & kLook));
      }
      rc = group(h, dp, h->plan_d.data() + L.off, L.f0, L.nf, static_cast<int>(lj - li), true,
                 nolook, lj < nl);
      h->main_dirty = true;
      li = lj;
      continue;
    }
    if (L.kind == 3) {
      // the pass's epoch is for another stream's consumer: the next association chunk runs on
      // the same (bulk) stream, behind the pass in stream order, so a run of them publishes once,
      // after its last pass (an epoch kernel per chunk cost ≈ 4.5 µs of each 106 µs chunk)
      rc = assoc_msg_group(h, dp, L.f0, L.nf, li + 1 < nl && h->plan_l[li + 1].kind != 3);
      ++li;
      continue;
    }
    if (L.kind == 1) {
      // (an owed epoch: k_assoc cannot poll it; the flush's start joined the bulk stream anyway)
      const bool poll = h->devsync && !h->serial && !h->epoch_owed;
      if (!poll && join_bulk(h)) return EKF_E_HIP;
      rc = assoc(h, dp, L.f0, L.nf, poll);
      // the chunk's factors and Σ pass on the bulk stream (with split CU masks the main stream
      // has 4 CUs per XCD: a pass there took 33 µs against 9 at N = 1024 fp32); the next
      // association joins the bulk stream first
      if (!rc) rc = group(h, dp, h->plan_d.data() + L.off, L.f0, L.nf, 1, true);
      h->main_dirty = true;
    }
    if (!rc && L.kind == 2) {
      if (join_bulk(h)) return EKF_E_HIP;
      rc = posterior_launch(h, dp, L.f0, L.nf);
      h->main_dirty = true;
      h->main_unordered = true;  // (k_posterior reads its descriptor; no bulk work follows it)
    }
    ++li;
  }
  h->plan_d.clear();
  h->plan_l.clear();
  for (int f = 0; f < h->F; ++f) forget_desc(h, f);
  return rc;
}

// Deferred submission (ekf_defer): callbacks append to the plan, which goes up with ONE upload and
// runs as one resident launch (or one pipelined run) once it is large or the caller synchronises.
constexpr size_t kFlushDesc = 8192;
int submit(ekf_ctx* h) {
  if (h->defer && h->plan_d.size() < kFlushDesc) return EKF_OK;
  return flush(h);
}

// Before any host access to device state: run what is planned, then wait for it.
// ekf_replay_device left the planning state on the device: bring it into the host mirror (behind
// everything enqueued so far) before the host plans or reads per-filter state again.
int adopt_device_plan(ekf_ctx* h) {
  if (!h->dev_plan) return EKF_OK;
  hipSetDevice(h->cfg.device);
  HIPCHK(hipMemcpyAsync(h->hstate, h->dstate[h->dstate_cur], h->F * sizeof(PlanState),
                        hipMemcpyDeviceToHost, h->plan_stream ? h->plan_stream : h->stream));
  if (drain(h)) return EKF_E_HIP;
  for (int f = 0; f < h->F; ++f) {
    const PlanState& ps = h->hstate[f];
    h->parity[f] = ps.parity;
    h->prev_m[f] = ps.prev_m;
    h->pending[f] = static_cast<char>(ps.pending);
    for (int i = 0; i < kMaxChunk; ++i) h->prev_ids[f][i] = ps.prev_ids[i];
    h->odom[f] = Pose2{ps.odom[0], ps.odom[1], ps.odom[2]};
    forget_desc(h, f);
  }
  h->dev_plan = false;
  return EKF_OK;
}

int settle(ekf_ctx* h) {
  if (int rc = flush(h)) return rc;
  if (drain(h)) return EKF_E_HIP;
  return adopt_device_plan(h);
}

// After a drain: did a device poll of this handle time out since the last report? Reported once
// (EKF_E_TIMEOUT); which filters it hit stays in their status (EKF_FLAG_TIMEOUT).
int take_fatal(ekf_ctx* h) {
  volatile unsigned* p = h->fatal_h;
  if (!p || *p == 0) return EKF_OK;
  *p = 0;
  return EKF_E_TIMEOUT;
}

// Association with the decisions read back (synchronous), kMaxAssoc markers per upload.
int assoc_sync(ekf_ctx* h, int f0, int nf, bool predict, bool posterior, int m_max, int* j_out,
               int* new_out) {
  int mm = 1;
  for (int k = 0; k < nf; ++k) mm = std::max(mm, static_cast<int>(h->msgs[k].size()));
  for (int i0 = 0; i0 < mm; i0 += kMaxAssoc) {
    const int i1 = std::min(mm, i0 + kMaxAssoc);
    plan_unknown(h, f0, nf, predict, posterior && i1 == mm, i0, i1);
    int rc = flush(h);
    if (rc) return rc;
    if (drain(h)) return EKF_E_HIP;
    for (int k = 0; k < nf; ++k) {
      FilterCtl c;
      HIPCHK(hipMemcpy(&c, h->ctl + f0 + k, sizeof(FilterCtl), hipMemcpyDeviceToHost));
      const int mf = static_cast<int>(h->msgs[k].size());
      for (int i = i0; i < std::min(i1, mf); ++i) {
        if (j_out) j_out[static_cast<size_t>(k) * m_max + i] = c.assoc_j[i % kMaxAssoc];
        if (new_out) new_out[static_cast<size_t>(k) * m_max + i] = c.assoc_new[i % kMaxAssoc];
      }
    }
  }
  return EKF_OK;
}

// Parse one message per filter (ekf_batch_sensor layout) into h->msgs.
int load_batch(ekf_ctx* h, int assoc_mode, int m_max, const int* counts, const int* ids,
               const int* actions, const double* rel_xy, const double* odom) {
  for (int f = 0; f < h->F; ++f) {
    const int c = counts[f];
    if (c < 0 || c > m_max) return EKF_E_ARG;
    if (!assoc_mode)
      for (int i = 0; i < c; ++i) {
        const size_t e = static_cast<size_t>(f) * m_max + i;
        if (actions && actions[e] == EKF_MARKER_DELETE) continue;
        if (ids[e] < 0 || ids[e] >= h->cfg.n_landmarks) return EKF_E_RANGE;
      }
  }
  for (int f = 0; f < h->F; ++f) {
    if (odom) h->odom[f] = Pose2{odom[3 * f], odom[3 * f + 1], odom[3 * f + 2]};
    h->absent[f] = counts[f] == 0;
    auto& mk = h->msgs[f];
    mk.clear();
    for (int i = 0; i < counts[f]; ++i) {
      const size_t e = static_cast<size_t>(f) * m_max + i;
      if (!assoc_mode && actions && actions[e] == EKF_MARKER_DELETE) continue;
      Marker k;
      k.id = assoc_mode ? -1 : ids[e];
      measure(rel_xy[2 * e], rel_xy[2 * e + 1], &k.zr, &k.zb);
      mk.push_back(k);
    }
  }
  return EKF_OK;
}

bool valid(ekf_ctx* h, int f) { return h && f >= 0 && f < h->F; }

}  // namespace

namespace ekfslam {

int handle_info(ekf_t h, HandleInfo* out) {
  if (!h || !out) return EKF_E_ARG;
  if (int rc = flush(h)) return rc;
  hipSetDevice(h->cfg.device);
  if (join_bulk(h)) return EKF_E_HIP;  // work enqueued on the main stream next sees the bulk's done
  out->F = h->F;
  out->N = h->cfg.n_landmarks;
  out->n = h->n;
  out->dtype = h->cfg.dtype;
  out->device = h->cfg.device;
  out->resident = h->resident;
  out->joseph = h->joseph;
  out->stream = h->stream;
  out->bulk = h->bulk ? h->bulk : h->stream;
  return EKF_OK;
}

int handle_parity(ekf_t h, int* parity) {
  if (!h || !parity) return EKF_E_ARG;
  if (int rc = adopt_device_plan(h)) return rc;
  for (int f = 0; f < h->F; ++f) parity[f] = h->parity[f];
  return EKF_OK;
}

int run_device_plan(ekf_t h, const MsgDesc* dd, const PlanEntry* dplan, int T,
                    const int* parity_after, const double* odom_after) {
  if (!h || T < 0 || !dd || !parity_after || !odom_after) return EKF_E_ARG;
  hipSetDevice(h->cfg.device);
  if (int r0 = adopt_device_plan(h)) return r0;
  int rc = EKF_OK;
  if (T > 0) {
    if (h->resident) {
      const PassArgs<double> a = args<double>(h, dd, 0);
      rc = timed(h, 4, h->stream, [&](hipEvent_t e0, hipEvent_t e1) {
        return launch_resident(a, dplan, T, 0, h->F, h->stream, e0, e1);
      });
    } else {
      // an owed Σ-pass epoch (the last flush's last pass published none): the chains take every
      // earlier pass as complete (PassArgs::first_ready), which holds once main has joined bulk
      if (h->epoch_owed && join_bulk(h)) return EKF_E_HIP;
      // the bulk stream reads these descriptors too (written on the main stream)
      HIPCHK(hipEventRecord(h->ev_chain, h->stream));
      HIPCHK(hipStreamWaitEvent(h->bulk, h->ev_chain, 0));
      const size_t F = static_cast<size_t>(h->F);
      if (h->devsync && !h->serial) {
        rc = group(h, dd, nullptr, 0, h->F, T, true, true);
      } else {
        for (int t = 0; t < T && !rc; ++t)
          rc = group(h, dd + t * F, nullptr, 0, h->F, 1, true, t == 0);
      }
      h->main_dirty = true;
    }
  }
  for (int f = 0; f < h->F; ++f) {
    h->parity[f] = parity_after[f];
    h->odom[f] = Pose2{odom_after[3 * f], odom_after[3 * f + 1], odom_after[3 * f + 2]};
    h->pending[f] = 0;
    h->prev_m[f] = -1;
    forget_desc(h, f);
  }
  return rc;
}

}  // namespace ekfslam


extern "C" {

void ekf_config_default(ekf_config* c) {
  if (!c) return;
  c->n_landmarks = 50;
  c->n_filters = 1;
  c->dtype = EKF_F64;
  c->q_noise = 1.0e-2;
  c->r_noise = 1.0e-2;
  c->init_var = 10e6;
  c->mah_gate = 2.0;
  c->device = 0;
}

const char* ekf_strerror(int s) {
  switch (s) {
    case EKF_OK: return "ok";
    case EKF_E_ARG: return "invalid argument";
    case EKF_E_RANGE: return "landmark index out of range / landmark capacity exhausted";
    case EKF_E_EMPTY: return "empty marker array";
    case EKF_E_NUMERIC: return "singular or non-finite innovation covariance";
    case EKF_E_HIP: return "HIP runtime error";
    case EKF_E_NOMEM: return "out of memory";
    case EKF_E_TIMEOUT:
      return "a device hand-off timed out: the state of the filters flagged EKF_FLAG_TIMEOUT is "
             "undefined (ekf_reset / ekf_set_state them)";
    default: return "unknown status";
  }
}

int ekf_create(ekf_t* out, const ekf_config* cfg_in) {
  if (!out) return EKF_E_ARG;
  *out = nullptr;
  ekf_config cfg;
  ekf_config_default(&cfg);
  if (cfg_in) cfg = *cfg_in;
  if (cfg.n_landmarks < 1 || cfg.n_filters < 1 || (cfg.dtype != EKF_F64 && cfg.dtype != EKF_F32))
    return EKF_E_ARG;
  ekf_ctx* h = new (std::nothrow) ekf_ctx;
  if (!h) return EKF_E_NOMEM;
  h->cfg = cfg;
  h->F = cfg.n_filters;
  h->n = 3 + 2 * cfg.n_landmarks;
  h->w = cfg.dtype == EKF_F32 ? 4 : 8;
  const int per_line = static_cast<int>(128 / h->w);
  h->ld = (h->n + per_line - 1) / per_line * per_line;
  h->ldk = (h->n + 63) / 64 * 64;
  h->sig_stride = static_cast<size_t>(h->n) * h->ld;
  h->x_stride = static_cast<size_t>((h->n + 15) / 16 * 16);
  h->km_stride = static_cast<size_t>(kMaxKW) * h->ldk;
  h->odom.assign(h->F, Pose2{});
  h->parity.assign(h->F, 0);
  h->pending.assign(h->F, 0);
  h->prev_m.assign(h->F, -1);
  h->stg_desc.assign(h->F, std::array<long, 2>{-1L, -1L});
  h->prev_ids.assign(h->F, std::array<int, kMaxChunk>{});
  h->msgs.resize(h->F);
  h->absent.assign(h->F, 0);
  auto fail = [&](int rc) {
    ekf_destroy(h);
    return rc;
  };
  if (hipSetDevice(cfg.device) != hipSuccess) return fail(EKF_E_HIP);
  if (const char* e = std::getenv("EKF_SERIAL")) h->serial = std::atoi(e) != 0;
  if (const char* e = std::getenv("EKF_DBG_ORDER")) h->dbg_order = static_cast<unsigned>(std::atoi(e));
  if (const char* e = std::getenv("EKF_ASSOC_MSG")) h->assoc_msg = std::atoi(e) != 0;
  {  // EKF_RESIDENT=0: the HBM pipeline at every size (tests compare the two)
    const char* e = std::getenv("EKF_RESIDENT");
    h->resident = cfg.dtype == EKF_F64 && h->n <= kResidentMaxN && !(e && std::atoi(e) == 0);
  }
  if (create_streams(h) != EKF_OK ||
      hipEventCreateWithFlags(&h->ev_chain, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_sig[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_sig[1], hipEventDisableTiming) != hipSuccess)
    return fail(EKF_E_HIP);
  // Many filters (no CU split, so event hand-offs): the Σ pass's waves hold every CU a chain or a
  // factor kernel needs, so nothing overlaps it anyway; one stream turns the two
  // cross-stream hops per message into kernel boundaries: swarm 1.12 → 1.15e7 corrections/s, with
  // the staging off (below) 1.17e7 (profiles/r4/r4s_*). EKF_SERIAL=0 keeps the two streams.
  {
    const char* e = std::getenv("EKF_SERIAL");
    if (!e && !h->devsync && h->F > kCuSplitMaxFilters) h->serial = true;
  }
  h->am_route = am_route(h);
  h->am_route_j = am_route(h, true);
  if (hipHostMalloc(reinterpret_cast<void**>(&h->fatal_h), 64,
                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
    return fail(EKF_E_NOMEM);
  *h->fatal_h = 0;
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&h->fatal_d), h->fatal_h, 0) != hipSuccess)
    return fail(EKF_E_HIP);
  const size_t sig_bytes = h->sig_stride * h->F * h->w;
  for (int p = 0; p < 2; ++p) {
    if (hipMalloc(&h->sig[p], sig_bytes) != hipSuccess) return fail(EKF_E_NOMEM);
    if (hipMalloc(&h->x[p], h->x_stride * h->F * sizeof(double)) != hipSuccess)
      return fail(EKF_E_NOMEM);
  }
  const size_t km_bytes = h->km_stride * h->F * h->w;
  if (hipMalloc(&h->kcat, km_bytes) != hipSuccess) return fail(EKF_E_NOMEM);
  if (hipMalloc(&h->mcat, km_bytes) != hipSuccess) return fail(EKF_E_NOMEM);
  if (hipMalloc(&h->ctl, sizeof(FilterCtl) * h->F) != hipSuccess) return fail(EKF_E_NOMEM);
  if (hipMalloc(&h->rec, 2 * sizeof(ChunkRec) * h->F) != hipSuccess) return fail(EKF_E_NOMEM);
  // staged rebuild operands (EKF_STAGE=0: every kLook chain gathers its own, tests compare the two)
  // The same many-filter handles skip it by default (EKF_STAGE=1 keeps it): there every message's
  // k_patch_stage runs on the serial critical path (≈ 18 µs for 512 filters), more than the chains'
  // own gathers cost (two rounds of ≈ 2 µs).
  const char* stage_env = std::getenv("EKF_STAGE");
  const size_t stage_bytes = 2 * h->F *
      (cfg.dtype == EKF_F32 ? sizeof(StageRec<float>) : sizeof(StageRec<double>));
  const bool stage_on = stage_env ? std::atoi(stage_env) != 0
                                  : (h->devsync || h->F <= kCuSplitMaxFilters);
  if (stage_on) {
    if (hipMalloc(&h->stage, stage_bytes) != hipSuccess) return fail(EKF_E_NOMEM);
    if (hipMemset(h->stage, 0, stage_bytes) != hipSuccess) return fail(EKF_E_HIP);
  }
  // (+ 3F words: PassArgs::dbg & 8's per-kernel launch epochs)
  if (h->dbg_order & (4096u | 8192u)) {
    const size_t b = sizeof(unsigned long long) * kDlogKinds * 64 * 64 * 8;
    if (hipMalloc(&h->dlog, b) != hipSuccess) return fail(EKF_E_NOMEM);
    if (hipMemset(h->dlog, 0, b) != hipSuccess) return fail(EKF_E_HIP);
  }
  const size_t sync_bytes = sizeof(unsigned) * (kSyncChain + 4 * static_cast<size_t>(h->F));
  if (hipMalloc(&h->sync, sync_bytes) != hipSuccess) return fail(EKF_E_NOMEM);
  if (hipMemset(h->sync, 0, sync_bytes) != hipSuccess) return fail(EKF_E_HIP);
  h->ddesc_cap = std::max(kDescInit, static_cast<size_t>(h->F) * 4);
  if (hipMalloc(&h->ddesc, sizeof(MsgDesc) * h->ddesc_cap) != hipSuccess) return fail(EKF_E_NOMEM);
  for (int i = 0; i < kRing; ++i)
    if (hipEventCreateWithFlags(&h->ring[i].ev, hipEventDisableTiming) != hipSuccess)
      return fail(EKF_E_HIP);
  if (int rc = reserve_upload(h, h->ddesc_cap)) return fail(rc);  // every pinned slot up front
  // Σ₀ = diag(0,0,0, init_var·I_2N), state = 0 (slam.cpp:127-132, :674)
  for (int p = 0; p < 2; ++p) {
    if (hipMemsetAsync(h->sig[p], 0, sig_bytes, h->stream) != hipSuccess) return fail(EKF_E_HIP);
    if (hipMemsetAsync(h->x[p], 0, h->x_stride * h->F * sizeof(double), h->stream) != hipSuccess)
      return fail(EKF_E_HIP);
  }
  // chunk records start zeroed: no kernel ever sees a previous process's bytes, whatever the
  // stream interleaving
  if (hipMemsetAsync(h->rec, 0, 2 * sizeof(ChunkRec) * h->F, h->stream) != hipSuccess)
    return fail(EKF_E_HIP);
  if (hipMemsetAsync(h->kcat, 0, km_bytes, h->stream) != hipSuccess ||
      hipMemsetAsync(h->mcat, 0, km_bytes, h->stream) != hipSuccess ||
      hipMemsetAsync(h->ctl, 0, sizeof(FilterCtl) * h->F, h->stream) != hipSuccess)
    return fail(EKF_E_HIP);
  hipError_t e = cfg.dtype == EKF_F32
                     ? launch_init_diag<float>(static_cast<float*>(h->sig[0]), h->sig_stride, h->n,
                                               h->ld, cfg.init_var, h->F, h->stream)
                     : launch_init_diag<double>(static_cast<double*>(h->sig[0]), h->sig_stride,
                                                h->n, h->ld, cfg.init_var, h->F, h->stream);
  if (e != hipSuccess || hipStreamSynchronize(h->stream) != hipSuccess) return fail(EKF_E_HIP);
  *out = h;
  return EKF_OK;
}

int ekf_destroy(ekf_t h) {
  if (!h) return EKF_E_ARG;
  hipSetDevice(h->cfg.device);
  if (h->bulk) hipStreamSynchronize(h->bulk);
  if (h->stream) hipStreamSynchronize(h->stream);
  for (int p = 0; p < 2; ++p) {
    if (h->sig[p]) hipFree(h->sig[p]);
    if (h->x[p]) hipFree(h->x[p]);
  }
  if (h->kcat) hipFree(h->kcat);
  if (h->mcat) hipFree(h->mcat);
  if (h->ctl) hipFree(h->ctl);
  if (h->rec) hipFree(h->rec);
  if (h->stage) hipFree(h->stage);
  if (h->ddesc) hipFree(h->ddesc);
  for (PlanState* p : h->dstate)
    if (p) hipFree(p);
  if (h->hstate) hipHostFree(h->hstate);
  if (h->fatal_h) hipHostFree(h->fatal_h);
  if (h->am.hist) hipFree(h->am.hist);
  if (h->am.cur) hipFree(h->am.cur);
  if (h->am.gran) hipFree(h->am.gran);
  for (int i = 0; i < kRing; ++i) {
    if (h->ring[i].p) hipHostFree(h->ring[i].p);
    if (h->ring[i].ev) hipEventDestroy(h->ring[i].ev);
  }
  for (auto& pe : h->pe) {
    for (auto e : pe.start) hipEventDestroy(e);
    for (auto e : pe.stop) hipEventDestroy(e);
  }
  for (auto e : h->pool) hipEventDestroy(e);
  if (h->ev_chain) hipEventDestroy(h->ev_chain);
  if (h->ev_join) hipEventDestroy(h->ev_join);
  if (h->sync) hipFree(h->sync);
  if (h->dlog) hipFree(h->dlog);
  for (hipEvent_t e : h->ev_sig)
    if (e) hipEventDestroy(e);
  for (hipEvent_t e : h->dbg_ev) hipEventDestroy(e);
  if (h->bulk) hipStreamDestroy(h->bulk);
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
  return EKF_OK;
}

int ekf_dims(ekf_t h, int* n, int* ld, int* nf) {
  if (!h) return EKF_E_ARG;
  if (n) *n = h->n;
  if (ld) *ld = h->ld;
  if (nf) *nf = h->F;
  return EKF_OK;
}

int ekf_get_path(ekf_t h, int* path) {
  if (!h || !path) return EKF_E_ARG;
  *path = h->resident ? EKF_PATH_RESIDENT : EKF_PATH_PIPELINE;
  return EKF_OK;
}

int ekf_set_odom(ekf_t h, int f, double theta, double x, double y) {
  if (!valid(h, f)) return EKF_E_ARG;
  if (int rc = adopt_device_plan(h)) return rc;
  h->odom[f] = Pose2{theta, x, y};
  return EKF_OK;
}

int ekf_fake_sensor(ekf_t h, int f, int m, const int* ids, const int* actions,
                    const double* rel_xy) {
  if (!valid(h, f) || m < 0 || (m > 0 && (!ids || !rel_xy))) return EKF_E_ARG;
  if (m == 0) return EKF_E_EMPTY;
  if (int rc = adopt_device_plan(h)) return rc;
  auto& mk = h->msgs[0];
  mk.clear();
  for (int i = 0; i < m; ++i) {
    if (actions && actions[i] == EKF_MARKER_DELETE) continue;
    if (ids[i] < 0 || ids[i] >= h->cfg.n_landmarks) return EKF_E_RANGE;
    Marker k;
    k.id = ids[i];
    measure(rel_xy[2 * i], rel_xy[2 * i + 1], &k.zr, &k.zb);
    mk.push_back(k);
  }
  hipSetDevice(h->cfg.device);
  plan_known(h, f, 1, true);
  return submit(h);
}

int ekf_sensor(ekf_t h, int f, int m, const double* rel_xy, int* assoc_out, int* is_new_out) {
  if (!valid(h, f) || m < 0 || (m > 0 && !rel_xy)) return EKF_E_ARG;
  if (m == 0) return EKF_E_EMPTY;
  if (int rc = adopt_device_plan(h)) return rc;
  auto& mk = h->msgs[0];
  mk.clear();
  for (int i = 0; i < m; ++i) {
    Marker k;
    k.id = -1;
    measure(rel_xy[2 * i], rel_xy[2 * i + 1], &k.zr, &k.zb);
    mk.push_back(k);
  }
  hipSetDevice(h->cfg.device);
  if (!assoc_out && !is_new_out) {
    plan_unknown(h, f, 1, true, true, 0, m);
    return submit(h);
  }
  const int rc = assoc_sync(h, f, 1, true, true, m, assoc_out, is_new_out);
  if (rc) return rc;
  {
    unsigned fl = 0;
    if (drain(h)) return EKF_E_HIP;
    if (int t = take_fatal(h)) return t;
    HIPCHK(hipMemcpy(&fl, &h->ctl[f].status, sizeof(unsigned), hipMemcpyDeviceToHost));
    if (fl & EKF_FLAG_RANGE) return EKF_E_RANGE;
  }
  return EKF_OK;
}

int ekf_batch_sensor(ekf_t h, int assoc_mode, int m_max, const int* counts, const int* ids,
                     const int* actions, const double* rel_xy, const double* odom) {
  if (!h || m_max < 0 || !counts || (m_max > 0 && !rel_xy) || (!assoc_mode && m_max > 0 && !ids))
    return EKF_E_ARG;
  if (int r0 = adopt_device_plan(h)) return r0;
  const int rc = load_batch(h, assoc_mode, m_max, counts, ids, actions, rel_xy, odom);
  if (rc) return rc;
  hipSetDevice(h->cfg.device);
  if (assoc_mode) {
    int mm = 1;
    for (int f = 0; f < h->F; ++f) mm = std::max(mm, static_cast<int>(h->msgs[f].size()));
    plan_unknown(h, 0, h->F, true, true, 0, mm, h->absent.data());
  } else {
    plan_known(h, 0, h->F, true, h->absent.data());
  }
  return submit(h);
}

int ekf_replay(ekf_t h, int assoc_mode, int T, int m_max, const int* counts, const int* ids,
               const int* actions, const double* rel_xy, const double* odom, double* out_pose) {
  if (!h || T < 0 || !counts || !odom || m_max < 0 || (m_max > 0 && !rel_xy) ||
      (!assoc_mode && m_max > 0 && !ids))
    return EKF_E_ARG;
  const size_t F = static_cast<size_t>(h->F);
  hipSetDevice(h->cfg.device);
  if (int rc = adopt_device_plan(h)) return rc;
  for (int t = 0; t < T; ++t) {
    const size_t o = static_cast<size_t>(t) * F * m_max;
    int rc = load_batch(h, assoc_mode, m_max, counts + t * F, ids ? ids + o : nullptr,
                        actions ? actions + o : nullptr, rel_xy + 2 * o, odom + 3 * F * t);
    if (rc) {
      flush(h);
      return rc;
    }
    if (assoc_mode) {
      int mm = 1;
      for (size_t f = 0; f < F; ++f) mm = std::max(mm, static_cast<int>(h->msgs[f].size()));
      plan_unknown(h, 0, h->F, true, true, 0, mm, h->absent.data());
    } else {
      plan_known(h, 0, h->F, true, h->absent.data());
    }
    // Many filters: upload and launch every ~kFlushDesc descriptors, so planning the next
    // messages on the host overlaps the GPU's work on these (one filter keeps the whole replay in
    // one upload and one persistent chain launch).
    if (!out_pose && h->plan_d.size() >= kFlushDesc) {
      rc = flush(h);
      if (rc) return rc;
    }
    if (out_pose) {
      rc = flush(h);
      if (rc) return rc;
      if (drain(h)) return EKF_E_HIP;
      for (size_t f = 0; f < F; ++f)
        HIPCHK(hipMemcpy(out_pose + 3 * (F * t + f), h->x[h->parity[f]] + f * h->x_stride,
                         3 * sizeof(double), hipMemcpyDeviceToHost));
    }
  }
  return submit(h);
}

// Known-association replay whose inputs are already in device memory: the descriptors are planned
// on the GPU (plan_kernels.hip) into the upload buffer, then the same launch groups as a flush.
// The planning state (parity, previous chunk, odometry) stays on the device between such calls.
int ekf_replay_device(ekf_t h, int T, int m_max, const int* d_counts, const int* d_ids,
                      const int* d_actions, const double* d_rel_xy, const double* d_odom) {
  if (!h || T < 0 || m_max < 0 || m_max > kMaxChunk || !d_counts || !d_odom ||
      (m_max > 0 && (!d_ids || !d_rel_xy)))
    return EKF_E_ARG;
  if (h->resident) return EKF_E_ARG;
  if (T == 0) return EKF_OK;
  // (Joseph form: one chunk per message too, kMaxJoseph = kMaxChunk, flagged kJoseph)
  hipSetDevice(h->cfg.device);
  if (int rc = flush(h)) return rc;  // what the host planned before runs first
  const size_t F = static_cast<size_t>(h->F);
  if (!h->dstate[0]) {
    for (PlanState*& p : h->dstate)
      if (hipMalloc(&p, F * sizeof(PlanState)) != hipSuccess) return EKF_E_NOMEM;
    if (hipHostMalloc(reinterpret_cast<void**>(&h->hstate), F * sizeof(PlanState),
                      hipHostMallocDefault) != hipSuccess)
      return EKF_E_NOMEM;
  }
  if (int rc = reserve_device(h, static_cast<size_t>(T) * F)) return rc;  // (no host staging)
  // device epochs: the planner runs on the bulk stream — ahead of the group's factor kernels and
  // Σ passes in stream order — and counts its descriptors, which the chain launch polls: the chain
  // starts beside the planner instead of behind a main → bulk event hop (≈ 6 µs of each replay)
  const bool beside = h->devsync && !h->serial;
  // the bulk stream may still read the last descriptors (an idle one reads nothing: no hop)
  if (((h->dbg_order & 2u) || hipStreamQuery(h->bulk) != hipSuccess) && join_bulk(h))
    return EKF_E_HIP;
  // ... and the main stream: work there that the bulk stream is not ordered after (a k_posterior
  // of ekf_posterior reads its descriptor in ddesc) must end before a planner on the bulk stream
  // rewrites ddesc. (Chains are covered: the bulk stream's factor kernels follow every chain
  // through its epoch or an event, so a planner enqueued behind them runs after it.)
  if (beside && h->main_unordered) {
    HIPCHK(hipEventRecord(h->ev_chain, h->stream));
    HIPCHK(hipStreamWaitEvent(h->bulk, h->ev_chain, 0));
    h->main_unordered = false;
  }
  hipStream_t ps = beside ? h->bulk : h->stream;
  if (!h->dev_plan) {  // the host mirror goes down once; later device replays chain on the device
    for (size_t f = 0; f < F; ++f) {
      PlanState& ps = h->hstate[f];
      ps = PlanState{};
      ps.parity = h->parity[f];
      ps.prev_m = h->prev_m[f];
      ps.pending = h->pending[f];
      for (int i = 0; i < kMaxChunk; ++i) ps.prev_ids[i] = h->prev_ids[f][i];
      ps.odom[0] = h->odom[f].theta;
      ps.odom[1] = h->odom[f].x;
      ps.odom[2] = h->odom[f].y;
    }
    HIPCHK(hipMemcpyAsync(h->dstate[h->dstate_cur], h->hstate, F * sizeof(PlanState),
                          hipMemcpyHostToDevice, ps));
    h->dev_plan = true;
  }
  ReplayArgs a{};
  a.counts = d_counts;
  a.ids = d_ids;
  a.actions = d_actions;
  a.rel = d_rel_xy;
  a.odom = d_odom;
  a.st_in = h->dstate[h->dstate_cur];
  a.st_out = h->dstate[h->dstate_cur ^ 1];
  a.desc = h->ddesc;
  a.T = T;
  a.joseph = h->joseph ? 1 : 0;
  a.F = h->F;
  a.M = m_max;
  a.N = h->cfg.n_landmarks;
  a.stage = h->stage != nullptr;
  a.plan_count = beside ? h->sync + kSyncPlan : nullptr;
  HIPCHK(launch_plan_replay(a, ps));
  h->dstate_cur ^= 1;
  h->plan_stream = ps;
  if (beside) {
    h->plan_total += static_cast<unsigned>(T) * static_cast<unsigned>(h->F);
    h->need_plan = h->plan_total;
  } else {
    // the bulk stream reads these descriptors too: one main → bulk hop (recorded before the
    // chain: behind a persistent chain launch the bulk kernels it waits for could never start)
    HIPCHK(hipEventRecord(h->ev_chain, h->stream));
    HIPCHK(hipStreamWaitEvent(h->bulk, h->ev_chain, 0));
  }
  h->main_dirty = false;
  const bool stg = h->stage != nullptr;
  int rc = EKF_OK;
  if (h->devsync && !h->serial) {
    // (the device planner stages only for chunks two on inside this replay: kStageOut needs next2)
    rc = group(h, h->ddesc, nullptr, 0, h->F, T, true, true, false, stg ? T - 2 : 0);
  } else {
    // Events: a chunk t ≥ 1 needs the Σ pass two back (kLook), or — no message of its filter
    // earlier in this replay — the passes before the replay, which the first chunk's join covers:
    // the wait on the pass two back suffices, and the chain of t runs beside the factor kernel and
    // Σ pass of t − 1 where the CUs allow (not a join of the whole bulk stream per message)
    for (int t = 0; t < T && !rc; ++t)
      rc = group(h, h->ddesc + static_cast<size_t>(t) * F, nullptr, 0, h->F, 1, true, t == 0, true,
                 stg && t + 2 < T ? 1 : 0);
  }
  h->main_dirty = true;
  if (!rc && (h->dbg_order & 32u) && drain(h)) return EKF_E_HIP;
  return rc;
}

int ekf_predict(ekf_t h, int f) {
  if (!valid(h, f)) return EKF_E_ARG;
  if (int rc = adopt_device_plan(h)) return rc;
  h->pending[f] = 1;
  return EKF_OK;
}

int ekf_correct(ekf_t h, int f, int id, double rx, double ry) {
  if (!valid(h, f)) return EKF_E_ARG;
  if (id < 0 || id >= h->cfg.n_landmarks) return EKF_E_RANGE;
  if (int rc = adopt_device_plan(h)) return rc;
  auto& mk = h->msgs[0];
  mk.clear();
  Marker k;
  k.id = id;
  measure(rx, ry, &k.zr, &k.zb);
  mk.push_back(k);
  hipSetDevice(h->cfg.device);
  plan_known(h, f, 1, false);
  return submit(h);
}

int ekf_associate_correct(ekf_t h, int f, double rx, double ry, int* j, int* is_new) {
  if (!valid(h, f)) return EKF_E_ARG;
  if (int rc = adopt_device_plan(h)) return rc;
  auto& mk = h->msgs[0];
  mk.clear();
  Marker k;
  k.id = -1;
  measure(rx, ry, &k.zr, &k.zb);
  mk.push_back(k);
  hipSetDevice(h->cfg.device);
  int jj = -1, nn = 0;
  const int rc = assoc_sync(h, f, 1, false, false, 1, &jj, &nn);
  if (rc) return rc;
  if (int t = take_fatal(h)) return t;  // (assoc_sync drained)
  if (j) *j = jj;
  if (is_new) *is_new = nn;
  if (jj < 0) return EKF_E_RANGE;
  return EKF_OK;
}

int ekf_posterior(ekf_t h, int f) {
  if (!valid(h, f)) return EKF_E_ARG;
  if (int rc = adopt_device_plan(h)) return rc;
  hipSetDevice(h->cfg.device);
  if (h->pending[f]) {  // fold the pending predict into a zero-marker pass, then the posterior
    h->msgs[0].clear();
    plan_known(h, f, 1, true);
  } else {
    plan_posterior(h, f);
  }
  return submit(h);
}

int ekf_flush(ekf_t h) {
  if (!h) return EKF_E_ARG;
  return flush(h);
}

int ekf_sync(ekf_t h) {
  if (!h) return EKF_E_ARG;
  // (a device replay's planning state stays on the device: the next host access adopts it)
  if (int rc = flush(h)) return rc;
  if (drain(h)) return EKF_E_HIP;
  return take_fatal(h);
}

int ekf_get_schedule(ekf_t h, int* flags) {
  if (!h || !flags) return EKF_E_ARG;
  *flags = (h->devsync ? EKF_SCHED_DEVSYNC : 0) | (h->serial ? EKF_SCHED_SERIAL : 0);
  return EKF_OK;
}

int ekf_get_assoc_route(ekf_t h, int* route) {
  if (!h || !route) return EKF_E_ARG;
  // (the route in effect: the Joseph form keeps the chunk route only where its kernel fits alike)
  *route = h->joseph && h->am_route_j != h->am_route ? EKF_ASSOC_MARKER : h->am_route;
  return EKF_OK;
}

int ekf_set_joseph(ekf_t h, int on) {
  if (!h) return EKF_E_ARG;
  if (int rc = flush(h)) return rc;  // what is planned runs with the form it was planned in
  if (h->joseph == (on != 0)) return EKF_OK;
  // a simple-form chain cannot rebuild from a Joseph chunk's record (its V columns): the first
  // chunk of each filter after a switch gathers its rows from Σ instead (no kLook)
  if (int rc = adopt_device_plan(h)) return rc;
  for (int f = 0; f < h->F; ++f) {
    h->prev_m[f] = -1;
    forget_desc(h, f);
  }
  h->joseph = on != 0;
  return EKF_OK;
}

int ekf_defer(ekf_t h, int on) {
  if (!h) return EKF_E_ARG;
  h->defer = on != 0;
  return on ? EKF_OK : flush(h);
}

// Σ₀ = diag(0,0,0, init_var·I_2N), state 0, t_map_odom identity, counter 0 (slam.cpp:127-139),
// on the device, for one filter or all (f < 0): a fresh run without reallocating.
int ekf_reset(ekf_t h, int f) {
  if (!h || f >= h->F) return EKF_E_ARG;
  if (int rc = settle(h)) return rc;
  hipSetDevice(h->cfg.device);
  const int f0 = f < 0 ? 0 : f, nf = f < 0 ? h->F : 1;
  for (int k = f0; k < f0 + nf; ++k) {
    h->parity[k] = 0;
    h->pending[k] = 0;
    h->prev_m[k] = -1;
    forget_desc(h, k);
  }
  const size_t sb = h->sig_stride * h->w;
  char* sig0 = static_cast<char*>(h->sig[0]) + f0 * sb;
  HIPCHK(hipMemsetAsync(sig0, 0, sb * nf, h->stream));
  HIPCHK(hipMemsetAsync(h->x[0] + f0 * h->x_stride, 0, h->x_stride * nf * sizeof(double),
                        h->stream));
  HIPCHK(hipMemsetAsync(h->ctl + f0, 0, sizeof(FilterCtl) * nf, h->stream));
  const hipError_t e =
      h->cfg.dtype == EKF_F32
          ? launch_init_diag<float>(reinterpret_cast<float*>(sig0), h->sig_stride, h->n, h->ld,
                                    h->cfg.init_var, nf, h->stream)
          : launch_init_diag<double>(reinterpret_cast<double*>(sig0), h->sig_stride, h->n, h->ld,
                                     h->cfg.init_var, nf, h->stream);
  if (e != hipSuccess) return EKF_E_HIP;
  return drain(h);
}

int ekf_get_pose(ekf_t h, int f, double* p) {
  if (!valid(h, f) || !p) return EKF_E_ARG;
  if (int rc = settle(h)) return rc;
  HIPCHK(hipMemcpy(p, h->x[h->parity[f]] + f * h->x_stride, 3 * sizeof(double),
                   hipMemcpyDeviceToHost));
  return EKF_OK;
}

int ekf_get_map_odom(ekf_t h, int f, double* p) {
  if (!valid(h, f) || !p) return EKF_E_ARG;
  if (int rc = settle(h)) return rc;
  HIPCHK(hipMemcpy(p, h->ctl[f].tmo, 3 * sizeof(double), hipMemcpyDeviceToHost));
  return EKF_OK;
}

int ekf_get_state(ekf_t h, int f, double* state, double* sigma, unsigned* counter) {
  if (!valid(h, f)) return EKF_E_ARG;
  if (int rc = settle(h)) return rc;
  const int p = h->parity[f];
  if (state)
    HIPCHK(hipMemcpy(state, h->x[p] + f * h->x_stride, h->n * sizeof(double),
                     hipMemcpyDeviceToHost));
  if (sigma) {
    std::vector<char> buf(h->sig_stride * h->w);
    const char* src = static_cast<const char*>(h->sig[p]) + f * h->sig_stride * h->w;
    HIPCHK(hipMemcpy(buf.data(), src, buf.size(), hipMemcpyDeviceToHost));
    for (int i = 0; i < h->n; ++i)
      for (int j = 0; j < h->n; ++j) {
        const size_t e = static_cast<size_t>(i) * h->ld + j;
        sigma[static_cast<size_t>(i) * h->n + j] =
            h->w == 4 ? reinterpret_cast<const float*>(buf.data())[e]
                      : reinterpret_cast<const double*>(buf.data())[e];
      }
  }
  if (counter) HIPCHK(hipMemcpy(counter, &h->ctl[f].counter, sizeof(unsigned), hipMemcpyDeviceToHost));
  return EKF_OK;
}

int ekf_set_state(ekf_t h, int f, const double* state, const double* sigma, const double* tmo,
                  unsigned counter) {
  if (!valid(h, f)) return EKF_E_ARG;
  if (int rc = settle(h)) return rc;
  h->prev_m[f] = -1;
  forget_desc(h, f);
  const int p = h->parity[f];
  if (state)
    HIPCHK(hipMemcpy(h->x[p] + f * h->x_stride, state, h->n * sizeof(double),
                     hipMemcpyHostToDevice));
  if (sigma) {
    std::vector<char> buf(h->sig_stride * h->w, 0);
    // fp64 pipeline: Σ is kept exactly symmetric (the symmetric Σ pass mirrors its upper triangle
    // and the factor kernel reads Σ_in[U, i] for Σ_in[i, U]), so the upper triangle is taken
    const bool sym = h->w == 8 && !h->resident;
    for (int i = 0; i < h->n; ++i)
      for (int j = 0; j < h->n; ++j) {
        const size_t e = static_cast<size_t>(i) * h->ld + j;
        const double v = sym && i > j ? sigma[static_cast<size_t>(j) * h->n + i]
                                      : sigma[static_cast<size_t>(i) * h->n + j];
        if (h->w == 4)
          reinterpret_cast<float*>(buf.data())[e] = static_cast<float>(v);
        else
          reinterpret_cast<double*>(buf.data())[e] = v;
      }
    char* dst = static_cast<char*>(h->sig[p]) + f * h->sig_stride * h->w;
    HIPCHK(hipMemcpy(dst, buf.data(), buf.size(), hipMemcpyHostToDevice));
  }
  if (tmo) HIPCHK(hipMemcpy(h->ctl[f].tmo, tmo, 3 * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(&h->ctl[f].counter, &counter, sizeof(unsigned), hipMemcpyHostToDevice));
  h->pending[f] = 0;
  return EKF_OK;
}

int ekf_get_status(ekf_t h, int f, unsigned* flags) {
  if (!valid(h, f) || !flags) return EKF_E_ARG;
  if (int rc = settle(h)) return rc;
  HIPCHK(hipMemcpy(flags, &h->ctl[f].status, sizeof(unsigned), hipMemcpyDeviceToHost));
  const unsigned z = 0;
  HIPCHK(hipMemcpy(&h->ctl[f].status, &z, sizeof(unsigned), hipMemcpyHostToDevice));
  return EKF_OK;
}

int ekf_profile_enable(ekf_t h, int enable) {
  if (!h) return EKF_E_ARG;
  h->prof = enable != 0;
  return EKF_OK;
}

int ekf_profile_read(ekf_t h, int kind, long long* launches, double* total_ms) {
  if (!h || kind < 0 || kind > 4) return EKF_E_ARG;
  if (int rc = settle(h)) return rc;
  auto& pe = h->pe[kind];
  for (size_t i = 0; i < pe.start.size(); ++i) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, pe.start[i], pe.stop[i]) == hipSuccess) h->prof_ms[kind] += ms;
    h->prof_launches[kind] += 1;
    h->pool.push_back(pe.start[i]);
    h->pool.push_back(pe.stop[i]);
  }
  pe.start.clear();
  pe.stop.clear();
  if (kind == 1) {  // a chain launch walks several chunks: report per chunk
    h->prof_launches[1] = h->prof_chunks;
    h->prof_chunks = 0;
  }
  if (launches) *launches = h->prof_launches[kind];
  if (total_ms) *total_ms = h->prof_ms[kind];
  h->prof_launches[kind] = 0;
  h->prof_ms[kind] = 0.0;
  return EKF_OK;
}

double ekf_normalize_angle(double rad) { return normalize_angle(rad); }

int ekf_debug_poison_lds(int device) {
  if (hipSetDevice(device) != hipSuccess) return EKF_E_HIP;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    return EKF_E_HIP;
  // a quiet NaN with a payload: NaN·0 = NaN, so any product with unwritten LDS poisons the result
  const unsigned long long nan = 0x7ff8dead0000beefull;
  if (launch_poison_lds(nan, 12 * (cus > 0 ? cus : 256), nullptr) != hipSuccess) return EKF_E_HIP;
  return hipDeviceSynchronize() == hipSuccess ? EKF_OK : EKF_E_HIP;
}

#ifdef EKF_DIAG_STAMPS
int ekfslam_diag_read_stamps(unsigned long long* out, int n);  // ekf_kernels.hip
// dev only (libekfslam_diag.so): the chain kernel's s_memtime stamps of filter 0's last chunk
int ekf_diag_stamps(unsigned long long* out, int n) { return ekfslam_diag_read_stamps(out, n); }
int ekfslam_res_read_stamps(unsigned long long* out, int n);  // ekf_resident.hip
// dev only: the resident kernel's stamps (filter flo, thread 0): 6 per correction
int ekf_diag_res_stamps(unsigned long long* out, int n) { return ekfslam_res_read_stamps(out, n); }
extern "C" int ekfslam_diag_read_am_stamps(unsigned long long* out);  // ekf_assoc.hip
// dev only: k_assoc_msg's s_memrealtime stamps, [2 workgroups][kMaxChunk + 1][8]
int ekf_diag_am_stamps(unsigned long long* out) { return ekfslam_diag_read_am_stamps(out); }
#endif

// dev only (tools/diag_handover.py): the PassArgs::dbg & 4 counters, sync[kSyncDbg + i], i < n ≤ 16
int ekf_debug_counters(ekf_t h, unsigned* out, int n) {
  if (!h || !out || n < 0 || n > 16) return EKF_E_ARG;
  if (int rc = settle(h)) return rc;
  HIPCHK(hipMemcpy(out, h->sync + kSyncDbg, n * sizeof(unsigned), hipMemcpyDeviceToHost));
  return EKF_OK;
}

// dev only: the PassArgs::dlog checksums (EKF_DBG_ORDER & 4096), kDlogKinds·64·64·8 words
int ekf_debug_log(ekf_t h, unsigned long long* out) {
  if (!h || !out || !h->dlog) return EKF_E_ARG;
  if (int rc = settle(h)) return rc;
  HIPCHK(hipMemcpy(out, h->dlog, sizeof(unsigned long long) * kDlogKinds * 64 * 64 * 8,
                   hipMemcpyDeviceToHost));
  return EKF_OK;
}

double ekf_sigma_pass_bytes(ekf_t h, int nf) {
  if (!h) return 0.0;
  const double n = h->n;
  // fp64: the symmetric pass (k_sigma_pass, SigmaTile64) reads the upper triangle of Σ_in only
  const double elems = h->w == 8 ? n * (n + 1) / 2 + n * n : 2.0 * n * n;
  return elems * static_cast<double>(h->w) * nf;
}

}  // extern "C"
