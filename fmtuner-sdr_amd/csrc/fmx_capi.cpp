// fmx_capi.cpp -- C ABI of libfmx: handle lifetime, per-channel parameter
// mirrors of the reference setters, resampler timing schedules, and the
// launch sequence that replaces one iteration of the reference's per-block
// body (src/main.cpp:1239-1308) for every channel of a handle.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "fmx_internal.h"
#include "fmx_synth.h"

namespace fmx {

#define HIP_TRY(expr)                                                                                   \
  do {                                                                                                  \
    hipError_t e__ = (expr);                                                                            \
    if (e__ != hipSuccess) {                                                                            \
      h->err = std::string(#expr) + ": " + hipGetErrorString(e__);                                      \
      return FMX_E_HIP;                                                                                 \
    }                                                                                                   \
  } while (0)

// Timing groups: channels whose resampler timing state is identical share
// one host-simulated output schedule (the schedule does not depend on the
// signal, only on the state and the number of inputs).
//
// Every step's schedules reach the GPU in ONE copy per set: slot b (step k
// mod FMX_NBUF) is [group map (C ints) | counts (cap ints) | schedules (G x
// stride)] in one device allocation, staged from a pinned host image of the
// same layout, copied by a small kernel on the stream of the set's only
// reader, right before it (the RDS set on sA before the front end, the
// audio set on sD before k_audio): stream order alone covers the slot, so
// no event joins the streams for it.  (Round 2 uploaded the next step's
// schedules one step early on sB: the front end then waited, through the
// upload's event, for the previous step's k_pll -- 35-50 us per step.)
#define FMX_HSLOTS 8 // pinned schedule images per timing set
// front-end completion events, a ring deeper than the image ring: a pinned
// image the front end of step s read (the speculated RDS schedule) is reused
// at the earliest FMX_HSLOTS / 2 steps later (at most two simulations per
// step), while evF[s % FMX_FRING] still marks that launch (round 4 bound the
// image to evA[s % FMX_NBUF], which the front end of step s + 3 re-binds: the
// host then waited for a later front end than the image's reader)
#define FMX_FRING (2 * FMX_HSLOTS)
// device schedule slots per timing set: one more than the intermediates'
// slots, so that the RDS slot the front end of step k fills for step k+1 was
// last read at step k-3 -- covered by the front end's one wait (evD(k-3))
#define FMX_SSLOTS (FMX_NBUF + 1)
struct TimingSet {
  float del = 1.0f;
  std::vector<ResampTiming> groups;
  std::vector<int> chan_group;
  int stride = 0, cap_groups = 0;
  int G = 0;   // groups in the last simulated step
  int cur = 0; // slot holding the schedules of the step being launched
  size_t slot_bytes = 0;
  unsigned char *d_slot[FMX_SSLOTS] = {};
  // pinned staging images, a ring deeper than the device slots: the image
  // reused at step k was copied at step k - FMX_HSLOTS, long complete, so the
  // host never blocks on it (with one image per device slot the host waited
  // 0.66 ms per step on the copy of step k-3 and woke late, ms-long GPU gaps)
  unsigned char *h_slot[FMX_HSLOTS] = {};
  const void *h_dev[FMX_HSLOTS] = {}; // the images' device-side addresses (mapped pinned memory)
  int hnext = 0, hcur = 0; // next image to fill, image of the last simulation
  hipEvent_t ev_h[FMX_HSLOTS] = {}; // recorded after a copy kernel's read of h_slot[i]
  hipEvent_t ev_use[FMX_HSLOTS] = {}; // the event marking the last read of h_slot[i]: ev_h[i], or the front end's evF
  bool ev_h_set[FMX_HSLOTS] = {};
  FmxSched *d_sched[FMX_SSLOTS] = {};
  int *d_count[FMX_SSLOTS] = {};
  int *d_group[FMX_SSLOTS] = {};
  hipStream_t up_stream = nullptr; // stream of the last copy into the slots (the set's reader)
  // one step of speculation (the RDS set of process_block): the next step's
  // schedules for the same n, simulated into pinned image spec_img and copied
  // into slot spec_slot by this step's front end (FeArgs::next_sched_*)
  bool spec = false;
  int spec_n = 0, spec_slot = -1, spec_G = 0, spec_img = -1;
  std::vector<ResampTiming> spec_groups;
};

struct Handle {
  fmx_config cfg{};
  int C = 0, device = 0, M = 1;
  int n_cu = 256;  // compute units of `device` (queried at create)
  // decimator input samples every channel has seen since its last reset
  // (capped at L-1): a full history lets the frontend take its VEC path
  long dec_fill = 0;
  std::string err;
  // sA: frontend, resets, uploads; sB: stereo PLL; sC: RDS; sD: audio.
  // Step k's frontend runs while step k-1's PLL / RDS kernels (latency-bound,
  // one lane per channel, a few SIMDs) and step k-1's audio still run; the
  // audio of step k overlaps the PLL of step k+1 (raw L/R double-buffered).
  hipStream_t sA = nullptr, sB = nullptr, sC = nullptr, sD = nullptr;
  hipStream_t sP = nullptr; // k_pilot's stream: sA, or its own (FMX_PILOT_STREAM A/B)
  hipEvent_t evA[FMX_NBUF] = {}, evB[FMX_NBUF] = {}, evC[FMX_NBUF] = {}, evD[FMX_NBUF] = {};
  hipEvent_t evP[FMX_NBUF] = {}; // k_pilot (sA, after k_fe8): k_pll's input
  hipEvent_t evR[FMX_NBUF] = {}; // k_rs on sA (FMX_RS_ON_A_MAXC): k_rds's input
  hipEvent_t evF[FMX_FRING] = {}; // process_block's front end of step k: evF[k % FMX_FRING]
  // host waits on pinned-image reuse (fmx_host_stats): waits, waits that
  // found the event pending (the host blocked), milliseconds blocked
  long host_waits = 0, host_stalls = 0;
  double host_stall_ms = 0.0;
  hipEvent_t evTmpB = nullptr, evTmpC = nullptr, evTmpD = nullptr, evTmpU = nullptr;
  bool evB_set[FMX_NBUF] = {}, evC_set[FMX_NBUF] = {}, evD_set[FMX_NBUF] = {};
  uint64_t step = 0;
  int st_idx = 0;
  FmxDesign *hdes = nullptr;
  FmxDesign *ddes = nullptr;
  DesignExtras ex;
  // parameters
  std::vector<FmxChanParam> hpar;
  FmxChanParam *dpar = nullptr;
  bool par_dirty = true;
  std::vector<int> w0, bw_mode, agc_ready;
  // state
  uint8_t *dec_hist = nullptr;
  int *dec_valid = nullptr;
  float *dc_v = nullptr, *agc = nullptr, *fd_prev = nullptr, *clip = nullptr;
  // RF level (computeSignalLevel arguments per channel; smoother state)
  std::vector<double> hsig;   // [C][4] gain*factor, bias, floor, ceil
  double *dsig = nullptr;
  float *sig_smooth = nullptr;
  unsigned long long *sig_sums[FMX_NBUF] = {}; // [C][6] byte sums of step k (front end -> k_audio)
  bool sig_dirty = true;
  unsigned long long *dbg = nullptr;  // stage clocks (FMX_DIAG builds with STAMPS=1 kernels only)
  float2_t *iq_hist = nullptr;
  float *st_hist = nullptr, *lr_hist = nullptr, *af_win = nullptr, *af_iir = nullptr;
  float *mono_win = nullptr, *mono_iir = nullptr, *rds_hist = nullptr, *ring = nullptr;
  FmxStereoState *st = nullptr;
  FmxRdsState *rds = nullptr;
  int *reset_mask = nullptr;
  std::vector<int> hmask;
  // process_block's channel resets of this step, per stream part (round 5):
  // the front-end part runs on sA at prepare time, the others on their
  // streams right before their kernels (fmx_capi.cpp process_block)
  std::vector<ResetList> rl_pending;
  int *mute = nullptr; // [C][2] retune fade/mute {remaining, total} (main.cpp:1310-1337)
  float *dec_scratch = nullptr; // [C][2 * block] complex, fmx_decimate_u8 (allocated on first use)
  // intermediates (double-buffered by step parity)
  float *mpx[FMX_NBUF] = {}, *pilot[FMX_NBUF] = {}, *rds_in[FMX_NBUF] = {};
  int *rds_count[FMX_NBUF] = {};
  float *rds_win[FMX_NBUF] = {};  // [C][32] the previous call's last MPX samples, k_fe8 -> k_rs
  float *lraw[FMX_NBUF] = {}, *rraw[FMX_NBUF] = {};
  int rds_stride = 0;
  // row stride (floats) of the MPX / pilot / raw L/R intermediates: the block
  // rounded up to 32 and, when that is a multiple of 256 (1 KB), one 128-B
  // line more (round 6), so that the rows a workgroup reads side by side do
  // not all fall into the same L2 sets (a build with -DFMX_ROW_PAD=0: the
  // block itself; 2048 channels 0.3481 -> 0.3412 ms, profiles/r06o_*)
  int row = 0;
  // the intermediate slot the last k_rds read (its RDS-rate input stays there
  // until the next RDS call): the ring refill's source (FmxRdsState::ring_ok)
  int rds_last_buf = -1;
  int ring_always = 0; // fmx_diag_set(FMX_DIAG_RDS_RING_ALWAYS): k_rds writes the ring every call
  // the call's PSK2 symbols, k_rds (sC) -> k_bits (sD), per slot (at most one
  // per decimation period)
  float *rds_sym[FMX_NBUF] = {}, *rds_sym_im[FMX_NBUF] = {};
  int *rds_sym_count[FMX_NBUF] = {};
  int sym_stride = 0;
  uint32_t block_index = 0;
  TimingSet t_af, t_mono, t_rds;
  // kernel timing
  bool timing = false;
  int timing_every = 1; // time the launches of every timing_every-th step (fmx_timing_enable)
#if FMX_DIAG
  // diagnostics build only (make variant V=diag KDEFS=-DFMX_DIAG=1): kernels
  // left out of process_block (FMX_DIAG_SKIP=rds,pll,audio; outputs invalid)
  bool skip_rds = false, skip_pll = false, skip_audio = false, skip_krs = false, skip_pilot = false;
  bool nowait_a = false; // FMX_DIAG_NOWAIT=1: the front end skips its cross-stream waits (outputs invalid)
#endif
  struct Pending {
    int k;
    hipEvent_t a, b;
    bool b_pool; // b from the pool (KTimer), else a stream's completion event (KBind)
  };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> pool;
  double kms[FMX_K_COUNT] = {};
  int klaunch[FMX_K_COUNT] = {};
  std::vector<void *> allocs;
};

static int dmalloc(Handle *h, void **p, size_t bytes) {
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) {
    h->err = std::string("hipMalloc failed: ") + hipGetErrorString(e);
    return FMX_E_NOMEM;
  }
  hipMemset(*p, 0, bytes);
  h->allocs.push_back(*p);
  return FMX_OK;
}
template <typename T> static int dalloc(Handle *h, T **p, size_t count) {
  return dmalloc(h, reinterpret_cast<void **>(p), count * sizeof(T));
}

// Events that only order work on this device (stream joins, kernel timing)
// skip the system-scope fence at record time (hipEventDisableSystemFence).
static unsigned ev_flags(bool timing) {
  return (timing ? 0u : static_cast<unsigned>(hipEventDisableTiming)) |
         static_cast<unsigned>(hipEventDisableSystemFence);
}

static hipEvent_t ev_get(Handle *h) {
  if (!h->pool.empty()) {
    hipEvent_t e = h->pool.back();
    h->pool.pop_back();
    return e;
  }
  hipEvent_t e;
  hipEventCreateWithFlags(&e, ev_flags(true));
  return e;
}

struct KTimer {
  Handle *h;
  int k;
  hipStream_t s;
  hipEvent_t a = nullptr, b = nullptr;
  bool on;
  KTimer(Handle *hh, int kk, hipStream_t ss)
      : h(hh), k(kk), s(ss), on(hh->timing && hh->step % static_cast<uint64_t>(hh->timing_every) == 0) {
    if (on) {
      a = ev_get(h);
      b = ev_get(h);
      hipEventRecord(a, s);
    }
  }
  ~KTimer() {
    if (on) {
      hipEventRecord(b, s);
      h->pending.push_back({k, a, b, true});
    }
  }
};

static void timing_take(Handle *h, const Handle::Pending &p, bool wait) {
  float ms = 0.0f;
  if (wait) hipEventSynchronize(p.b);
  hipEventElapsedTime(&ms, p.a, p.b);
  h->kms[p.k] += ms;
  h->klaunch[p.k]++;
  h->pool.push_back(p.a);
  if (p.b_pool) h->pool.push_back(p.b);
}

// The pending timings up to the last one ending on `e`, waited for: `e` is
// about to be bound to a new launch.
static void timing_release(Handle *h, hipEvent_t e) {
  size_t last = 0;
  for (size_t k = 0; k < h->pending.size(); ++k)
    if (h->pending[k].b == e) last = k + 1;
  for (size_t k = 0; k < last; ++k) timing_take(h, h->pending[k], true);
  h->pending.erase(h->pending.begin(), h->pending.begin() + static_cast<std::ptrdiff_t>(last));
}

// process_block's launches: the stream's completion event `done` (evF / evC /
// evB / evD, or none) is bound to the kernel itself through hipExtLaunchKernel
// (set_launch_events), and with timing on a pool event takes its start (and
// its end when there is no `done`): no marker packets between the kernels of
// a stream (each marker was a packet the next kernel and every cross-stream
// waiter queued behind).  A kernel left out (diagnostics) or a failed launch
// records `done` as a marker.
struct KBind {
  Handle *h;
  int k;
  hipStream_t s;
  hipEvent_t a = nullptr, done;
  bool on, bound = false, own = false; // own: `done` from the pool (timing only)
  KBind(Handle *hh, int kk, hipStream_t ss, hipEvent_t d)
      : h(hh), k(kk), s(ss), done(d), on(hh->timing && hh->step % static_cast<uint64_t>(hh->timing_every) == 0) {
    if (on) {
      if (done) timing_release(h, done);
      a = ev_get(h);
      if (!done) {
        done = ev_get(h);
        own = true;
      }
    }
    set_launch_events(a, done);
  }
  // after a successful launch call
  void launched() { bound = true; }
  ~KBind() {
    set_launch_events(nullptr, nullptr);
    if (bound) {
      if (on) h->pending.push_back({k, a, done, own});
    } else {
      if (on) h->pool.push_back(a);
      if (own) h->pool.push_back(done);
      else if (done) hipEventRecord(done, s);
    }
  }
};

// the pending timings whose end event has completed, without blocking
// (process_block, every step while timing is on): keeps the event pool
// recycled, so the timed region never creates events -- creating them as the
// pool ran dry stalled the host for 3-6 ms every 5-6 steps (rocprofv3
// timeline: the GPU idle, the next step's work queued late)
static void harvest_timing(Handle *h) {
  size_t k = 0;
  for (; k < h->pending.size(); ++k) {
    auto &p = h->pending[k];
    if (hipEventQuery(p.b) != hipSuccess) break;
    timing_take(h, p, false);
  }
  h->pending.erase(h->pending.begin(), h->pending.begin() + static_cast<std::ptrdiff_t>(k));
}

static void collect_timing(Handle *h) {
  for (auto &p : h->pending) timing_take(h, p, true);
  h->pending.clear();
}

/* ---------------- timing sets ---------------- */
// slot layout: group map, counts, then the schedules 16-B aligned
static size_t tset_sched_off(const Handle *h, const TimingSet &t) {
  return (sizeof(int) * (static_cast<size_t>(h->C) + t.cap_groups) + 15) & ~static_cast<size_t>(15);
}
static FmxSched *tset_hsched(const Handle *h, TimingSet &t, int b) {
  return reinterpret_cast<FmxSched *>(t.h_slot[b] + tset_sched_off(h, t)); // b: host image
}
static void tset_free_slots(Handle *h, TimingSet &t) {
  for (int b = 0; b < FMX_SSLOTS; ++b) {
    if (t.d_slot[b]) {
      h->allocs.erase(std::remove(h->allocs.begin(), h->allocs.end(), static_cast<void *>(t.d_slot[b])),
                      h->allocs.end());
      hipFree(t.d_slot[b]);
    }
    t.d_slot[b] = nullptr;
  }
  for (int i = 0; i < FMX_HSLOTS; ++i) {
    if (t.h_slot[i]) hipHostFree(t.h_slot[i]);
    t.h_slot[i] = nullptr;
  }
}
static int tset_alloc_slots(Handle *h, TimingSet &t) {
  const size_t off = tset_sched_off(h, t);
  t.slot_bytes = (off + sizeof(FmxSched) * static_cast<size_t>(t.stride) * t.cap_groups + 15) & ~static_cast<size_t>(15);
  int rc;
  for (int b = 0; b < FMX_SSLOTS; ++b) {
    if ((rc = dalloc(h, &t.d_slot[b], t.slot_bytes)) != FMX_OK) return rc;

    t.d_group[b] = reinterpret_cast<int *>(t.d_slot[b]);
    t.d_count[b] = t.d_group[b] + h->C;
    t.d_sched[b] = reinterpret_cast<FmxSched *>(t.d_slot[b] + off);
  }
  for (int i = 0; i < FMX_HSLOTS; ++i) {
    HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&t.h_slot[i]), t.slot_bytes, hipHostMallocMapped));
    std::memset(t.h_slot[i], 0, t.slot_bytes);
    void *dp = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&dp, t.h_slot[i], 0));
    t.h_dev[i] = dp;
    if (!t.ev_h[i]) HIP_TRY(hipEventCreateWithFlags(&t.ev_h[i], ev_flags(false)));
  }
  return FMX_OK;
}
// cap: timing groups the slots hold before a reallocation (which synchronises
// the device): the AF / mono sets take a group per distinct post-reset
// timing state -- a live receiver's retunes leave a bounded number of them
// (the 240k -> 32k phase repeats every 15 blocks of 4096) -- the RDS set one
static int tset_init(Handle *h, TimingSet &t, float del, int max_in, int cap) {
  t.del = del;
  ResampTiming r;
  timing_reset(r);
  r.del = del;
  t.groups.assign(1, r);
  t.chan_group.assign(static_cast<size_t>(h->C), 0);
  t.stride = static_cast<int>(std::ceil(static_cast<double>(max_in) / std::max(0.5, (double)del))) + 8;
  t.cap_groups = std::max(1, std::min(cap, h->C));
  return tset_alloc_slots(h, t);
}
// channel c's resampler was reset (liquid resamp_reset): move it to a group
// in the post-reset state, creating the group if needed; drop empty groups.
static void tset_reset_channel(TimingSet &t, int c) {
  ResampTiming fresh;
  timing_reset(fresh);
  fresh.del = t.del;
  int g = -1;
  for (size_t i = 0; i < t.groups.size(); ++i)
    if (timing_equal(t.groups[i], fresh)) {
      g = static_cast<int>(i);
      break;
    }
  if (g < 0) {
    t.groups.push_back(fresh);
    g = static_cast<int>(t.groups.size()) - 1;
  }
  t.chan_group[static_cast<size_t>(c)] = g;
}

static void tset_compact(TimingSet &t) {
  std::vector<int> used(t.groups.size(), 0);
  for (int g : t.chan_group) used[static_cast<size_t>(g)] = 1;
  std::vector<int> remap(t.groups.size(), -1);
  std::vector<ResampTiming> ng;
  for (size_t i = 0; i < t.groups.size(); ++i)
    if (used[i]) {
      // merge groups whose state became identical
      int found = -1;
      for (size_t j = 0; j < ng.size(); ++j)
        if (timing_equal(ng[j], t.groups[i])) found = static_cast<int>(j);
      if (found < 0) {
        ng.push_back(t.groups[i]);
        found = static_cast<int>(ng.size()) - 1;
      }
      remap[i] = found;
    }
  for (int &g : t.chan_group) g = remap[static_cast<size_t>(g)];
  if (ng.empty()) {
    ResampTiming r;
    timing_reset(r);
    r.del = t.del;
    ng.push_back(r);
  }
  t.groups = ng;
}

// Wait until the last reader of pinned image i is done (counted: a wait that
// finds the event pending blocks the host).
static hipError_t image_wait(Handle *h, TimingSet &t, int i) {
  if (!t.ev_h_set[i]) return hipSuccess;
  h->host_waits++;
  hipError_t q = hipEventQuery(t.ev_use[i]);
  if (q == hipSuccess) return hipSuccess;
  if (q != hipErrorNotReady) return q;
  h->host_stalls++;
  const auto t0 = std::chrono::steady_clock::now();
  q = hipEventSynchronize(t.ev_use[i]);
  h->host_stall_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return q;
}

// Simulate n inputs for every group into the pinned image of slot `buf`
// (the caller uploads it); returns the largest output count in *max_count.
static int tset_simulate(Handle *h, TimingSet &t, int n, int buf, int *max_count) {
  tset_compact(t);
  const int G = static_cast<int>(t.groups.size());
  if (G > t.cap_groups) {
    HIP_TRY(hipDeviceSynchronize());
    tset_free_slots(h, t);
    t.cap_groups = G * 2;
    for (int i = 0; i < FMX_HSLOTS; ++i) t.ev_h_set[i] = false;
    int rc;
    if ((rc = tset_alloc_slots(h, t)) != FMX_OK) return rc;
  }
  // the previous copy out of this pinned image must have run
  const int hb = t.hnext;
  t.hnext = (hb + 1) % FMX_HSLOTS;
  t.hcur = hb;
  HIP_TRY(image_wait(h, t, hb));
  FmxSched *hs = tset_hsched(h, t, hb);
  int *hc = reinterpret_cast<int *>(t.h_slot[hb]) + h->C;
  int mx = 0;
  for (int g = 0; g < G; ++g) {
    const int k = timing_run(t.groups[static_cast<size_t>(g)], n, hs + static_cast<size_t>(g) * t.stride, t.stride);
    if (k > t.stride) {
      h->err = "resampler schedule overflow";
      return FMX_E_CAPACITY;
    }
    hc[g] = k;
    mx = std::max(mx, k);
  }
  std::memcpy(t.h_slot[hb], t.chan_group.data(), sizeof(int) * h->C);
  t.G = G;
  if (max_count) *max_count = mx;
  return FMX_OK;
}
static int tset_upload(Handle *h, TimingSet &t, int buf, hipStream_t s) {
  const size_t bytes = tset_sched_off(h, t) + sizeof(FmxSched) * static_cast<size_t>(t.stride) * t.G;
  // a copy kernel reading the mapped pinned image, not hipMemcpyAsync: the
  // runtime's small host-to-device copy blocked the host until the stream
  // reached it (round 2: 0.65 ms per step, up to 9 ms)
  if (t.up_stream && t.up_stream != s) { // the slot's last reader ran on another stream (stage calls vs process_block)
    HIP_TRY(hipEventRecord(h->evTmpU, t.up_stream));
    HIP_TRY(hipStreamWaitEvent(s, h->evTmpU, 0));
  }
  if (launch_copy16(t.h_dev[t.hcur], t.d_slot[buf], (bytes + 15) / 16, s) != FMX_OK) return FMX_E_HIP;
  HIP_TRY(hipEventRecord(t.ev_h[t.hcur], s));
  t.ev_use[t.hcur] = t.ev_h[t.hcur];
  t.ev_h_set[t.hcur] = true;
  t.up_stream = s;
  return FMX_OK;
}
// Simulate n inputs and upload the schedules into slot `buf` on stream s,
// the stream of the set's reader.
static int tset_advance(Handle *h, TimingSet &t, int n, int buf, hipStream_t s, int *max_count) {
  int rc;
  t.spec = false; // any other advance voids a speculated next step
  if ((rc = tset_simulate(h, t, n, buf, max_count)) != FMX_OK) return rc;
  if ((rc = tset_upload(h, t, buf, s)) != FMX_OK) return rc;
  t.cur = buf;
  return FMX_OK;
}

// process_block's RDS set: take the schedules speculated last step when this
// step has the same n (the slot was filled by the previous front end), else
// simulate and upload as usual.
static int tset_take_or_advance(Handle *h, TimingSet &t, int n, int buf, hipStream_t s) {
  if (t.spec && t.spec_n == n && t.spec_slot == buf) {
    t.groups = t.spec_groups;
    t.G = t.spec_G;
    t.hcur = t.spec_img;
    t.cur = buf;
    t.up_stream = s;
    t.spec = false;
    return FMX_OK;
  }
  return tset_advance(h, t, n, buf, s, nullptr);
}
// Simulate the NEXT step (same n) into a pinned image for slot `slot`; the
// front end launched next copies it (one 16-B word per thread of its first
// workgroups, grid of `threads` threads).  Returns the words to copy, 0 when
// nothing is speculated (schedules that would not fit the slot or the grid).
static unsigned tset_speculate(Handle *h, TimingSet &t, int n, int slot, size_t threads) {
  t.spec = false;
  const int G = static_cast<int>(t.groups.size());
  const size_t bytes = tset_sched_off(h, t) + sizeof(FmxSched) * static_cast<size_t>(t.stride) * G;
  const size_t n16 = (bytes + 15) / 16;
  if (G > t.cap_groups || n16 > threads) return 0;
  const int hb = t.hnext;
  if (image_wait(h, t, hb) != hipSuccess) return 0;
  t.spec_groups = t.groups;
  FmxSched *hs = tset_hsched(h, t, hb);
  int *hc = reinterpret_cast<int *>(t.h_slot[hb]) + h->C;
  for (int g = 0; g < G; ++g) {
    const int k = timing_run(t.spec_groups[static_cast<size_t>(g)], n, hs + static_cast<size_t>(g) * t.stride, t.stride);
    if (k > t.stride) return 0;
    hc[g] = k;
  }
  std::memcpy(t.h_slot[hb], t.chan_group.data(), sizeof(int) * h->C);
  t.hnext = (hb + 1) % FMX_HSLOTS;
  t.spec = true;
  t.spec_n = n;
  t.spec_slot = slot;
  t.spec_G = G;
  t.spec_img = hb;
  return static_cast<unsigned>(n16);
}

// Make sA wait for everything queued on sB, sC and sD (used before resets,
// parameter uploads and the single-stream stage entry points).
static int join_into_A(Handle *h) {
  HIP_TRY(hipEventRecord(h->evTmpB, h->sB));
  HIP_TRY(hipEventRecord(h->evTmpC, h->sC));
  HIP_TRY(hipEventRecord(h->evTmpD, h->sD));
  HIP_TRY(hipStreamWaitEvent(h->sA, h->evTmpB, 0));
  HIP_TRY(hipStreamWaitEvent(h->sA, h->evTmpC, 0));
  HIP_TRY(hipStreamWaitEvent(h->sA, h->evTmpD, 0));
  return FMX_OK;
}

static bool dec_warm(const Handle *h) { return h->M > 1 && h->dec_fill >= h->hdes->dec_len - 1; }
static void dec_advance(Handle *h, int n_out) {
  h->dec_fill = std::min<long>(h->hdes->dec_len - 1, h->dec_fill + (long)n_out * h->M);
}

static ResetArgs reset_args(Handle *h) {
  ResetArgs r{};
  r.des = h->ddes;
  r.C = h->C;
  r.mask = h->reset_mask;
  r.st = h->st;
  r.rds = h->rds;
  r.ring = h->ring;
  r.dec_hist = h->dec_hist;
  r.dec_valid = h->dec_valid;
  r.dc_v = h->dc_v;
  r.iq_hist = h->iq_hist;
  r.agc = h->agc;
  r.fd_prev = h->fd_prev;
  r.st_hist = h->st_hist;
  r.lr_hist = h->lr_hist;
  r.af_win = h->af_win;
  r.af_iir = h->af_iir;
  r.mono_win = h->mono_win;
  r.mono_iir = h->mono_iir;
  r.rds_hist = h->rds_hist;
  r.mute = h->mute;
  r.rds_prev = h->rds_last_buf >= 0 ? h->rds_in[h->rds_last_buf] : nullptr;
  r.rds_stride = h->rds_stride;
  return r;
}

static int apply_resets(Handle *h) {
  bool any = false;
  for (int v : h->hmask) {
    any |= (v != 0);
    if (v & (RS_DECIM | RS_CREATE)) h->dec_fill = 0;
  }
  if (!any) return FMX_OK;
  int rc = join_into_A(h);
  if (rc != FMX_OK) return rc;
  HIP_TRY(hipMemcpyAsync(h->reset_mask, h->hmask.data(), sizeof(int) * h->C, hipMemcpyHostToDevice, h->sA));
  rc = launch_reset(reset_args(h), h->sA);
  if (rc != FMX_OK) {
    h->err = "reset kernel launch failed";
    return rc;
  }
  std::fill(h->hmask.begin(), h->hmask.end(), 0);
  return FMX_OK;
}

static int sync_params(Handle *h) {
  if (h->sig_dirty) {
    int rc = join_into_A(h);
    if (rc != FMX_OK) return rc;
    HIP_TRY(hipMemcpyAsync(h->dsig, h->hsig.data(), sizeof(double) * h->hsig.size(), hipMemcpyHostToDevice, h->sA));
    h->sig_dirty = false;
  }
  if (!h->par_dirty) return FMX_OK;
  int rc = join_into_A(h);
  if (rc != FMX_OK) return rc;
  HIP_TRY(hipMemcpyAsync(h->dpar, h->hpar.data(), sizeof(FmxChanParam) * h->C, hipMemcpyHostToDevice, h->sA));
  h->par_dirty = false;
  return FMX_OK;
}

static int prepare(Handle *h) {
  int rc = sync_params(h);
  if (rc != FMX_OK) return rc;
  return apply_resets(h);
}

// the pending lists' `part` on stream s (the part's owner)
static int launch_reset_parts(Handle *h, int part, hipStream_t s) {
  for (const ResetList &L : h->rl_pending) {
    if (launch_reset_list(reset_args(h), L, part, h->st_idx, s) != FMX_OK) {
      h->err = "reset kernel launch failed";
      return FMX_E_HIP;
    }
  }
  return FMX_OK;
}

// process_block's resets without draining the pipeline: up to
// FMX_RESET_LISTS_MAX lists of FMX_RESET_LIST channels (kernel arguments, no
// upload) whose parts run on the stream that owns each part's state, right
// before that stream's kernel of this step -- after the previous step's
// kernel of the same stream, before this step's.  Object creation, or more
// channels than the lists hold (FMX_RESET_LISTS_MAX x FMX_RESET_LIST), take
// the joined path (prepare).  Lists a failed call left with parts unlaunched
// (an error return between the part launches below) go back into hmask whole:
// the next call resets those channels again in every part, so no channel is
// left half reset.  One retune per block at 4096 channels costs
// nothing measurable: 0.638 against 0.640 ms per step (profiles/
// r05h_retune_ab.txt); with round 4's join (and the handle on k_frontend)
// 1.01 ms (r05d), with the join alone 0.82 (r05e).
#define FMX_RESET_LISTS_MAX 4
static int prepare_pipelined(Handle *h) {
  int rc = sync_params(h);
  if (rc != FMX_OK) return rc;
  for (const ResetList &L : h->rl_pending)
    for (int i = 0; i < L.n; ++i) h->hmask[static_cast<size_t>(L.ch[i])] |= L.m[i];
  h->rl_pending.clear();
  int cnt = 0;
  bool create = false;
  for (int v : h->hmask) {
    cnt += (v != 0);
    create |= (v & RS_CREATE) != 0;
  }
  if (cnt == 0) return FMX_OK;
  if (create || cnt > FMX_RESET_LISTS_MAX * FMX_RESET_LIST) return apply_resets(h);
  ResetList L{};
  for (int c = 0; c < h->C; ++c) {
    const int v = h->hmask[static_cast<size_t>(c)];
    if (v == 0) continue;
    if (v & RS_DECIM) h->dec_fill = 0;
    L.ch[L.n] = c;
    L.m[L.n] = v;
    if (++L.n == FMX_RESET_LIST) {
      h->rl_pending.push_back(L);
      L = ResetList{};
    }
  }
  if (L.n > 0) h->rl_pending.push_back(L);
  std::fill(h->hmask.begin(), h->hmask.end(), 0);
  return launch_reset_parts(h, RSP_FRONT, h->sA);
}


/* ---------------- reference setters (host mirrors) ---------------- */
static void set_bandwidth(Handle *h, int c, int bw) { // fm_demod.cpp:168-204
  const int sel = bandwidth_select(bw, h->w0[static_cast<size_t>(c)]);
  if (sel == h->bw_mode[static_cast<size_t>(c)]) return;
  h->bw_mode[static_cast<size_t>(c)] = sel;
  h->hpar[static_cast<size_t>(c)].iqsel = sel;
  h->hmask[static_cast<size_t>(c)] |= RS_IQFIR;
  h->par_dirty = true;
}
static void set_deemph(Handle *h, int c, int code) { // main.cpp:699-708 -> both objects
  h->hpar[static_cast<size_t>(c)].deemph = code;
  if (code != FMX_DEEMPH_OFF) h->hmask[static_cast<size_t>(c)] |= RS_DEEMPH;
  h->par_dirty = true;
}
// setDeemphasis(tau_us) with any tau (fm_demod.cpp:50-62, af_post_processor.cpp:31-45):
// tau <= 0 disables it (filter state kept), else alpha = dt / (tau + dt) in
// float and the IIR re-created
static void set_deemph_us(Handle *h, int c, int tau_us) {
  FmxChanParam &p = h->hpar[static_cast<size_t>(c)];
  if (tau_us <= 0) {
    p.deemph = FMX_DEEMPH_OFF;
  } else {
    const float tau = static_cast<float>(tau_us) * 1e-6f;
    const float dt = 1.0f / static_cast<float>(h->cfg.out_rate);
    p.deemph = 3;
    p.deemph_alpha = dt / (tau + dt);
    h->hmask[static_cast<size_t>(c)] |= RS_DEEMPH;
  }
  h->par_dirty = true;
}
// setDeviation: kf = (float)(deviation / Fs), freqdem re-created (r_prev = 0)
static void set_deviation(Handle *h, int c, int hz) {
  const float kf = static_cast<float>(static_cast<double>(hz) / static_cast<double>(h->hdes->fs));
  h->hpar[static_cast<size_t>(c)].fd_ref = static_cast<float>(1.0 / (2.0 * 3.14159265358979323846 * static_cast<double>(kf)));
  h->hmask[static_cast<size_t>(c)] |= RS_FREQDEM;
  h->par_dirty = true;
}
static void set_agc(Handle *h, int c, int mode) { // fm_demod.cpp:210-217
  h->hpar[static_cast<size_t>(c)].agc = mode;
  if (mode != FMX_AGC_OFF) {
    h->agc_ready[static_cast<size_t>(c)] = 1;
    h->hmask[static_cast<size_t>(c)] |= RS_AGC;
  }
  h->par_dirty = true;
}

static void destroy(Handle *h) {
  if (!h) return;
  if (h->sA) hipStreamSynchronize(h->sA);
  if (h->sB) hipStreamSynchronize(h->sB);
  if (h->sC) hipStreamSynchronize(h->sC);
  if (h->sD) hipStreamSynchronize(h->sD);
  if (h->sP) hipStreamSynchronize(h->sP);
  for (auto &p : h->pending) {
    hipEventDestroy(p.a);
    if (p.b_pool) hipEventDestroy(p.b);
  }
  for (auto e : h->pool) hipEventDestroy(e);
  for (TimingSet *t : {&h->t_af, &h->t_mono, &h->t_rds}) {
    tset_free_slots(h, *t);
    for (hipEvent_t e : t->ev_h)
      if (e) hipEventDestroy(e);
  }
  for (void *p : h->allocs) hipFree(p);
  for (int b = 0; b < FMX_NBUF; ++b)
    for (hipEvent_t e : {h->evA[b], h->evB[b], h->evC[b], h->evD[b], h->evP[b], h->evR[b]})
      if (e) hipEventDestroy(e);
  for (hipEvent_t e : h->evF)
    if (e) hipEventDestroy(e);
  if (h->evTmpB) hipEventDestroy(h->evTmpB);
  if (h->evTmpC) hipEventDestroy(h->evTmpC);
  if (h->evTmpD) hipEventDestroy(h->evTmpD);
  if (h->evTmpU) hipEventDestroy(h->evTmpU);
  if (h->sP && h->sP != h->sA) hipStreamDestroy(h->sP);
  if (h->sD && h->sD != h->sA) hipStreamDestroy(h->sD);
  if (h->sC && h->sC != h->sA) hipStreamDestroy(h->sC);
  if (h->sB && h->sB != h->sA) hipStreamDestroy(h->sB);
  if (h->sA) hipStreamDestroy(h->sA);
  delete h->hdes;
  delete h;
}

static int create(const fmx_config *cfg, int n, int device, Handle **out) {
  auto *h = new (std::nothrow) Handle();
  if (!h) return FMX_E_NOMEM;
  *out = h;
  h->cfg = *cfg;
  h->C = n;
  h->device = device;
  if (n <= 0 || cfg->block <= 0 || cfg->block > 32768) {
    h->err = "n_channels must be > 0 and block in 1..32768";
    return FMX_E_INVALID;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    h->err = "no HIP device available";
    return FMX_E_NODEVICE;
  }
  if (device < 0 || device >= ndev) {
    h->err = "device index out of range";
    return FMX_E_INVALID;
  }
  HIP_TRY(hipSetDevice(device));
  {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && v > 0) h->n_cu = v;
  }
  h->hdes = new FmxDesign();
  int rc = design_build(*cfg, h->hdes, &h->ex, &h->err);
  if (rc != FMX_OK) return rc;
  h->M = h->hdes->M;
  if (h->M > 1 && !((h->M == 10 && h->hdes->dec_tpp == 28) || (h->M == 8 && h->hdes->dec_tpp == 28) ||
                    (h->M == 4 && h->hdes->dec_tpp == 20) || (h->M == 2 && h->hdes->dec_tpp == 12))) {
    h->err = "decimation factor has no kernel instantiation (supported M: 1, 2, 4, 8, 10)";
    return FMX_E_INVALID;
  }
  if (h->hdes->af_del < 3.0f) {
    h->err = "dsp_rate / out_rate must be >= 3";
    return FMX_E_INVALID;
  }
  HIP_TRY(hipStreamCreateWithFlags(&h->sA, hipStreamNonBlocking));
  // The product library reads no environment: its outputs and its schedule
  // depend only on the configuration and the calls.  A diagnostics build
  // (FMX_DIAG=1, never the shipped libfmx.so) adds FMX_SERIAL=1 (every kernel
  // on one stream: isolated per-kernel times) and FMX_DIAG_SKIP.
  bool serial = false;
#if FMX_DIAG
  if (const char *e = std::getenv("FMX_DIAG_SKIP")) {
    const std::string v(e);
    h->skip_rds = v.find("rds") != std::string::npos;
    h->skip_pll = v.find("pll") != std::string::npos;
    h->skip_audio = v.find("audio") != std::string::npos;
    h->skip_krs = v.find("krs") != std::string::npos;      // k_rs alone (the bound of fusing it into k_rds)
    h->skip_pilot = v.find("pilot") != std::string::npos;  // k_pilot alone
  }
  if (const char *e = std::getenv("FMX_SERIAL"); e && e[0] == '1') serial = true;
  if (const char *e = std::getenv("FMX_DIAG_NOWAIT"); e && e[0] == '1') h->nowait_a = true;
  if (const char *e = std::getenv("FMX_DIAG_SAPRIO"); e && e[0] == '1') {
    int lo = 0, hi = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_TRY(hipStreamDestroy(h->sA));
    HIP_TRY(hipStreamCreateWithPriority(&h->sA, hipStreamNonBlocking, hi));
  }
#endif
#ifndef FMX_PILOT_STREAM
#define FMX_PILOT_STREAM 0 // A/B: k_pilot on a fifth stream (after the front end's event) instead of sA
#endif
  if (serial) {
    h->sB = h->sC = h->sD = h->sP = h->sA;
  } else {
    HIP_TRY(hipStreamCreateWithFlags(&h->sB, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&h->sC, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&h->sD, hipStreamNonBlocking));
    h->sP = h->sA;
    if (FMX_PILOT_STREAM) HIP_TRY(hipStreamCreateWithFlags(&h->sP, hipStreamNonBlocking));
  }
  for (int b = 0; b < FMX_NBUF; ++b) {
    HIP_TRY(hipEventCreateWithFlags(&h->evA[b], ev_flags(true)));
    HIP_TRY(hipEventCreateWithFlags(&h->evB[b], ev_flags(true)));
    HIP_TRY(hipEventCreateWithFlags(&h->evP[b], ev_flags(true)));
    HIP_TRY(hipEventCreateWithFlags(&h->evR[b], ev_flags(true)));
    HIP_TRY(hipEventCreateWithFlags(&h->evC[b], ev_flags(true)));
    HIP_TRY(hipEventCreateWithFlags(&h->evD[b], ev_flags(true)));
  }
  for (hipEvent_t &e : h->evF) HIP_TRY(hipEventCreateWithFlags(&e, ev_flags(true)));
  HIP_TRY(hipEventCreateWithFlags(&h->evTmpB, ev_flags(false)));
  HIP_TRY(hipEventCreateWithFlags(&h->evTmpC, ev_flags(false)));
  HIP_TRY(hipEventCreateWithFlags(&h->evTmpD, ev_flags(false)));
  HIP_TRY(hipEventCreateWithFlags(&h->evTmpU, ev_flags(false)));
  if ((rc = dalloc(h, &h->ddes, 1)) != FMX_OK) return rc;
  HIP_TRY(hipMemcpy(h->ddes, h->hdes, sizeof(FmxDesign), hipMemcpyHostToDevice));
  const size_t C = static_cast<size_t>(n);
#ifndef FMX_ROW_PAD
#define FMX_ROW_PAD 1
#endif
  h->row = cfg->block;
  if (FMX_ROW_PAD) {
    h->row = (cfg->block + 31) & ~31;
    if (h->row % 256 == 0) h->row += 32;
  }
  const size_t B = static_cast<size_t>(h->row);
  // parameters: the reference objects as main.cpp:640-710 configures them
  h->hpar.assign(C, FmxChanParam{});
  h->w0.assign(C, 194000);
  h->bw_mode.assign(C, 0);
  h->agc_ready.assign(C, 0);
  h->hmask.assign(C, 0);
  for (size_t c = 0; c < C; ++c) {
    FmxChanParam &p = h->hpar[c];
    p.iqsel = FMX_IQ_CTOR;
    p.agc = 0;
    p.blend = std::clamp(cfg->blend, 0, 2);
    p.force_mono = cfg->force_mono;
    p.force_stereo = cfg->force_stereo;
    p.deemph = std::clamp(cfg->deemphasis, 0, 2);
  }
  if ((rc = dalloc(h, &h->dpar, C)) != FMX_OK) return rc;
  // state
  if ((rc = dalloc(h, &h->dec_hist, C * 2 * FMX_MAX_DEC)) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->dec_valid, C)) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->dc_v, C * 2)) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->agc, C * 2)) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->fd_prev, C * 2)) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->clip, C)) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->dsig, C * 4)) != FMX_OK) return rc;
#if FMX_DIAG
  if (const char *e = std::getenv("FMX_STAMPS"); e && e[0] == '1') {
    if ((rc = dalloc(h, &h->dbg, 48)) != FMX_OK) return rc; // [0,8) frontend, [8,16) k_rds, [16,32) k_pll, [32,48) sub-stage clocks
    HIP_TRY(hipMemset(h->dbg, 0, 48 * sizeof(unsigned long long)));
  }
#endif
  if ((rc = dalloc(h, &h->sig_smooth, C * 2)) != FMX_OK) return rc;
  for (int b = 0; b < FMX_NBUF; ++b)
    if ((rc = dalloc(h, &h->sig_sums[b], C * 6)) != FMX_OK) return rc;
  HIP_TRY(hipMemset(h->sig_smooth, 0, sizeof(float) * 2 * C));
  h->hsig.resize(static_cast<size_t>(C) * 4);
  for (int c = 0; c < C; ++c) {  // gain 0, config.h:27-29 defaults
    h->hsig[4 * c] = 0.0;
    h->hsig[4 * c + 1] = -4.0;
    h->hsig[4 * c + 2] = -55.0;
    h->hsig[4 * c + 3] = -19.0;
  }
  if ((rc = dalloc(h, &h->iq_hist, C * (FMX_IQ_MAXLEN - 1))) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->st_hist, FMX_ST_BUFS * C * FMX_HIST)) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->lr_hist, C * 2 * (FMX_LR_LEN - 1))) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->af_win, C * 64)) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->af_iir, C * 4)) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->mono_win, C * 32)) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->mono_iir, C * 2)) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->rds_hist, C * 32)) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->ring, C * 2 * FMX_RDS_RING)) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->st, C)) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->rds, C)) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->reset_mask, C)) != FMX_OK) return rc;
  if ((rc = dalloc(h, &h->mute, C * 2)) != FMX_OK) return rc;
  // intermediates
  for (int b = 0; b < FMX_NBUF; ++b) {
    if ((rc = dalloc(h, &h->mpx[b], C * B)) != FMX_OK) return rc;
    if ((rc = dalloc(h, &h->pilot[b], C * B)) != FMX_OK) return rc;
  }
  for (int b = 0; b < FMX_NBUF; ++b) {
    // pair tiles (whole groups of 2 channels); k_audio's XCD order reads octets
    if ((rc = dalloc(h, &h->lraw[b], ((C + 7) & ~static_cast<size_t>(7)) * B)) != FMX_OK) return rc;
    if ((rc = dalloc(h, &h->rraw[b], ((C + 7) & ~static_cast<size_t>(7)) * B)) != FMX_OK) return rc;
  }
  if ((rc = tset_init(h, h->t_rds, h->hdes->rds_del, cfg->block, 4)) != FMX_OK) return rc;
  if ((rc = tset_init(h, h->t_af, h->hdes->af_del, cfg->block, 64)) != FMX_OK) return rc;
  if ((rc = tset_init(h, h->t_mono, h->hdes->af_del, cfg->block, 64)) != FMX_OK) return rc;
  h->rds_stride = (h->t_rds.stride + 63) & ~63; // 256-B rows: k_rds stages 16-B aligned pieces
  h->sym_stride = (h->rds_stride / FMX_RDS_DECIM + 8 + 3) & ~3;
  for (int b = 0; b < FMX_NBUF; ++b) {
    if ((rc = dalloc(h, &h->rds_sym[b], C * static_cast<size_t>(h->sym_stride))) != FMX_OK) return rc;
    if ((rc = dalloc(h, &h->rds_sym_im[b], C)) != FMX_OK) return rc;
    if ((rc = dalloc(h, &h->rds_sym_count[b], C)) != FMX_OK) return rc;
    if ((rc = dalloc(h, &h->rds_in[b], C * static_cast<size_t>(h->rds_stride))) != FMX_OK) return rc;
    if ((rc = dalloc(h, &h->rds_count[b], C)) != FMX_OK) return rc;
    if ((rc = dalloc(h, &h->rds_win[b], C * 32)) != FMX_OK) return rc;
  }
  // construct every object (RS_CREATE) then apply main.cpp's configuration
  std::fill(h->hmask.begin(), h->hmask.end(), static_cast<int>(RS_CREATE));
  for (int c = 0; c < n; ++c) {
    h->w0[static_cast<size_t>(c)] = std::clamp(cfg->w0_bandwidth_hz, 0, 400000);
    set_agc(h, c, std::clamp(cfg->dsp_agc, 0, 2));
    set_deemph(h, c, std::clamp(cfg->deemphasis, 0, 2));
    if (cfg->bandwidth_hz >= 0) set_bandwidth(h, c, cfg->bandwidth_hz); // -1: keep the ctor filter
  }
  rc = prepare(h);
  if (rc != FMX_OK) return rc;
  HIP_TRY(hipStreamSynchronize(h->sA));
  return FMX_OK;
}

static FeArgs fe_args(Handle *h, int n, int mode, int buf) {
  FeArgs a{};
  a.des = h->ddes;
  a.des_fs = h->hdes->fs;
  a.par = h->dpar;
  a.C = h->C;
  a.n = n;
  a.in_mode = mode;
  a.st_hist_rd = h->st_hist + static_cast<size_t>(h->st_idx) * h->C * FMX_HIST;
  a.st_hist_wr = h->st_hist + static_cast<size_t>((h->st_idx + 1) % FMX_ST_BUFS) * h->C * FMX_HIST;
  a.dec_hist = h->dec_hist;
  a.dec_valid = h->dec_valid;
  a.dc_v = h->dc_v;
  a.iq_hist = h->iq_hist;
  a.agc = h->agc;
  a.fd_prev = h->fd_prev;
  a.rds_hist = h->rds_hist;
  a.clip_out = h->clip;
  a.dbg = h->dbg;
  a.rds_count = h->rds_count[buf];
  a.rds_sched = h->t_rds.d_sched[h->t_rds.cur];
  a.rds_sched_n = h->t_rds.d_count[h->t_rds.cur];
  a.rds_group = h->t_rds.d_group[h->t_rds.cur];
  a.rds_sched_stride = h->t_rds.stride;
  return a;
}

static AudioArgs audio_args(Handle *h, int n, int mode, TimingSet *t) {
  AudioArgs a{};
  a.des = h->ddes;
  a.par = h->dpar;
  a.C = h->C;
  a.n = n;
  a.mode = mode;
  a.lr_hist = h->lr_hist;
  a.af_win = h->af_win;
  a.af_iir = h->af_iir;
  a.mono_win = h->mono_win;
  a.mono_iir = h->mono_iir;
  if (t) {
    a.sched = t->d_sched[t->cur];
    a.sched_n = t->d_count[t->cur];
    a.group = t->d_group[t->cur];
    a.sched_stride = t->stride;
  }
  return a;
}

// k_audio of a process_block step evaluates the step's RF levels from the
// front end's byte sums (computeSignalLevel over the call's n * M IQ samples)
static void audio_signal_level(Handle *h, AudioArgs &a, const fmx_block_out *o, int buf, int n) {
  if (!o->d_signal) return;
  a.sig_out = o->d_signal;
  a.sig_sums = h->sig_sums[buf];
  a.sig_samples = static_cast<long>(n) * h->M;
  a.sig_par = h->dsig;
  a.sig_smooth = h->sig_smooth;
}

// raw L/R (k_pll -> k_audio) in pair tiles when the block is whole 16-sample tiles
static int lr_tiled(const Handle *h) { return (h->row % 16 == 0) ? 1 : 0; }

static PllArgs pll_args(Handle *h, int n, const float *mpx, int mpx_stride, int buf) {
  PllArgs a{};
  a.des = h->ddes;
  a.par = h->dpar;
  a.C = h->C;
  a.n = n;
  a.pilot = h->pilot[buf];
  a.pilot_stride = h->row;
  a.mpx = mpx;
  a.mpx_stride = mpx_stride;
  a.st_hist_rd = h->st_hist + static_cast<size_t>(h->st_idx) * h->C * FMX_HIST;
  a.lraw = h->lraw[buf];
  a.rraw = h->rraw[buf];
  a.lr_stride = h->row;
  a.lr_tiled = lr_tiled(h);
  a.st = h->st;
  a.dbg = h->dbg ? h->dbg + 16 : nullptr;
  a.n_cu = h->n_cu;
  return a;
}

static RdsArgs rds_args(Handle *h, int buf) {
  RdsArgs a{};
  a.des = h->ddes;
  a.C = h->C;
  a.in = h->rds_in[buf];
  a.in_stride = h->rds_stride;
  a.in_count = h->rds_count[buf];
  a.st = h->rds;
  a.ring = h->ring;
  a.block_index = h->block_index;
  a.dbg = h->dbg ? h->dbg + 8 : nullptr;
  a.sym = h->rds_sym[buf];
  a.sym_stride = h->sym_stride;
  a.sym_count = h->rds_sym_count[buf];
  a.sym_last_im = h->rds_sym_im[buf];
  a.in_prev = h->rds_last_buf >= 0 ? h->rds_in[h->rds_last_buf] : nullptr;
  a.ring_always = h->ring_always;
  return a;
}

static int check_n(Handle *h, int n) {
  if (n < 0 || n > h->cfg.block) {
    h->err = "n exceeds the handle's block size";
    return FMX_E_CAPACITY;
  }
  return FMX_OK;
}

// end of a step: advance the stereo-history rotation and the step counter
static void step_done(Handle *h, bool stereo_hist_written) {
  if (stereo_hist_written) h->st_idx = (h->st_idx + 1) % FMX_ST_BUFS;
  h->step++;
}

#if FMX_DIAG
#define FMX_SKIP(k) (h->skip_##k)
#else
#define FMX_SKIP(k) false
#endif

// One reference block for every channel (main.cpp:1239-1308), on four
// streams: sA front end, sC RDS, sB stereo PLL, sD audio.  Per step k (slot
// buf = k mod FMX_NBUF of the intermediates):
//   sA: [wait evD(k-3)] [RDS schedule copy] k_fe8 -> evF(k), k_pilot -> evP(k)
//   sC: [wait evF(k)] k_rs, k_rds -> evC(k)
//   sB: [wait evP(k)] k_pll -> evB(k)
//   sD: [wait evC(k)] k_bits, [wait evB(k)] [audio schedule copy] k_audio -> evD(k)
// evD(k) therefore marks every reader of slot buf done (k_audio waits for
// k_rds as well as k_pll), so the front end of step k+3 -- the next writer of
// the slot, and through evP of the raw L/R slot k_pll writes -- needs ONE
// cross-stream wait.  The resampler schedules go on the stream of their only
// reader, right before it.  Front end k+1 runs while k_pll / k_rs / k_rds /
// k_audio of step k (and k-1) still run.  (Measured and rejected in round 4:
// k_rs on sD ahead of k_audio, with k_audio no longer waiting for k_rds --
// 0.427 -> 0.437 ms per step at 2 048 channels, 0.744 -> 0.753 at 4 096,
// profiles/r04k_ab_rs_stream.txt.)
static int process_block(Handle *h, const uint8_t *d_iq, size_t iq_stride, int n, const fmx_block_out *o) {
  int rc;
  if ((rc = check_n(h, n)) != FMX_OK) return rc;
  if (!o || !o->d_pcm_l || !o->d_pcm_r || !o->d_pcm_count || !d_iq) {
    h->err = "process_block: d_iq, d_pcm_l, d_pcm_r and d_pcm_count are required";
    return FMX_E_INVALID;
  }
  if (n == 0) return FMX_OK;
  if ((rc = prepare_pipelined(h)) != FMX_OK) return rc;
  if (h->timing) harvest_timing(h);
  const bool stereo = h->cfg.stereo != 0;
  const bool rds = h->cfg.rds != 0;
  const int buf = static_cast<int>(h->step % FMX_NBUF);
  const int prev = (buf + FMX_NBUF - 1) % FMX_NBUF;
  // slot buf was last read by step k-FMX_NBUF; a caller-owned MPX buffer by
  // step k-1's readers
#if FMX_DIAG
  const bool wait_a = !h->nowait_a;
#else
  constexpr bool wait_a = true;
#endif
  // An event the host already sees complete needs no barrier packet on sA:
  // each costs the front end ~5 us at its launch even when its event
  // completed long before.  With the bench's timing on,
  // step k-3's audio has finished by the time step k is submitted.
  auto wait_pending = [](hipStream_t s, hipEvent_t e) {
    return hipEventQuery(e) == hipSuccess ? hipSuccess : hipStreamWaitEvent(s, e, 0);
  };
  if (!wait_a) {
  } else if (o->d_mpx && h->evD_set[prev]) HIP_TRY(wait_pending(h->sA, h->evD[prev]));
  else if (h->evD_set[buf]) HIP_TRY(wait_pending(h->sA, h->evD[buf]));
  // RDS resampler schedule of this step (read by k_rs, or by the front end):
  // the slot the previous front end filled when the speculation holds, else a
  // copy kernel on sA; then the next step's, copied by this front end into
  // slot k+1 of FMX_SSLOTS, last read by step k-3's k_rs (sC) -- before
  // evD(k-3), which the front end waits for: no second wait
  const int rslot = static_cast<int>(h->step % FMX_SSLOTS), nrslot = static_cast<int>((h->step + 1) % FMX_SSLOTS);
  if (rds && (rc = tset_take_or_advance(h, h->t_rds, n, rslot, h->sA)) != FMX_OK) return rc;
  const unsigned spec16 = rds ? tset_speculate(h, h->t_rds, n, nrslot, static_cast<size_t>(h->C) * 256) : 0u;
  float *mpx = o->d_mpx ? o->d_mpx : h->mpx[buf];
  const int mpx_stride = o->d_mpx ? o->mpx_stride : h->row;
  hipEvent_t evFE = h->evF[h->step % FMX_FRING];
  bool use_rs = false, pil_k = false;
  // ---- front end (sA) ----
  {
    FeArgs a = fe_args(h, n, h->M > 1 ? FE_IN_U8_DECIM : FE_IN_U8_DIRECT, buf);
    a.iq = d_iq;
    a.iq_stride = iq_stride;
    a.mpx_out = mpx;
    a.mpx_stride = mpx_stride;
    a.do_demod = 1;
    if (stereo) {
      a.pilot_out = h->pilot[buf];
      a.pilot_stride = h->row;
    }
    if (rds) {
      a.rds_out = h->rds_in[buf];
      a.rds_stride = h->rds_stride;
    }
    // the RDS resampler of a k_fe8 step runs as k_rs (MFMA tiles of 16
    // channels x 16 outputs on the handle's one RDS schedule)
    // (16 outputs' windows span <= 15 del + 31 samples: inside k_rs's 64 for del <= 2.1)
    // k_rs takes one resampler schedule for all channels: the RDS timing set
    // is never reset per channel (SubcarrierSet::reset, subcarrier.cpp:108)
    const bool fe8 = frontend_is_fe8(a, h->M, h->hdes->dec_tpp);
    use_rs = rds && h->hdes->rds_del <= 2.1f && h->t_rds.G == 1 && fe8;
    // the pilot BPF of a k_fe8 step runs as k_pilot (after it, on sA): k_fe8
    // writes the MPX and the stereo history rows k_pilot starts from
    // (FMX_FE_PILOT, A/B: inside k_fe8's RS = true instance, no k_pilot)
#ifndef FMX_FE_PILOT
#define FMX_FE_PILOT 0
#endif
    pil_k = stereo && fe8 && !FMX_FE_PILOT;
    if (pil_k) {
      a.pilot_out = nullptr;
      a.st_hist_out = 1;
    }
    if (use_rs) a.rds_win_out = h->rds_win[buf];
    a.clip_out = o->d_clip_ratio ? o->d_clip_ratio : h->clip;
    a.sig_sums = o->d_signal ? h->sig_sums[buf] : nullptr;
    if (spec16) {
      a.next_sched_src = h->t_rds.h_dev[h->t_rds.spec_img];
      a.next_sched_dst = h->t_rds.d_slot[nrslot];
      a.next_sched_n16 = spec16;
    }
    KBind t(h, fe8 ? FMX_K_FRONTEND : FMX_K_FRONTEND_GENERIC, h->sA, evFE);
    if ((rc = launch_frontend_m(a, h->M, h->hdes->dec_tpp, h->sA, dec_warm(h))) != FMX_OK) {
      h->err = "frontend launch failed";
      h->t_rds.spec = false; // the next step's schedule was not copied
      return rc;
    }
    t.launched();
    dec_advance(h, n);
  }
  if (spec16) { // the pinned image is reused FMX_HSLOTS simulations later: its read ends with the front end
    h->t_rds.ev_use[h->t_rds.spec_img] = evFE;
    h->t_rds.ev_h_set[h->t_rds.spec_img] = true;
  }
  // ---- pilot BPF (after the front end; read by k_pll): on sA, or with
  // FMX_PILOT_ON_B on sB ahead of k_pll ----
#ifndef FMX_PILOT_ON_B
#define FMX_PILOT_ON_B 0
#endif
  hipStream_t sPil = FMX_PILOT_ON_B ? h->sB : h->sP;
  if (pil_k && (FMX_PILOT_ON_B || sPil != h->sA)) HIP_TRY(hipStreamWaitEvent(sPil, evFE, 0));
  // FMX_PILOT_SPLIT_PCT (A/B): that share of the channels (rounded down to 8)
  // has its pilot BPF on sB, ahead of k_pll, the rest stays on sA
#ifndef FMX_PILOT_SPLIT_PCT
#define FMX_PILOT_SPLIT_PCT 0
#endif
  const int pil_cB = (pil_k && !FMX_PILOT_ON_B && sPil == h->sA && h->sB != h->sA)
                         ? ((h->C * FMX_PILOT_SPLIT_PCT / 100) & ~7) : 0;
  auto run_pilot = [&](int c0, int cn, hipStream_t s, hipEvent_t done) -> int {
    PilotArgs p{};
    p.des = h->ddes;
    p.des_pilot_len = h->hdes->pilot_len;
    p.C = cn;
    p.n = n;
    p.mpx = mpx + static_cast<size_t>(c0) * mpx_stride;
    p.mpx_stride = mpx_stride;
    p.st_hist_rd = h->st_hist + (static_cast<size_t>(h->st_idx) * h->C + c0) * FMX_HIST;
    p.out = h->pilot[buf] + static_cast<size_t>(c0) * h->row;
    p.out_stride = h->row;
    KBind t(h, FMX_K_PILOT, s, done);
    if (!FMX_SKIP(pll) && !FMX_SKIP(pilot)) {
      if (launch_pilot(p, s) != FMX_OK) {
        h->err = "pilot launch failed";
        return FMX_E_HIP;
      }
      t.launched();
    }
    return FMX_OK;
  };
  if (pil_k && (rc = run_pilot(0, h->C - pil_cB, sPil, h->evP[buf])) != FMX_OK) return rc;
  if (pil_cB > 0) {
    HIP_TRY(hipStreamWaitEvent(h->sB, evFE, 0));
    if ((rc = run_pilot(h->C - pil_cB, pil_cB, h->sB, nullptr)) != FMX_OK) return rc;
  }
  // ---- RDS (sC): the 240k -> 171k resampler (k_rs), then k_rds ----
  // (FMX_RS_ON_A_MAXC: up to that many channels k_rs runs on sA behind
  // k_pilot instead, so that the RDS stream holds only k_rds -- A/B)
#ifndef FMX_RS_ON_A_MAXC
#define FMX_RS_ON_A_MAXC 0
#endif
  const bool rs_on_a = rds && use_rs && h->C <= FMX_RS_ON_A_MAXC && h->sA != h->sC;
  auto run_rs = [&](hipStream_t s, hipEvent_t done) -> int {
    RsArgs r{};
    r.des = h->ddes;
    r.C = h->C;
    r.n = n;
    r.mpx = mpx;
    r.mpx_stride = mpx_stride;
    r.win = h->rds_win[buf];
    r.sched = h->t_rds.d_sched[h->t_rds.cur];
    r.sched_n = h->t_rds.d_count[h->t_rds.cur];
    r.group = h->t_rds.d_group[h->t_rds.cur];
    r.sched_stride = h->t_rds.stride;
    r.out = h->rds_in[buf];
    r.out_stride = h->rds_stride;
    // <= FMX_RS_TMAX output tiles per workgroup (8 parts of 23 tiles at a
    // 4096-sample block); from 256 channel groups (4096 channels) on, <= 46:
    // about half as many workgroups beside the other streams' (round 6, with
    // k_rs's schedule no longer staged in LDS): 4096 ch 0.5790 -> 0.5707 and
    // 0.5804 -> 0.5718 ms in two 4-rep A/Bs; at 2048 ch the longer parts were
    // slower, 0.3453 -> 0.3638 (profiles/r06k_ab_rs_parts_*.txt, r06m_*).
    // Fewer channels, finer parts: with few channel groups k_rs is latency --
    // one wave per part walking its tiles -- so below 2048 channels parts of
    // <= 6 tiles (1024 ch 0.2809 -> 0.2444 ms, 256 ch 0.2465 -> 0.2033) and
    // <= 12 at 2048 (0.3410 -> 0.3379, 0.3445 -> 0.3420 in r06c)
    // (profiles/r06z4_*, r06z5_*)
    const int rs_groups = (h->C + 15) / 16;
    const int rs_tiles = (h->t_rds.stride + 15) / 16,
              rs_tmax = rs_groups >= 256 ? 46 : (rs_groups >= 128 ? FMX_RS_TMAX : 6);
    r.parts = std::max(1, (rs_tiles + rs_tmax - 1) / rs_tmax);
    KBind t(h, FMX_K_RS, s, done);
    if (!FMX_SKIP(rds) && !FMX_SKIP(krs)) {
      if (launch_rs(r, s) != FMX_OK) {
        h->err = "rds resampler launch failed";
        return FMX_E_HIP;
      }
      t.launched();
    }
    return FMX_OK;
  };
  if (rs_on_a && (rc = run_rs(h->sA, h->evR[buf])) != FMX_OK) return rc;
  // FMX_RS_AFTER_PILOT (A/B): the RDS stream starts behind k_pilot instead of
  // beside it (k_rs then shares the CUs with the next k_fe8 and k_pll, the
  // co-residency its 16.5 KB LDS was sized for, not with k_pilot)
#ifndef FMX_RS_AFTER_PILOT
#define FMX_RS_AFTER_PILOT 0
#endif
  HIP_TRY(hipStreamWaitEvent(h->sC, rs_on_a ? h->evR[buf] : ((FMX_RS_AFTER_PILOT && pil_k) ? h->evP[buf] : evFE), 0));
  if ((rc = launch_reset_parts(h, RSP_RDS, h->sC)) != FMX_OK) return rc;
  if (rds) {
    RdsArgs a = rds_args(h, buf);
    a.groups = o->d_groups;
    a.groups_stride = o->d_groups ? o->groups_stride : 0;
    a.group_count = o->d_group_count;
    // FMX_RDS_FUSED: k_rds produces the 171 kHz samples itself (k_rs's MFMA
    // tiles inside its rounds): no k_rs launch, no 171 kHz rows in HBM
    const bool fused = FMX_RDS_FUSED && use_rs && !rs_on_a;
    if (fused) {
      a.fused = 1;
      a.n = n;
      a.mpx = mpx;
      a.mpx_stride = mpx_stride;
      a.win = h->rds_win[buf];
      a.sched = h->t_rds.d_sched[h->t_rds.cur];
      a.sched_n = h->t_rds.d_count[h->t_rds.cur];
      a.group = h->t_rds.d_group[h->t_rds.cur];
      a.sched_stride = h->t_rds.stride;
    } else if (use_rs && !rs_on_a && (rc = run_rs(h->sC, nullptr)) != FMX_OK) {
      return rc;
    }
    KBind t(h, FMX_K_RDS, h->sC, h->evC[buf]);
    if (!FMX_SKIP(rds)) {
      if ((rc = launch_rds_sym(a, h->sC)) != FMX_OK) {
        h->err = "rds launch failed";
        return rc;
      }
      t.launched();
      if (!a.fused) h->rds_last_buf = buf;
    }
  } else {
    if (o->d_group_count) HIP_TRY(hipMemsetAsync(o->d_group_count, 0, sizeof(int) * h->C, h->sC));
    HIP_TRY(hipEventRecord(h->evC[buf], h->sC));
  }
  h->evC_set[buf] = true;
  // ---- stereo PLL (sB) ----
  if (!(pil_k && FMX_PILOT_ON_B)) HIP_TRY(hipStreamWaitEvent(h->sB, pil_k ? h->evP[buf] : evFE, 0));
  if ((rc = launch_reset_parts(h, RSP_STEREO, h->sB)) != FMX_OK) return rc;
  if (stereo) {
    PllArgs a = pll_args(h, n, mpx, mpx_stride, buf);
    a.stereo_out = o->d_stereo;
    a.pilot_tenths_out = o->d_pilot_tenths;
    a.indicator_out = o->d_stereo_indicator;
    KBind t(h, FMX_K_STEREO, h->sB, h->evB[buf]);
    if (!FMX_SKIP(pll)) {
      if ((rc = launch_pll(a, h->sB)) != FMX_OK) {
        h->err = "pll launch failed";
        return rc;
      }
      t.launched();
    }
  } else {
    if (o->d_stereo) HIP_TRY(hipMemsetAsync(o->d_stereo, 0, sizeof(int) * h->C, h->sB));
    if (o->d_pilot_tenths) HIP_TRY(hipMemsetAsync(o->d_pilot_tenths, 0, sizeof(int) * h->C, h->sB));
    if (o->d_stereo_indicator) HIP_TRY(hipMemsetAsync(o->d_stereo_indicator, 0, sizeof(int) * h->C, h->sB));
    HIP_TRY(hipEventRecord(h->evB[buf], h->sB));
  }
  h->evB_set[buf] = true;
  // ---- audio (sD): after the PLL (stereo) / the front end (mono), and
  // after k_rds, so that evD closes the step ----
  // the RDS bit decoders (k_bits) over k_rds's symbols of slot buf, here
  // rather than behind k_rds on sC: the RDS stream's step is k_rs + k_rds
  // only, k_bits runs beside the next step's k_rs.  It waits for k_rds
  // alone, ahead of the PLL wait, so that it runs beside the tail of k_pll
  // and k_audio starts as soon as k_pll ends
  HIP_TRY(hipStreamWaitEvent(h->sD, h->evC[buf], 0));
  if ((rc = launch_reset_parts(h, RSP_BITS, h->sD)) != FMX_OK) return rc;
  if (rds && !FMX_SKIP(rds)) {
    RdsArgs a = rds_args(h, buf);
    a.groups = o->d_groups;
    a.groups_stride = o->d_groups ? o->groups_stride : 0;
    a.group_count = o->d_group_count;
    KBind t(h, FMX_K_BITS, h->sD, nullptr);
    if ((rc = launch_bits(a, h->sD)) != FMX_OK) {
      h->err = "rds bit decoder launch failed";
      return rc;
    }
    t.launched();
  }
  HIP_TRY(hipStreamWaitEvent(h->sD, h->evB[buf], 0));
  if ((rc = launch_reset_parts(h, RSP_AUDIO, h->sD)) != FMX_OK) return rc;
  h->rl_pending.clear();
  TimingSet *tau = stereo ? &h->t_af : &h->t_mono;
  if ((rc = tset_advance(h, *tau, n, buf, h->sD, nullptr)) != FMX_OK) return rc;
  {
    AudioArgs a = audio_args(h, n, stereo ? 0 : 3, tau);
    if (stereo) {
      a.in_l = h->lraw[buf];
      a.in_r = h->rraw[buf];
      a.in_stride = h->row;
#ifdef FMX_AB_NO_LR // A/B only: every channel reads the first pair's rows (L2-resident)
      a.in_stride = 0;
#endif
      a.in_tiled = lr_tiled(h);
      a.cap = h->cfg.block;
    } else {
      a.in_l = mpx;
      a.in_r = nullptr;
      a.in_stride = mpx_stride;
      a.cap = 1 << 30;
    }
    a.out_l = o->d_pcm_l;
    a.out_r = o->d_pcm_r;
    a.out_stride = o->pcm_stride;
    a.out_count = o->d_pcm_count;
    a.clamp = 1;
    a.mute = h->mute;
    a.mute_fade = h->cfg.out_rate / 200;
    audio_signal_level(h, a, o, buf, n);
    KBind t(h, FMX_K_AUDIO, h->sD, h->evD[buf]);
    if (!FMX_SKIP(audio)) {
      if ((rc = launch_audio(a, h->sD)) != FMX_OK) {
        h->err = "audio launch failed";
        return rc;
      }
      t.launched();
    }
  }
  h->evD_set[buf] = true;
  h->block_index++;
  step_done(h, stereo);
  return FMX_OK;
}

// Stage entry points run every kernel on sA after the pipelined streams
// have drained into it.
static int stage_begin(Handle *h, int n) {
  int rc;
  if ((rc = check_n(h, n)) != FMX_OK) return rc;
  if ((rc = prepare(h)) != FMX_OK) return rc;
  return join_into_A(h);
}
// later pipelined work on sB / sC / sD must see the stage's results
static int stage_end(Handle *h) {
  const int buf = static_cast<int>(h->step % FMX_NBUF);
  HIP_TRY(hipEventRecord(h->evA[buf], h->sA));
  HIP_TRY(hipStreamWaitEvent(h->sB, h->evA[buf], 0));
  HIP_TRY(hipStreamWaitEvent(h->sC, h->evA[buf], 0));
  HIP_TRY(hipStreamWaitEvent(h->sD, h->evA[buf], 0));
  return FMX_OK;
}

} // namespace fmx

using namespace fmx;


static Handle *H(void *p) { return static_cast<Handle *>(p); }

extern "C" {

int fmx_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int fmx_create(const fmx_config *cfg, int n_channels, int device, void **handle) {
  if (!cfg || !handle) return FMX_E_INVALID;
  Handle *h = nullptr;
  int rc = create(cfg, n_channels, device, &h);
  *handle = h;
  return rc;
}

int fmx_destroy(void *handle) {
  destroy(H(handle));
  return FMX_OK;
}

const char *fmx_last_error(void *handle) { return handle ? H(handle)->err.c_str() : "null handle"; }

int fmx_sync(void *handle) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  HIP_TRY(hipStreamSynchronize(h->sC));
  HIP_TRY(hipStreamSynchronize(h->sD));
  HIP_TRY(hipStreamSynchronize(h->sB));
  HIP_TRY(hipStreamSynchronize(h->sA));
  return FMX_OK;
}

int fmx_num_channels(void *handle) { return handle ? H(handle)->C : 0; }

int fmx_host_stats(void *handle, double *out, int n) {
  Handle *h = H(handle);
  if (!h || !out || n < 0) return FMX_E_INVALID;
  const double v[3] = {static_cast<double>(h->host_waits), static_cast<double>(h->host_stalls), h->host_stall_ms};
  for (int i = 0; i < n && i < 3; ++i) out[i] = v[i];
  h->host_waits = h->host_stalls = 0;
  h->host_stall_ms = 0.0;
  return FMX_OK;
}

int fmx_diag_set(void *handle, int what, int value) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  if (what != FMX_DIAG_RDS_RING_ALWAYS) {
    h->err = "unknown diagnostic setting";
    return FMX_E_INVALID;
  }
  h->ring_always = value != 0;
  return FMX_OK;
}

int fmx_diag_rds_ring(void *handle, int channel, float *out) {
  Handle *h = H(handle);
  if (!h || !out) return FMX_E_INVALID;
  if (channel < 0 || channel >= h->C) {
    h->err = "channel out of range";
    return FMX_E_INVALID;
  }
  // every stream's work done, the ring of every checkpointed channel
  // refilled (a valid state transition: the ring is what k_rds would have
  // written), then the channel's row oldest first
  int rc = join_into_A(h);
  if (rc != FMX_OK) return rc;
  if ((rc = launch_ring_fill(reset_args(h), h->sA)) != FMX_OK) return rc;
  HIP_TRY(hipStreamSynchronize(h->sA));
  std::vector<float> row(2 * FMX_RDS_RING);
  FmxRdsState st{};
  HIP_TRY(hipMemcpy(row.data(), h->ring + static_cast<size_t>(channel) * 2 * FMX_RDS_RING, sizeof(float) * row.size(),
                    hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&st, h->rds + channel, sizeof(st), hipMemcpyDeviceToHost));
  for (int k = 0; k < FMX_RDS_RING; ++k) {
    const uint32_t idx = (st.ring_pos - FMX_RDS_RING + static_cast<uint32_t>(k)) & (FMX_RDS_RING - 1);
    out[2 * k] = row[2 * idx];
    out[2 * k + 1] = row[2 * idx + 1];
  }
  return FMX_OK;
}

static int reset_channels(Handle *h, int channel, int extra) {
  if (channel < -1 || channel >= h->C) {
    h->err = "channel out of range";
    return FMX_E_INVALID;
  }
  const int c0 = (channel < 0) ? 0 : channel, c1 = (channel < 0) ? h->C : channel + 1;
  for (int c = c0; c < c1; ++c) {
    int m = RS_DECIM | RS_DEMOD | RS_STEREO | RS_AF | RS_RDS | extra;
    if (h->agc_ready[static_cast<size_t>(c)]) m |= RS_AGC;
    int &hm = h->hmask[static_cast<size_t>(c)];
    if (m & RS_MUTE) hm &= 0xFFFF; // the latest mute length wins
    hm |= m;
    tset_reset_channel(h->t_af, c);
    tset_reset_channel(h->t_mono, c);
  }
  return FMX_OK;
}

int fmx_reset(void *handle, int channel) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  return reset_channels(h, channel, 0);
}

int fmx_retune(void *handle, int channel, int mute_samples) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  // kRetuneMuteSamples = OUTPUT_RATE / 25 (main.cpp:696-697)
  const int len = (mute_samples < 0) ? h->cfg.out_rate / 25 : mute_samples;
  if (len > 65535) {
    h->err = "mute_samples must be <= 65535";
    return FMX_E_INVALID;
  }
  // a newer mute replaces any mute still running (main.cpp:1034-1035)
  return reset_channels(h, channel, RS_MUTE | static_cast<int>(static_cast<unsigned>(len) << 16));
}

int fmx_set_param(void *handle, int channel, int key, int value) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  if (channel < -1 || channel >= h->C) {
    h->err = "channel out of range";
    return FMX_E_INVALID;
  }
  const int c0 = (channel < 0) ? 0 : channel, c1 = (channel < 0) ? h->C : channel + 1;
  for (int c = c0; c < c1; ++c) {
    FmxChanParam &p = h->hpar[static_cast<size_t>(c)];
    switch (key) {
      case FMX_PARAM_BANDWIDTH_HZ: set_bandwidth(h, c, value); break;
      case FMX_PARAM_BANDWIDTH_MODE: set_bandwidth(h, c, tef_bandwidth_hz(value)); break;
      case FMX_PARAM_W0_HZ: h->w0[static_cast<size_t>(c)] = std::clamp(value, 0, 400000); break;
      case FMX_PARAM_DEEMPHASIS: set_deemph(h, c, std::clamp(value, 0, 2)); break;
      case FMX_PARAM_DEEMPH_US: set_deemph_us(h, c, value); break;
      case FMX_PARAM_DEVIATION_HZ:
        if (value <= 0) {
          h->err = "deviation must be > 0 Hz";
          return FMX_E_INVALID;
        }
        set_deviation(h, c, value);
        break;
      case FMX_PARAM_DSP_AGC: set_agc(h, c, std::clamp(value, 0, 2)); break;
      case FMX_PARAM_BLEND:
        p.blend = std::clamp(value, 0, 2);
        h->par_dirty = true;
        break;
      case FMX_PARAM_FORCE_MONO:
        p.force_mono = value != 0;
        h->par_dirty = true;
        break;
      case FMX_PARAM_FORCE_STEREO:
        p.force_stereo = value != 0;
        h->par_dirty = true;
        break;
      default: h->err = "unknown parameter key"; return FMX_E_INVALID;
    }
  }
  return FMX_OK;
}

/* diagnostic: frontend stage clocks (s_memtime ticks summed over
 * workgroups) when the handle was created with FMX_STAMPS=1 */
int fmx_debug_stamps(void *handle, unsigned long long *out, int n) {
  Handle *h = H(handle);
  if (!h || !h->dbg || n < 8) return FMX_E_INVALID;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out, h->dbg, (n >= 48 ? 48 : n >= 32 ? 32 : n >= 16 ? 16 : 8) * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return FMX_OK;
}

int fmx_set_signal_params(void *handle, int channel, int applied_gain_db, double gain_comp_factor, double bias_db,
                          double floor_dbfs, double ceil_dbfs) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  if (channel >= h->C) {
    h->err = "channel out of range";
    return FMX_E_INVALID;
  }
  const int c0 = (channel < 0) ? 0 : channel, c1 = (channel < 0) ? h->C : channel + 1;
  for (int c = c0; c < c1; ++c) {
    // computeSignalLevel: compensated = (dbfs - gain * factor) + bias
    h->hsig[4 * c] = static_cast<double>(applied_gain_db) * gain_comp_factor;
    h->hsig[4 * c + 1] = bias_db;
    h->hsig[4 * c + 2] = floor_dbfs;
    h->hsig[4 * c + 3] = ceil_dbfs;
  }
  h->sig_dirty = true;
  return FMX_OK;
}

int fmx_process_block(void *handle, const uint8_t *d_iq, size_t iq_stride, int n, const fmx_block_out *out) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  return process_block(h, d_iq, iq_stride, n, out);
}

int fmx_decimate(void *handle, const uint8_t *d_iq, size_t iq_stride, int n_out, float *d_out, int out_stride) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  int rc;
  if ((rc = stage_begin(h, n_out)) != FMX_OK) return rc;
  if (n_out == 0) return FMX_OK;
  if (h->M == 1) {
    h->err = "fmx_decimate needs iq_rate > dsp_rate";
    return FMX_E_INVALID;
  }
  FeArgs a = fe_args(h, n_out, FE_IN_U8_DECIM, 0);
  a.iq = d_iq;
  a.iq_stride = iq_stride;
  a.bb_out = d_out;
  a.bb_stride = out_stride;
  a.do_demod = 0;
  a.clip_out = nullptr;
  {
    KTimer t(h, FMX_K_FRONTEND, h->sA);
    if ((rc = launch_frontend_m(a, h->M, h->hdes->dec_tpp, h->sA, dec_warm(h))) != FMX_OK) return rc;
    dec_advance(h, n_out);
  }
  return stage_end(h);
}

int fmx_decimate_u8(void *handle, const uint8_t *d_iq, size_t iq_stride, int n_out, uint8_t *d_out,
                    size_t out_stride) {
  Handle *h = H(handle);
  if (!h || !d_out) return FMX_E_INVALID;
  int rc;
  if ((rc = check_n(h, n_out)) != FMX_OK) return rc;
  if (!h->dec_scratch && (rc = dalloc(h, &h->dec_scratch, static_cast<size_t>(h->C) * 2 * h->cfg.block)) != FMX_OK)
    return rc;
  if ((rc = fmx_decimate(handle, d_iq, iq_stride, n_out, h->dec_scratch, 2 * h->cfg.block)) != FMX_OK) return rc;
  if ((rc = launch_iq_to_u8(h->dec_scratch, 2 * h->cfg.block, h->C, n_out, d_out, out_stride, h->sA)) != FMX_OK)
    return rc;
  return stage_end(h);
}

static int demod_common(Handle *h, int mode, const void *d_in, size_t in_stride, int n, float *d_mpx,
                        int mpx_stride, float *d_mono, int mono_stride, int *d_mono_count, float *d_clip) {
  int rc;
  if ((rc = stage_begin(h, n)) != FMX_OK) return rc;
  if (n == 0) return FMX_OK;
  const int buf = static_cast<int>(h->step % FMX_NBUF);
  float *mpx = d_mpx ? d_mpx : h->mpx[buf];
  const int ms = d_mpx ? mpx_stride : h->row;
  {
    FeArgs a = fe_args(h, n, mode, buf);
    if (mode == FE_IN_CF) {
      a.in_f = static_cast<const float *>(d_in);
      a.in_stride = static_cast<int>(in_stride);
    } else {
      a.iq = static_cast<const uint8_t *>(d_in);
      a.iq_stride = in_stride;
    }
    a.mpx_out = mpx;
    a.mpx_stride = ms;
    a.do_demod = 1;
    if (d_clip) a.clip_out = d_clip;
    KTimer t(h, FMX_K_FRONTEND, h->sA);
    if ((rc = launch_frontend_m(a, 1, 1, h->sA)) != FMX_OK) return rc;
  }
  if (d_mono) {
    if ((rc = tset_advance(h, h->t_mono, n, buf, h->sA, nullptr)) != FMX_OK) return rc;
    AudioArgs a = audio_args(h, n, 2, &h->t_mono);
    a.in_l = mpx;
    a.in_stride = ms;
    a.out_l = d_mono;
    a.out_r = d_mono;
    a.out_stride = mono_stride;
    a.out_count = d_mono_count;
    a.cap = 1 << 30;
    a.clamp = 0;
    KTimer t(h, FMX_K_AUDIO, h->sA);
    if ((rc = launch_audio(a, h->sA)) != FMX_OK) return rc;
  } else if (d_mono_count) {
    HIP_TRY(hipMemsetAsync(d_mono_count, 0, sizeof(int) * h->C, h->sA));
  }
  return stage_end(h);
}

int fmx_demod(void *handle, const float *d_iq_cf, int in_stride, int n, float *d_mpx, int mpx_stride, float *d_mono,
              int mono_stride, int *d_mono_count) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  return demod_common(h, FE_IN_CF, d_iq_cf, static_cast<size_t>(in_stride), n, d_mpx, mpx_stride, d_mono,
                      mono_stride, d_mono_count, nullptr);
}

int fmx_demod_u8(void *handle, const uint8_t *d_iq, size_t iq_stride, int n, float *d_mpx, int mpx_stride,
                 float *d_mono, int mono_stride, int *d_mono_count, float *d_clip_ratio) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  return demod_common(h, FE_IN_U8_DIRECT, d_iq, iq_stride, n, d_mpx, mpx_stride, d_mono, mono_stride,
                      d_mono_count, d_clip_ratio);
}

int fmx_downsample(void *handle, const float *d_mpx, int mpx_stride, int n, float *d_out, int out_stride,
                   int *d_count) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  int rc;
  if ((rc = stage_begin(h, n)) != FMX_OK) return rc;
  if (n == 0) return FMX_OK;
  const int buf = static_cast<int>(h->step % FMX_NBUF);
  if ((rc = tset_advance(h, h->t_mono, n, buf, h->sA, nullptr)) != FMX_OK) return rc;
  AudioArgs a = audio_args(h, n, 2, &h->t_mono);
  a.in_l = d_mpx;
  a.in_stride = mpx_stride;
  a.out_l = d_out;
  a.out_r = d_out;
  a.out_stride = out_stride;
  a.out_count = d_count;
  a.cap = 1 << 30;
  a.clamp = 0;
  {
    KTimer t(h, FMX_K_AUDIO, h->sA);
    if ((rc = launch_audio(a, h->sA)) != FMX_OK) return rc;
  }
  return stage_end(h);
}

int fmx_stereo(void *handle, const float *d_mpx, int mpx_stride, int n, float *d_left, float *d_right, int lr_stride,
               int *d_stereo, int *d_pilot_tenths) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  int rc;
  if ((rc = stage_begin(h, n)) != FMX_OK) return rc;
  if (n == 0) return FMX_OK;
  const int buf = static_cast<int>(h->step % FMX_NBUF);
  {
    FeArgs a = fe_args(h, n, FE_IN_MPX, buf);
    a.in_f = d_mpx;
    a.in_stride = mpx_stride;
    a.pilot_out = h->pilot[buf];
    a.pilot_stride = h->row;
    a.do_demod = 0;
    a.clip_out = nullptr;
    KTimer t(h, FMX_K_FRONTEND, h->sA);
    if ((rc = launch_frontend_m(a, 1, 1, h->sA)) != FMX_OK) return rc;
  }
  {
    PllArgs a = pll_args(h, n, d_mpx, mpx_stride, buf);
    a.stereo_out = d_stereo;
    a.pilot_tenths_out = d_pilot_tenths;
    KTimer t(h, FMX_K_STEREO, h->sA);
    if ((rc = launch_pll(a, h->sA)) != FMX_OK) return rc;
  }
  {
    AudioArgs a = audio_args(h, n, 4, nullptr);
    a.in_l = h->lraw[buf];
    a.in_r = h->rraw[buf];
    a.in_stride = h->row;
    a.in_tiled = lr_tiled(h);
    a.lr_out_l = d_left;
    a.lr_out_r = d_right;
    a.lr_out_stride = lr_stride;
    KTimer t(h, FMX_K_AUDIO, h->sA);
    if ((rc = launch_audio(a, h->sA)) != FMX_OK) return rc;
  }
  rc = stage_end(h);
  step_done(h, true);
  return rc;
}

int fmx_afpost(void *handle, const float *d_left, const float *d_right, int in_stride, int n, float *d_out_l,
               float *d_out_r, int out_stride, int cap, int *d_count) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  int rc;
  if ((rc = stage_begin(h, n)) != FMX_OK) return rc;
  if (n == 0 || cap <= 0) return FMX_OK;
  // AFPostProcessor::process stops consuming input once outCapacity outputs
  // are written; only the no-truncation case is supported here.
  std::vector<ResampTiming> saved = h->t_af.groups;
  std::vector<int> saved_map = h->t_af.chan_group;
  int mx = 0;
  const int buf = static_cast<int>(h->step % FMX_NBUF);
  if ((rc = tset_advance(h, h->t_af, n, buf, h->sA, &mx)) != FMX_OK) return rc;
  if (mx > cap) {
    h->t_af.groups = saved;
    h->t_af.chan_group = saved_map;
    h->err = "fmx_afpost: outCapacity smaller than the produced sample count is not supported";
    return FMX_E_CAPACITY;
  }
  AudioArgs a = audio_args(h, n, 1, &h->t_af);
  a.in_l = d_left;
  a.in_r = d_right;
  a.in_stride = in_stride;
  a.out_l = d_out_l;
  a.out_r = d_out_r;
  a.out_stride = out_stride;
  a.out_count = d_count;
  a.cap = cap;
  a.clamp = 0;
  {
    KTimer t(h, FMX_K_AUDIO, h->sA);
    if ((rc = launch_audio(a, h->sA)) != FMX_OK) return rc;
  }
  return stage_end(h);
}

int fmx_rds(void *handle, const float *d_mpx, int mpx_stride, int n, fmx_rds_group *d_groups, int groups_stride,
            int *d_group_count) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  int rc;
  if ((rc = stage_begin(h, n)) != FMX_OK) return rc;
  if (n == 0) {
    if (d_group_count) HIP_TRY(hipMemsetAsync(d_group_count, 0, sizeof(int) * h->C, h->sA));
    return FMX_OK;
  }
  const int buf = static_cast<int>(h->step % FMX_NBUF);
  if ((rc = tset_advance(h, h->t_rds, n, static_cast<int>(h->step % FMX_SSLOTS), h->sA, nullptr)) != FMX_OK) return rc;
  {
    FeArgs a = fe_args(h, n, FE_IN_MPX, buf);
    a.in_f = d_mpx;
    a.in_stride = mpx_stride;
    a.rds_out = h->rds_in[buf];
    a.rds_stride = h->rds_stride;
    a.do_demod = 0;
    a.clip_out = nullptr;
    KTimer t(h, FMX_K_FRONTEND, h->sA);
    if ((rc = launch_frontend_m(a, 1, 1, h->sA)) != FMX_OK) return rc;
  }
  RdsArgs a = rds_args(h, buf);
  a.groups = d_groups;
  a.groups_stride = d_groups ? groups_stride : 0;
  a.group_count = d_group_count;
  {
    KTimer t(h, FMX_K_RDS, h->sA);
    if ((rc = launch_rds(a, h->sA)) != FMX_OK) return rc;
    h->rds_last_buf = buf;
  }
  h->block_index++;
  return stage_end(h);
}

int fmx_malloc(void *handle, void **d_ptr, size_t bytes) {
  Handle *h = H(handle);
  if (!h || !d_ptr) return FMX_E_INVALID;
  HIP_TRY(hipSetDevice(h->device));
  hipError_t e = hipMalloc(d_ptr, bytes ? bytes : 16);
  if (e != hipSuccess) {
    h->err = hipGetErrorString(e);
    return FMX_E_NOMEM;
  }
  return FMX_OK;
}
int fmx_free(void *handle, void *d_ptr) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  HIP_TRY(hipFree(d_ptr));
  return FMX_OK;
}
int fmx_memcpy_h2d(void *handle, void *d_dst, const void *h_src, size_t bytes) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(d_dst, h_src, bytes, hipMemcpyHostToDevice));
  return FMX_OK;
}
int fmx_memcpy_d2h(void *handle, void *h_dst, const void *d_src, size_t bytes) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(h_dst, d_src, bytes, hipMemcpyDeviceToHost));
  return FMX_OK;
}
int fmx_memset(void *handle, void *d_ptr, int value, size_t bytes) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  HIP_TRY(hipMemsetAsync(d_ptr, value, bytes, h->sA));
  HIP_TRY(hipStreamSynchronize(h->sA));
  return FMX_OK;
}

int fmx_timing_enable(void *handle, int enable) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  if (h->timing && !enable) {
    (void)hipDeviceSynchronize();
    collect_timing(h);
  }
  h->timing = enable != 0;
  h->timing_every = enable > 1 ? enable : 1;
  // events for the timed region up front (creating them on the way stalls the host)
  while (h->timing && h->pool.size() < 256) {
    hipEvent_t e;
    HIP_TRY(hipEventCreateWithFlags(&e, ev_flags(true)));
    h->pool.push_back(e);
  }
  for (int k = 0; k < FMX_K_COUNT; ++k) {
    h->kms[k] = 0.0;
    h->klaunch[k] = 0;
  }
  return FMX_OK;
}

int fmx_kernel_times(void *handle, double *ms, int *launches, int n) {
  Handle *h = H(handle);
  if (!h) return FMX_E_INVALID;
  (void)hipDeviceSynchronize();
  collect_timing(h);
  for (int k = 0; k < n && k < FMX_K_COUNT; ++k) {
    if (ms) ms[k] = h->kms[k];
    if (launches) launches[k] = h->klaunch[k];
  }
  return FMX_OK;
}

/* ---------------- synthetic input ---------------- */
static uint16_t rds_crc10(uint16_t data) {
  uint32_t reg = 0;
  for (int i = 15; i >= 0; --i) {
    const uint32_t bit = ((data >> i) & 1u) ^ ((reg >> 9) & 1u);
    reg = (reg << 1) & 0x3FFu;
    if (bit) reg ^= 0x1B9u; // g(x) = x^10+x^8+x^7+x^5+x^4+x^3+1
  }
  return static_cast<uint16_t>(reg);
}

// Known RDS test groups: PI = 0x1000 + ch, 0A PS groups
// alternating with 2A RadioText groups.
static void rds_group_words(uint32_t ch, int g, uint16_t w[4]) {
  const uint16_t pi = static_cast<uint16_t>(0x1000u + ch);
  const uint16_t pty = static_cast<uint16_t>(ch % 32u);
  char ps[9];
  std::snprintf(ps, sizeof(ps), "FM%05u ", static_cast<unsigned>(ch % 100000u));
  char rt[96];
  std::snprintf(rt, sizeof(rt), "MI355X channel %05u radiotext test pattern 0123456789 abcdefghij",
                static_cast<unsigned>(ch % 100000u));
  w[0] = pi;
  if ((g & 1) == 0) { // 0A
    const int seg = (g / 2) % 4;
    w[1] = static_cast<uint16_t>((0u << 12) | (0u << 11) | (pty << 5) | (1u << 3) | static_cast<unsigned>(seg));
    w[2] = 0xE0CD;
    w[3] = static_cast<uint16_t>((static_cast<uint8_t>(ps[2 * seg]) << 8) | static_cast<uint8_t>(ps[2 * seg + 1]));
  } else { // 2A
    const int seg = (g / 2) % 16;
    w[1] = static_cast<uint16_t>((2u << 12) | (0u << 11) | (pty << 5) | static_cast<unsigned>(seg));
    w[2] = static_cast<uint16_t>((static_cast<uint8_t>(rt[4 * seg]) << 8) | static_cast<uint8_t>(rt[4 * seg + 1]));
    w[3] = static_cast<uint16_t>((static_cast<uint8_t>(rt[4 * seg + 2]) << 8) |
                                 static_cast<uint8_t>(rt[4 * seg + 3]));
  }
}

int fmx_synth_rds_bits(const fmx_synth_config *cfg, uint32_t ch0, int n_ch, uint8_t *h_bits, uint16_t *h_groups) {
  if (!cfg || n_ch < 0 || cfg->n_bits <= 0) return FMX_E_INVALID;
  static const uint16_t kOffset[4] = {0x0FC, 0x198, 0x168, 0x1B4}; // A, B, C, D
  const int nb = cfg->n_bits;
  const int ng = nb / 104 + 1;
  for (int ci = 0; ci < n_ch; ++ci) {
    const uint32_t ch = ch0 + static_cast<uint32_t>(ci);
    uint8_t prev = 0;
    for (int g = 0; g < ng; ++g) {
      uint16_t w[4];
      rds_group_words(ch, g, w);
      if (h_groups && g < nb / 104)
        for (int k = 0; k < 4; ++k) h_groups[(static_cast<size_t>(ci) * (nb / 104) + g) * 4 + k] = w[k];
      for (int blk = 0; blk < 4; ++blk) {
        const uint32_t word = (static_cast<uint32_t>(w[blk]) << 10) | (rds_crc10(w[blk]) ^ kOffset[blk]);
        for (int b = 25; b >= 0; --b) {
          const int idx = g * 104 + blk * 26 + (25 - b);
          if (idx >= nb) break;
          const uint8_t d = static_cast<uint8_t>((word >> b) & 1u);
          prev = static_cast<uint8_t>(d ^ prev); // differential encoding
          if (h_bits) h_bits[static_cast<size_t>(ci) * nb + idx] = prev;
        }
      }
    }
  }
  return FMX_OK;
}

int fmx_synth_host(const fmx_synth_config *cfg, uint32_t ch0, int n_ch, int64_t sample0, int n_samples,
                   const uint8_t *h_bits, uint8_t *h_out, size_t out_stride, int threads) {
  if (!cfg || !h_out || n_ch < 0 || n_samples < 0) return FMX_E_INVALID;
  if (threads < 1) threads = 1;
  auto work = [&](int t) {
    for (int ci = t; ci < n_ch; ci += threads) {
      const uint32_t ch = ch0 + static_cast<uint32_t>(ci);
      const fmx_synth_chan cp = fmx_synth_channel(cfg, ch);
      const uint8_t *b = h_bits ? h_bits + static_cast<size_t>(ci) * cfg->n_bits : nullptr;
      uint8_t *o = h_out + static_cast<size_t>(ci) * out_stride;
      for (int i = 0; i < n_samples; ++i) fmx_synth_sample(cfg, ch, &cp, sample0 + i, b, o + 2 * static_cast<size_t>(i));
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < threads; ++t) th.emplace_back(work, t);
  work(0);
  for (auto &x : th) x.join();
  return FMX_OK;
}

int fmx_synth_device(void *handle, const fmx_synth_config *cfg, uint32_t ch0, int n_ch, int64_t sample0,
                     int n_samples, const uint8_t *d_bits, uint8_t *d_out, size_t out_stride) {
  Handle *h = H(handle);
  if (!h || !cfg) return FMX_E_INVALID;
  return launch_synth(*cfg, ch0, n_ch, sample0, n_samples, d_bits, d_out, out_stride, h->sA);
}

/* ---------------- diagnostics (no GPU needed) ---------------- */
static double f16_value(uint16_t h) {
  const int e = (h >> 10) & 31;
  const double m = static_cast<double>(h & 0x3FF);
  const double v = (e == 0) ? std::ldexp(m, -24) : std::ldexp(m + 1024.0, e - 25);
  return (h & 0x8000u) ? -v : v;
}
int fmx_design_taps(const fmx_config *cfg, int which, float *out, int cap) {
  if (!cfg) return FMX_E_INVALID;
  FmxDesign *d = new FmxDesign();
  DesignExtras ex;
  std::string err;
  int rc = design_build(*cfg, d, &ex, &err);
  if (rc != FMX_OK) {
    delete d;
    return rc;
  }
  std::vector<float> v;
  switch (which) {
    case 0: v.assign(d->dec_taps_raw, d->dec_taps_raw + d->dec_len); break;
    case 1: {
      const int sel = bandwidth_select(cfg->bandwidth_hz, std::clamp(cfg->w0_bandwidth_hz, 0, 400000));
      const int idx = (sel == 0) ? FMX_IQ_CTOR : sel;
      v.assign(d->iq_taps[idx], d->iq_taps[idx] + d->iq_len[idx]);
      break;
    }
    case 2: v.assign(d->pilot_taps, d->pilot_taps + d->pilot_len); break;
    case 3: v.assign(d->lr_taps, d->lr_taps + FMX_LR_LEN); break;
    case 4: v = ex.proto_af; break;
    case 5: v = ex.proto_rds; break;
    case 6: v.assign(d->rds_fir, d->rds_fir + FMX_RDS_FIR); break;
    case 7: v = ex.rrc; break;
    case 8: v = ex.rrc_d; break;
    case 10: { // k_fe8 MFMA pilot BPF taps back from the f16 hi/lo fragments (row 0 lanes), as pilot_taps
      const int P = d->pilot_len, P8 = ((P + 6) & ~7) + 1;
      for (int k = 0; k < P; ++k) {
        const int dd = P8 - 1 - k; // = 32 ks + 8 g + j with row 0
        const int ks = dd / 32, gg = (dd % 32) / 8, j = dd % 8, l = 16 * gg;
        const double q = f16_value(d->pilot_frag[ks][0][l][j]) + f16_value(d->pilot_frag[ks][1][l][j]);
        v.push_back(static_cast<float>(q / 4096.0));
      }
      break;
    }
    case 12: // k_audio MFMA L/R FIR taps back from the f16 hi/lo fragments (row 0 lanes), as case 3
      for (int k = 0; k < FMX_LR_LEN; ++k) {
        const int dd = FMX_LR_LEN - 1 - k; // = 32 ks + 8 g + j with row 0
        const int ks = dd / 32, gg = (dd % 32) / 8, j = dd % 8, l = 16 * gg;
        const double q = f16_value(d->lr_frag[ks][0][l][j]) + f16_value(d->lr_frag[ks][1][l][j]);
        v.push_back(static_cast<float>(q / 4096.0));
      }
      break;
    case 11: { // k_fe8 MFMA IQ FIR taps back from the f16 hi/lo fragments (row 0 lanes), as case 1
      const int sel = bandwidth_select(cfg->bandwidth_hz, std::clamp(cfg->w0_bandwidth_hz, 0, 400000));
      const int idx = (sel == 0) ? FMX_IQ_CTOR : sel;
      const int P = d->iq_len[idx], P8 = ((P + 6) & ~7) + 1;
      for (int k = 0; k < P; ++k) {
        const int dd = P8 - 1 - k;
        const int ks = dd / 32, gg = (dd % 32) / 8, j = dd % 8, l = 16 * gg;
        const double q = f16_value(d->iq_frag[idx][ks][0][l][j]) + f16_value(d->iq_frag[idx][ks][1][l][j]);
        v.push_back(static_cast<float>(q / 4096.0));
      }
      break;
    }
    case 13: // k_fe8 MFMA decimator taps back from the f16 hi/lo A fragments (row 0 lanes), as dec_taps_raw
      for (int k = 0; k < d->dec_len; ++k) {
        const int dd = d->dec_len - k;
        const int ks = dd / 32, gg = (dd % 32) / 8, j = dd % 8, l = 16 * gg;
        const double q = f16_value(d->dec_frag[ks][0][l][j]) + f16_value(d->dec_frag[ks][1][l][j]);
        v.push_back(static_cast<float>(q / 65536.0 * 127.5));
      }
      break;
    case 9: { // the same fragments' rows 1..15 (lane l = 16 g + r): every row holds the taps shifted by M r
      const int M = d->M;
      for (int r = 0; r < 16; ++r)
        for (int k = 0; k < d->dec_len; ++k) {
          const int dd = d->dec_len - k + M * r;
          const int ks = dd / 32, gg = (dd % 32) / 8, j = dd % 8, l = 16 * gg + r;
          const double q = f16_value(d->dec_frag[ks][0][l][j]) + f16_value(d->dec_frag[ks][1][l][j]);
          v.push_back(static_cast<float>(q / 65536.0 * 127.5));
        }
      break;
    }
    case 14: { // k_fe8's flat LDS tap window (dec_q16) against the A fragments: 1 where the entry process_block's
               // decimator reads for (K step, lane, element, hi / lo) equals dec_frag's, for every K step it runs
      const int M = d->M, KS = (15 * M + d->dec_len + 1 + 31) / 32;
      for (int ks = 0; ks < KS; ++ks)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j)
            for (int sh = 0; sh < 2; ++sh) {
              const int i = 32 * ks + 8 * (l >> 4) + j + 15 * M - M * (l & 15);
              v.push_back(i >= 0 && i < FMX_DEC_QN && d->dec_q16[sh][i] == d->dec_frag[ks][sh][l][j] ? 1.0f : 0.0f);
            }
      break;
    }
    case 15: { // k_pilot's flat LDS tap window (pilot_q16) against pilot_frag, as case 14
      for (int ks = 0; ks < d->pilot_ks; ++ks)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j)
            for (int sh = 0; sh < 2; ++sh) {
              const int base = 32 * ks + 8 * (l >> 4) + 15 - (l & 15), c = base & 1, i = base - c + j;
              v.push_back(i >= 0 && i < FMX_PILOT_QN && d->pilot_q16[c][sh][i] == d->pilot_frag[ks][sh][l][j] ? 1.0f : 0.0f);
            }
      break;
    }
    case 16: { // k_fe8's flat LDS IQ FIR windows (iq_q16) against iq_frag, every design, as case 15
      for (int i = 0; i < FMX_IQ_DESIGNS; ++i)
        for (int ks = 0; ks < d->iq_ks[i]; ++ks)
          for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 8; ++j)
              for (int sh = 0; sh < 2; ++sh) {
                const int base = 32 * ks + 8 * (l >> 4) + 15 - (l & 15), c = base & 1, e = base - c + j;
                v.push_back(e >= 0 && e < FMX_IQ_QN && d->iq_q16[i][c][sh][e] == d->iq_frag[i][ks][sh][l][j] ? 1.0f : 0.0f);
              }
      break;
    }
    case 17: { // k_audio's flat LDS L/R FIR window (lr_q16) against lr_frag, as case 15
      for (int ks = 0; ks < FMX_LR_KS; ++ks)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j)
            for (int sh = 0; sh < 2; ++sh) {
              const int base = 32 * ks + 8 * (l >> 4) + 15 - (l & 15), c = base & 1, e = base - c + j;
              v.push_back(e >= 0 && e < FMX_LR_QN && d->lr_q16[c][sh][e] == d->lr_frag[ks][sh][l][j] ? 1.0f : 0.0f);
            }
      break;
    }
    default: delete d; return FMX_E_INVALID;
  }
  delete d;
  const int n = static_cast<int>(v.size());
  if (out) std::memcpy(out, v.data(), sizeof(float) * static_cast<size_t>(std::min(n, cap)));
  return n;
}

/* host simulation of the resampler schedule (tests) */
int fmx_resamp_schedule(float del, int n_in, int *packed, float *mu, int cap) {
  ResampTiming t;
  timing_reset(t);
  t.del = del;
  std::vector<FmxSched> s(static_cast<size_t>(std::max(cap, 1)));
  int k = timing_run(t, n_in, s.data(), cap);
  for (int i = 0; i < std::min(k, cap); ++i) {
    if (packed) packed[i] = s[static_cast<size_t>(i)].packed;
    if (mu) mu[i] = s[static_cast<size_t>(i)].mu;
  }
  return k;
}

} // extern "C"
