// lincheck_abi.hip — host side of liblincheck.so: device plans, batching, capacity growth,
// multi-GPU key sharding and the extern "C" entry points declared in include/lincheck.h.
//
// Replaces, at the drop-in boundary, the call the reference makes through
//   (checker/linearizable {:model m :algorithm :linear})   register.clj:109-111, counter.clj:135-137
// and, for many keys at once, jepsen.independent/checker's per-key loop (register.clj:106).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lincheck.h"
#include "bounds.hpp"
#include "ctab.hpp"
#include "dense.hpp"
#include "wide.hpp"
#include "encode.hpp"
#include "keys.hpp"
#include "pool.hpp"
#include "search.hpp"

namespace lc {
namespace {

void set_err(char* err, int32_t len, const char* fmt, ...) {
  if (!err || len <= 0) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(err, (size_t)len, fmt, ap);
  va_end(ap);
}

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) {                                                        \
      last_error = std::string(#expr) + ": " + hipGetErrorString(e_);              \
      return e_ == hipErrorOutOfMemory ? LC_E_MEMORY : LC_E_DEVICE;                \
    }                                                                              \
  } while (0)

// for extern "C" entry points without a plan: message into the caller's err buffer
#define HIP_CHECK_MSG(expr)                                                        \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) {                                                        \
      set_err(err, err_len, "%s: %s", #expr, hipGetErrorString(e_));               \
      return e_ == hipErrorOutOfMemory ? LC_E_MEMORY : LC_E_DEVICE;                \
    }                                                                              \
  } while (0)

std::mutex& device_mutex(int dev) {
  static std::mutex mus[64];
  return mus[dev & 63];
}

bool debug() {
  static int d = -1;
  if (d < 0) {
    const char* e = getenv("LC_DEBUG");
    d = (e && *e && *e != '0') ? 1 : 0;
  }
  return d == 1;
}

int bits_for(int64_t n) {  // bits to represent values 0..n-1
  int b = 0;
  while ((1ll << b) < n) ++b;
  return b;
}

struct DevArray {
  void* p = nullptr;
  size_t bytes = 0;
  ~DevArray() { release(); }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  hipError_t ensure(size_t n) {
    if (n <= bytes && p) return hipSuccess;
    release();
    if (n == 0) n = 8;
    hipError_t e = hipMalloc(&p, n);
    if (e == hipSuccess) bytes = n;
    else p = nullptr;
    return e;
  }
  template <typename T>
  T* as() const { return (T*)p; }
};

// One launch that zeroes a run's small control buffers (instead of a memset each: every
// hipMemsetAsync is a fill kernel and a host API call of its own, ~8 per dense run)
struct ZeroSpans {
  uint32_t* p[8];
  uint32_t n[8];  // 4-byte words
  int k = 0;
  void add(void* ptr, size_t bytes) {
    p[k] = (uint32_t*)ptr;
    n[k] = (uint32_t)((bytes + 3) / 4);
    ++k;
  }
};
__global__ void __launch_bounds__(256) zero_spans_kernel(ZeroSpans z) {
  const uint32_t stride = gridDim.x * 256u;
  for (int s = 0; s < z.k; ++s)
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < z.n[s]; i += stride) z.p[s][i] = 0u;
}
hipError_t zero_spans(const ZeroSpans& z, hipStream_t s) {
  if (z.k == 0) return hipSuccess;
  hipLaunchKernelGGL(zero_spans_kernel, dim3(32), dim3(256), 0, s, z);
  return hipGetLastError();
}

}  // namespace
}  // namespace lc

using namespace lc;

struct lc_plan {
  int device = 0;
  int model = 0;
  int64_t max_configs = 0;
  Encoded enc;
  std::string last_error;
  // batches of histories (global ids) sharing one packed key layout (grid kernel)
  struct Batch {
    std::vector<int> hs;
    int mask_bits, state_bits, hist_bits;
  };
  std::vector<Batch> batches;
  int path = 0;  // 0 auto (dense tables, then grid), 1 keys kernel first, 2 grid kernel only
  int nwg = 0, cell_cap = 256, f_cap = 65536, spill_log = 17;
  int64_t ovf_cap = 1 << 18;
  int knwg = 0;
  int64_t kfcap = 1 << 18, klcap = 1 << 18;
  int kspill_log = 18;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // device copies of the encoded history
  DevArray d_step_off, d_step_slot, d_inv_off, d_inv_slot, d_inv_kind, d_inv_a, d_inv_b, d_init;
  DevArray d_beg, d_end, d_kshift, d_kbits, d_order, d_queue;  // keys kernel (all histories)
  DevArray d_bbeg, d_bend, d_binit;                           // grid batch gathers
  // per-history work state
  DevArray d_live, d_opk, d_opa, d_opb, d_status, d_fail, d_nonempty, d_explored;
  // grid-kernel per-owner storage
  DevArray d_flist, d_fcount, d_cells, d_cellcnt, d_ovf, d_ovfcnt, d_spill, d_spillpos;
  DevArray d_bar, d_produced, d_running, d_flags, d_stats, d_stamps;
  // keys-kernel per-workgroup storage
  DevArray d_kscratch, d_kspill, d_kspillpos, d_kstatus, d_kfail, d_kexplored;
  // dense closure tables (narrow cas-register histories; dense.hpp)
  std::vector<int> dense_b, dense_w, dense_x, dense_m;  // block / wave / wide / mid teams, heaviest first
  // counter histories on closure tables (ctab.hip), heaviest first
  std::vector<int> dense_c;
  int dgrid_c = 0;
  // LC_CTAB_MAXW (0: counters take the grid kernel, tests): widest counter on the closure tables;
  // past CTAB_LMAX (one workgroup's LDS) only as a tile team, to CTAB_TEAM_LMAX
  int ctab_maxw = CTAB_TEAM_LMAX;
  int ctab_pipe = 3;          // LC_CTAB_PIPE: bit 0 double-buffered tables, bit 1 chunks from an LDS counter
  // counter tile teams (ctab_team_kernel): LC_CTAB_TEAM=0 keeps every counter on one
  // workgroup; histories of live width >= LC_CTAB_TEAM_MINW get 2^T tiles, T = LC_CTAB_TEAM_T or,
  // by default, width - 15 (tiles of 15 local slots: 2^9 words, double-buffered). r5e/r5f sweeps
  // (one MI355X): c2c4 (width 20) 117 ms on one workgroup, 123 / 82 / 61 / 48 / 46 / 47 ms at
  // T = 1..6; c5x 38.9 s -> 19.7 / 13.5 / 10.1 / 9.7 / 10.0 s at T = 2..6; c2c (width 16) 31.8 ms
  // alone, 37-41 ms as a team (its super-layers are one pass of ~430 words: latency, not issue)
  int ctab_team = 1, ctab_team_minw = 17, ctab_team_t = 0;
  std::vector<int8_t> ctab_T;  // per history: team slots (0: one workgroup)
  std::vector<char> ctab_grid;  // per history: a counter the tables could not run (run_ctab)
  DevArray d_cstats;
  DevArray d_dpack, d_dwords, d_dqueue, d_dstatus, d_dfail, d_dexpl;
  DevArray d_dres;  // run_dense's results in one block: explored | status | fail | stats | abort | stamps
  // histories wider than the LDS tile teams hold: tables in HBM (wide.hip)
  std::vector<int> dense_wd;
  std::vector<char> wide_ok;
  std::vector<std::vector<uint32_t>> wide_streams;  // per history (built by dense_sink)
  DevArray d_wtab, d_wstream, d_wmeta, d_wres, d_wbar;
  DevArray d_ctmeta, d_ctmirror, d_ctctl, d_ctord;  // counter tile teams
  int wide_maxw = WIDE_LMAX, wide_minw = 0;  // LC_WIDE_MAXW (0: off) / LC_WIDE_MINW (tests)
  int wide_grid = 0;  // LC_WIDE_GRID: at most this many workgroups for the HBM tables (0: all resident)
  int wide_watchdog_ms = 20000;  // LC_WIDE_WATCHDOG_MS: a grid barrier's longest wait
  bool wide_force_abort = false;  // LC_WIDE_FORCE_ABORT=1 (tests): the abort word set before launch
  int wide_stall_hist = -1, wide_stall_wg = -1;  // LC_WIDE_STALL=h:wg (tests): a real barrier stall
  bool wide_pipe = true;  // LC_WIDE_PIPE=0: one step at a time (a grid barrier per popcount layer)
  int wide_split = 0;     // LC_WIDE_SPLIT: at least this many split bits (2^split slabs; tests)
  // counters on the HBM tables (wctr_pipe_kernel, §3.13): widths past the tile teams up to
  // LC_WCTR_MAXW (0: off, they take the grid kernel); LC_WCTR_MINW routes narrower ones (tests)
  int wctr_maxw = WCTR_LMAX, wctr_minw = 0;
  // the dense kernels' inputs inside d_dpack (one upload): step streams, per-history stream
  // begin / step count / table width, and the queue order
  uint32_t* dp_stream = nullptr;
  int64_t* dp_sbeg = nullptr;
  int32_t *dp_nst = nullptr, *dp_ord = nullptr;
  int8_t* dp_lm = nullptr;
  char* hpack = nullptr;  // pinned staging of d_dpack (kept across calls)
  size_t hpack_bytes = 0;
  // per history: how many of its steps have live width L (L = 0..32), for the team planner's
  // step-time models (a sum over 33 widths instead of over every step)
  struct WidthHist {
    uint32_t c[33];
    uint32_t steps() const {
      uint32_t s = 0;
      for (uint32_t x : c) s += x;
      return s;
    }
  };
  std::vector<WidthHist> widths;
  DevArray d_tany, d_tanyoff, d_tdone;
  DevArray d_dstamps, d_dlhist, d_tstamps, d_mirror, d_tflags, d_ctl, d_abort, d_wgteam, d_tbase, d_tbits, d_tlbits, d_thist;
  struct StepBytes { double lds, hbm; };
  std::vector<StepBytes> dalg_tot;  // [n_hist] every step's (a history that passes runs them all)
  // team layout last uploaded by run_dense (one launch): unchanged across runs of a plan
  std::vector<int32_t> up_wgteam, up_base, up_hist, up_anyoff;
  std::vector<int8_t> up_bits, up_lbits;
  void* up_ptr = nullptr;
  unsigned long long* hstage = nullptr;  // pinned: the run's results, copied in one go
  size_t hstage_bytes = 0;
  int64_t dstream_words = 0;
  int dgrid_b = 0, dgrid_w = 0, dgrid_m = 0;
  int tile_cap = 256, dense_maxw = DENSE_WIDE_LMAX;  // LC_TILE_WGS / LC_DENSE_MAXW (tests)
  int tile_lbits = DENSE_LMAX;                        // LC_TILE_LBITS: local slots per tile
  int wide_from = 99, wide_lbits = DENSE_LMAX;        // LC_TILE_WIDE=w:b: b local slots from width w
  // LC_PIPE: bits 0/1/2 = BLOCK/WAVE/TILE teams overlap steps (0: one at a time); bit 3 = tile
  // teams without per-step team barriers (finished teams then join the BLOCK queue); bit 4 =
  // MID teams for widths 12..14 (needs bit 0); bit 5 = one pass per running segment (r1 form;
  // default: segments packed over the team); bit 6 = WAVE histories on the big kernel's waves
  // (no dense_wave_kernel); bit 7 = MID histories (widths 12..mid_maxw) as 4-wave teams inside
  // big workgroups (no dense_mid_kernel); bit 8 = tagged tile-team mirror words (readers poll
  // the data; by default chain plans only); bit 9 = double-buffered tables (a step after an
  // in-word return starts one super-layer after its predecessor, not two); bit 10 = WAVE
  // histories of at most 9 slots in one wave's registers; bit 11 = their closure as a whole-table
  // fixpoint for steps of at most 7 slots (r3d A/B, 3 runs each: C1 0.523 -> 0.428 ms, C3 11.57
  // -> 11.59 ms); bit 12 = X of a step after a hi return from its inputs (off); bit 13 = tile
  // teams on global popcount layers (off); bit 14 = XCD-compact workgroup roles in the big
  // kernel (r3l A/B, 2 runs each: C3 11.64 -> 11.55 ms, C2 and 8-way shares unchanged); bit 16 =
  // tile teams pre-poll their credit tokens a super-layer early (r3n: -0.5 to -1 %); bit 17 = a
  // credit window of 16 super-layers instead of 8 (r3y, 2 runs each: C2 30.09 -> 29.76, C3 11.52
  // -> 11.39, C4 736 -> 729 ms, 8-way shares 0/1 unchanged).
  // Default 217039 = 1|2|4|8|64|128|256|512|1024|2048|16384|65536|131072, with the planner.
  int dense_pipe = 217039;
  bool pipe_env = false;  // LC_PIPE given: its bits as they are
  std::vector<int> plan_lb;  // team planner: local slots per tile (0: not a team)
  bool plan_off = false;     // LC_TEAM_PLAN=0: every wide history keeps 17-bit tiles
  hipStream_t stream2 = nullptr, stream3 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_b0 = nullptr, ev_b1 = nullptr, ev_w0 = nullptr, ev_w1 = nullptr;  // per dense kernel
  hipEvent_t ev_m0 = nullptr, ev_m1 = nullptr, ev_join3 = nullptr;
  bool spill_clean = false, kspill_clean = false;
  // results
  std::vector<int32_t> status, fail_step;
  std::vector<unsigned long long> explored;
  double stats[LC_STATS_N] = {0};
  // lc_plan_create phases (ms): encode, hipSetDevice (+ runtime init), streams/events/occupancy,
  // uploads, build_dense (reported as stats 20..24)
  double phase_ms[5] = {0};
  int32_t max_t = INT32_MAX;  // failure-frontier dump mode (grid kernel)
  bool report = false;        // + per-config last-op tags (search.hpp tag_shift; one history)
  int64_t entry_bytes() const { return model == LC_MODEL_CAS_REGISTER ? 8 : 16; }
  int state_bits_of(int h) const {
    return model == LC_MODEL_CAS_REGISTER ? bits_for(enc.n_states[h]) : 0;
  }

  ~lc_plan() {
    if (ev0) hipEventDestroy(ev0);
    if (ev1) hipEventDestroy(ev1);
    if (ev_fork) hipEventDestroy(ev_fork);
    if (ev_join) hipEventDestroy(ev_join);
    if (ev_join3) hipEventDestroy(ev_join3);
    for (hipEvent_t e : {ev_b0, ev_b1, ev_w0, ev_w1, ev_m0, ev_m1})
      if (e) hipEventDestroy(e);
    if (stream2) hipStreamDestroy(stream2);
    if (stream3) hipStreamDestroy(stream3);
    if (stream) hipStreamDestroy(stream);
    if (hstage) hipHostFree(hstage);
    if (hpack) hipHostFree(hpack);
  }

  void flag_wide() {
    for (int h = 0; h < enc.n_hist; ++h) {  // [state | mask] of one history must fit 63 bits
      if (!enc.err[h] && enc.live_max[h] + state_bits_of(h) > 63) {
        enc.err[h] = LC_H_WIDE;
        enc.errmsg[h] = "pending ops + state bits exceed the 63-bit packed config";
      }
    }
  }

  void make_batches(const std::vector<int>& ids) {
    batches.clear();
    size_t i = 0;
    while (i < ids.size()) {
      Batch b;
      int mb = 1, sb = 0;
      while (i < ids.size() && (int)b.hs.size() < HMAX) {
        const int h = ids[i];
        int mb2 = std::max(mb, enc.live_max[h]);
        int sb2 = std::max(sb, state_bits_of(h));
        int hb2 = bits_for((int64_t)b.hs.size() + 1);
        if (!b.hs.empty() && mb2 + sb2 + hb2 > 63) break;
        mb = mb2;
        sb = sb2;
        b.hs.push_back(h);
        ++i;
      }
      b.mask_bits = mb;
      b.state_bits = sb;
      b.hist_bits = bits_for((int64_t)b.hs.size());
      batches.push_back(std::move(b));
    }
  }

  template <typename V>
  int upload(DevArray& d, const V& v) {
    using T = typename V::value_type;
    HIP_TRY(d.ensure(std::max<size_t>(v.size(), 1) * sizeof(T)));
    if (!v.empty()) HIP_TRY(hipMemcpy(d.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return 0;
  }

  int init_device() {
    auto t0 = std::chrono::steady_clock::now();
    auto ms_since = [](std::chrono::steady_clock::time_point t) {
      return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    };
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipFree(nullptr));  // forces runtime/context initialisation into this phase
    phase_ms[1] = ms_since(t0);
    t0 = std::chrono::steady_clock::now();
    if (!stream) HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    if (!ev0) HIP_TRY(hipEventCreate(&ev0));
    if (!ev1) HIP_TRY(hipEventCreate(&ev1));
    if (!stream2) HIP_TRY(hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking));
    if (!stream3) HIP_TRY(hipStreamCreateWithFlags(&stream3, hipStreamNonBlocking));
    if (!ev_fork) HIP_TRY(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
    if (!ev_join) HIP_TRY(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
    if (!ev_join3) HIP_TRY(hipEventCreateWithFlags(&ev_join3, hipEventDisableTiming));
    for (hipEvent_t* e : {&ev_b0, &ev_b1, &ev_w0, &ev_w1, &ev_m0, &ev_m1})
      if (!*e) HIP_TRY(hipEventCreate(e));
    {
      // occupancy queries (hipGetDeviceProperties ~ms each) once per device and model; the
      // caller holds the device mutex
      static struct { bool ok; int nwg, db, dw, dm, knwg, dc; } cache[64][4];
      auto& c = cache[device & 63][model & 3];
      if (!c.ok) {
        // (LC_PHASES: the first query of a kernel loads the library's code object onto the
        // device, once per process; each query is timed so the one-time cost is attributed)
        const double t_ev = ms_since(t0);
        auto t1 = std::chrono::steady_clock::now();
        c.nwg = search_grid_size(model);
        const double t_search = ms_since(t1);
        t1 = std::chrono::steady_clock::now();
        c.db = dense_grid_size(DENSE_BIG);
        c.dw = dense_grid_size(DENSE_WAVE);
        c.dm = dense_grid_size(DENSE_MID);
        const double t_dense = ms_since(t1);
        t1 = std::chrono::steady_clock::now();
        c.knwg = keys_grid_size(model);
        c.dc = ctab_grid_size();
        c.ok = c.nwg > 0 && c.knwg > 0;
        if (debug() || getenv("LC_PHASES"))
          fprintf(stderr, "[lincheck] first use of device %d: streams+events %.2f ms, occupancy queries: search %.2f "
                  "dense %.2f keys %.2f ms\n", device, t_ev, t_search, t_dense, ms_since(t1));
      }
      nwg = c.nwg, dgrid_b = c.db, dgrid_w = c.dw, dgrid_m = c.dm, knwg = c.knwg, dgrid_c = c.dc;
    }
    if (nwg <= 0 || knwg <= 0) {
      last_error = "search kernels cannot be resident (occupancy 0)";
      return LC_E_DEVICE;
    }
    reset_knobs();  // a reused plan (lc_check's per-device cache) must not keep an earlier call's env
    const char* e = getenv("LC_PATH");
    if (e && !strcmp(e, "keys")) path = 1;
    if (e && !strcmp(e, "grid")) path = 2;
    if (e && !strcmp(e, "dense")) path = 0;
    // dense-path knobs (tests): workgroups tile teams may take per launch, widest history
    if ((e = getenv("LC_TILE_WGS")) && atoi(e) > 0) tile_cap = atoi(e);
    if ((e = getenv("LC_DENSE_MAXW")) && atoi(e) > 0) dense_maxw = std::min(atoi(e), DENSE_WIDE_LMAX);
    if ((e = getenv("LC_WIDE_MAXW"))) wide_maxw = std::max(0, std::min(atoi(e), WIDE_LMAX));
    if ((e = getenv("LC_WIDE_MINW"))) wide_minw = std::max(0, atoi(e));
    if ((e = getenv("LC_WIDE_PIPE"))) wide_pipe = atoi(e) != 0;
    if ((e = getenv("LC_WIDE_SPLIT"))) wide_split = std::max(0, std::min(atoi(e), WIDE_MAX_SPLIT));
    if ((e = getenv("LC_WCTR_MAXW"))) wctr_maxw = std::max(0, std::min(atoi(e), WCTR_LMAX));
    if ((e = getenv("LC_WCTR_MINW"))) wctr_minw = std::max(0, atoi(e));
    if ((e = getenv("LC_WIDE_GRID"))) wide_grid = std::max(0, atoi(e));
    if ((e = getenv("LC_WIDE_WATCHDOG_MS")) && atoi(e) >= 0) wide_watchdog_ms = atoi(e);
    if ((e = getenv("LC_WIDE_FORCE_ABORT"))) wide_force_abort = atoi(e) != 0;
    if ((e = getenv("LC_WIDE_STALL")) && strchr(e, ':')) {
      wide_stall_hist = atoi(e);
      wide_stall_wg = atoi(strchr(e, ':') + 1);
    }
    if ((e = getenv("LC_CTAB_MAXW"))) ctab_maxw = std::max(0, std::min(atoi(e), CTAB_TEAM_LMAX));
    if ((e = getenv("LC_CTAB_PIPE"))) ctab_pipe = atoi(e);
    if ((e = getenv("LC_CTAB_TEAM"))) ctab_team = atoi(e);
    if ((e = getenv("LC_CTAB_TEAM_MINW"))) ctab_team_minw = atoi(e);
    if ((e = getenv("LC_CTAB_TEAM_T"))) ctab_team_t = std::max(0, std::min(atoi(e), CTAB_TEAM_MAXB));
    if ((e = getenv("LC_TILE_LBITS")) && atoi(e) > 0) tile_lbits = std::max(12, std::min(atoi(e), DENSE_LMAX));
    if ((e = getenv("LC_PIPE"))) dense_pipe = atoi(e), pipe_env = true;
    if ((e = getenv("LC_TEAM_PLAN"))) plan_off = atoi(e) == 0;
    if ((e = getenv("LC_PLAN_K")) && atof(e) > 0) plan_k16 = atof(e);
    if ((e = getenv("LC_PLAN_X")) && atof(e) > 0) plan_x = atof(e);
    if ((e = getenv("LC_PLAN_KB")) && atof(e) > 0) plan_kb = atof(e);
    if ((e = getenv("LC_PLAN_ROT"))) plan_rot = atoi(e) != 0;
    if ((e = getenv("LC_PLAN_TM")) && atof(e) > 0) plan_tm = atof(e);
    if ((e = getenv("LC_PLAN_LBMIN")) && atoi(e) >= 4) plan_lbmin = atoi(e);
    if ((e = getenv("LC_TEAM_ROT"))) team_rot = std::max(-1, atoi(e));
    if ((e = getenv("LC_TEAM_ROT_LB"))) rot_min_lb = atoi(e);
    if ((e = getenv("LC_TEAM_ROT_CHAIN"))) rot_chain_lb = atoi(e);
    if ((e = getenv("LC_TEAM_ROT_CHAIN_MIN"))) rot_chain_min = atoi(e);
    if ((e = getenv("LC_BATCH_HIST"))) batch_hist = atoi(e);
    if ((e = getenv("LC_MID_MAXW")) && atoi(e) > DENSE_WAVE_LMAX && atoi(e) <= DENSE_MID_LMAX) mid_maxw = atoi(e);
    if ((e = getenv("LC_TILE_WIDE")) && strchr(e, ':')) {
      wide_from = atoi(e);
      wide_lbits = std::max(12, std::min(atoi(strchr(e, ':') + 1), DENSE_LMAX));
    }
    // test hooks: shrink the keys kernel's per-workgroup capacities to force the fallback
    if ((e = getenv("LC_KCAP")) && atoll(e) > 0) kfcap = klcap = atoll(e);
    // test hooks: tiny cells / overflow buckets exercise the overflow and regrow paths
    if ((e = getenv("LC_CELLCAP")) && atoi(e) > 0) cell_cap = atoi(e);
    if ((e = getenv("LC_OVFCAP")) && atoll(e) > 0) ovf_cap = atoll(e);
    phase_ms[2] = ms_since(t0);
    return 0;
  }

  // Every env-derived knob back to its default before init_device reads the environment, so a
  // plan reused across lc_check calls (cached_plan) sees only the current environment. The grid
  // kernel's capacities keep what earlier runs grew them to (never below the defaults): a
  // regrow is a whole re-run of the batch.
  void reset_knobs() {
    path = 0;
    tile_cap = 256, dense_maxw = DENSE_WIDE_LMAX, tile_lbits = DENSE_LMAX;
    wide_maxw = WIDE_LMAX, wide_minw = 0, wide_pipe = true, wide_grid = 0, wide_split = 0;
    wctr_maxw = WCTR_LMAX, wctr_minw = 0;
    ctab_maxw = CTAB_TEAM_LMAX, ctab_pipe = 3, wide_watchdog_ms = 20000, wide_force_abort = false;
    ctab_team = 1, ctab_team_minw = 17, ctab_team_t = 0;
    wide_stall_hist = wide_stall_wg = -1;
    wide_from = 99, wide_lbits = DENSE_LMAX;
    dense_pipe = 217039, pipe_env = false, plan_off = false;
    plan_k16 = -1, plan_x = 1.2, plan_kb = 0.45, plan_rot = false, plan_tm = 1.0, plan_lbmin = 12, team_rot = -1, rot_min_lb = 16, rot_chain_lb = 14, rot_chain_min = 14, batch_hist = 600, mid_maxw = 0;
    rot_keep_inword = !(getenv("LC_SLOTS") && strcmp(getenv("LC_SLOTS"), "lff") == 0);
    kfcap = klcap = 1 << 18;
    cell_cap = 256;
    ovf_cap = std::max<int64_t>(grown_ovf, 1 << 18);
    f_cap = std::max(grown_f, 65536);
    spill_log = std::max(grown_spill, 17);
  }
  int64_t grown_ovf = 0;  // capacities run_grid grew (kept across reuses)
  int grown_f = 0, grown_spill = 0;

  int upload_encoded() {
    flag_wide();
    grid_up = false;  // the grid / keys kernels' arrays go up when a run first needs them
    HIP_TRY(d_queue.ensure(8));
    auto t0 = std::chrono::steady_clock::now();
    const int rc = build_dense();
    phase_ms[4] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
  }
  bool grid_up = false;

  // the encoded histories as the grid and keys kernels read them (every history; the dense
  // kernels read only their step streams, so a check the dense tables decide never uploads these)
  int upload_grid() {
    if (grid_up) return 0;
    const int n = enc.n_hist;
    std::vector<int64_t> init(n);
    std::vector<int32_t> beg(n), end(n), order(n);
    std::vector<int8_t> ksh(n), kbi(n);
    std::vector<double> cost(n);
    for (int h = 0; h < n; ++h) {
      init[h] = model == LC_MODEL_COUNTER ? enc.init_value : 0;  // (register: nil; leader: {})
      beg[h] = enc.step_off[h];
      end[h] = enc.step_off[h + 1];
      ksh[h] = (int8_t)enc.live_max[h];
      kbi[h] = (int8_t)state_bits_of(h);
      order[h] = h;
      // heaviest first: frontier width grows with the pending window
      cost[h] = (double)enc.n_steps(h) * (1.0 + enc.live_max[h]) * (1.0 + enc.live_max[h]);
    }
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return cost[a] > cost[b]; });
    int rc;
    if ((rc = upload(d_step_off, enc.step_off))) return rc;
    if ((rc = upload(d_step_slot, enc.step_slot))) return rc;
    if ((rc = upload(d_inv_off, enc.inv_off))) return rc;
    if ((rc = upload(d_inv_slot, enc.inv_slot))) return rc;
    if ((rc = upload(d_inv_kind, enc.inv_kind))) return rc;
    if ((rc = upload(d_inv_a, enc.inv_a))) return rc;
    if ((rc = upload(d_inv_b, enc.inv_b))) return rc;
    if ((rc = upload(d_init, init))) return rc;
    if ((rc = upload(d_beg, beg))) return rc;
    if ((rc = upload(d_end, end))) return rc;
    if ((rc = upload(d_kshift, ksh))) return rc;
    if ((rc = upload(d_kbits, kbi))) return rc;
    if ((rc = upload(d_order, order))) return rc;
    grid_up = true;
    return 0;
  }

  // Algorithmic bytes of one dense step with live slots `live` and ninv invocations
  // (DESIGN.md §3.4). LDS: the closure visits the words w over live hi slots (We =
  // 2^popcount(live >> 3)), reading each (8 B) and its pulls (8 B per set bit: He / 2 on
  // average) and writing it; the return reads half the table's 2^H words and writes all.
  // HBM: the step's stream words; a tile-team step (slots >= 17 live) also writes every
  // visited word to its tile's mirror once and reads each cross-tile predecessor (te / 2 per
  // word on average, te live team slots) plus the return's half.
  static StepBytes step_alg_bytes(uint32_t live, int ninv) {
    const int L = 32 - __builtin_clz(live);
    const int H = L > 3 ? L - 3 : 0;
    const int He = __builtin_popcount(live >> 3);
    const double W = (double)(1ull << H), We = (double)(1ull << He);
    StepBytes b{8.0 * We * (2.0 + 0.5 * He) + 12.0 * W, 4.0 * (1 + ninv)};
    const int te = __builtin_popcount(live >> DENSE_LMAX);
    if (te) b.hbm += 8.0 * We * (1.0 + 0.5 * te + 0.5);
    return b;
  }
  // bytes of the steps history h ran (all of them, or up to its failing step)
  StepBytes dense_hist_bytes(int h, int fail_t) const {
    if (fail_t < 0) return dalg_tot[h];
    StepBytes b{0, 0};  // a failing history: its steps up to fail_t, from its stream (in hpack)
    const uint32_t* w = (const uint32_t*)hpack + ((const int64_t*)(hpack + o_sbeg))[h];
    const uint32_t* const e = w + dense_nw[h];
    for (int t = 0; w < e && t <= fail_t; ++t) {
      const uint32_t hdr = *w++;
      int ninv = 0;
      while (w < e && (*w & DENSE_OPW)) ++w, ++ninv;
      const StepBytes sb = step_alg_bytes(hdr & DENSE_LIVE_MASK, ninv);
      b.lds += sb.lds, b.hbm += sb.hbm;
    }
    return b;
  }

  // local slots per tile of wide history h: the team planner's choice, else tile_lbits
  // (LC_TILE_LBITS / LC_TILE_WIDE), raised where the team would not fit the chip's workgroups
  int team_lbits(int h) const {
    int grid_log = 0;
    while ((2 << grid_log) <= dgrid_b) ++grid_log;
    const int lw = enc.live_max[h];
    if (plan_lb[h] > 0 && plan_lb[h] < DENSE_LMAX) return plan_lb[h];  // team planner
    const int want = lw >= wide_from ? std::min(wide_lbits, tile_lbits) : tile_lbits;
    return std::min(DENSE_LMAX, std::max(lw - grid_log, std::min(want, lw - 1)));
  }

  // Step streams for the dense closure-table kernels (format: dense.hpp). Eligible:
  // cas-register, <= DENSE_MAX_STATES register values, live width <= dense_maxw.
  // ---- dense step streams, built in three parts around the encoder (plan_build):
  //   dense_prepare (before encode): the pinned staging layout, per history an upper-bound
  //     stream range (its entry count: every entry yields at most one word), knobs;
  //   dense_sink (inside encode, on the worker that just encoded history h, its arrays still in
  //     cache): eligibility, the step stream words, the width histogram and byte model;
  //   build_dense (after encode): team classes, planner, rotation, queue order, ONE async H2D.
  // Eligible: cas-register, <= DENSE_MAX_STATES register values, live width <= dense_maxw,
  // <= DENSE_MAX_NINV invocations per step.
  bool dense_on = false;
  std::vector<char> dense_ok;
  std::vector<double> dense_cost;
  std::vector<int64_t> dense_nw;  // words of each history's step stream
  size_t o_sbeg = 0, o_nst = 0, o_ord = 0, o_lm = 0, pack_bytes = 0;
  int64_t pack_words = 0;
  int dense_prepare(int n, const int64_t* hist_off) {
    dense_b.clear();
    dense_w.clear();
    dense_x.clear();
    dense_m.clear();
    dense_wd.clear();
    dense_c.clear();
    dense_on = (model == LC_MODEL_CAS_REGISTER && path == 0 && dgrid_b > 0 && dgrid_w > 0 && dgrid_m > 0) ||
               (model == LC_MODEL_COUNTER && path == 0 && dgrid_c > 0 && ctab_maxw > 0);
    if (!dense_on) return 0;
    dense_ok.assign(n, 0);
    wide_ok.assign(n, 0);
    ctab_T.assign(n, 0);
    ctab_grid.assign(n, 0);
    if ((int)wide_streams.size() < n) wide_streams.resize(n);
    dense_cost.assign(n, 0.0);
    dense_nw.assign(n, 0);
    widths.resize(n);
    dalg_tot.resize(n);
    plan_lb.assign(n, 0);
    // history h's range: its entry count + 1 words (every entry yields at most one word; the +1
    // holds the terminator the decoders need: a step's op words are counted up to the first word
    // without DENSE_OPW, which must not be a neighbour's stale word)
    // (a counter step stream has two words per invocation: twice the entry count bounds it)
    pack_words = (model == LC_MODEL_COUNTER ? 2 : 1) * (hist_off[n] - hist_off[0]) + n;
    // everything the dense kernels read goes up in ONE async copy from a pinned staging buffer
    // (kept across calls: no page faults, DMA at full rate): [words | sbeg | nsteps | order | lmax]
    o_sbeg = ((size_t)pack_words * 4 + 7) & ~(size_t)7;
    o_nst = o_sbeg + (size_t)n * 8;
    o_ord = o_nst + (size_t)n * 4;
    o_lm = o_ord + (size_t)n * 4;
    pack_bytes = o_lm + (size_t)n + 8;
    if (hpack_bytes < pack_bytes) {
      if (hpack) HIP_TRY(hipHostFree(hpack));
      hpack = nullptr;
      hpack_bytes = 0;
      HIP_TRY(hipHostMalloc(&hpack, pack_bytes + pack_bytes / 4, hipHostMallocDefault));
      hpack_bytes = pack_bytes + pack_bytes / 4;
    }
    int64_t* const sbeg = (int64_t*)(hpack + o_sbeg);
    const int64_t mul = model == LC_MODEL_COUNTER ? 2 : 1;
    for (int h = 0; h < n; ++h) sbeg[h] = mul * (hist_off[h] - hist_off[0]) + h;
    return 0;
  }
  // lc_failure_configs on the HBM tables: run_wide stops each history after wide_stop steps (-1:
  // all), and records the tables' layout of its last launch
  int wide_stop = -1;
  bool wide_last_ranked = false, wide_ran = false;
  int wide_last_hm = 0, wide_last_split = 0;
  bool keep_inv_arrays = false;  // lc_failure_configs: its grid re-run needs every history's
  // returns true when h's step stream was built (its invocation arrays are then not needed)
  bool dense_sink(int h, const HistView& v) {
    if (!dense_on) return false;
    if (model == LC_MODEL_COUNTER) return ctab_sink(h, v);
    int32_t* const nst = (int32_t*)(hpack + o_nst);
    int8_t* const lm = (int8_t*)(hpack + o_lm);
    dalg_tot[h] = StepBytes{0, 0};
    nst[h] = 0;
    lm[h] = 0;
    bool ok = !v.err && v.n_states <= DENSE_MAX_STATES;
    int64_t max_ninv = 0;  // a step's words must fit the decoders' window
    for (int64_t t = 0; t < v.n_steps; ++t) max_ninv = std::max(max_ninv, v.step_ninv[t]);
    // wider than the LDS tile teams can hold (or from LC_WIDE_MINW on, tests): tables in HBM.
    // (LC_DENSE_MAXW below 24 sends the widths between it and 25 to the grid kernel, as before.)
    const int wmin = wide_minw > 0 ? wide_minw : DENSE_WIDE_LMAX + 1;
    if (ok && max_ninv <= WIDE_MAX_NINV && v.live_max >= wmin && v.live_max <= wide_maxw) {
      wide_sink(h, v);
      return false;  // (its invocation arrays stay: lc_failure_configs re-runs it on the grid kernel)
    }
    ok = ok && max_ninv <= DENSE_MAX_NINV && v.live_max <= dense_maxw;
    dense_ok[h] = ok;
    if (!ok) return false;
    nst[h] = (int32_t)v.n_steps;
    lm[h] = (int8_t)std::max(1, v.live_max);
    WidthHist& wh = widths[h];
    std::fill(wh.c, wh.c + 33, 0u);
    uint32_t* out = (uint32_t*)hpack + ((const int64_t*)(hpack + o_sbeg))[h];
    uint32_t live = 0;
    int64_t q = 0;
    double cost = 0;
    StepBytes tot{0, 0};
    for (int64_t t = 0; t < v.n_steps; ++t) {
      if (t > 0) live &= ~(1u << v.step_slot[t - 1]);
      const int64_t q1 = q + v.step_ninv[t];
      for (int64_t k = q; k < q1; ++k) live |= 1u << v.inv_slot[k];
      const uint32_t j = v.step_slot[t];
      *out++ = live | (j << DENSE_J_SHIFT);
      for (int64_t k = q; k < q1; ++k) {
        const int64_t a = v.inv_a[k], b = v.inv_b[k];
        const uint32_t am = a == R_ANY ? 0xffu : (a == R_NEVER ? 0u : (1u << a));
        const uint32_t bm = b < 0 ? 0u : (1u << b);
        *out++ = (uint32_t)v.inv_slot[k] | (am << 8) | (bm << 16) | DENSE_OPW;
      }
      const int L = 32 - __builtin_clz(live);
      cost += (double)(1u << L) * L;
      ++wh.c[L];
      const StepBytes sb = step_alg_bytes(live, (int)(q1 - q));
      tot.lds += sb.lds, tot.hbm += sb.hbm;
      q = q1;
    }
    dalg_tot[h] = tot;
    dense_cost[h] = cost;
    dense_nw[h] = out - ((uint32_t*)hpack + ((const int64_t*)(hpack + o_sbeg))[h]);
    *out = 0u;  // the terminator (no DENSE_OPW): the last step's op words end here
    return !keep_inv_arrays;
  }

  // A wide history's step stream (wide.hpp: two header words, then its op words), into its own
  // buffer: wide histories are rare, and the upper-bound layout of the others has no room for
  // the second header word.
  void wide_sink(int h, const HistView& v) {
    std::vector<uint32_t>& out = wide_streams[h];
    out.clear();
    uint64_t live = 0;
    int64_t q = 0;
    for (int64_t t = 0; t < v.n_steps; ++t) {
      if (t > 0) live &= ~(1ull << v.step_slot[t - 1]);
      const int64_t q1 = q + v.step_ninv[t];
      for (int64_t k = q; k < q1; ++k) live |= 1ull << v.inv_slot[k];
      out.push_back((uint32_t)(live & 0x7fffffffu));
      out.push_back((uint32_t)(live >> 31) & 0x7fffffffu);
      out.push_back((uint32_t)v.step_slot[t]);
      for (int64_t k = q; k < q1; ++k) {
        const int64_t a = v.inv_a[k], b = v.inv_b[k];
        const uint32_t am = a == R_ANY ? 0xffu : (a == R_NEVER ? 0u : (1u << a));
        const uint32_t bm = b < 0 ? 0u : (1u << b);
        out.push_back((uint32_t)v.inv_slot[k] | (am << 8) | (bm << 16) | DENSE_OPW);
      }
      q = q1;
    }
    out.push_back(0u);
    wide_ok[h] = 1;
  }

  // A wide counter history's step stream (wide.hip's counter format: three header words, then
  // ctab.hpp's two words per invocation), into its own buffer as wide_sink's.
  void wctr_sink(int h, const HistView& v) {
    std::vector<uint32_t>& out = wide_streams[h];
    out.clear();
    const int64_t init = enc.init_value;
    uint64_t live = 0;
    int64_t q = 0;
    for (int64_t t = 0; t < v.n_steps; ++t) {
      if (t > 0) live &= ~(1ull << v.step_slot[t - 1]);
      const int64_t q1 = q + v.step_ninv[t];
      for (int64_t k = q; k < q1; ++k) live |= 1ull << v.inv_slot[k];
      out.push_back((uint32_t)(live & 0x7fffffffu));
      out.push_back((uint32_t)(live >> 31) & 0x7fffffffu);
      out.push_back((uint32_t)v.step_slot[t]);
      for (int64_t k = q; k < q1; ++k) {
        uint32_t fl = 0;
        int64_t req = 0;
        counter_req(v.inv_kind[k], v.inv_a[k], v.inv_b[k], init, fl, req);
        const int64_t delta = (v.inv_kind[k] & C_SUB) ? -v.inv_b[k] : v.inv_b[k];
        out.push_back((uint32_t)v.inv_slot[k] | (fl << 8) | ((uint32_t)(uint8_t)(int8_t)delta << 16) | DENSE_OPW);
        out.push_back(((uint32_t)(req + CTAB_REQ_BIAS) & 0x3fffffffu) | DENSE_OPW);
      }
      q = q1;
    }
    out.push_back(0u);
    wide_ok[h] = 1;
  }

  // CounterModel.step's requirement of one op (counter.clj:102-127), relative to the initial
  // value: a read of v needs v; an :ok *-and-get [d new] needs new - d (or new + d); flags CT_UNC
  // (steps from any config) / CT_NEVER (from none: a pre- and post-condition that disagree, or a
  // value out of the int32 range no config reaches)
  static void counter_req(uint8_t kind, int64_t a, int64_t b, int64_t init, uint32_t& fl, int64_t& req) {
    const int64_t delta = (kind & C_SUB) ? -b : b;
    fl = 0;
    req = 0;
    if (!(kind & (C_PRE_EQ | C_POST_EQ))) {
      fl = CT_UNC;
      return;
    }
    int64_t r_pre = 0, r_post = 0;
    bool never = false;
    if (kind & C_PRE_EQ) never |= __builtin_sub_overflow(a, init, &r_pre);
    if (kind & C_POST_EQ) never |= __builtin_sub_overflow(a, init, &r_post) || __builtin_sub_overflow(r_post, delta, &r_post);
    req = (kind & C_PRE_EQ) ? r_pre : r_post;
    if ((kind & C_PRE_EQ) && (kind & C_POST_EQ) && r_pre != r_post) never = true;
    if (req >= CTAB_REQ_BIAS || req < -CTAB_REQ_BIAS) never = true;
    if (never) fl = CT_NEVER, req = 0;
  }

  // A counter history's step stream for the closure tables (ctab.hpp): each op as its delta and
  // the value, relative to the initial one, the counter must hold before it (CounterModel.step,
  // counter.clj:102-127: a read of v needs v; an :ok *-and-get [d new] needs new - d, or new + d
  // for decr; both a pre- and a post-condition that disagree: never). Eligible: the table fits
  // one workgroup's LDS (live width <= ctab_maxw), |delta| <= CTAB_DMAX, the deltas' absolute sum
  // below CTAB_SUM_MAX (every config value then fits the kernel's int32 sums), at most
  // CTAB_MAX_NINV invocations per step. The others take the grid kernel.
  bool ctab_sink(int h, const HistView& v) {
    int32_t* const nst = (int32_t*)(hpack + o_nst);
    int8_t* const lm = (int8_t*)(hpack + o_lm);
    nst[h] = 0;
    lm[h] = 0;
    dense_ok[h] = 0;
    // the counter tables' conditions on the ops (either layout): deltas within the EQ range, their
    // absolute sum bounded, no leader ops, a step's invocations within the decoder's window
    bool elig = !v.err;
    int64_t ni = 0, max_ninv = 0;
    for (int64_t t = 0; t < v.n_steps; ++t) ni += v.step_ninv[t], max_ninv = std::max(max_ninv, v.step_ninv[t]);
    int64_t dsum = 0;
    for (int64_t k = 0; k < ni && elig; ++k) {
      const int64_t d = v.inv_b[k];
      if ((v.inv_kind[k] & C_LEADER) || d > CTAB_DMAX || d < -CTAB_DMAX) elig = false;
      dsum += d < 0 ? -d : d;
    }
    if (!elig || dsum >= CTAB_SUM_MAX) return false;
    // past the tile teams (or from LC_WCTR_MINW on, tests): the HBM tables (§3.13)
    const int cmin = wctr_minw > 0 ? wctr_minw : CTAB_TEAM_LMAX + 1;
    if (v.live_max >= cmin && v.live_max <= wctr_maxw && max_ninv <= WCTR_MAX_NINV) {
      wctr_sink(h, v);
      return false;  // (its invocation arrays stay: lc_failure_configs re-runs it on the grid kernel)
    }
    const bool ok = v.live_max <= ctab_maxw && (v.live_max <= CTAB_LMAX || ctab_team) && max_ninv <= CTAB_MAX_NINV;
    if (!ok) return false;
    dense_ok[h] = 1;
    nst[h] = (int32_t)v.n_steps;
    lm[h] = (int8_t)std::max(1, v.live_max);
    // a tile team (ctab_team_kernel) for a wide history: its team slots are the top T positions
    // of the table. Slot labels are arbitrary (a mask is a set), so the T hi slots live in the
    // most steps take those positions (every step then spreads over the tiles; crashed ops, live
    // for good and never returning, are the best team slots); the other hi slots keep their order.
    const int Lh = v.live_max;
    int T = 0;
    if (ctab_team && Lh >= ctab_team_minw)
      T = ctab_team_t > 0 ? ctab_team_t : std::max(1, std::min(CTAB_TEAM_MAXB, Lh - 15));
    if (Lh - T < CTAB_LO + 1) T = 0;
    if (Lh > CTAB_LMAX && (T == 0 || Lh - T > CTAB_LO + 13)) {  // (tiles of <= 2^13 words)
      dense_ok[h] = 0;
      nst[h] = 0;
      return false;
    }
    ctab_T[h] = (int8_t)T;
    uint32_t pi[32];
    for (int k = 0; k < 32; ++k) pi[k] = (uint32_t)k;
    if (T > 0) {
      int64_t cnt[32] = {0};
      uint32_t lv = 0;
      int64_t q = 0;
      for (int64_t t = 0; t < v.n_steps; ++t) {
        if (t > 0) lv &= ~(1u << v.step_slot[t - 1]);
        for (int64_t k = q; k < q + v.step_ninv[t]; ++k) lv |= 1u << v.inv_slot[k];
        q += v.step_ninv[t];
        for (uint32_t m = lv; m; m &= m - 1) ++cnt[__builtin_ctz(m)];
      }
      std::vector<int> hi;
      for (int k = CTAB_LO; k < Lh; ++k) hi.push_back(k);
      std::stable_sort(hi.begin(), hi.end(), [&](int a, int b) { return cnt[a] > cnt[b]; });
      std::vector<char> team(32, 0);
      for (int i = 0; i < T; ++i) team[hi[i]] = 1, pi[hi[i]] = (uint32_t)(Lh - T + i);
      uint32_t nxt = CTAB_LO;
      for (int k = CTAB_LO; k < Lh; ++k)
        if (!team[k]) pi[k] = nxt++;
    }
    auto relabel = [&](uint32_t m) {
      uint32_t r = 0;
      for (; m; m &= m - 1) r |= 1u << pi[__builtin_ctz(m)];
      return r;
    };
    uint32_t* const out0 = (uint32_t*)hpack + ((const int64_t*)(hpack + o_sbeg))[h];
    uint32_t* out = out0;
    const int64_t init = enc.init_value;
    uint32_t live = 0;
    int64_t q = 0;
    double cost = 0;
    for (int64_t t = 0; t < v.n_steps; ++t) {
      if (t > 0) live &= ~(1u << v.step_slot[t - 1]);
      const int64_t q1 = q + v.step_ninv[t];
      for (int64_t k = q; k < q1; ++k) live |= 1u << v.inv_slot[k];
      *out++ = relabel(live) | (pi[v.step_slot[t]] << DENSE_J_SHIFT);
      for (int64_t k = q; k < q1; ++k) {
        const uint8_t kind = v.inv_kind[k];
        const int64_t delta = (kind & C_SUB) ? -v.inv_b[k] : v.inv_b[k];
        uint32_t fl = 0;
        int64_t req = 0;
        counter_req(kind, v.inv_a[k], v.inv_b[k], init, fl, req);
        *out++ = pi[v.inv_slot[k]] | (fl << 8) | ((uint32_t)(uint8_t)(int8_t)delta << 16) | DENSE_OPW;
        *out++ = ((uint32_t)(req + CTAB_REQ_BIAS) & 0x3fffffffu) | DENSE_OPW;
      }
      const int L = live ? 32 - __builtin_clz(live) : 0;
      cost += std::ldexp(1.0, std::max(0, L - CTAB_LO)) + 8.0;
      q = q1;
    }
    dense_cost[h] = cost;
    dense_nw[h] = out - out0;
    *out = 0u;  // the terminator (no DENSE_OPW)
    // (a history wider than one workgroup's table keeps its invocation arrays: should its team
    // not fit the launch, it takes the grid kernel)
    return !keep_inv_arrays && Lh <= CTAB_LMAX;
  }

  int build_dense() {
    const auto t_build = std::chrono::steady_clock::now();
    auto ms_since_build = [&] {
      return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_build).count();
    };
    if (!dense_on) return 0;
    const int n = enc.n_hist;
    std::vector<char>& ok = dense_ok;
    std::vector<double>& cost = dense_cost;
    uint32_t* const words = (uint32_t*)hpack;
    int64_t* const sbeg = (int64_t*)(hpack + o_sbeg);
    int32_t* const ordp = (int32_t*)(hpack + o_ord);
    const double t_fill = ms_since_build();
    up_ptr = nullptr;  // (a new layout: upload the team tables again)
    for (int h = 0; h < n; ++h)
      if (wide_ok[h]) dense_wd.push_back(h);
    for (int h = 0; h < n; ++h) {
      if (!ok[h]) continue;
      if (model == LC_MODEL_COUNTER) {
        dense_c.push_back(h);
        continue;
      }
      const int lw = enc.live_max[h];
      // MID teams (several per CU) take the narrower BLOCK histories when BLOCK steps are pipelined
      (lw <= DENSE_WAVE_LMAX ? dense_w
       : ((dense_pipe & 129) == 129 ? lw <= mid_width() : lw <= DENSE_MID_LMAX && (dense_pipe & 17) == 17) ? dense_m
       : lw <= DENSE_LMAX ? dense_b : dense_x).push_back(h);
    }
    plan_teams(widths);
    const double t_plan = ms_since_build();
    // LC_TEAM_ROT=r: a tile team's slots relabelled so its r lowest slots (the ones live in
    // almost every step) become the top r team bits and the others move down r places. Slot
    // labels are arbitrary (masks are sets), so the answer is unchanged; what changes is which
    // tiles work in a step: with low slots as team bits every tile holds a share of every step,
    // instead of tile 0 holding every step whole.
    // Default (LC_TEAM_ROT unset): full rotation for teams whose tiles hold >= rot_min_lb local
    // slots when the plan is a batch (throughput: rotated big tiles are the cheapest teams) or
    // at least 40 % of the history's steps are wide anyway (C4, lb 16: 1.85 s -> 0.90 s). A
    // chain plan's mostly-narrow histories keep their narrow steps on tile 0 alone, off the
    // exchange (a C3 125-key share: 8.2 ms unrotated, 8.9 rotated), and so do narrower tiles
    // (C2, lb 13: 35.4 ms, 39.7 rotated).
    if (team_rot != 0)
      for (int h : dense_x) {
        const int lw = enc.live_max[h], lb = team_lbits(h);
        // auto (will_rotate): a batch plan's big-tile teams, or mostly-wide histories, and a
        // chain plan's widest teams (14-slot tiles, >= 4 team bits: 16+ tiles), which gain from it
        // too (r3i, every 8-way C3 share rotated and not: w21/lb14 8.46 -> 7.37 ms and 6.64 ->
        // 6.22, w18/lb14 6.24 -> 5.91; w17/lb14 (3 team bits) 6.62 -> 6.86, and 13-slot tiles
        // lose at every width: w19/lb13 6.39 -> 7.08, w20/lb13 6.34 -> 7.05)
        if (team_rot < 0 && !will_rotate(widths[h], lw, lb)) continue;
        const int r = team_rot < 0 ? lw - lb : std::min(team_rot, lw - lb);
        if (r <= 0) continue;
        // with the encoder's slot policy the in-word slots 0..2 hold the soonest-returning ops:
        // they stay in the word, and slots 3..r+2 (the most used of the rest) become the team bits
        const int keep = rot_keep_inword ? 3 : 0;
        uint32_t perm[32];
        for (int k = 0; k < 32; ++k)
          perm[k] = k >= lw || k < keep ? (uint32_t)k
                    : k < keep + r    ? (uint32_t)(lw - r + (k - keep))
                                      : (uint32_t)(k - r);
        uint32_t* w = words + sbeg[h];
        uint32_t* const e = w + dense_nw[h];
        while (w < e) {
          const uint32_t x = *w;
          if (x & DENSE_OPW) {
            *w = (x & ~0xffu) | perm[x & 31u];
          } else {
            uint32_t live = 0;
            for (uint32_t m = x & DENSE_LIVE_MASK; m; m &= m - 1) live |= 1u << perm[__builtin_ctz(m)];
            *w = live | (perm[(x >> DENSE_J_SHIFT) & 31u] << DENSE_J_SHIFT);
          }
          ++w;
        }
      }
    pool_block_us = 0, pool_mid_us = 0, pool_wave_us = 0;  // the BLOCK pool's planned work
    for (int h : dense_b) pool_block_us += est_block_us(widths[h]);
    if (dense_pipe & 128) for (int h : dense_m) pool_mid_us += est_mid_us(widths[h]) / 4.0;
    if (dense_pipe & 64) for (int h : dense_w) pool_wave_us += 7.9 * (double)widths[h].steps() / 16.0;
    auto heavy_first = [&](int a, int b) { return cost[a] > cost[b]; };
    std::stable_sort(dense_b.begin(), dense_b.end(), heavy_first);
    std::stable_sort(dense_w.begin(), dense_w.end(), heavy_first);
    std::stable_sort(dense_x.begin(), dense_x.end(), heavy_first);
    std::stable_sort(dense_m.begin(), dense_m.end(), heavy_first);
    std::stable_sort(dense_c.begin(), dense_c.end(), heavy_first);
    {
      int32_t* o = ordp;
      for (const std::vector<int>* ids : {&dense_b, &dense_w, &dense_x, &dense_m, &dense_c})
        o = std::copy(ids->begin(), ids->end(), o);
    }
    dstream_words = pack_words;
    const double t_rot = ms_since_build();
    HIP_TRY(d_dpack.ensure(pack_bytes));
    HIP_TRY(hipMemcpyAsync(d_dpack.p, hpack, pack_bytes, hipMemcpyHostToDevice, stream));
    char* const dp = (char*)d_dpack.p;
    dp_stream = (uint32_t*)dp;
    dp_sbeg = (int64_t*)(dp + o_sbeg);
    dp_nst = (int32_t*)(dp + o_nst);
    dp_ord = (int32_t*)(dp + o_ord);
    dp_lm = (int8_t*)(dp + o_lm);
    int rc;
    if (!d_dwords.p) {
      std::vector<uint32_t> wl(1u << DENSE_WORD_BITS);
      dense_word_list(DENSE_WORD_BITS, wl.data());
      if ((rc = upload(d_dwords, wl))) return rc;
    }
    if (debug() || getenv("LC_PHASES"))
      fprintf(stderr, "[lincheck] build_dense (ms from its start; streams built in encode): classes %.2f  team plan %.2f  rotation+order %.2f  "
              "upload issued %.2f\n", t_fill, t_plan, t_rot, ms_since_build());
    HIP_TRY(d_dqueue.ensure(16));
    HIP_TRY(d_dstatus.ensure((size_t)std::max(n, 1) * 4));
    HIP_TRY(d_dfail.ensure((size_t)std::max(n, 1) * 4));
    HIP_TRY(d_dexpl.ensure((size_t)std::max(n, 1) * 8));
    return 0;
  }

  // Team planner (pipelined tile teams, LC_PIPE bits 2|3): how many local slots each tile of a
  // team holds. A history's time is the chain of its steps, so the launch lasts as long as the
  // slowest history, or the pool (BLOCK histories, heaviest first, then WAVE histories 16 per
  // workgroup) on the workgroups the teams leave, whichever is later. Greedy: while the slowest
  // single history bounds that makespan, give it tiles of one slot fewer (twice the
  // workgroups; a BLOCK history becomes a 2-tile team) if that shortens it and the pool, on
  // fewer workgroups, still ends before the new makespan. Step-time models (us; least-squares
  // fits to MI355X LC_DEBUG history times, r2c-r2h), L = the step's live width:
  //   BLOCK step   4.67 + 0.00266 * 2^(L-3)
  //   team step    1.59 + 0.0043 * 2^(min(L,lb)-3) + (L > lb) * (3.87 + 1.57 * (L - lb))
  //   WAVE step    7.9 (16 histories share a workgroup)
  static double est_block_us(const WidthHist& ws) {
    double t = 0;
    for (int L = 0; L <= 32; ++L)
      if (ws.c[L]) t += ws.c[L] * (4.67 + 0.00266 * std::ldexp(1.0, std::max(0, L - 3)));
    return t;
  }
  // MID step (4-wave team, LC_PIPE bit 7)   4.9 + 0.0016 * 2^(L-3)  (r2t LC_DEBUG, C3)
  static double est_mid_us(const WidthHist& ws) {
    double t = 0;
    for (int L = 0; L <= 32; ++L)
      if (ws.c[L]) t += ws.c[L] * (4.9 + 0.0016 * std::ldexp(1.0, std::max(0, L - 3)));
    return t;
  }
  double pool_block_us = 0, pool_mid_us = 0, pool_wave_us = 0;  // the planned pool's work (WG-us)
  uint32_t mirror_seq = 0;  // tagged mirrors: launches since the buffer was last zeroed
  int team_rot = -1;       // LC_TEAM_ROT: tile-team slot rotation (build_dense; -1 auto)
  int rot_min_lb = 16;     // LC_TEAM_ROT_LB: auto rotation from this tile size
  int rot_chain_lb = 14;   // LC_TEAM_ROT_CHAIN: a chain plan's teams of this tile size (>= 4 team bits)
  int rot_chain_min = 14;  // LC_TEAM_ROT_CHAIN_MIN: ... and of the smaller tile sizes down to this one
  // rotation keeps slots 0..2 in the word (the encoder's slot policy; LC_SLOTS=lff: rotate them too)
  bool rot_keep_inword = !(getenv("LC_SLOTS") && strcmp(getenv("LC_SLOTS"), "lff") == 0);
  // LC_MID_MAXW: widest MID history when they run in big workgroups (bit 7); by default 13 for
  // a batch plan (four per CU is the cheaper throughput) and 12 for a chain plan, where a MID
  // team's longer step (w14: 7.7 us against 4.9 as a BLOCK team) becomes a chain of its own
  // (r2cd: 4-way shares 9.92 -> 9.67 ms at the slowest rank). r4r LC_DEBUG on C3: the MID pool
  // ended at 10.5 ms (its w14 histories at 8.0 us per step), the BLOCK pool at 8.1, the WAVE pool
  // at 5.6; with w14 histories as BLOCK teams (r4s, twice each) C3 11.00-11.08 -> 10.70-10.71 ms
  int mid_maxw = 0;
  int mid_width() const { return mid_maxw > 0 ? mid_maxw : batch_plan() ? 13 : 12; }
  // LC_PLAN_K: scales the team model's VALU term. The model was fitted on unrotated teams;
  // rotated teams (auto from lb 16) spread every step over the tiles, so fewer tiles serve. A
  // batch plan (many histories sharing the chip) is throughput-bound and wants them (r2rot4/5
  // sweep on C3: 0.4-0.45 -> 11.7 ms, 0.7 -> 13.4-13.6); a plan of a few histories is their
  // chain and keeps a higher factor (C2: 0.7 -> 35.5 ms, 0.4 -> 39.1 ms; rank shares: 1.0, r2cd).
  double plan_k16 = -1;  // < 0: 0.45 for a batch plan, else 1.0 (r2cd)
  // LC_PLAN_X: the team model's cost per team bit (us per step). Fitted at 1.57 (r2c-r2h); 1.2
  // with a 12-slot floor (LC_PLAN_LBMIN) lets C2 take 12-slot tiles: 29.6 -> 28.1 ms, the 8-way C3
  // shares, C3 and C4 unchanged (r3ag-r3ai)
  double plan_x = 1.2;
  double plan_kb = 0.45;  // LC_PLAN_KB: the batch plan's VALU factor
  bool plan_rot = false;  // LC_PLAN_ROT: the team model knows which teams will be rotated
  // LC_PLAN_TM: a batch plan's team estimates times this (r3n LC_DEBUG: rotated 17-slot teams
  // took 1.3-1.8x their estimate while the BLOCK pool took 0.95x of its own)
  double plan_tm = 1.0;
  int plan_lbmin = 12;  // LC_PLAN_LBMIN: the team planner's smallest tile (local slots)
  // A batch plan (LC_BATCH_HIST: more than 600 histories, e.g. C3 on one GPU) fills the chip,
  // so the launch is throughput-bound; fewer histories leave workgroups idle and the launch is
  // its slowest chain (r2rot6-8: C3 1000 keys 11.8 ms batch / 16.2 unrotated; a 250-key share
  // 8.2-9.5 ms as a chain plan, 9.6-9.9 as a batch plan).
  int batch_hist = 600;  // (r2bh: a 500-key share as a chain plan: slowest rank 11.3 -> 10.9 ms)
  bool batch_plan() const { return enc.n_hist > batch_hist; }
  // Will build_dense rotate history h's team of lb-slot tiles? (the rule documented there)
  bool will_rotate(const WidthHist& ws, int lw, int lb) const {
    if (team_rot == 0 || lw <= lb) return false;
    if (team_rot > 0) return true;
    int wide = 0;
    for (int L = lb + 1; L <= 32; ++L) wide += (int)ws.c[L];
    const bool mostly_wide = 10 * wide >= 4 * (int)ws.steps();
    const bool chain_widest = !batch_plan() && lb <= rot_chain_lb && lb >= std::min(rot_chain_min, rot_chain_lb) && lw - lb >= 4;
    return chain_widest || (lb >= rot_min_lb && (batch_plan() || mostly_wide));
  }
  // lw: the history's widest step. A rotated team (LC_PLAN_ROT, r3) has its t = lw - lb team
  // bits among the slots live in almost every step: every step is spread over the tiles (local
  // width L - t) and pays the exchange; unrotated, a step of width L <= lb runs on tile 0 alone.
  double est_team_us(const WidthHist& ws, int lb, int lw = 0) const {
    const double k = plan_k16 > 0 ? plan_k16 : batch_plan() ? plan_kb : 1.0;
    const bool rot = plan_rot && lw > lb && will_rotate(ws, lw, lb);
    const int tb = rot ? lw - lb : 0;
    double t = 0;
    for (int L = 0; L <= 32; ++L) {
      if (!ws.c[L]) continue;
      const int Lloc = rot ? std::max(3, L - tb) : std::min<int>(L, lb);
      double u = 1.59 + 0.0043 * k * std::ldexp(1.0, std::max(0, std::min(Lloc, lb) - 3));
      if (rot) u += 3.87 + plan_x * tb;
      else if (L > lb) u += 3.87 + plan_x * (L - lb);
      t += ws.c[L] * u;
    }
    return batch_plan() ? t * plan_tm : t;
  }
  void plan_teams(const std::vector<WidthHist>& ws) {
    const bool pipe_teams = (dense_pipe & 12) == 12;
    const int maxb = (dense_pipe & DENSE_PIPE_SERIAL_SEGS) ? DENSE_TEAM_MAXB_SERIAL : DENSE_TEAM_MAXB;
    const int cap = std::min(dgrid_b, tile_cap);
    for (int h : dense_x) plan_lb[h] = DENSE_LMAX;
    if (!pipe_teams || getenv("LC_TILE_LBITS") || getenv("LC_TILE_WIDE") || plan_off) return;
    auto wgs = [&](int h, int lb) { return enc.live_max[h] > lb ? 1 << (enc.live_max[h] - lb) : 1; };
    std::vector<double> est(enc.n_hist, 0.0);
    std::vector<char> in_block(enc.n_hist, 0);
    int team_wgs = 0;
    for (int h : dense_x) team_wgs += wgs(h, DENSE_LMAX), est[h] = est_team_us(ws[h], DENSE_LMAX, enc.live_max[h]);
    double pool = 0;
    for (int h : dense_b) in_block[h] = 1, est[h] = est_block_us(ws[h]), pool += est[h];
    if (dense_pipe & 64)  // WAVE histories on the big kernel's waves, 16 per workgroup
      for (int h : dense_w) pool += 7.9 * (double)ws[h].steps() / 16.0;
    if (dense_pipe & 128)  // MID histories on the big kernel's waves, 4 per workgroup
      for (int h : dense_m) pool += est_mid_us(ws[h]) / 4.0;
    std::vector<int> cand(dense_x);
    for (int h : dense_b)
      if (enc.live_max[h] >= 14) cand.push_back(h);
    for (int iter = 0; iter < 4096 && !cand.empty(); ++iter) {
      int best = cand[0];
      for (int h : cand) if (est[h] > est[best]) best = h;
      const int block_wgs = std::max(1, dgrid_b - team_wgs);
      if (est[best] <= pool / block_wgs) break;  // the pool bounds the launch
      const int lw = enc.live_max[best];
      const int cur = in_block[best] ? lw : plan_lb[best];
      double second = 0;  // the slowest other history
      for (int h : cand) if (h != best) second = std::max(second, est[h]);
      // every smaller tile size the team limits allow: the one with the smallest makespan
      int nlb = -1, extra = 0;
      double t_new = est[best], m_best = est[best];
      for (int lb = cur - 1; lb >= plan_lbmin && lw - lb <= maxb; --lb) {
        const int x = wgs(best, lb) - (in_block[best] ? 1 : wgs(best, cur));
        if (team_wgs + x > cap || dgrid_b - team_wgs - x < 1) break;
        const double t = est_team_us(ws[best], lb, lw);
        const double pool_new = (pool - (in_block[best] ? est[best] : 0.0)) / (dgrid_b - team_wgs - x);
        const double m = std::max(std::max(t, second), pool_new);
        if (m < m_best - 1.0) nlb = lb, extra = x, t_new = t, m_best = m;
      }
      if (nlb < 0) break;
      if (in_block[best]) {
        in_block[best] = 0;
        pool -= est[best];
        dense_b.erase(std::find(dense_b.begin(), dense_b.end(), best));
        dense_x.push_back(best);
      }
      team_wgs += extra;
      plan_lb[best] = nlb;
      est[best] = t_new;
    }
    if (debug()) {
      fprintf(stderr, "[lincheck] team plan: %zu teams, %d team workgroups, block pool est %.0f us on %d wgs:",
              dense_x.size(), team_wgs, pool / std::max(1, dgrid_b - team_wgs), dgrid_b - team_wgs);
      for (int h : dense_x) fprintf(stderr, " h%d:w%d/lb%d(%.0fus)", h, enc.live_max[h], plan_lb[h], est[h]);
      fprintf(stderr, "\n");
    }
  }

  // Dense closure-table kernels: the big kernel (tile teams first, then BLOCK histories) on
  // one stream, the wave kernel beside it on a second stream. Wide histories whose tile
  // teams do not fit one launch (tile_cap workgroups) run in further big-kernel launches.
  int run_dense(float* ms) {
    const int nb = (int)dense_b.size(), nw = (int)dense_w.size(), nx = (int)dense_x.size();
    const int nm = (int)dense_m.size();
    if (nb + nw + nx + nm == 0) return 0;
    const int n = enc.n_hist;
    // the results in ONE device block, copied back in one transfer: explored (8 B per history) |
    // status (4) | fail step (4) | one stats block per kernel (big, wave, MID) | the abort word |
    // per-history start / end stamps (32; the chain-bound figure, stats 39..41)
    const size_t n1 = (size_t)std::max(n, 1);
    const size_t o_st = n1 * 8, o_fs = o_st + n1 * 4, o_ss = (o_fs + n1 * 4 + 7) & ~(size_t)7,
                 o_ab = o_ss + 3 * SS_N * 8, o_sp = o_ab + 16, r_bytes = o_sp + n1 * 32;
    HIP_TRY(d_dres.ensure(r_bytes));
    char* const rb = (char*)d_dres.p;
    ZeroSpans z0;  // (one launch)
    z0.add(d_dqueue.p, 16);
    z0.add(rb, n1 * 8);                          // explored
    z0.add(rb + o_ss, 3 * SS_N * 8 + 16 + n1 * 32);  // stats, abort word, stamps
    DenseParams p{};
    p.sbeg = dp_sbeg;
    p.nsteps = dp_nst;
    p.lmax = dp_lm;
    p.words = d_dwords.as<uint32_t>();
    p.stream = dp_stream;
    p.stream_words = dstream_words;
    p.status = (int32_t*)(rb + o_st);
    p.fail_step = (int32_t*)(rb + o_fs);
    p.explored = (unsigned long long*)rb;
    p.stats = (unsigned long long*)(rb + o_ss);
    p.pipe = dense_pipe;
    p.stamps = (unsigned long long*)(rb + o_sp);
    if (debug()) {
      HIP_TRY(d_dlhist.ensure((64 * LH_N + 32) * 8));
      HIP_TRY(hipMemsetAsync(d_dlhist.p, 0, (64 * LH_N + 32) * 8, stream));
      p.lhist = d_dlhist.as<unsigned long long>();
    }
    // tile teams: one per wide history, 2^(width - 17) workgroups; packed into launches of at
    // most `cap` workgroups (the first launch also runs the BLOCK histories)
    const int cap = std::max(1, std::min(tile_cap, dgrid_b));
    std::vector<std::vector<int>> launches(1);
    int used = 0;
    // local slots per tile: tile_lbits (<= DENSE_LMAX, the LDS tile), raised where the team
    // would not fit the chip's workgroups; a team larger than `cap` gets a launch of its own
    auto lbits_of = [&](int h) { return team_lbits(h); };
    for (int h : dense_x) {
      const int g = 1 << (enc.live_max[h] - lbits_of(h));
      if (used + g > cap && !launches.back().empty()) {
        launches.emplace_back();
        used = 0;
      }
      launches.back().push_back(h);
      used += g;
    }
    size_t max_wgs = 0, max_teams = 0;
    std::vector<std::vector<int32_t>> l_wgteam(launches.size()), l_base(launches.size()), l_hist(launches.size());
    std::vector<std::vector<int8_t>> l_bits(launches.size()), l_lbits(launches.size());
    for (size_t l = 0; l < launches.size(); ++l) {
      int b = 0;
      for (int h : launches[l]) {
        const int t = enc.live_max[h] - lbits_of(h);
        // the kernel trusts these: a tile is at most the 17-bit LDS table and a team's
        // workgroups must all be resident at once
        if (lbits_of(h) > DENSE_LMAX || lbits_of(h) < 4 || t < 1 || (1 << t) > dgrid_b) {
          last_error = "dense tile team shape out of range";
          return LC_E_INTERNAL;
        }
        l_base[l].push_back(b);
        l_bits[l].push_back((int8_t)t);
        l_lbits[l].push_back((int8_t)lbits_of(h));
        l_hist[l].push_back(h);
        for (int r = 0; r < (1 << t); ++r) l_wgteam[l].push_back((int32_t)l_base[l].size() - 1);
        b += 1 << t;
      }
      max_wgs = std::max(max_wgs, l_wgteam[l].size());
      max_teams = std::max(max_teams, l_base[l].size());
    }
    // pipelined teams: per team one survivor bit per step (+ the last return), in u32 words
    std::vector<std::vector<int32_t>> l_anyoff(launches.size());
    size_t max_anyw = 0;
    for (size_t l = 0; l < launches.size(); ++l) {
      int32_t o = 0;
      for (int h : launches[l]) {
        l_anyoff[l].push_back(o);
        o += enc.n_steps(h) / 32 + 1;
      }
      max_anyw = std::max(max_anyw, (size_t)o);
    }
    // pipelined teams pull over at most DENSE_TEAM_MAXB team bits per tile (5 with serial segments)
    // (LC_TILE_LBITS below 17 can make more): such launches use the per-step team loop
    int pipe_mode = dense_pipe;
    for (size_t l = 0; l < launches.size(); ++l)
      for (int8_t t : l_bits[l])
        if (t > ((dense_pipe & DENSE_PIPE_SERIAL_SEGS) ? DENSE_TEAM_MAXB_SERIAL : DENSE_TEAM_MAXB)) pipe_mode &= ~4;
    // tagged mirror words (bit 8): packed pipelined teams only; a tag holds the step in its
    // low 20 bits above a launch sequence, so histories of 2^20 steps or more use tokens
    if (!(pipe_mode & 4) || (pipe_mode & DENSE_PIPE_SERIAL_SEGS)) pipe_mode &= ~256;
    // by default only chain plans: a batch plan's teams are throughput-bound and the doubled
    // mirror traffic costs it ~2 % (C3 12.2 -> 12.5 ms), while C2 / C4 gain 6 % / 10 % (r2tag)
    if (!pipe_env && batch_plan()) pipe_mode &= ~256;
    for (int h : dense_x)
      if (enc.n_steps(h) >= (1 << 20) - 1) pipe_mode &= ~256;
    p.pipe = pipe_mode;
    if (max_wgs) {
      const size_t slots = (pipe_mode & 4) ? DENSE_MRING : 2;  // 2: the per-step loop's buffers
      const size_t mbytes = (max_wgs * slots << (DENSE_LMAX - 3)) * 8 * ((pipe_mode & 256) ? 2 : 1);
      HIP_TRY(d_tdone.ensure(max_wgs * 8));
      if (mbytes > d_mirror.bytes || !d_mirror.p) mirror_seq = 0;  // fresh buffer: zeroed below
      HIP_TRY(d_mirror.ensure(mbytes));
      HIP_TRY(d_tany.ensure(std::max<size_t>(max_anyw, 1) * 4));
      HIP_TRY(d_tanyoff.ensure(max_teams * 4));
      HIP_TRY(d_tflags.ensure(max_wgs * 8));
      HIP_TRY(d_ctl.ensure(max_teams * dense_ctl_bytes()));
      HIP_TRY(d_wgteam.ensure(max_wgs * 4));
      HIP_TRY(d_tbase.ensure(max_teams * 4));
      HIP_TRY(d_tbits.ensure(max_teams));
      HIP_TRY(d_tlbits.ensure(max_teams));
      HIP_TRY(d_thist.ensure(max_teams * 4));
    }
    HIP_TRY(zero_spans(z0, stream));
    // LC_PIPE bit 6 (default): WAVE histories run on the big kernel's waves after its BLOCK queue
    const bool wave_in_big = (dense_pipe & 64) != 0;
    HIP_TRY(hipEventRecord(ev0, stream));
    if (nw && !wave_in_big) {
      HIP_TRY(hipEventRecord(ev_fork, stream));
      HIP_TRY(hipStreamWaitEvent(stream2, ev_fork, 0));
      DenseParams q = p;
      q.n = nw;
      q.order = dp_ord + nb;
      q.queue = d_dqueue.as<int32_t>() + 1;
      q.stats = p.stats + SS_N;
      HIP_TRY(hipEventRecord(ev_w0, stream2));
      HIP_TRY(launch_dense(q, DENSE_WAVE, std::min(dgrid_w, (nw + 3) / 4), stream2));
      HIP_TRY(hipEventRecord(ev_w1, stream2));
      HIP_TRY(hipEventRecord(ev_join, stream2));
    }
    // LC_PIPE bit 7: MID histories run on the big kernel's waves, four per workgroup
    const bool mid_in_big = (dense_pipe & 128) != 0;
    if (nm && !mid_in_big) {
      if (!nw || wave_in_big) HIP_TRY(hipEventRecord(ev_fork, stream));
      HIP_TRY(hipStreamWaitEvent(stream3, ev_fork, 0));
      DenseParams q = p;
      q.n = nm;
      q.order = dp_ord + nb + nw + nx;
      q.queue = d_dqueue.as<int32_t>() + 2;
      q.stats = p.stats + 2 * SS_N;
      HIP_TRY(hipEventRecord(ev_m0, stream3));
      // wave + MID workgroups stay within one per CU: either fits beside a big-kernel
      // workgroup, two of them do not, and every tile-team workgroup must be resident
      const int wgrid = nw && !wave_in_big ? std::min(dgrid_w, (nw + 3) / 4) : 0;
      const int mgrid = std::min(nm, dgrid_m - wgrid);
      if (mgrid > 0) HIP_TRY(launch_dense(q, DENSE_MID, mgrid, stream3));
      HIP_TRY(hipEventRecord(ev_m1, stream3));
      HIP_TRY(hipEventRecord(ev_join3, stream3));
    }
    HIP_TRY(hipEventRecord(ev_b0, stream));
    for (size_t l = 0; l < launches.size(); ++l) {
      const int nt = (int)l_base[l].size(), twgs = (int)l_wgteam[l].size();
      DenseParams q = p;
      q.n = l == 0 ? nb : 0;
      q.order = dp_ord;
      q.queue = d_dqueue.as<int32_t>();
      q.n2 = l == 0 ? nm : 0;
      q.order2 = dp_ord + nb + nw + nx;
      q.queue2 = d_dqueue.as<int32_t>() + 2;
      q.n_team_wgs = twgs;
      q.n_w = 0;
      if (l == 0 && wave_in_big) {
        q.n_w = nw;
        q.order_w = dp_ord + nb;
        q.queue_w = d_dqueue.as<int32_t>() + 1;
      }
      if (nt) {
        // the team tables: uploaded when the layout (or a buffer) changed, else still in place
        // from the last run of this plan (one launch)
        const bool same = launches.size() == 1 && up_ptr == d_wgteam.p && up_wgteam == l_wgteam[l] &&
                          up_base == l_base[l] && up_bits == l_bits[l] && up_lbits == l_lbits[l] &&
                          up_hist == l_hist[l] && up_anyoff == l_anyoff[l] && d_tbase.p && d_tanyoff.p;
        if (!same) {
          HIP_TRY(hipMemcpyAsync(d_wgteam.p, l_wgteam[l].data(), twgs * 4, hipMemcpyHostToDevice, stream));
          HIP_TRY(hipMemcpyAsync(d_tbase.p, l_base[l].data(), nt * 4, hipMemcpyHostToDevice, stream));
          HIP_TRY(hipMemcpyAsync(d_tbits.p, l_bits[l].data(), nt, hipMemcpyHostToDevice, stream));
          HIP_TRY(hipMemcpyAsync(d_tlbits.p, l_lbits[l].data(), nt, hipMemcpyHostToDevice, stream));
          HIP_TRY(hipMemcpyAsync(d_thist.p, l_hist[l].data(), nt * 4, hipMemcpyHostToDevice, stream));
          HIP_TRY(hipMemcpyAsync(d_tanyoff.p, l_anyoff[l].data(), nt * 4, hipMemcpyHostToDevice, stream));
          if (launches.size() == 1) {
            up_wgteam = l_wgteam[l], up_base = l_base[l], up_bits = l_bits[l], up_lbits = l_lbits[l];
            up_hist = l_hist[l], up_anyoff = l_anyoff[l];
            up_ptr = d_wgteam.p;
          } else {
            up_ptr = nullptr;
          }
        }
        ZeroSpans zt;
        zt.add(d_tflags.p, (size_t)twgs * 8);
        zt.add(d_tdone.p, (size_t)twgs * 8);
        zt.add(d_ctl.p, (size_t)nt * dense_ctl_bytes());
        zt.add(d_tany.p, std::max<size_t>(max_anyw, 1) * 4);
        HIP_TRY(zero_spans(zt, stream));
        q.done = d_tdone.as<unsigned long long>();
        q.team_any = d_tany.as<uint32_t>();
        q.team_any_off = d_tanyoff.as<int32_t>();
        q.wg_team = d_wgteam.as<int32_t>();
        q.team_base = d_tbase.as<int32_t>();
        q.team_bits = d_tbits.as<int8_t>();
        q.team_lbits = d_tlbits.as<int8_t>();
        q.team_hist = d_thist.as<int32_t>();
        q.mirror = d_mirror.as<uint64_t>();
        if (q.pipe & 256) {  // a fresh tag range per launch; the buffer is zeroed every 4096
          if ((mirror_seq & 0xfffu) == 0) HIP_TRY(hipMemsetAsync(d_mirror.p, 0, d_mirror.bytes, stream));
          q.mirror_tag = (mirror_seq & 0xfffu) << 20;
          ++mirror_seq;
        }
        q.flags = d_tflags.as<unsigned long long>();
        q.ctl = d_ctl.p;
        q.abort = (int32_t*)(rb + o_ab);
        if (debug() && l == 0) {
          HIP_TRY(d_tstamps.ensure((size_t)twgs * 64));
          HIP_TRY(hipMemsetAsync(d_tstamps.p, 0, (size_t)twgs * 64, stream));
          q.tstamps = d_tstamps.as<unsigned long long>();
        }
      }
      // WAVE histories: 16 per workgroup, or one per workgroup under LC_PIPE bit 18 (PIPE_WSPREAD)
      const int wave_wgs = (q.pipe & 262144) ? q.n_w : (q.n_w + 15) / 16;
      const int grid = twgs + std::max(0, std::min(dgrid_b - twgs, q.n + q.n2 + wave_wgs));
      // BLOCK-pool workgroups that start on the MID queue: its share of the pool's work
      q.mid_first = 0;
      if (mid_in_big && q.n2 > 0) {
        const int pool_wgs = grid - twgs - wave_wgs;
        const double tot = pool_block_us + pool_mid_us + pool_wave_us;
        const double share = tot > 0 ? pool_mid_us / tot : 0.0;
        q.mid_first = std::max(0, std::min({(q.n2 + 3) / 4, pool_wgs, (int)std::lround(share * (grid - twgs))}));
      }
      if (grid > 0) HIP_TRY(launch_dense(q, DENSE_BIG, grid, stream));
    }
    HIP_TRY(hipEventRecord(ev_b1, stream));
    if (nw && !wave_in_big) HIP_TRY(hipStreamWaitEvent(stream, ev_join, 0));
    if (nm && !mid_in_big) HIP_TRY(hipStreamWaitEvent(stream, ev_join3, 0));
    HIP_TRY(hipEventRecord(ev1, stream));
    // the result block into one pinned buffer: one transfer behind the kernels, one wait
    if (hstage_bytes < r_bytes) {
      if (hstage) HIP_TRY(hipHostFree(hstage));
      hstage = nullptr;
      HIP_TRY(hipHostMalloc(&hstage, r_bytes, hipHostMallocDefault));
      hstage_bytes = r_bytes;
    }
    char* const hb = reinterpret_cast<char*>(hstage);
    HIP_TRY(hipMemcpyAsync(hb, rb, r_bytes, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    float t = 0;
    HIP_TRY(hipEventElapsedTime(&t, ev0, ev1));
    *ms += t;
    const unsigned long long* const ex = reinterpret_cast<const unsigned long long*>(hb);
    const int32_t* const st = reinterpret_cast<const int32_t*>(hb + o_st);
    const int32_t* const fs = reinterpret_cast<const int32_t*>(hb + o_fs);
    const unsigned long long* const ss3 = reinterpret_cast<const unsigned long long*>(hb + o_ss);
    const int32_t* const abw = reinterpret_cast<const int32_t*>(hb + o_ab);
    const unsigned long long* const stamp = reinterpret_cast<const unsigned long long*>(hb + o_sp);
    if (*abw) {
      last_error = "dense tile-team watchdog fired (a team workgroup was not resident)";
      return LC_E_INTERNAL;
    }
    unsigned long long ss[SS_N];
    for (int i = 0; i < SS_N; ++i) ss[i] = ss3[i] + ss3[SS_N + i] + ss3[2 * SS_N + i];
    for (const std::vector<int>* ids : {&dense_b, &dense_w, &dense_x, &dense_m})
      for (int h : *ids) {
        status[h] = st[h], fail_step[h] = fs[h], explored[h] = ex[h];
        note_chain(h, stamp[4 * h], stamp[4 * h + 1]);
      }
    stats[1] += (nw && !wave_in_big ? 1 : 0) + (nm && !mid_in_big ? 1 : 0) + (double)launches.size();
    stats[12] += nb + nw + nx + nm;
    stats[13] += t;
    // per-kernel time (events on each kernel's own stream) and algorithmic bytes of the steps
    // each kernel ran: 14/15 big/wave ms, 16/17 big HBM/LDS bytes, 18/19 wave HBM/LDS bytes
    float tb = 0, tw = 0;
    HIP_TRY(hipEventElapsedTime(&tb, ev_b0, ev_b1));
    if (nw && !wave_in_big) HIP_TRY(hipEventElapsedTime(&tw, ev_w0, ev_w1));
    float tm = 0;  // the MID kernel runs beside both; its steps are counted with the wave kernel's
    if (nm && !mid_in_big) HIP_TRY(hipEventElapsedTime(&tm, ev_m0, ev_m1));
    stats[14] += tb;
    stats[15] += std::max(tw, tm);
    for (const std::vector<int>* ids : {&dense_b, &dense_x, &dense_w, &dense_m})
      for (int h : *ids) {
        const StepBytes b = dense_hist_bytes(h, fs[h]);
        const int k = ((ids == &dense_w && !wave_in_big) || (ids == &dense_m && !mid_in_big)) ? 18 : 16;
        stats[k] += b.hbm;
        stats[k + 1] += b.lds;
      }
    stats[2] += (double)ss[SS_STEPS];
    stats[4] += (double)ss[SS_FOUT] + (nb + nw + nx + nm);  // frontier in = previous frontier out (+ initial)
    stats[6] += (double)ss[SS_FOUT];
    // per kernel (SURVEY §8(d) terms): 25..27 big F_in / F_out / explored, 28..30 wave (+MID);
    // a history's frontier out of every step but its last is the next step's frontier in
    {
      double ex_big = 0, ex_wave = 0;
      for (const std::vector<int>* ids : {&dense_b, &dense_x}) for (int h : *ids) ex_big += (double)ex[h];
      for (const std::vector<int>* ids : {&dense_w, &dense_m})
        for (int h : *ids)
          ((ids == &dense_w ? wave_in_big : mid_in_big) ? ex_big : ex_wave) += (double)ex[h];
      const double fo_big = (double)ss3[SS_FOUT], fo_wave = (double)(ss3[SS_N + SS_FOUT] + ss3[2 * SS_N + SS_FOUT]);
      stats[25] += fo_big + (nb + nx + (wave_in_big ? nw : 0) + (mid_in_big ? nm : 0));
      stats[26] += fo_big;
      stats[27] += ex_big;
      stats[28] += fo_wave + ((wave_in_big ? 0 : nw) + (mid_in_big ? 0 : nm));
      stats[29] += fo_wave;
      stats[30] += ex_wave;
    }
    if (debug()) {
      fprintf(stderr, "[lincheck] dense: %d block + %d wave + %d tile-team histories (%zu launch(es), %zu team "
              "workgroups): %.3f ms, steps=%llu Fout=%llu\n", nb, nw, nx, launches.size(), max_wgs, t,
              ss[SS_STEPS], ss[SS_FOUT]);
      dense_report(stamp);
      std::vector<unsigned long long> LH(64 * LH_N + 32);
      if (hipMemcpy(LH.data(), d_dlhist.p, LH.size() * 8, hipMemcpyDeviceToHost) == hipSuccess)
        for (int kind = 0; kind < 3; ++kind)
          for (int wv = 0; wv < 2; ++wv) {
            const unsigned long long* q = &LH[64 * LH_N + kind * 10 + wv * 5];
            if (!q[4]) continue;
            const double n = (double)q[4];
            fprintf(stderr, "[lincheck]   pipelined %s teams, %s: per super-layer cycles: ring %.0f segments %.0f "
                    "decode+start %.0f barrier %.0f (%.0f super-layers)\n", kind == 0 ? "WAVE" : kind == 1 ? "BLOCK" : "MID",
                    wv == 0 ? "wave 0" : "decoder wave", q[0] / n, q[1] / n, q[2] / n, q[3] / n, n);
          }
      if (LH[64 * LH_N + 31])  // the big kernel's workgroups: shader clock over the 100-MHz clock
        fprintf(stderr, "[lincheck]   big kernel: mean core clock %.0f MHz over its workgroups' lifetimes\n",
                100.0 * (double)LH[64 * LH_N + 30] / (double)LH[64 * LH_N + 31]);
      if (hipMemcpy(LH.data(), d_dlhist.p, LH.size() * 8, hipMemcpyDeviceToHost) == hipSuccess)
        for (int k = 0; k < 64; ++k) {
          const unsigned long long* e = &LH[k * LH_N];
          if (!e[0]) continue;
          const int L = k & 31;
          const double s = (double)e[0];
          fprintf(stderr, "[lincheck]   %s step width %2d: %8llu steps %7.2f us/step  nonzero words %8.1f -> %8.1f "
                  "of %d  explored %8.1f\n", k >= 32 ? "block" : "wave ", L, e[0], e[1] / s / 100.0, e[2] / s,
                  e[3] / s, 1 << (L > 3 ? L - 3 : 0), e[4] / s);
        }
      if (!launches[0].empty()) {  // phase split of every tile team of the first launch
        std::vector<unsigned long long> TS(l_wgteam[0].size() * 8);
        if (hipMemcpy(TS.data(), d_tstamps.p, TS.size() * 8, hipMemcpyDeviceToHost) == hipSuccess)
          for (size_t tm = 0; tm < l_hist[0].size(); ++tm) {
            const int g0 = 1 << l_bits[0][tm], b0 = l_base[0][tm];
            for (int r = 0; r < g0; ++r) {
              if (r > 1 && r != g0 - 1 && tm > 0) continue;  // ranks 0, 1, last of later teams
              const unsigned long long* T = &TS[(size_t)(b0 + r) * 8];
              const double st = std::max(1.0, (double)T[5]);
              fprintf(stderr, (p.pipe & 4) ? "[lincheck]     tile team h=%d lb=%d rank %2d: per super-layer us: wait %.2f "
                      "compute %.2f publish %.2f credit %.2f - %.2f (%.0f super-layers)\n" : "[lincheck]     tile team "
                      "h=%d lb=%d rank %2d: per team step us: wait %.1f compute %.1f publish %.1f return %.1f barrier %.1f (%.0f steps)\n",
                      l_hist[0][tm], (int)l_lbits[0][tm], r, T[0] / st / 100, T[1] / st / 100, T[2] / st / 100,
                      T[3] / st / 100, T[4] / st / 100, st);
            }
          }
      }
    }
    return 0;
  }

  // LC_DEBUG: per-team spans and the slowest histories (s_memrealtime, 100 MHz)
  void dense_report(const unsigned long long* T) {  // T: the host copy of the stamps [n][4]
    const std::vector<int>* lists[4] = {&dense_b, &dense_w, &dense_x, &dense_m};
    const char* names[4] = {"block", "wave", "wide", "mid"};
    unsigned long long t0 = ~0ull;
    for (auto* ids : lists)
      for (int h : *ids) t0 = std::min(t0, T[4 * h]);
    for (int team = 0; team < 4; ++team) {
      const std::vector<int>& ids = *lists[team];
      if (ids.empty()) continue;
      unsigned long long first = ~0ull, last = 0;
      double by_l_us[64] = {0}, by_l_steps[64] = {0};
      std::vector<std::pair<double, int>> dur;
      for (int h : ids) {
        first = std::min(first, T[4 * h]);
        last = std::max(last, T[4 * h + 1]);
        const double us = (double)(T[4 * h + 1] - T[4 * h]) / 100.0;
        dur.push_back({us, h});
        by_l_us[enc.live_max[h]] += us;
        by_l_steps[enc.live_max[h]] += enc.n_steps(h);
      }
      std::sort(dur.rbegin(), dur.rend());
      fprintf(stderr, "[lincheck]   %s teams: start %.1f us, end %.1f us after the first dequeue\n", names[team],
              (first - t0) / 100.0, (last - t0) / 100.0);
      for (int i = 0; i < (int)dur.size() && i < 4; ++i) {
        const int h = dur[i].second;
        fprintf(stderr, "[lincheck]     slowest #%d: h=%d width=%d steps=%d %.1f us (start %.1f)", i, h,
                enc.live_max[h], enc.n_steps(h), dur[i].first, (T[4 * h] - t0) / 100.0);
        if (T[4 * h + 3])
          fprintf(stderr, " team steps %llu: %.1f us (%.1f us each)", T[4 * h + 3], T[4 * h + 2] / 100.0,
                  T[4 * h + 2] / 100.0 / (double)T[4 * h + 3]);
        fprintf(stderr, "\n");
      }
      for (int l = 0; l < 64; ++l)
        if (by_l_steps[l] > 0)
          fprintf(stderr, "[lincheck]     width %2d: %.3f us per step over %.0f steps\n", l,
                  by_l_us[l] / by_l_steps[l], by_l_steps[l]);
    }
  }

  int ensure_grid(int nh) {
    HIP_TRY(d_live.ensure(2ull * nh * 8));
    HIP_TRY(d_opk.ensure(2ull * nh * 64));
    HIP_TRY(d_opa.ensure(2ull * nh * 64 * 8));
    HIP_TRY(d_opb.ensure(2ull * nh * 64 * 8));
    HIP_TRY(d_status.ensure((size_t)nh * 4));
    HIP_TRY(d_fail.ensure((size_t)nh * 4));
    HIP_TRY(d_nonempty.ensure(2ull * nh * 4));
    HIP_TRY(d_explored.ensure((size_t)nh * 8));
    HIP_TRY(d_bbeg.ensure((size_t)nh * 4));
    HIP_TRY(d_bend.ensure((size_t)nh * 4));
    HIP_TRY(d_binit.ensure((size_t)nh * 8));
    const size_t E = (size_t)entry_bytes();
    HIP_TRY(d_flist.ensure(2ull * nwg * f_cap * E));
    HIP_TRY(d_fcount.ensure(2ull * nwg * 4));
    HIP_TRY(d_cells.ensure(2ull * nwg * nwg * cell_cap * E));
    HIP_TRY(d_cellcnt.ensure(2ull * nwg * nwg * 4));
    HIP_TRY(d_ovf.ensure(2ull * nwg * ovf_cap * E));
    HIP_TRY(d_ovfcnt.ensure(2ull * nwg * 4));
    size_t sp = (size_t)nwg << spill_log;
    if (d_spill.bytes < sp * 8) {
      HIP_TRY(d_spill.ensure(sp * 8));
      spill_clean = false;
    }
    HIP_TRY(d_spillpos.ensure(sp * 4));
    HIP_TRY(d_bar.ensure(sizeof(GridBar)));
    HIP_TRY(d_produced.ensure(4 * 8));
    HIP_TRY(d_running.ensure(4 * 4));
    HIP_TRY(d_flags.ensure(FL_N * 4));
    HIP_TRY(d_stats.ensure(SS_N * 8));
    return 0;
  }

  void add_stats(const unsigned long long* ss) {
    stats[1] += 1;
    stats[2] += (double)ss[SS_STEPS];
    stats[3] += (double)ss[SS_PHASES];
    stats[4] += (double)ss[SS_FIN];
    stats[5] += (double)ss[SS_CAND];
    stats[6] += (double)ss[SS_FOUT];
    stats[11] += (double)ss[SS_SPILL];
  }

  // keys kernel over every history; returns 0 or LC_E_*
  int run_keys(float* ms) {
    const int n = enc.n_hist;
    const size_t E = (size_t)entry_bytes();
    HIP_TRY(d_kscratch.ensure((size_t)knwg * (2 * kfcap + 2 * klcap) * E));
    const size_t sp = (size_t)knwg << kspill_log;
    if (d_kspill.bytes < sp * 8) {
      HIP_TRY(d_kspill.ensure(sp * 8));
      kspill_clean = false;
    }
    HIP_TRY(d_kspillpos.ensure(sp * 4));
    HIP_TRY(d_kstatus.ensure((size_t)std::max(n, 1) * 4));
    HIP_TRY(d_kfail.ensure((size_t)std::max(n, 1) * 4));
    HIP_TRY(d_kexplored.ensure((size_t)std::max(n, 1) * 8));
    HIP_TRY(d_stats.ensure(SS_N * 8));
    std::vector<int32_t> st0(n);
    for (int h = 0; h < n; ++h) st0[h] = enc.err[h] ? ST_SKIP : ST_RUNNING;
    if (n) HIP_TRY(hipMemcpyAsync(d_kstatus.p, st0.data(), n * 4, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipMemsetAsync(d_queue.p, 0, 8, stream));
    HIP_TRY(hipMemsetAsync(d_stats.p, 0, SS_N * 8, stream));
    if (!kspill_clean) {
      HIP_TRY(hipMemsetAsync(d_kspill.p, 0xff, sp * 8, stream));
      kspill_clean = true;
    }
    KeysParams p{};
    p.n_hist = n;
    p.model = model;
    p.kshift = d_kshift.as<int8_t>();
    p.kbits = d_kbits.as<int8_t>();
    p.fcap = kfcap;
    p.lcap = klcap;
    p.spill_log = kspill_log;
    p.step_beg = d_beg.as<int32_t>();
    p.step_end = d_end.as<int32_t>();
    p.step_slot = d_step_slot.as<uint8_t>();
    p.inv_off = d_inv_off.as<int64_t>();
    p.inv_slot = d_inv_slot.as<uint8_t>();
    p.inv_kind = d_inv_kind.as<uint8_t>();
    p.inv_a = d_inv_a.as<int64_t>();
    p.inv_b = d_inv_b.as<int64_t>();
    p.init_st = d_init.as<int64_t>();
    p.order = d_order.as<int32_t>();
    p.queue = d_queue.as<int32_t>();
    p.status = d_kstatus.as<int32_t>();
    p.fail_step = d_kfail.as<int32_t>();
    p.explored = d_kexplored.as<unsigned long long>();
    p.scratch = d_kscratch.p;
    p.spill = d_kspill.as<uint64_t>();
    p.spill_pos = d_kspillpos.as<uint32_t>();
    p.stats = d_stats.as<unsigned long long>();
    const int grid = std::min(knwg, std::max(1, n));
    HIP_TRY(hipEventRecord(ev0, stream));
    HIP_TRY(launch_keys(p, grid, stream));
    HIP_TRY(hipEventRecord(ev1, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    float t = 0;
    HIP_TRY(hipEventElapsedTime(&t, ev0, ev1));
    *ms += t;
    std::vector<int32_t> st(n), fs(n);
    std::vector<unsigned long long> ex(n);
    if (n) {
      HIP_TRY(hipMemcpy(st.data(), d_kstatus.p, n * 4, hipMemcpyDeviceToHost));
      HIP_TRY(hipMemcpy(fs.data(), d_kfail.p, n * 4, hipMemcpyDeviceToHost));
      HIP_TRY(hipMemcpy(ex.data(), d_kexplored.p, n * 8, hipMemcpyDeviceToHost));
    }
    unsigned long long ss[SS_N];
    HIP_TRY(hipMemcpy(ss, d_stats.p, sizeof(ss), hipMemcpyDeviceToHost));
    add_stats(ss);
    int ncap = 0;
    for (int h = 0; h < n; ++h) {
      status[h] = st[h];
      fail_step[h] = fs[h];
      explored[h] = ex[h];
      ncap += st[h] == ST_CAPACITY;
    }
    if (debug())
      fprintf(stderr,
              "[lincheck] keys kernel: %d histories on %d workgroups: %.2f ms, steps=%llu Fin=%llu "
              "cand=%llu Fout=%llu spill=%llu -> %d over capacity\n",
              n, grid, t, ss[SS_STEPS], ss[SS_FIN], ss[SS_CAND], ss[SS_FOUT], ss[SS_SPILL], ncap);
    return 0;
  }

  // grid kernel on one batch; returns 0, LC_E_* on hard errors, 1/2 when capacities must grow
  int run_batch(const Batch& bt, float* ms) {
    const int nh = (int)bt.hs.size();
    int rc = ensure_grid(nh);
    if (rc) return rc;
    std::vector<int32_t> st0(nh), beg(nh), end(nh);
    std::vector<int64_t> init(nh);
    for (int i = 0; i < nh; ++i) {
      const int h = bt.hs[i];
      st0[i] = enc.err[h] ? ST_SKIP : ST_RUNNING;
      beg[i] = enc.step_off[h];
      end[i] = enc.step_off[h + 1];
      init[i] = model == LC_MODEL_COUNTER ? enc.init_value : 0;
    }
    HIP_TRY(hipMemcpyAsync(d_status.p, st0.data(), nh * 4, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipMemcpyAsync(d_bbeg.p, beg.data(), nh * 4, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipMemcpyAsync(d_bend.p, end.data(), nh * 4, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipMemcpyAsync(d_binit.p, init.data(), nh * 8, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipMemsetAsync(d_live.p, 0, 2ull * nh * 8, stream));
    HIP_TRY(hipMemsetAsync(d_fail.p, 0xff, (size_t)nh * 4, stream));
    HIP_TRY(hipMemsetAsync(d_nonempty.p, 0, 2ull * nh * 4, stream));
    HIP_TRY(hipMemsetAsync(d_explored.p, 0, (size_t)nh * 8, stream));
    if (!spill_clean) {
      HIP_TRY(hipMemsetAsync(d_spill.p, 0xff, ((size_t)nwg << spill_log) * 8, stream));
      spill_clean = true;
    }
    HIP_TRY(hipMemsetAsync(d_bar.p, 0, sizeof(GridBar), stream));
    HIP_TRY(hipMemsetAsync(d_ovfcnt.p, 0, 2ull * nwg * 4, stream));
    HIP_TRY(hipMemsetAsync(d_produced.p, 0, 32, stream));
    HIP_TRY(hipMemsetAsync(d_running.p, 0, 16, stream));
    HIP_TRY(hipMemsetAsync(d_flags.p, 0, FL_N * 4, stream));
    HIP_TRY(hipMemsetAsync(d_stats.p, 0, SS_N * 8, stream));

    SearchParams p{};
    p.n_hist = nh;
    p.nwg = nwg;
    p.mask_bits = bt.mask_bits;
    p.state_shift = bt.mask_bits;
    p.hist_shift = bt.mask_bits + bt.state_bits;
    p.tag_shift = 0;
    if (report) {  // one history: the hist field is empty, the 6-bit tag sits above the state
      p.tag_shift = bt.mask_bits + bt.state_bits;
      p.hist_shift = p.tag_shift + 6;
    }
    p.cell_cap = cell_cap;
    p.f_cap = f_cap;
    p.spill_log = spill_log;
    p.max_t = max_t;
    p.model = model;
    p.step_beg = d_bbeg.as<int32_t>();
    p.step_end = d_bend.as<int32_t>();
    p.step_slot = d_step_slot.as<uint8_t>();
    p.inv_off = d_inv_off.as<int64_t>();
    p.inv_slot = d_inv_slot.as<uint8_t>();
    p.inv_kind = d_inv_kind.as<uint8_t>();
    p.inv_a = d_inv_a.as<int64_t>();
    p.inv_b = d_inv_b.as<int64_t>();
    p.init_st = d_binit.as<int64_t>();
    p.live = d_live.as<uint64_t>();
    p.op_kind = d_opk.as<uint8_t>();
    p.op_a = d_opa.as<int64_t>();
    p.op_b = d_opb.as<int64_t>();
    p.status = d_status.as<int32_t>();
    p.fail_step = d_fail.as<int32_t>();
    p.nonempty = d_nonempty.as<uint32_t>();
    p.explored = d_explored.as<unsigned long long>();
    p.flist = d_flist.p;
    p.fcount = d_fcount.as<uint32_t>();
    p.cells = d_cells.p;
    p.cell_cnt = d_cellcnt.as<uint32_t>();
    p.ovf = d_ovf.p;
    p.ovf_cnt = d_ovfcnt.as<uint32_t>();
    p.ovf_cap = ovf_cap;
    p.spill = d_spill.as<uint64_t>();
    p.spill_pos = d_spillpos.as<uint32_t>();
    p.bar = d_bar.as<GridBar>();
    p.produced = d_produced.as<unsigned long long>();
    p.running = d_running.as<unsigned>();
    p.flags = d_flags.as<int32_t>();
    p.stats = d_stats.as<unsigned long long>();
    p.stamps = nullptr;
    if (debug()) {
      HIP_TRY(d_stamps.ensure((size_t)nwg * 8 * 8));
      HIP_TRY(hipMemsetAsync(d_stamps.p, 0, (size_t)nwg * 64, stream));
      p.stamps = d_stamps.as<unsigned long long>();
    }

    HIP_TRY(hipEventRecord(ev0, stream));
    HIP_TRY(launch_search(p, stream));
    HIP_TRY(hipEventRecord(ev1, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    float t = 0;
    HIP_TRY(hipEventElapsedTime(&t, ev0, ev1));
    *ms += t;

    int32_t flags[FL_N];
    HIP_TRY(hipMemcpy(flags, d_flags.p, sizeof(flags), hipMemcpyDeviceToHost));
    unsigned long long ss[SS_N];
    HIP_TRY(hipMemcpy(ss, d_stats.p, sizeof(ss), hipMemcpyDeviceToHost));
    if (debug())
      fprintf(stderr,
              "[lincheck] grid batch %d hist bits m%d s%d h%d nwg=%d cell_cap=%d ovf_cap=%lld f_cap=%d "
              "spill_log=%d: %.2f ms, steps=%llu phases=%llu Fin=%llu cand=%llu Fout=%llu "
              "spill=%llu flags abort=%d ovf=%d spillfull=%d\n",
              nh, bt.mask_bits, bt.state_bits, bt.hist_bits, nwg, cell_cap, (long long)ovf_cap, f_cap, spill_log, t,
              ss[SS_STEPS], ss[SS_PHASES], ss[SS_FIN], ss[SS_CAND], ss[SS_FOUT], ss[SS_SPILL],
              flags[FL_ABORT], flags[FL_OVERFLOW], flags[FL_SPILL]);
    if (debug()) {
      std::vector<unsigned long long> T((size_t)nwg * 8);
      HIP_TRY(hipMemcpy(T.data(), d_stamps.p, T.size() * 8, hipMemcpyDeviceToHost));
      double m[8] = {0};
      for (int w = 0; w < nwg; ++w)
        for (int i = 0; i < 8; ++i) m[i] += (double)T[(size_t)w * 8 + i] / nwg;
      const double ph = std::max(1.0, (double)ss[SS_PHASES]);
      fprintf(stderr,
              "[lincheck]   mean us per phase (s_memrealtime): barrier %.2f  X-hist %.2f  "
              "X-expand %.2f  prefix %.2f  process %.2f  publish %.2f  step-end %.2f (phases %.0f)\n",
              m[0] / ph / 100, m[1] / ph / 100, m[2] / ph / 100, m[3] / ph / 100, m[4] / ph / 100,
              m[5] / ph / 100, m[6] / ph / 100, ph);
    }
    if (flags[FL_ABORT]) {
      last_error = "search kernel watchdog: grid barrier timed out";
      return LC_E_INTERNAL;
    }
    if (flags[FL_SPILL]) {
      spill_clean = false;  // a full spill table may hold stale entries
      return 2;
    }
    if (flags[FL_OVERFLOW]) return 1;

    std::vector<int32_t> st(nh), fs(nh);
    std::vector<unsigned long long> ex(nh);
    HIP_TRY(hipMemcpy(st.data(), d_status.p, nh * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(fs.data(), d_fail.p, nh * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(ex.data(), d_explored.p, nh * 8, hipMemcpyDeviceToHost));
    for (int i = 0; i < nh; ++i) {
      const int h = bt.hs[i];
      status[h] = st[i];
      fail_step[h] = fs[i];
      explored[h] = ex[i];
    }
    add_stats(ss);
    return 0;
  }

  size_t device_budget() {
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return 0;
    return free_b;
  }

  // The slowest history of the run (device clock stamps at its dequeue and its end, 100 MHz):
  // stats 39..41 = its microseconds, RETURN steps and live width. Against the kernel time it
  // says how much of the launch is one history's dependent chain of steps.
  void note_chain(int h, unsigned long long t0, unsigned long long t1) {
    if (!t0 || t1 < t0) return;
    const double us = (double)(t1 - t0) / 100.0;
    if (us > stats[39]) stats[39] = us, stats[40] = enc.n_steps(h), stats[41] = enc.live_max[h];
  }

  // Counter histories on closure tables (ctab.hip): one launch, one history per 1024-thread
  // workgroup (dequeued heaviest first), their step streams already in d_dpack.
  int run_ctab(float* ms) {
    const int nc = (int)dense_c.size();
    if (!nc) return 0;
    const int n = enc.n_hist;
    HIP_TRY(d_cstats.ensure(16));
    ZeroSpans z;
    z.add((char*)d_dqueue.p + 12, 4);
    z.add(d_cstats.p, 16);
    z.add(d_dexpl.p, (size_t)std::max(n, 1) * 8);
    HIP_TRY(zero_spans(z, stream));
    CtabParams p{};
    p.n = nc;
    p.order = dp_ord + (dense_b.size() + dense_w.size() + dense_x.size() + dense_m.size());
    p.sbeg = dp_sbeg;
    p.nsteps = dp_nst;
    p.lmax = dp_lm;
    p.words = d_dwords.as<uint32_t>();
    p.stream = dp_stream;
    p.stream_words = dstream_words;
    p.queue = (int32_t*)((char*)d_dqueue.p + 12);
    p.status = d_dstatus.as<int32_t>();
    p.fail_step = d_dfail.as<int32_t>();
    p.explored = d_dexpl.as<unsigned long long>();
    p.stats = d_cstats.as<unsigned long long>();
    p.pipe = ctab_pipe;
    HIP_TRY(d_dstamps.ensure((size_t)std::max(n, 1) * 32));
    HIP_TRY(hipMemsetAsync(d_dstamps.p, 0, (size_t)std::max(n, 1) * 32, stream));
    p.stamps = d_dstamps.as<unsigned long long>();
    if (debug()) {
      HIP_TRY(d_dlhist.ensure(16 * 12 * 8));
      HIP_TRY(hipMemsetAsync(d_dlhist.p, 0, 16 * 12 * 8, stream));
      p.prof = d_dlhist.as<unsigned long long>();
    }
    // tile teams first (cooperative launches, each as many teams as fit the chip, the heaviest
    // histories first), then every other counter history one per workgroup; all write the same
    // result arrays
    std::vector<int32_t> singles;
    std::vector<std::vector<int>> team_launches;
    int n_team_hist = 0;
    {
      const int cap = std::min(ctab_team_max_wgs(), 256);
      std::vector<int> cand;
      for (int h : dense_c)
        if (ctab_T[h] > 0 && (1 << ctab_T[h]) <= cap) cand.push_back(h);
      std::stable_sort(cand.begin(), cand.end(), [&](int a, int b) { return dense_cost[a] > dense_cost[b]; });
      std::vector<char> in_team(n, 0);
      int used = cap;
      for (int h : cand) {
        const int g = 1 << ctab_T[h];
        if (used + g > cap) team_launches.emplace_back(), used = 0;
        team_launches.back().push_back(h);
        used += g;
        in_team[h] = 1;
        ++n_team_hist;
      }
      for (int h : dense_c)
        if (!in_team[h]) {
          if (enc.live_max[h] > CTAB_LMAX) ctab_grid[h] = 1;  // (no team: the grid kernel)
          else singles.push_back(h);
        }
    }
    HIP_TRY(hipEventRecord(ev0, stream));
    int team_wgs = 0;
    for (const std::vector<int>& hs : team_launches) {
      std::vector<int32_t> t_hist, t_base, t_anyoff, wg_team;
      std::vector<int8_t> t_bits;
      int anyw_acc = 0;
      for (int h : hs) {
        const int g = 1 << ctab_T[h];
        t_hist.push_back(h), t_base.push_back((int32_t)wg_team.size()), t_bits.push_back(ctab_T[h]);
        t_anyoff.push_back(anyw_acc);
        for (int r = 0; r < g; ++r) wg_team.push_back((int32_t)t_hist.size() - 1);
        anyw_acc += enc.n_steps(h) / 32 + 2;
      }
      team_wgs = std::max(team_wgs, (int)wg_team.size());
      const int nt = (int)t_hist.size(), g = (int)wg_team.size();
      int lbmax = 0;
      size_t anyw = 0;
      for (int k = 0; k < nt; ++k) {
        lbmax = std::max(lbmax, enc.live_max[t_hist[k]] - t_bits[k]);
        anyw = std::max(anyw, (size_t)t_anyoff[k] + enc.n_steps(t_hist[k]) / 32 + 2);
      }
      const int mshift = std::max(0, lbmax - CTAB_LO);
      const size_t meta = (size_t)g * 4 + (size_t)nt * 13 + 64;
      HIP_TRY(d_ctmeta.ensure(meta));
      std::vector<char> mb(meta, 0);
      memcpy(mb.data(), wg_team.data(), (size_t)g * 4);
      memcpy(mb.data() + (size_t)g * 4, t_base.data(), (size_t)nt * 4);
      memcpy(mb.data() + (size_t)g * 4 + nt * 4, t_hist.data(), (size_t)nt * 4);
      memcpy(mb.data() + (size_t)g * 4 + nt * 8, t_anyoff.data(), (size_t)nt * 4);
      memcpy(mb.data() + (size_t)g * 4 + nt * 12, t_bits.data(), (size_t)nt);
      HIP_TRY(hipMemcpyAsync(d_ctmeta.p, mb.data(), meta, hipMemcpyHostToDevice, stream));
      HIP_TRY(d_ctmirror.ensure(((size_t)g * CT_MRING) << mshift << 3));
      const size_t ctl_b = (size_t)g * 8 + anyw * 4 + (size_t)nt * 256 + 64;
      HIP_TRY(d_ctctl.ensure(ctl_b));
      HIP_TRY(hipMemsetAsync(d_ctctl.p, 0, ctl_b, stream));
      CtabTeamParams tp{};
      tp.c = p;
      tp.n_teams = nt;
      const char* mp = (const char*)d_ctmeta.p;
      tp.wg_team = (const int32_t*)mp;
      tp.team_base = (const int32_t*)(mp + (size_t)g * 4);
      tp.team_hist = (const int32_t*)(mp + (size_t)g * 4 + nt * 4);
      tp.team_any_off = (const int32_t*)(mp + (size_t)g * 4 + nt * 8);
      tp.team_bits = (const int8_t*)(mp + (size_t)g * 4 + nt * 12);
      char* cp = (char*)d_ctctl.p;
      tp.flags = (unsigned long long*)cp;
      tp.anyv = (uint32_t*)(cp + (size_t)g * 8);
      tp.ctl = (unsigned*)(cp + (size_t)g * 8 + anyw * 4);
      tp.abort = (int32_t*)(cp + (size_t)g * 8 + anyw * 4 + (size_t)nt * 256);
      tp.mirror = d_ctmirror.as<uint64_t>();
      tp.mshift = mshift;
      tp.watchdog = 2000000000ull;  // 20 s
      HIP_TRY(launch_ctab_team(tp, g, stream));
      int32_t ab = 0;
      HIP_TRY(hipMemcpyAsync(&ab, tp.abort, 4, hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipStreamSynchronize(stream));  // (the next launch reuses the team buffers)
      if (ab) {
        last_error = "counter tile-team watchdog fired";
        return LC_E_INTERNAL;
      }
      if (debug())
        for (int k = 0; k < nt; ++k)
          fprintf(stderr, "[lincheck] ctab team: h=%d width=%d steps=%d tiles=%d (lb %d)\n", t_hist[k],
                  enc.live_max[t_hist[k]], enc.n_steps(t_hist[k]), 1 << t_bits[k], enc.live_max[t_hist[k]] - t_bits[k]);
    }
    if (!singles.empty()) {
      // the single-workgroup kernel's queue: its histories, heaviest first (as build_dense ordered them)
      HIP_TRY(d_ctord.ensure(singles.size() * 4));
      std::vector<int32_t> so;
      std::vector<char> is_single(n, 0);
      for (int h : singles) is_single[h] = 1;
      const int32_t* hord = reinterpret_cast<const int32_t*>(hpack + o_ord) +
                            (dense_b.size() + dense_w.size() + dense_x.size() + dense_m.size());
      for (int i = 0; i < nc; ++i)
        if (is_single[hord[i]]) so.push_back(hord[i]);
      if (so.size() != singles.size()) so.assign(singles.begin(), singles.end());
      HIP_TRY(hipMemcpyAsync(d_ctord.p, so.data(), so.size() * 4, hipMemcpyHostToDevice, stream));
      CtabParams q = p;
      q.n = (int)so.size();
      q.order = d_ctord.as<int32_t>();
      HIP_TRY(launch_ctab(q, std::min((int)so.size(), dgrid_c), stream));
    }
    const int grid = team_wgs + std::min((int)singles.size(), dgrid_c);
    HIP_TRY(hipEventRecord(ev1, stream));
    const size_t need = (size_t)n * 32 + 16;
    if (hstage_bytes < need) {
      if (hstage) HIP_TRY(hipHostFree(hstage));
      hstage = nullptr;
      HIP_TRY(hipHostMalloc(&hstage, need, hipHostMallocDefault));
      hstage_bytes = need;
    }
    unsigned long long* const ex = hstage;
    int32_t* const st = reinterpret_cast<int32_t*>(hstage + n);
    int32_t* const fs = st + n;
    unsigned long long* const cs = reinterpret_cast<unsigned long long*>(fs + n);
    unsigned long long* const stamp = cs + 2;  // [n][2]
    HIP_TRY(hipMemcpyAsync(stamp, d_dstamps.p, (size_t)n * 16, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(ex, d_dexpl.p, (size_t)n * 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(st, d_dstatus.p, (size_t)n * 4, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(fs, d_dfail.p, (size_t)n * 4, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(cs, d_cstats.p, 16, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    float t = 0;
    HIP_TRY(hipEventElapsedTime(&t, ev0, ev1));
    *ms += t;
    double expl = 0;
    for (int h : dense_c) {
      if (ctab_grid[h]) continue;
      status[h] = st[h], fail_step[h] = fs[h], explored[h] = ex[h];
      expl += (double)ex[h];
      note_chain(h, stamp[2 * h], stamp[2 * h + 1]);
    }
    stats[1] += 1;
    stats[2] += (double)cs[1];
    stats[4] += (double)cs[0] + nc;  // frontier in = previous frontier out (+ the initial config)
    stats[6] += (double)cs[0];
    stats[12] += nc;
    stats[13] += t;
    stats[34] += nc - (int)std::count(ctab_grid.begin(), ctab_grid.end(), (char)1);
    stats[42] += (double)n_team_hist;
    stats[35] += t;
    stats[36] += (double)cs[0] + nc;
    stats[37] += (double)cs[0];
    stats[38] += expl;
    if (debug()) {
      fprintf(stderr, "[lincheck] ctab: %d counter histories on %d workgroups: %.3f ms, steps=%llu Fout=%llu\n", nc,
              grid, t, cs[1], cs[0]);
      std::vector<unsigned long long> T((size_t)n * 4);
      if (hipMemcpy(T.data(), d_dstamps.p, (size_t)n * 16, hipMemcpyDeviceToHost) == hipSuccess)
        for (int i = 0; i < nc && i < 4; ++i) {
          const int h = dense_c[i];
          fprintf(stderr, "[lincheck]   h=%d width=%d steps=%d: %.1f us (%.3f us/step)\n", h, enc.live_max[h],
                  enc.n_steps(h), (T[2 * h + 1] - T[2 * h]) / 100.0,
                  (T[2 * h + 1] - T[2 * h]) / 100.0 / std::max(1, enc.n_steps(h)));
        }
      // per wave: ring, words, decode+start, barrier cycles, super-layers, words closed, then (LC_DEBUG
      // word phases, serialised by their marks) hi sums + pulls, gates | closure, to the word, sweeps, pulls
      unsigned long long P[16 * 12];
      if (hipMemcpy(P, d_dlhist.p, sizeof(P), hipMemcpyDeviceToHost) == hipSuccess)
        for (int wv = 0; wv < 16; ++wv)
          if (const unsigned long long *q = P + 8 * wv, *r = P + 128 + 4 * wv; q[4])
            fprintf(stderr, "[lincheck]   wave %2d%s: per super-layer cycles: ring %.0f words %.0f decode+start %.0f "
                    "barrier %.0f; %.1f words (%llu super-layers)%s\n", wv, wv == 15 ? " (decoder)" : "",
                    q[0] / (double)q[4], q[1] / (double)q[4], q[2] / (double)q[4], q[3] / (double)q[4],
                    q[5] / (double)q[4], q[4],
                    r[1] ? ("; words phase (LC_CT_WORDPROF build): to-word " + std::to_string(r[1] / q[4]) + " sums " +
                            std::to_string((q[6] - r[3]) / q[4]) + " pulls " + std::to_string(r[3] / q[4]) + " gates " +
                            std::to_string(q[7] / q[4]) + " closure " + std::to_string(r[0] / q[4]))
                               .c_str()
                         : "");
    }
    return 0;
  }

  // lc_failure_configs for history 0 on the HBM tables: the frontier before
  // its failing RETURN t and every config's :last-op, from the tables themselves. Knossos's
  // per-config :last-op: config (m, v) of that frontier was either produced by step
  // t-1's closure linearizing t-1's returning op j (then that op is its last), or carried through
  // that return from (m + j, v) in step t-1's frontier (then it keeps that config's). The closure
  // produced (m + j, v) iff some state u of the FINAL step t-1 table at mask m steps to v under
  // j's op (T_j(B[m]): R at masks holding j, dense.hip §3.1), so the walk needs one word per
  // config per step back. A run stopped after step S - 1 (wide_stop = S) leaves the final tables of
  // steps S - 1 and S - 2 in place; deeper walks re-run to an earlier stop. Returns
  // LC_E_CONFIGS when the frontier outgrows the dump (the report is then unavailable).
  struct RepCfg {
    uint64_t mask;
    int state, last_step;  // state id (0 = nil); the step whose closure produced it (-1: initial)
  };
  // Failure report of a counter history on the HBM tables (wctr_pipe_kernel), as wide_report:
  // the run stopped before the failing RETURN t, step t - 1's table dumped through its returning
  // slot (wctr_dump_kernel: masks), each config's :last-op walked back. At step s a config of
  // mask m (without j_s) was produced by linearizing j_s last iff m is in step s's table and j_s's
  // requirement holds at m (CounterModel.step, counter.clj:102-127: S(m) = req - base, or j_s
  // unconstrained); else it was carried and held j_s already (m | j_s one step earlier).
  // out: (mask, value = init + base + S(mask), producing step) per config.
  struct CtrCfg {
    uint64_t mask;
    int64_t value;
    int last_step;
  };
  int wctr_report(int t_fail, std::vector<CtrCfg>& out) {
    out.clear();
    const int64_t init = enc.init_value;
    if (t_fail <= 0) {
      out.push_back({0ull, init, -1});
      return 0;
    }
    // per step (the decoder's state): live slots, j, base, j's delta / requirement / flags, and
    // the slot deltas (for the sums of the walk and the values)
    const std::vector<uint32_t>& ws = wide_streams[0];
    std::vector<uint64_t> live_s;
    std::vector<int> j_s;
    std::vector<int64_t> base_s;
    std::vector<std::array<int8_t, 64>> d_s;
    std::vector<int32_t> req_s;
    std::vector<uint32_t> fl_s;
    {
      std::array<int8_t, 64> d{};
      int32_t req[64] = {0};
      uint32_t fl[64];
      for (int k = 0; k < 64; ++k) fl[k] = CT_UNC;
      int64_t base = 0;
      size_t q = 0;
      while (q + 2 < ws.size() && (int)live_s.size() < t_fail) {
        if (!j_s.empty()) base += d_s.back()[j_s.back()];
        const uint64_t live = (uint64_t)ws[q] | ((uint64_t)ws[q + 1] << 31);
        const int j = (int)ws[q + 2];
        q += 3;
        for (; q + 1 < ws.size() && (ws[q] & DENSE_OPW); q += 2) {
          const uint32_t a = ws[q], b = ws[q + 1], sl = a & 63u;
          fl[sl] = (a >> 8) & 0xffu;
          d[sl] = (int8_t)(uint8_t)((a >> 16) & 0xffu);
          req[sl] = (int32_t)(b & 0x3fffffffu) - CTAB_REQ_BIAS;
        }
        live_s.push_back(live), j_s.push_back(j), base_s.push_back(base), d_s.push_back(d);
        req_s.push_back(req[j]), fl_s.push_back(fl[j]);
      }
      if ((int)live_s.size() < t_fail) {
        last_error = "failure configs: the wide counter stream ends before the failing step";
        return LC_E_INTERNAL;
      }
    }
    auto sum_of = [&](uint64_t m, int s) {
      int64_t v = 0;
      for (; m; m &= m - 1) v += d_s[s][__builtin_ctzll(m)];
      return v;
    };
    auto run_to = [&](int stop) -> int {
      wide_stop = stop;
      wide_ran = false;
      const int rc = run();
      wide_stop = -1;
      if (rc) return rc;
      if (!wide_ran) {
        last_error = "failure configs: the history did not run on the HBM tables";
        return LC_E_CONFIGS;
      }
      return 0;
    };
    int rc = run_to(t_fail);
    if (rc) return rc;
    const int64_t tw = (int64_t)1 << wide_last_hm;
    auto table_of = [&](int s) { return d_wtab.as<uint64_t>() + ((s & 1) ? tw : 0); };
    WideDumpParams dp{};
    dp.ranked = 1;
    dp.Hm = wide_last_hm;
    dp.split = 0;
    const int64_t cap = (int64_t)1 << 22;
    DevArray d_masks, d_cnt;
    HIP_TRY(d_masks.ensure((size_t)cap * 8));
    HIP_TRY(d_cnt.ensure(8));
    HIP_TRY(hipMemsetAsync(d_cnt.p, 0, 8, stream));
    dp.tab = table_of(t_fail - 1);
    dp.jp = j_s[t_fail - 1];
    dp.lv = live_s[t_fail - 1] & ~(1ull << dp.jp);
    dp.cap = cap;
    dp.masks = d_masks.as<uint64_t>();
    dp.count = d_cnt.as<unsigned long long>();
    HIP_TRY(launch_wctr_dump(dp, stream));
    unsigned long long cnt = 0;
    HIP_TRY(hipMemcpyAsync(&cnt, d_cnt.p, 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    if ((int64_t)cnt > cap) {
      last_error = "failure configs unavailable: the pre-failure frontier holds " + std::to_string(cnt) +
                   " configs, more than the dump's " + std::to_string(cap);
      return LC_E_CONFIGS;
    }
    std::vector<uint64_t> masks(cnt);
    HIP_TRY(hipMemcpy(masks.data(), d_masks.p, cnt * 8, hipMemcpyDeviceToHost));
    // the value: the ops returned before step t_fail plus the mask's (slot deltas as of step
    // t_fail - 1: a slot invoked at t_fail is fresh, never in the mask)
    const int64_t base_f = base_s[t_fail - 1] + d_s[t_fail - 1][j_s[t_fail - 1]];
    out.resize(cnt);
    std::vector<uint64_t> cur(cnt);
    std::vector<int> open;
    for (size_t i = 0; i < cnt; ++i) {
      out[i] = {masks[i], init + base_f + sum_of(masks[i], t_fail - 1), -2};
      cur[i] = masks[i];
      open.push_back((int)i);
    }
    int S = t_fail;
    DevArray d_hw, d_words;
    std::vector<uint64_t> hw, words;
    for (int st = t_fail - 1; st >= 0 && !open.empty(); --st) {
      if (st < S - 2) {
        S = st + 1;
        if ((rc = run_to(S))) return rc;
      }
      hw.resize(open.size());
      for (size_t k = 0; k < open.size(); ++k) hw[k] = cur[open[k]] >> 6;
      HIP_TRY(d_hw.ensure(hw.size() * 8));
      HIP_TRY(d_words.ensure(hw.size() * 8));
      HIP_TRY(hipMemcpy(d_hw.p, hw.data(), hw.size() * 8, hipMemcpyHostToDevice));
      dp.tab = table_of(st);
      HIP_TRY(launch_wide_gather(dp, d_hw.as<uint64_t>(), d_words.as<uint64_t>(), (int)hw.size(), stream));
      words.resize(hw.size());
      HIP_TRY(hipMemcpyAsync(words.data(), d_words.p, words.size() * 8, hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipStreamSynchronize(stream));
      const int j = j_s[st];
      std::vector<int> still;
      for (size_t k = 0; k < open.size(); ++k) {
        const int i = open[k];
        const bool in_tab = (words[k] >> (cur[i] & 63u)) & 1u;
        bool produced = in_tab;
        if (produced && !(fl_s[st] & CT_UNC))
          produced = !(fl_s[st] & CT_NEVER) && sum_of(cur[i], st) == (int64_t)req_s[st] - base_s[st];
        if (produced) out[i].last_step = st;
        else cur[i] |= 1ull << j, still.push_back(i);
      }
      open.swap(still);
    }
    if (!open.empty()) {
      last_error = "failure configs: a config's :last-op walk reached the history's start";
      return LC_E_CONFIGS;
    }
    return 0;
  }

  int wide_report(int t_fail, std::vector<RepCfg>& out) {
    out.clear();
    if (t_fail <= 0) {  // the failing RETURN is the first: its frontier is the initial config
      out.push_back({0ull, 0, -1});
      return 0;
    }
    // per step: live slots, returning slot, its op's (amask, bmask) (wide_sink's stream)
    const std::vector<uint32_t>& ws = wide_streams[0];
    std::vector<uint64_t> live_s;
    std::vector<int> j_s;
    std::vector<uint32_t> am_s, bm_s;
    {
      uint32_t am[64] = {0}, bm[64] = {0};
      size_t q = 0;
      while (q + 2 < ws.size() && (int)live_s.size() < t_fail) {
        const uint64_t live = (uint64_t)ws[q] | ((uint64_t)ws[q + 1] << 31);
        const int j = (int)ws[q + 2];
        q += 3;
        for (; q < ws.size() && (ws[q] & DENSE_OPW); ++q) {
          const uint32_t w = ws[q], sl = w & 63u;
          am[sl] = (w >> 8) & 0xffu, bm[sl] = (w >> 16) & 0xffu;
        }
        live_s.push_back(live), j_s.push_back(j), am_s.push_back(am[j]), bm_s.push_back(bm[j]);
      }
      if ((int)live_s.size() < t_fail) {
        last_error = "failure configs: the wide step stream ends before the failing step";
        return LC_E_INTERNAL;
      }
    }
    auto run_to = [&](int stop) -> int {
      wide_stop = stop;
      wide_ran = false;
      const int rc = run();
      wide_stop = -1;
      if (rc) return rc;
      if (!wide_ran) {
        last_error = "failure configs: the history did not run on the HBM tables";
        return LC_E_CONFIGS;
      }
      return 0;
    };
    int rc = run_to(t_fail);
    if (rc) return rc;
    const int64_t tw = (int64_t)1 << wide_last_hm;
    auto table_of = [&](int s) { return d_wtab.as<uint64_t>() + ((s & 1) ? tw : 0); };
    WideDumpParams d{};
    d.ranked = wide_last_ranked ? 1 : 0;
    d.Hm = wide_last_hm;
    d.split = wide_last_split;
    // the dump: the frontier before step t_fail
    const int64_t cap = (int64_t)1 << 22;
    DevArray d_masks, d_states, d_cnt;
    HIP_TRY(d_masks.ensure((size_t)cap * 8));
    HIP_TRY(d_states.ensure((size_t)cap));
    HIP_TRY(d_cnt.ensure(8));
    HIP_TRY(hipMemsetAsync(d_cnt.p, 0, 8, stream));
    d.tab = table_of(t_fail - 1);
    d.jp = j_s[t_fail - 1];
    d.lv = live_s[t_fail - 1] & ~(1ull << d.jp);
    d.cap = cap;
    d.masks = d_masks.as<uint64_t>();
    d.states = d_states.as<uint8_t>();
    d.count = d_cnt.as<unsigned long long>();
    HIP_TRY(launch_wide_dump(d, stream));
    unsigned long long cnt = 0;
    HIP_TRY(hipMemcpyAsync(&cnt, d_cnt.p, 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    if ((int64_t)cnt > cap) {
      last_error = "failure configs unavailable: the pre-failure frontier holds " + std::to_string(cnt) +
                   " configs, more than the dump's " + std::to_string(cap);
      return LC_E_CONFIGS;
    }
    std::vector<uint64_t> masks(cnt);
    std::vector<uint8_t> states(cnt);
    HIP_TRY(hipMemcpy(masks.data(), d_masks.p, cnt * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(states.data(), d_states.p, cnt, hipMemcpyDeviceToHost));
    out.resize(cnt);
    std::vector<uint64_t> cur(cnt);
    std::vector<int> open;
    for (size_t i = 0; i < cnt; ++i) {
      out[i] = {masks[i], (int)states[i], -2};
      cur[i] = masks[i];
      open.push_back((int)i);
    }
    // the walk, one step back per round: tables of steps S - 1, S - 2 are in place
    int S = t_fail;
    DevArray d_hw, d_words;
    std::vector<uint64_t> hw;
    std::vector<uint64_t> words;
    for (int st = t_fail - 1; st >= 0 && !open.empty(); --st) {
      if (st < S - 2) {
        S = st + 1;
        if ((rc = run_to(S))) return rc;
      }
      hw.resize(open.size());
      for (size_t k = 0; k < open.size(); ++k) hw[k] = cur[open[k]] >> 3;
      HIP_TRY(d_hw.ensure(hw.size() * 8));
      HIP_TRY(d_words.ensure(hw.size() * 8));
      HIP_TRY(hipMemcpy(d_hw.p, hw.data(), hw.size() * 8, hipMemcpyHostToDevice));
      d.tab = table_of(st);
      HIP_TRY(launch_wide_gather(d, d_hw.as<uint64_t>(), d_words.as<uint64_t>(), (int)hw.size(), stream));
      words.resize(hw.size());
      HIP_TRY(hipMemcpyAsync(words.data(), d_words.p, words.size() * 8, hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipStreamSynchronize(stream));
      const uint32_t am = am_s[st], bm = bm_s[st];
      const int j = j_s[st];
      std::vector<int> still;
      for (size_t k = 0; k < open.size(); ++k) {
        const int i = open[k];
        const int pm = (int)(cur[i] & 7u), v = out[i].state;
        auto has = [&](int u) { return (words[k] >> (8 * u + pm)) & 1u; };
        bool produced = false;  // CASRegister.step of j's op from some state at mask cur (a6)
        if (am == 0) {
          produced = false;  // names a value the register never holds
        } else if (bm) {
          const int dst = __builtin_ctz(bm);
          if (v == dst) {
            if (am == 0xffu) {  // write: from any state
              for (int u = 0; u < 8 && !produced; ++u) produced = has(u);
            } else {  // cas a -> dst
              produced = has(__builtin_ctz(am));
            }
          }
        } else if (am == 0xffu) {
          produced = has(v);  // read nil: every state stays
        } else {
          produced = v == __builtin_ctz(am) && has(v);  // read a
        }
        if (produced) out[i].last_step = st;
        else cur[i] |= 1ull << j, still.push_back(i);
      }
      open.swap(still);
    }
    if (!open.empty()) {
      last_error = "failure configs: a config's :last-op walk reached the history's start";
      return LC_E_CONFIGS;
    }
    return 0;
  }

  // The wide histories (tables in HBM), one persistent launch over the whole GPU, one history
  // after another. `ran` stays false when the two tables do not fit the device (they then take
  // the grid kernel, as before).
  // Counter histories on the HBM tables (wctr_pipe_kernel, §3.13): run_wide's launch with the
  // counter layout (2^(lmax - 6) words per table, no slabs) and the counter stream format.
  int run_wctr(float* ms, bool& ran) {
    const int nwd = (int)dense_wd.size();
    std::vector<int64_t> sbeg(nwd), aoff(nwd);
    std::vector<int32_t> nst(nwd);
    std::vector<int8_t> lmx(nwd);
    std::vector<uint32_t> words;
    int lmax = 0;
    int64_t abits = 0;
    for (int i = 0; i < nwd; ++i) {
      const int h = dense_wd[i];
      sbeg[i] = (int64_t)words.size();
      nst[i] = wide_stop >= 0 ? std::min(enc.n_steps(h), wide_stop) : enc.n_steps(h);
      lmx[i] = (int8_t)enc.live_max[h];
      lmax = std::max(lmax, (int)enc.live_max[h]);
      words.insert(words.end(), wide_streams[h].begin(), wide_streams[h].end());
      aoff[i] = abits, abits += nst[i] / 32 + 1;
    }
    words.resize(words.size() + 64, 0u);  // the decoder reads a 64-word window
    if (lmax > WCTR_LMAX) {
      last_error = "wide counter tables: a history wider than WCTR_LMAX";
      return LC_E_INTERNAL;
    }
    const int64_t tw = (int64_t)1 << std::max(0, lmax - 6);
    if (d_wtab.ensure((size_t)tw * 16) != hipSuccess) {
      (void)hipGetLastError();
      return 0;  // (the tables do not fit: the grid kernel)
    }
    int rc;
    if ((rc = upload(d_wstream, words))) return rc;
    if (!d_dwords.p) {
      std::vector<uint32_t> wl(1u << DENSE_WORD_BITS);
      dense_word_list(DENSE_WORD_BITS, wl.data());
      if ((rc = upload(d_dwords, wl))) return rc;
    }
    const size_t m_sb = (size_t)nwd * 8, m_ns = (size_t)nwd * 4;
    HIP_TRY(d_wmeta.ensure(2 * m_sb + m_ns + (size_t)nwd + 8));
    HIP_TRY(hipMemcpy(d_wmeta.p, sbeg.data(), m_sb, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy((char*)d_wmeta.p + m_sb, aoff.data(), m_sb, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy((char*)d_wmeta.p + 2 * m_sb, nst.data(), m_ns, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy((char*)d_wmeta.p + 2 * m_sb + m_ns, lmx.data(), (size_t)nwd, hipMemcpyHostToDevice));
    const size_t r_bytes = (size_t)nwd * 24 + 32 + (size_t)abits * 4;
    HIP_TRY(d_wres.ensure(r_bytes));
    HIP_TRY(d_wbar.ensure(wide_bar_bytes() + 8));
    HIP_TRY(hipMemsetAsync(d_wres.p, 0, r_bytes, stream));
    HIP_TRY(hipMemsetAsync(d_wbar.p, 0, wide_bar_bytes() + 8, stream));
    WideParams p{};
    p.n = nwd;
    p.sbeg = (const int64_t*)d_wmeta.p;
    p.anyv_off = (const int64_t*)((char*)d_wmeta.p + m_sb);
    p.nsteps = (const int32_t*)((char*)d_wmeta.p + 2 * m_sb);
    p.lmax = (const int8_t*)((char*)d_wmeta.p + 2 * m_sb + m_ns);
    p.pipe = 1;
    p.stream = d_wstream.as<uint32_t>();
    p.words = d_dwords.as<uint32_t>();
    p.tab = d_wtab.as<uint64_t>();
    p.tab_words = tw;
    unsigned long long* const rex = d_wres.as<unsigned long long>();
    p.explored = rex;
    p.any = rex + nwd;
    p.status = (int32_t*)(rex + 2 * nwd);
    p.fail_step = p.status + nwd;
    p.stats = (unsigned long long*)(p.fail_step + nwd);
    p.anyv = (uint32_t*)(p.stats + 4);
    p.bar = d_wbar.as<unsigned>();
    p.abort = (int32_t*)((char*)d_wbar.p + wide_bar_bytes());
    p.watchdog = (uint64_t)wide_watchdog_ms * 100000ull;
    const int gmax = wctr_grid_size();
    const int grid = wide_grid > 0 ? std::min(wide_grid, gmax) : gmax;
    if (grid < 1) {
      last_error = "wide counter kernel: no resident workgroups";
      return LC_E_INTERNAL;
    }
    HIP_TRY(hipEventRecord(ev0, stream));
    HIP_TRY(launch_wctr(p, grid, stream));
    HIP_TRY(hipEventRecord(ev1, stream));
    std::vector<unsigned long long> res((r_bytes + 7) / 8);
    int32_t ab = 0;
    HIP_TRY(hipMemcpyAsync(res.data(), d_wres.p, r_bytes, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(&ab, p.abort, 4, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    float t = 0;
    HIP_TRY(hipEventElapsedTime(&t, ev0, ev1));
    *ms += t;
    const int32_t* st = (const int32_t*)(res.data() + 2 * nwd);
    const int32_t* fs = st + nwd;
    const unsigned long long* ss = (const unsigned long long*)(fs + nwd);
    for (int i = 0; i < nwd; ++i) {
      const int h = dense_wd[i];
      const bool unfinished = st[i] != ST_VALID && st[i] != ST_INVALID;
      status[h] = ab && unfinished ? ST_ABORTED : st[i], fail_step[h] = fs[i], explored[h] = res[i];
    }
    stats[1] += 1;
    stats[2] += (double)ss[1];
    stats[12] += nwd;
    stats[13] += t;
    stats[31] += nwd;
    stats[32] += t;
    stats[34] += nwd;  // (counter histories on closure tables)
    stats[35] += t;
    stats[37] += (double)ss[0];
    for (int i = 0; i < nwd; ++i) stats[38] += (double)res[i];
    stats[43] = std::max(stats[43], 1.0);
    wide_last_ranked = true, wide_last_hm = std::max(0, lmax - 6), wide_last_split = 0;
    wide_ran = true;
    // algorithmic bytes as run_wide's: per step and live word its X, its pulls and its store
    double alg = 0;
    for (int i = 0; i < nwd; ++i) {
      const std::vector<uint32_t>& ws = wide_streams[dense_wd[i]];
      size_t q = 0;
      for (int tt = 0; tt < nst[i] && q + 2 < ws.size(); ++tt) {
        if (fs[i] >= 0 && tt > fs[i] + 1) break;
        const int n = __builtin_popcountll(((uint64_t)ws[q] | ((uint64_t)ws[q + 1] << 31)) >> 6);
        alg += std::ldexp(1.0, n) * (n / 2.0 + 2.0) * 8.0;
        q += 3;
        while (q < ws.size() && (ws[q] & DENSE_OPW)) ++q;
      }
    }
    stats[33] += alg;
    if (debug())
      fprintf(stderr, "[lincheck] wide counters: %d histories (tables of 2^%d words in HBM), %.3f ms, steps=%llu "
              "Fout=%llu; words visited %llu, stored nonzero %llu\n", nwd, std::max(0, lmax - 6), t, ss[1], ss[0],
              ss[2], ss[3]);
    ran = true;
    return 0;
  }

  int run_wide(float* ms, bool& ran) {
    if (model == LC_MODEL_COUNTER) return run_wctr(ms, ran);
    const int nwd = (int)dense_wd.size();
    std::vector<int64_t> sbeg(nwd);
    std::vector<int32_t> nst(nwd);
    std::vector<int8_t> lmx(nwd);
    std::vector<uint32_t> words;
    int lmax = 0;
    for (int i = 0; i < nwd; ++i) {
      const int h = dense_wd[i];
      sbeg[i] = (int64_t)words.size();
      nst[i] = wide_stop >= 0 ? std::min(enc.n_steps(h), wide_stop) : enc.n_steps(h);
      lmx[i] = (int8_t)enc.live_max[h];
      lmax = std::max(lmax, (int)enc.live_max[h]);
      words.insert(words.end(), wide_streams[h].begin(), wide_streams[h].end());
    }
    words.resize(words.size() + 64, 0u);  // the decoders read a 64-word window
    const int64_t tw = (int64_t)1 << std::max(0, lmax - 3);
    if (d_wtab.ensure((size_t)tw * 16) != hipSuccess) {
      (void)hipGetLastError();
      return 0;
    }
    int rc;
    if ((rc = upload(d_wstream, words))) return rc;
    if (!d_dwords.p) {
      std::vector<uint32_t> wl(1u << DENSE_WORD_BITS);
      dense_word_list(DENSE_WORD_BITS, wl.data());
      if ((rc = upload(d_dwords, wl))) return rc;
    }
    // meta: sbeg | anyv_off | nsteps | lmax; results: explored | any | status | fail | stats[4] |
    // the pipelined kernel's per-step bits
    std::vector<int64_t> aoff(nwd);
    int64_t abits = 0;
    for (int i = 0; i < nwd; ++i) aoff[i] = abits, abits += nst[i] / 32 + 1;
    const size_t m_sb = (size_t)nwd * 8, m_ns = (size_t)nwd * 4;
    HIP_TRY(d_wmeta.ensure(2 * m_sb + m_ns + (size_t)nwd + 8));
    HIP_TRY(hipMemcpy(d_wmeta.p, sbeg.data(), m_sb, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy((char*)d_wmeta.p + m_sb, aoff.data(), m_sb, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy((char*)d_wmeta.p + 2 * m_sb, nst.data(), m_ns, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy((char*)d_wmeta.p + 2 * m_sb + m_ns, lmx.data(), (size_t)nwd, hipMemcpyHostToDevice));
    const size_t r_bytes = (size_t)nwd * 24 + 32 + (size_t)abits * 4;
    HIP_TRY(d_wres.ensure(r_bytes));
    HIP_TRY(d_wbar.ensure(wide_bar_bytes() + 8));
    HIP_TRY(hipMemsetAsync(d_wres.p, 0, r_bytes, stream));
    HIP_TRY(hipMemsetAsync(d_wbar.p, 0, wide_bar_bytes() + 8, stream));
    if (wide_force_abort) {  // (tests: the path a fired watchdog takes, without waiting 20 s for one)
      static const int32_t one = 1;
      HIP_TRY(hipMemcpyAsync((char*)d_wbar.p + wide_bar_bytes(), &one, 4, hipMemcpyHostToDevice, stream));
    }
    WideParams p{};
    p.n = nwd;
    p.sbeg = (const int64_t*)d_wmeta.p;
    p.anyv_off = (const int64_t*)((char*)d_wmeta.p + m_sb);
    p.nsteps = (const int32_t*)((char*)d_wmeta.p + 2 * m_sb);
    p.lmax = (const int8_t*)((char*)d_wmeta.p + 2 * m_sb + m_ns);
    // (the one-step kernel's prefix tables stop at WIDE_NOPIPE_LMAX: wider tables always pipeline)
    // slabs (§3.10): a slab's local index is 32-bit, so past 2^32 words the top hi bits split
    // the table; LC_WIDE_SPLIT asks for more split bits (the rank split, tests), never leaving a
    // slab without a hi bit of its own
    const int hm = std::max(0, lmax - 3);
    p.split = std::min(std::max(wide_split, hm - WIDE_SLAB_BITS), std::max(0, hm - 1));
    p.pipe = wide_pipe || lmax > WIDE_NOPIPE_LMAX || p.split > 0 ? 1 : 0;
    wide_last_ranked = p.pipe != 0, wide_last_hm = hm, wide_last_split = p.split;
    p.stream = d_wstream.as<uint32_t>();
    p.words = d_dwords.as<uint32_t>();
    p.tab = d_wtab.as<uint64_t>();
    p.tab_words = tw;
    unsigned long long* const rex = d_wres.as<unsigned long long>();
    p.explored = rex;
    p.any = rex + nwd;
    p.status = (int32_t*)(rex + 2 * nwd);
    p.fail_step = p.status + nwd;
    p.stats = (unsigned long long*)(p.fail_step + nwd);
    p.anyv = (uint32_t*)(p.stats + 4);
    p.bar = d_wbar.as<unsigned>();
    p.abort = (int32_t*)((char*)d_wbar.p + wide_bar_bytes());
    p.watchdog = (uint64_t)wide_watchdog_ms * 100000ull;
    const int grid = wide_grid > 0 ? std::min(wide_grid, wide_grid_size(p.pipe)) : wide_grid_size(p.pipe);
    if (wide_stall_hist >= 0 && wide_stall_wg >= 0 && wide_stall_wg < grid) {
      p.stall = (int32_t*)((char*)d_wbar.p + wide_bar_bytes() + 4);  // (zeroed with the barrier)
      p.stall_hist = wide_stall_hist;
      p.stall_wg = wide_stall_wg;
    }
    if (grid < 1) {
      last_error = "wide kernel: no resident workgroups";
      return LC_E_INTERNAL;
    }
    HIP_TRY(hipEventRecord(ev0, stream));
    HIP_TRY(launch_wide(p, grid, stream));
    HIP_TRY(hipEventRecord(ev1, stream));
    std::vector<unsigned long long> res((r_bytes + 7) / 8);
    int32_t ab = 0;
    HIP_TRY(hipMemcpyAsync(res.data(), d_wres.p, r_bytes, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(&ab, p.abort, 4, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    float t = 0;
    HIP_TRY(hipEventElapsedTime(&t, ev0, ev1));
    *ms += t;
    const int32_t* st = (const int32_t*)(res.data() + 2 * nwd);
    const int32_t* fs = st + nwd;
    const unsigned long long* ss = (const unsigned long long*)(fs + nwd);
    // a watchdog abort (a grid barrier stalled: the cooperative grid assumes the whole
    // device, so another user of it can starve a workgroup) leaves the histories it had not
    // finished undecided (LC_H_ABORTED, :unknown); the finished ones and the rest of the call
    // keep their answers
    for (int i = 0; i < nwd; ++i) {
      const int h = dense_wd[i];
      const bool unfinished = st[i] != ST_VALID && st[i] != ST_INVALID;
      status[h] = ab && unfinished ? ST_ABORTED : st[i], fail_step[h] = fs[i], explored[h] = res[i];
    }
    if (ab && debug()) fprintf(stderr, "[lincheck] wide: grid barrier watchdog fired after %.1f ms\n", t);
    stats[1] += 1;
    stats[2] += (double)ss[1];
    stats[12] += nwd;  // (dense histories: LDS or HBM tables)
    stats[13] += t;
    stats[31] += nwd;
    stats[32] += t;
    stats[43] = std::max(stats[43], (double)(1 << p.split));
    // algorithmic bytes: every live word of every step read as X, pulled by its popcount-q
    // successors... counted from the reader: X (8 B) + popcount pulls (8 B each) + its store
    double alg = 0;
    for (int i = 0; i < nwd; ++i) {
      const int h = dense_wd[i];
      const std::vector<uint32_t>& ws = wide_streams[h];
      const int fs_i = fs[i];
      size_t q = 0;
      for (int tt = 0; tt < enc.n_steps(h) && q + 2 < ws.size(); ++tt) {
        if (fs_i >= 0 && tt > fs_i + 1) break;
        const int n = __builtin_popcountll(((uint64_t)ws[q] | ((uint64_t)ws[q + 1] << 31)) >> 3);
        alg += std::ldexp(1.0, n) * (n / 2.0 + 2.0) * 8.0;
        q += 3;
        while (q < ws.size() && (ws[q] & DENSE_OPW)) ++q;
      }
    }
    stats[33] += alg;
    if (debug())
      fprintf(stderr, "[lincheck] wide: %d histories (tables of 2^%d words in HBM), %.3f ms, steps=%llu Fout=%llu; "
              "words visited %llu, stored nonzero %llu (%.2f %%)\n", nwd, std::max(0, lmax - 3), t, ss[1], ss[0], ss[2],
              ss[3], 100.0 * (double)ss[3] / (double)std::max(1ull, ss[2]));
    ran = true;
    wide_ran = true;
    return 0;
  }

  int run_grid(const std::vector<int>& ids, float* ms) {
    make_batches(ids);
    for (size_t bi = 0; bi < batches.size(); ++bi) {
      const Batch& bt = batches[bi];
      int rc;
      for (int attempt = 0;; ++attempt) {
        rc = run_batch(bt, ms);
        if (rc <= 0) break;
        // grow what overflowed, bounded by max_configs and free HBM
        const size_t E = (size_t)entry_bytes();
        size_t need = 0;
        if (rc == 2) {
          spill_log += 2;
          need = ((size_t)nwg << spill_log) * 12;
        } else {
          ovf_cap *= 4;
          f_cap *= 2;
          need = 2ull * nwg * ovf_cap * E + 2ull * nwg * f_cap * E;
        }
        bool over_cfg = max_configs > 0 && (int64_t)nwg * f_cap > 4 * max_configs;
        if (over_cfg || need > device_budget() * 9 / 10 || attempt > 6 || spill_log > 24) {
          // capacity exhausted: the batch's histories are undecided (Knossos: :unknown)
          for (int h : bt.hs) status[h] = enc.err[h] ? ST_SKIP : ST_CAPACITY;
          rc = 0;
          break;
        }
        d_ovf.release();
        d_flist.release();
      }
      grown_ovf = std::max(grown_ovf, ovf_cap);
      grown_f = std::max(grown_f, f_cap);
      grown_spill = std::max(grown_spill, spill_log);
      if (rc < 0) return rc;
    }
    return 0;
  }

  int run() {
    HIP_TRY(hipSetDevice(device));
    status.assign(enc.n_hist, ST_SKIP);
    fail_step.assign(enc.n_hist, -1);
    explored.assign(enc.n_hist, 0);
    std::fill(stats, stats + LC_STATS_N, 0.0);
    for (int i = 0; i < 5; ++i) stats[20 + i] = phase_ms[i];
    float ms = 0;
    int rc = 0;
    std::vector<int> grid_ids;
    const bool keys = max_t == INT32_MAX && path == 1;
    const bool dense = max_t == INT32_MAX && path == 0 &&
                       (dense_b.size() + dense_w.size() + dense_x.size() + dense_m.size()) > 0;
    std::vector<char> done(enc.n_hist, 0);
    if (dense) {
      rc = run_dense(&ms);
      if (rc) return rc;
      for (int h : dense_b) done[h] = 1;
      for (int h : dense_w) done[h] = 1;
      for (int h : dense_x) done[h] = 1;
      for (int h : dense_m) done[h] = 1;
    }
    if (max_t == INT32_MAX && path == 0 && dense_on && !dense_c.empty()) {
      if ((rc = run_ctab(&ms))) return rc;
      for (int h : dense_c)
        if (!ctab_grid[h]) done[h] = 1;
    }
    if (max_t == INT32_MAX && path == 0 && dense_on && !dense_wd.empty()) {
      bool ran = false;
      if ((rc = run_wide(&ms, ran))) return rc;
      if (ran)
        for (int h : dense_wd) done[h] = 1;
    }
    if (keys) {
      if ((rc = upload_grid())) return rc;
      rc = run_keys(&ms);
      if (rc) return rc;
      for (int h = 0; h < enc.n_hist; ++h)
        if (status[h] == ST_CAPACITY) grid_ids.push_back(h);
    } else {
      for (int h = 0; h < enc.n_hist; ++h)
        if (!enc.err[h] && !done[h]) grid_ids.push_back(h);
    }
    if (!grid_ids.empty()) {
      if ((rc = upload_grid())) return rc;
      rc = run_grid(grid_ids, &ms);
      if (rc) return rc;
    }
    stats[0] = ms;
    stats[7] = 0;
    for (auto x : explored) stats[7] += (double)x;
    stats[8] = (double)entry_bytes();
    // bytes_alg = F_in*C + N_cand*(C+8) + F_out*C
    const double C = stats[8];
    stats[9] = stats[4] * C + stats[5] * (C + 8) + stats[6] * C;
    stats[10] = keys ? knwg : nwg;
    return 0;
  }

  void results(int8_t* v, int64_t* fi, int64_t* finv, int64_t* pok, int64_t* ex,
               int32_t* er) const {
    for (int h = 0; h < enc.n_hist; ++h) {
      int8_t valid = LC_UNKNOWN;
      int32_t code = enc.err[h];
      int64_t a = -1, b = -1, c = -1;
      switch (status[h]) {
        case ST_VALID: valid = LC_VALID; break;
        case ST_INVALID: {
          valid = LC_INVALID;
          const int64_t g = (int64_t)enc.step_off[h] + fail_step[h];
          a = enc.step_cmp_idx[g];
          b = enc.step_inv_idx[g];
          c = fail_step[h] > 0 ? enc.step_cmp_idx[g - 1] : -1;
          break;
        }
        case ST_CAPACITY: code = LC_H_CAPACITY; break;
        case ST_ABORTED: code = LC_H_ABORTED; break;
        case ST_MODEL: code = LC_H_MODEL; break;
        default: break;
      }
      if (v) v[h] = valid;
      if (fi) fi[h] = a;
      if (finv) finv[h] = b;
      if (pok) pok[h] = c;
      if (ex) ex[h] = (int64_t)explored[h];
      if (er) er[h] = code;
    }
  }
};

namespace {

// Encode histories and upload them into plan `reuse` (its device buffers, streams and events
// kept: lc_check's per-device cached plan) or into a new plan.
// `pre` (lc_check with n_gpus > 1): the whole batch already encoded once; this plan takes its
// histories `pre_hs` (hist_off = their entry offsets) by copying their encoded arrays
// (encoded_subset) and builds its dense step streams from them, with no second encode.
int plan_build(int device, int model, int64_t init_value, int n_hist, const int64_t* hist_off,
               const HistArrays& a, int64_t max_configs, lc_plan** out, std::string& msg,
               lc_plan* reuse = nullptr, bool keep_inv_arrays = false, const Encoded* pre = nullptr,
               const std::vector<int>* pre_hs = nullptr) {
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point t) {
    return std::chrono::duration<double, std::milli>(clk::now() - t).count();
  };
  std::unique_ptr<lc_plan> fresh(reuse ? nullptr : new lc_plan());
  lc_plan* const p = reuse ? reuse : fresh.get();
  p->device = device;
  p->model = model;
  p->max_configs = max_configs;
  p->max_t = INT32_MAX;
  p->report = false;
  p->keep_inv_arrays = keep_inv_arrays;
  std::fill(p->phase_ms, p->phase_ms + 5, 0.0);
  int rc = p->init_device();  // records phase_ms[1] (hipSetDevice) and [2] (streams, occupancy)
  auto t = clk::now();
  // the dense step streams are written by the encoder's workers as each history is encoded
  if (!rc) rc = p->dense_prepare(n_hist, hist_off);
  if (!rc && pre) {
    // the dense sink reads each history from the batch's encoding; the per-invocation arrays
    // of the histories it takes are not copied (as the single-shard encode leaves them out)
    const HistSink sink = [p](int h, const HistView& v) { return p->dense_sink(h, v); };
    encoded_subset(*pre, *pre_hs, p->enc, p->dense_on ? &sink : nullptr);
  } else if (!rc) {
    const HistSink sink = [p](int h, const HistView& v) { return p->dense_sink(h, v); };
    encode(model, init_value, n_hist, hist_off, a, p->enc, p->dense_on ? &sink : nullptr);
  }
  p->phase_ms[0] = ms_since(t);
  t = clk::now();
  if (!rc) rc = p->upload_encoded();  // records phase_ms[4] (build_dense)
  p->phase_ms[3] = ms_since(t) - p->phase_ms[4];
  if (debug() || getenv("LC_PHASES"))
    fprintf(stderr, "[lincheck] plan_create phases (ms): encode %.2f  hipSetDevice %.2f  streams+occupancy %.2f  "
            "uploads %.2f  build_dense %.2f\n", p->phase_ms[0], p->phase_ms[1], p->phase_ms[2], p->phase_ms[3],
            p->phase_ms[4]);
  if (rc) {
    msg = p->last_error;
    return rc;
  }
  *out = reuse ? reuse : fresh.release();
  return 0;
}

// lc_check's plan per device, reused from call to call (buffers grow to the largest check);
// guarded by the device mutex. Never destroyed by a static destructor (at process exit the HIP
// runtime may be torn down before this library's destructors run): lc_release frees them
// explicitly, and a process that never calls it leaves them to the OS.
lc_plan*& cached_slot(int dev) {
  static lc_plan* plans[64];
  return plans[dev & 63];
}
lc_plan* cached_plan(int dev) {
  lc_plan*& c = cached_slot(dev);
  if (!c) c = new lc_plan();
  return c;
}

bool valid_args(int model, int n_hist, const int64_t* hist_off, const int32_t* process,
                const int8_t* type, const int8_t* f, const int64_t* v0, const int64_t* v1,
                const int8_t* vflags, char* err, int32_t err_len) {
  if (model != LC_MODEL_CAS_REGISTER && model != LC_MODEL_COUNTER && model != LC_MODEL_LEADER) {
    set_err(err, err_len, "unknown model kind %d", model);
    return false;
  }
  if (n_hist < 0 || !hist_off) {
    set_err(err, err_len, "n_hist < 0 or hist_off NULL");
    return false;
  }
  for (int h = 0; h < n_hist; ++h)
    if (hist_off[h + 1] < hist_off[h]) {
      set_err(err, err_len, "hist_off not monotone at %d", h);
      return false;
    }
  if (hist_off[n_hist] > hist_off[0] && (!process || !type || !f || !v0 || !v1 || !vflags)) {
    set_err(err, err_len, "NULL history array");
    return false;
  }
  return true;
}

// Longest-processing-time split of histories over G shards by entry count: heaviest first,
// each to the least-loaded shard (lowest index on ties); deterministic. Host only.
void lpt_shards(int n_hist, const int64_t* off, int G, int32_t* out_shard) {
  std::vector<int> order(n_hist);
  for (int h = 0; h < n_hist; ++h) order[h] = h;
  std::stable_sort(order.begin(), order.end(),
                   [&](int x, int y) { return off[x + 1] - off[x] > off[y + 1] - off[y]; });
  std::vector<int64_t> load(G, 0);
  for (int h : order) {
    const int g = (int)(std::min_element(load.begin(), load.end()) - load.begin());
    out_shard[h] = g;
    load[g] += off[h + 1] - off[h];
  }
}

// Modeled time (us) of each history's dependent chain of RETURN steps on the dense kernels,
// with the team planner's step models (lc_plan::est_*; MI355X LC_DEBUG fits) as the history
// would run in a shard of a few hundred keys (a chain plan): WAVE (width <= 11) 7.9 us per
// step, MID (12..14) 4.9 + 0.0016 * 2^(L-3), BLOCK (15..17) 4.67 + 0.00266 * 2^(L-3), wider a
// tile team of 16-slot tiles, 1.59 + 0.0043 * 2^(min(L,16)-3) + [L > 16] (3.87 + 1.57 (L-16)).
// Width 25..WIDE_LMAX (the HBM tables, a whole GPU each, one after another): per step ~7 us of
// grid barriers plus its 2^n live words' X, pulls and store (8 B each) at ~1.3 TB/s (r3t/r3u:
// 55 us per step at width 27, 190 at width 30 on the crash ramp). Counter histories and
// histories no table takes (the grid kernel) cost their entry count (one unit per entry). Host
// only.
void history_costs_of(const Encoded& enc, const int64_t* off, std::vector<double>& cost) {
  const int n_hist = enc.n_hist;
  cost.assign(n_hist, 0.0);
  if (enc.model != LC_MODEL_CAS_REGISTER) {
    for (int h = 0; h < n_hist; ++h) cost[h] = (double)(off[h + 1] - off[h]);
    return;
  }
  for (int h = 0; h < n_hist; ++h) {
    const int lw = enc.live_max[h];
    if (enc.err[h] || enc.n_states[h] > DENSE_MAX_STATES || lw > WIDE_LMAX) {
      cost[h] = (double)(off[h + 1] - off[h]);
      continue;
    }
    uint64_t live = 0;
    double t = 0;
    if (lw > DENSE_WIDE_LMAX) {  // the HBM tables
      for (int64_t g = enc.step_off[h]; g < enc.step_off[h + 1]; ++g) {
        if (g > enc.step_off[h]) live &= ~(1ull << enc.step_slot[g - 1]);
        for (int64_t q = enc.inv_off[g]; q < enc.inv_off[g + 1]; ++q) live |= 1ull << enc.inv_slot[q];
        const int n = __builtin_popcountll(live >> 3);
        t += 7.0 + std::ldexp(1.0, n) * (n / 2.0 + 2.0) * 8.0 / 1.3e6;
      }
      cost[h] = t;
      continue;
    }
    for (int64_t g = enc.step_off[h]; g < enc.step_off[h + 1]; ++g) {
      if (g > enc.step_off[h]) live &= ~(1ull << enc.step_slot[g - 1]);
      for (int64_t q = enc.inv_off[g]; q < enc.inv_off[g + 1]; ++q) live |= 1ull << enc.inv_slot[q];
      const int L = live ? 64 - __builtin_clzll(live) : 0;
      const double w = std::ldexp(1.0, std::max(0, std::min(L, 16) - 3));
      t += lw <= DENSE_WAVE_LMAX ? 7.9
           : lw <= 14            ? 4.9 + 0.0016 * w
           : lw <= DENSE_LMAX    ? 4.67 + 0.00266 * std::ldexp(1.0, std::max(0, L - 3))
                                 : 1.59 + 0.0043 * w + (L > 16 ? 3.87 + 1.57 * (L - 16) : 0.0);
    }
    cost[h] = t;
  }
}
void history_costs(int model, int64_t init_value, int n_hist, const int64_t* off, const HistArrays& a,
                   std::vector<double>& cost) {
  Encoded enc;
  if (model == LC_MODEL_CAS_REGISTER) encode(model, init_value, n_hist, off, a, enc);
  else enc.model = model, enc.n_hist = n_hist;
  history_costs_of(enc, off, cost);
}

// LPT over G shards by cost: heaviest first, each to the least-loaded shard (lowest index on
// ties); deterministic. Host only.
void lpt_by_cost(int n_hist, const std::vector<double>& cost, int G, int32_t* out_shard) {
  std::vector<int> order(n_hist);
  for (int h = 0; h < n_hist; ++h) order[h] = h;
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return cost[x] > cost[y]; });
  std::vector<double> load(G, 0.0);
  for (int h : order) {
    const int g = (int)(std::min_element(load.begin(), load.end()) - load.begin());
    out_shard[h] = g;
    load[g] += cost[h];
  }
}

// state of the most recent lc_check on this thread (for lc_failure_configs)
struct LastCheck {
  int model = 0, device = 0;
  int64_t init_value = 0;
  std::vector<int64_t> off, index, v0, v1;
  std::vector<int32_t> process;
  std::vector<int8_t> type, f, vflags;
  std::vector<int8_t> valid;
  bool have = false;
};
thread_local LastCheck g_last;

}  // namespace

extern "C" {

int32_t lc_abi_version(void) { return LC_ABI_VERSION; }

int32_t lc_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int32_t lc_plan_create(int32_t device, int32_t model_kind, int64_t init_value, int32_t n_hist,
                       const int64_t* hist_off, const int64_t* index, const int32_t* process,
                       const int8_t* type, const int8_t* f, const int64_t* v0, const int64_t* v1,
                       const int8_t* vflags, int64_t max_configs, lc_plan** out, char* err,
                       int32_t err_len) {
  if (!out) return LC_E_ARG;
  *out = nullptr;
  if (!valid_args(model_kind, n_hist, hist_off, process, type, f, v0, v1, vflags, err, err_len))
    return LC_E_ARG;
  const auto t0 = std::chrono::steady_clock::now();
  // the first HIP call of the process initialises the runtime: counted with hipSetDevice
  if (lc_device_count() <= device || device < 0) {
    set_err(err, err_len, "no HIP device %d (the checker has no CPU fallback)", device);
    return LC_E_DEVICE;
  }
  const double count_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  std::lock_guard<std::mutex> g(device_mutex(device));
  HistArrays a{hist_off[n_hist] - hist_off[0], index, process, type, f, v0, v1, vflags};
  std::string msg;
  int rc = plan_build(device, model_kind, init_value, n_hist, hist_off, a, max_configs, out, msg);
  if (rc) set_err(err, err_len, "%s", msg.c_str());
  else (*out)->phase_ms[1] += count_ms;
  return rc;
}

int32_t lc_plan_run(lc_plan* p, char* err, int32_t err_len) {
  if (!p) return LC_E_ARG;
  std::lock_guard<std::mutex> g(device_mutex(p->device));
  int rc = p->run();
  if (rc) set_err(err, err_len, "%s", p->last_error.c_str());
  return rc;
}

int32_t lc_plan_results(lc_plan* p, int8_t* out_valid, int64_t* out_fail_idx, int64_t* out_fail_inv,
                        int64_t* out_prev_ok, int64_t* out_explored, int32_t* out_err) {
  if (!p) return LC_E_ARG;
  p->results(out_valid, out_fail_idx, out_fail_inv, out_prev_ok, out_explored, out_err);
  return 0;
}

int32_t lc_plan_stats(lc_plan* p, double* stats, int32_t n) {
  if (!p || !stats) return LC_E_ARG;
  for (int i = 0; i < n && i < LC_STATS_N; ++i) stats[i] = p->stats[i];
  for (int i = 20; i < 25 && i < n; ++i) stats[i] = p->phase_ms[i - 20];  // creation phases, run or not
  return 0;
}

void lc_plan_destroy(lc_plan* p) {
  if (!p) return;
  std::lock_guard<std::mutex> g(device_mutex(p->device));
  hipSetDevice(p->device);
  delete p;
}

int32_t lc_check(int32_t model_kind, int64_t init_value, int32_t n_hist, const int64_t* hist_off,
                 const int64_t* index, const int32_t* process, const int8_t* type, const int8_t* f,
                 const int64_t* v0, const int64_t* v1, const int8_t* vflags, int32_t n_gpus,
                 int64_t max_configs, int32_t flags, int8_t* out_valid, int64_t* out_fail_idx,
                 int64_t* out_fail_inv, int64_t* out_prev_ok, int64_t* out_explored,
                 int32_t* out_err, char* err, int32_t err_len) {
  if (!valid_args(model_kind, n_hist, hist_off, process, type, f, v0, v1, vflags, err, err_len))
    return LC_E_ARG;
  const int ndev = lc_device_count();
  if (ndev <= 0) {
    set_err(err, err_len, "no HIP device visible (the checker has no CPU fallback)");
    return LC_E_DEVICE;
  }
  // shards: one per requested GPU; more shards than visible devices are multiplexed over
  // them (shard g on device g % ndev, serialised by the device mutex; results do not change)
  int G = n_gpus <= 0 ? ndev : n_gpus;
  G = std::max(1, std::min(G, std::max(1, n_hist)));

  // the caller's arrays, rebased to the first history (no copy)
  const int64_t b0 = hist_off[0];
  std::vector<int64_t> off0(hist_off, hist_off + n_hist + 1);
  for (auto& x : off0) x -= b0;
  auto at = [&](auto* ptr) { return ptr ? ptr + b0 : ptr; };
  const int64_t* cidx = at(index);
  const int32_t* cpr = at(process);
  const int8_t *cty = at(type), *cf = at(f), *cvf = at(vflags);
  const int64_t *cv0 = at(v0), *cv1 = at(v1);
  g_last = LastCheck();

  // bounds pre-filter for counters (sound rejection only; never changes a verdict's index)
  if (model_kind == LC_MODEL_COUNTER && (flags & LC_FLAG_BOUNDS_ONLY)) {
    std::vector<int8_t> bounds_ok(n_hist, 1);
    std::vector<int64_t> bounds_bad(n_hist, -1);
    int rc = lc_counter_bounds(init_value, n_hist, off0.data(), cidx, cpr, cty, cf, cv0, cv1, cvf,
                               bounds_ok.data(), bounds_bad.data(), err, err_len);
    if (rc) return rc;
    for (int h = 0; h < n_hist; ++h) {
      if (out_valid) out_valid[h] = bounds_ok[h] ? LC_UNKNOWN : LC_INVALID;
      if (out_fail_idx) out_fail_idx[h] = bounds_bad[h];
      if (out_fail_inv) out_fail_inv[h] = -1;
      if (out_prev_ok) out_prev_ok[h] = -1;
      if (out_explored) out_explored[h] = 0;
      if (out_err) out_err[h] = 0;
    }
    return 0;
  }

  // shard histories over devices: longest-processing-time on each history's modeled chain time
  // (lc_shard_histories_by_cost; a shard lasts as long as its slowest chains)
  std::vector<std::vector<int>> shard(G);
  // n_gpus > 1: the batch is encoded ONCE (its modeled costs split it; each shard's plan then
  // copies its histories' encoded arrays instead of gathering and re-encoding the raw ones)
  Encoded all;
  if (G > 1) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    encode(model_kind, init_value, n_hist, off0.data(), HistArrays{off0[n_hist], cidx, cpr, cty, cf, cv0, cv1, cvf},
           all);
    const auto t1 = clk::now();
    std::vector<int32_t> of(n_hist);
    std::vector<double> cost;
    history_costs_of(all, off0.data(), cost);
    lpt_by_cost(n_hist, cost, G, of.data());
    if (debug() || getenv("LC_PHASES"))
      fprintf(stderr, "[lincheck] lc_check(n_gpus=%d): one encode %.2f ms, cost split %.2f ms\n", G,
              std::chrono::duration<double, std::milli>(t1 - t0).count(),
              std::chrono::duration<double, std::milli>(clk::now() - t1).count());
    for (int h = 0; h < n_hist; ++h) shard[of[h]].push_back(h);
  } else {
    for (int h = 0; h < n_hist; ++h) shard[0].push_back(h);
  }
  std::vector<int> rcs(G, 0);
  std::vector<std::string> msgs(G);
  std::vector<int8_t> verdict(n_hist, LC_UNKNOWN);
  auto work = [&](int g) {
    const std::vector<int>& hs = shard[g];
    if (hs.empty()) return;
    // one shard: the caller's arrays in place; several: this shard's histories of the batch
    // encoded once above (only their entry offsets here, for the dense streams' layout)
    std::vector<int64_t> off(1, 0);
    const HistArrays a{off0[n_hist], cidx, cpr, cty, cf, cv0, cv1, cvf};
    const int64_t* offp = off0.data();
    if (G > 1) {
      for (int h : hs) off.push_back(off.back() + off0[h + 1] - off0[h]);
      offp = off.data();
    }
    const int dev = g % ndev;
    std::lock_guard<std::mutex> lk(device_mutex(dev));
    lc_plan* p = nullptr;
    int rc = plan_build(dev, model_kind, init_value, (int)hs.size(), offp, a, max_configs, &p, msgs[g],
                        cached_plan(dev), false, G > 1 ? &all : nullptr, &hs);
    if (!rc) {
      rc = p->run();
      if (rc) msgs[g] = p->last_error;
    }
    if (!rc) {
      const size_t m = hs.size();
      std::vector<int8_t> v(m);
      std::vector<int64_t> fi(m), fv(m), po(m), ex(m);
      std::vector<int32_t> er(m);
      p->results(v.data(), fi.data(), fv.data(), po.data(), ex.data(), er.data());
      for (size_t k = 0; k < m; ++k) {
        const int h = hs[k];
        verdict[h] = v[k];
        if (out_valid) out_valid[h] = v[k];
        if (out_fail_idx) out_fail_idx[h] = fi[k];
        if (out_fail_inv) out_fail_inv[h] = fv[k];
        if (out_prev_ok) out_prev_ok[h] = po[k];
        if (out_explored) out_explored[h] = ex[k];
        if (out_err) out_err[h] = er[k];
      }
    }
    rcs[g] = rc;  // (p is the device's cached plan: kept for the next call)
  };
  if (G == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int g = 0; g < G; ++g) th.emplace_back(work, g);
    for (auto& t : th) t.join();
  }
  for (int g = 0; g < G; ++g)
    if (rcs[g]) {
      set_err(err, err_len, "shard %d (device %d): %s", g, g % ndev, msgs[g].c_str());
      return rcs[g];
    }
  // keep the invalid histories (only) for lc_failure_configs; the others get empty runs
  g_last.model = model_kind;
  g_last.init_value = init_value;
  g_last.off.assign(n_hist + 1, 0);
  for (int h = 0; h < n_hist; ++h)
    g_last.off[h + 1] = g_last.off[h] + (verdict[h] == LC_INVALID ? off0[h + 1] - off0[h] : 0);
  const int64_t nk = g_last.off[n_hist];
  g_last.index.resize(nk), g_last.process.resize(nk), g_last.type.resize(nk), g_last.f.resize(nk);
  g_last.v0.resize(nk), g_last.v1.resize(nk), g_last.vflags.resize(nk);
  for (int h = 0; h < n_hist; ++h) {
    if (verdict[h] != LC_INVALID) continue;
    const int64_t sb = off0[h], m = off0[h + 1] - sb, o = g_last.off[h];
    for (int64_t i = 0; i < m; ++i) g_last.index[o + i] = cidx ? cidx[sb + i] : i;  // :index or position
    std::copy_n(cpr + sb, m, g_last.process.data() + o);
    std::copy_n(cty + sb, m, g_last.type.data() + o);
    std::copy_n(cf + sb, m, g_last.f.data() + o);
    std::copy_n(cv0 + sb, m, g_last.v0.data() + o);
    std::copy_n(cv1 + sb, m, g_last.v1.data() + o);
    std::copy_n(cvf + sb, m, g_last.vflags.data() + o);
  }
  g_last.valid = verdict;
  g_last.have = true;
  return 0;
}

int32_t lc_release(int32_t device) {
  const int ndev = lc_device_count();
  for (int d = 0; d < std::min(ndev, 64); ++d) {
    if (device >= 0 && d != device) continue;
    std::lock_guard<std::mutex> lk(device_mutex(d));
    lc_plan*& c = cached_slot(d);
    if (!c) continue;
    hipSetDevice(d);
    hipDeviceSynchronize();
    delete c;
    c = nullptr;
  }
  // the calling thread's encoder buffers (kept between calls) go too
  encode_trim();
  return 0;
}

int32_t lc_check_stats(int32_t device, double* stats, int32_t n) {
  if (device < 0 || device >= 64 || !stats) return LC_E_ARG;
  std::lock_guard<std::mutex> lk(device_mutex(device));
  lc_plan* c = cached_slot(device);
  if (!c) return LC_E_ARG;
  return lc_plan_stats(c, stats, n);
}

int32_t lc_shard_histories_by_cost(int32_t model_kind, int64_t init_value, int32_t n_hist,
                                   const int64_t* hist_off, const int64_t* index, const int32_t* process,
                                   const int8_t* type, const int8_t* f, const int64_t* v0, const int64_t* v1,
                                   const int8_t* vflags, int32_t n_shards, int32_t* out_shard,
                                   double* out_cost_us, char* err, int32_t err_len) {
  if (n_shards < 1 || (n_hist > 0 && !out_shard)) {
    set_err(err, err_len, "n_shards < 1 or out_shard NULL");
    return LC_E_ARG;
  }
  if (!valid_args(model_kind, n_hist, hist_off, process, type, f, v0, v1, vflags, err, err_len))
    return LC_E_ARG;
  const int64_t b0 = hist_off[0];
  std::vector<int64_t> off0(hist_off, hist_off + n_hist + 1);
  for (auto& x : off0) x -= b0;
  auto at = [&](auto* ptr) { return ptr ? ptr + b0 : ptr; };
  HistArrays a{off0[n_hist], at(index), at(process), at(type), at(f), at(v0), at(v1), at(vflags)};
  std::vector<double> cost;
  history_costs(model_kind, init_value, n_hist, off0.data(), a, cost);
  lpt_by_cost(n_hist, cost, n_shards, out_shard);
  if (out_cost_us) std::copy(cost.begin(), cost.end(), out_cost_us);
  return 0;
}

int32_t lc_shard_histories(int32_t n_hist, const int64_t* hist_off, int32_t n_shards, int32_t* out_shard) {
  if (n_hist < 0 || n_shards < 1 || (n_hist > 0 && (!hist_off || !out_shard))) return LC_E_ARG;
  for (int h = 0; h < n_hist; ++h)
    if (hist_off[h + 1] < hist_off[h]) return LC_E_ARG;
  lpt_shards(n_hist, hist_off, n_shards, out_shard);
  return 0;
}

int32_t lc_failure_configs(int32_t hist, int32_t k, int64_t* state, int8_t* is_nil,
                           int64_t* linearized, int32_t* n_lin, int64_t* last_op, int32_t* n_out,
                           int64_t* pending, int32_t* n_pending, int64_t* out_last_op, char* err,
                           int32_t err_len) {
  const LastCheck& L = g_last;
  if (!L.have || hist < 0 || hist + 1 >= (int)L.off.size()) {
    set_err(err, err_len, "no checked history %d on this thread", hist);
    return LC_E_ARG;
  }
  if (L.valid[hist] != LC_INVALID) {  // (only invalid histories are kept)
    set_err(err, err_len, "history %d is not invalid", hist);
    return LC_E_ARG;
  }
  const int64_t b = L.off[hist], e = L.off[hist + 1];
  int64_t off[2] = {0, e - b};
  HistArrays a{e - b, L.index.data() + b, L.process.data() + b, L.type.data() + b, L.f.data() + b,
               L.v0.data() + b, L.v1.data() + b, L.vflags.data() + b};
  std::lock_guard<std::mutex> lk(device_mutex(0));
  lc_plan* p = nullptr;
  std::string msg;
  int rc = plan_build(0, L.model, L.init_value, 1, off, a, 0, &p, msg, nullptr, true);
  if (rc) {
    set_err(err, err_len, "%s", msg.c_str());
    return rc;
  }
  std::unique_ptr<lc_plan> hold(p);
  rc = p->run();  // find the failing step
  if (rc) {
    set_err(err, err_len, "%s", p->last_error.c_str());
    return rc;
  }
  if (p->status[0] != ST_INVALID) {
    set_err(err, err_len, "history %d is not invalid", hist);
    return LC_E_ARG;
  }
  const int t_fail = p->fail_step[0];
  // a history wider than the LDS tables was decided on the HBM tables (wide.hip), which keep no
  // per-config :last-op; its grid-kernel re-run can take minutes at these widths (the crash
  // ramp's width-27 history did not finish in 3), so the report stops here unless asked
  // (LC_WIDE_CONFIGS=1). The verdict, failing op and explored count stand.
  const Encoded& en = p->enc;
  // the pending ops at the failing RETURN, by slot (replayed slot assignments)
  int64_t slot_inv[64];
  for (int s = 0; s < 64; ++s) slot_inv[s] = -1;
  for (int t = 0; t <= t_fail; ++t) {
    const int64_t g = en.step_off[0] + t;
    if (t > 0) slot_inv[en.step_slot[g - 1]] = -1;
    for (int64_t q = en.inv_off[g]; q < en.inv_off[g + 1]; ++q) slot_inv[en.inv_slot[q]] = en.inv_index[q];
  }
  auto last_of_step = [&](int s) -> int64_t {  // :ok completion of step s's returning op
    return s >= 0 ? en.step_cmp_idx[en.step_off[0] + s] : -1;
  };
  // emit: configs (state id, slot mask, producing step) sorted by (state, mask), the first k
  auto emit = [&](std::vector<lc_plan::RepCfg>& all, int mask_bits) -> int32_t {
    std::sort(all.begin(), all.end(), [](const lc_plan::RepCfg& x, const lc_plan::RepCfg& y) {
      return x.state != y.state ? x.state < y.state : x.mask < y.mask;
    });
    int np = 0;
    for (int s = 0; s < 64; ++s)
      if (slot_inv[s] >= 0) {
        if (pending) pending[np] = slot_inv[s];
        ++np;
      }
    if (n_pending) *n_pending = np;
    int64_t newest = -1;
    for (const auto& c : all) newest = std::max(newest, last_of_step(c.last_step));
    if (out_last_op) *out_last_op = newest;
    int out = 0;
    for (const auto& c : all) {
      if (out >= k) break;
      int64_t val = 0;
      int8_t nil = 0;
      if (c.state == 0) nil = 1;
      else val = en.state_val[en.state_off[0] + c.state - 1];
      int nl = 0;
      for (int s = 0; s < mask_bits; ++s)
        if ((c.mask >> s) & 1) {
          if (linearized) linearized[(size_t)out * 64 + nl] = slot_inv[s];
          ++nl;
        }
      if (state) state[out] = val;
      if (is_nil) is_nil[out] = nil;
      if (n_lin) n_lin[out] = nl;
      if (last_op) last_op[out] = last_of_step(c.last_step);
      ++out;
    }
    if (n_out) *n_out = out;
    return 0;
  };
  // a history wider than the LDS tables was decided on the HBM tables (wide.hip): its report
  // comes from the tables (a stopped re-run, the frontier dumped, each config's :last-op walked
  // back), not from the grid kernel, which takes minutes at these widths (LC_WIDE_CONFIGS=0
  // forces the grid-kernel re-run, for tests)
  // (the route is the check's own: LC_WIDE_MINW sends narrower histories there too, for tests)
  if (p->enc.model == LC_MODEL_CAS_REGISTER && !p->dense_wd.empty() &&
      !(getenv("LC_WIDE_CONFIGS") && atoi(getenv("LC_WIDE_CONFIGS")) == 0)) {
    std::vector<lc_plan::RepCfg> all;
    rc = p->wide_report(t_fail, all);
    if (rc) {
      set_err(err, err_len, "%s", p->last_error.c_str());
      return rc;
    }
    return emit(all, WIDE_LMAX);
  }
  // a counter decided on the HBM counter tables (wctr_pipe_kernel): the same, from those tables
  if (p->enc.model == LC_MODEL_COUNTER && !p->dense_wd.empty() &&
      !(getenv("LC_WIDE_CONFIGS") && atoi(getenv("LC_WIDE_CONFIGS")) == 0)) {
    std::vector<lc_plan::CtrCfg> all;
    rc = p->wctr_report(t_fail, all);
    if (rc) {
      set_err(err, err_len, "%s", p->last_error.c_str());
      return rc;
    }
    std::sort(all.begin(), all.end(), [](const lc_plan::CtrCfg& x, const lc_plan::CtrCfg& y) { return x.mask < y.mask; });
    {
      std::vector<lc_plan::RepCfg> none;
      emit(none, 0);  // the pending ops and an empty output, then the configs below
    }
    int64_t newest = -1;
    for (const auto& c : all) newest = std::max(newest, last_of_step(c.last_step));
    if (out_last_op) *out_last_op = newest;
    int out = 0;
    for (const auto& c : all) {
      if (out >= k) break;
      int nl = 0;
      for (int s = 0; s < 64; ++s)
        if ((c.mask >> s) & 1) {
          if (linearized) linearized[(size_t)out * 64 + nl] = slot_inv[s];
          ++nl;
        }
      if (state) state[out] = c.value;
      if (is_nil) is_nil[out] = 0;
      if (n_lin) n_lin[out] = nl;
      if (last_op) last_op[out] = last_of_step(c.last_step);
      ++out;
    }
    if (n_out) *n_out = out;
    return 0;
  }
  // stop before the failing RETURN: the frontier it saw stays in flist (the grid kernel: the
  // dense tables keep no config lists), each config tagged with the step that emitted it. A key
  // with no room for the 6-bit tag, or a tagged frontier (a config once per route) that outgrows
  // the lists, falls back to the untagged dump: the same configs, each with the
  // previous :ok op as its :last-op (what the report shows without per-config tags)
  bool tagged = p->enc.live_max[0] + p->state_bits_of(0) + 6 <= 63;
  for (;;) {
    p->max_t = t_fail;
    p->report = tagged;
    rc = p->run();
    if (rc) {
      set_err(err, err_len, "%s", p->last_error.c_str());
      return rc;
    }
    if (p->status[0] == ST_RUNNING) break;
    if (tagged) {
      tagged = false;
      continue;
    }
    // the grid kernel's frontier lists overflowed before step t_fail (the verdict itself may
    // have come from the dense tables, which have no such limit): the lists are partial
    set_err(err, err_len, "failure configs unavailable: the pre-failure frontier of history %d exceeds the "
            "grid kernel's capacity (status %d)", hist, p->status[0]);
    return LC_E_CONFIGS;
  }
  // read the frontier lists of buffer (t_fail & 1): (config, tag) entries; per config the most
  // recent tag wins (age = steps since the emitting closure; a carried config is at most
  // width-many RETURNs old, < 64)
  const lc_plan::Batch& bt = p->batches[0];
  const int par = t_fail & 1;
  const int tag_shift = bt.mask_bits + bt.state_bits;
  std::vector<uint32_t> fc(2 * p->nwg);
  HIP_CHECK_MSG(hipMemcpy(fc.data(), p->d_fcount.p, fc.size() * 4, hipMemcpyDeviceToHost));
  const size_t E = (size_t)p->entry_bytes();
  std::vector<uint8_t> buf((size_t)p->f_cap * E);
  struct Cfg { uint64_t cfg; int64_t val; int age; };
  std::vector<Cfg> all;
  for (int w = 0; w < p->nwg; ++w) {
    const uint32_t n = std::min<uint32_t>(fc[(size_t)par * p->nwg + w], (uint32_t)p->f_cap);
    if (!n) continue;
    HIP_CHECK_MSG(hipMemcpy(buf.data(), (char*)p->d_flist.p + ((size_t)par * p->nwg + w) * p->f_cap * E, n * E,
                            hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i) {
      uint64_t key;
      memcpy(&key, buf.data() + i * E, 8);
      int64_t val = 0;
      if (L.model != LC_MODEL_CAS_REGISTER) memcpy(&val, buf.data() + i * E + 8, 8);
      const int tag = tagged ? (int)((key >> tag_shift) & 63) : (t_fail - 1) & 63;  // untagged: age 0
      all.push_back({key & ((1ull << tag_shift) - 1), val, (t_fail - 1 - tag) & 63});
    }
  }
  // one entry per config (its youngest tag), in config order
  std::sort(all.begin(), all.end(), [](const Cfg& x, const Cfg& y) {
    return x.cfg != y.cfg ? x.cfg < y.cfg : x.age < y.age;
  });
  all.erase(std::unique(all.begin(), all.end(), [](const Cfg& x, const Cfg& y) { return x.cfg == y.cfg; }),
            all.end());
  if (L.model == LC_MODEL_CAS_REGISTER) {
    const uint64_t sm = (1ull << bt.state_bits) - 1;
    std::vector<lc_plan::RepCfg> rep;
    rep.reserve(all.size());
    for (const Cfg& c : all)
      rep.push_back({c.cfg & ((1ull << bt.mask_bits) - 1), (int)((c.cfg >> bt.mask_bits) & sm),
                     t_fail == 0 ? -1 : t_fail - 1 - c.age});
    return emit(rep, bt.mask_bits);
  }
  // counter / leader: the value is the config's second word
  {
    std::vector<lc_plan::RepCfg> none;
    emit(none, 0);  // the pending ops and an empty output, then the configs below
  }
  auto last_index = [&](int age) -> int64_t {  // :ok completion of the emitting step's op
    const int s = t_fail - 1 - age;
    return s >= 0 ? en.step_cmp_idx[en.step_off[0] + s] : -1;
  };
  int64_t newest = -1;
  for (const Cfg& c : all) newest = std::max(newest, last_index(c.age));
  if (out_last_op) *out_last_op = newest;
  int out = 0;
  for (const Cfg& c : all) {
    if (out >= k) break;
    int nl = 0;
    for (int s = 0; s < bt.mask_bits; ++s)
      if ((c.cfg >> s) & 1) {
        if (linearized) linearized[(size_t)out * 64 + nl] = slot_inv[s];
        ++nl;
      }
    if (state) state[out] = c.val;
    if (is_nil) is_nil[out] = 0;
    if (n_lin) n_lin[out] = nl;
    if (last_op) last_op[out] = t_fail == 0 ? -1 : last_index(c.age);
    ++out;
  }
  if (n_out) *n_out = out;
  return 0;
}

}  // extern "C"
