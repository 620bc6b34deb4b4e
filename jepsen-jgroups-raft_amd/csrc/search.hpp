// search.hpp — device-side search parameters shared by the kernel and the host plan.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace lc {

constexpr int BLOCK = 1024;           // threads per workgroup (16 waves)
constexpr int S_LOG = 13;             // LDS closure-set table: 8192 x 8 B = 64 KiB
constexpr int O_LOG = 12;             // LDS frontier-out table: 4096 x 8 B = 32 KiB
constexpr int HMAX = 4096;            // histories per launch (LDS explored counters)
constexpr int WGMAX = 512;            // owners (workgroups) per launch
constexpr int PROBE_LIMIT = 32;       // LDS probes before spilling to the HBM table
constexpr uint64_t EMPTY = ~0ull;
constexpr uint64_t MARK = 1ull << 63; // "returned directly" routing marker

enum : int32_t { ST_RUNNING = 0, ST_VALID = 1, ST_INVALID = 2, ST_CAPACITY = 3, ST_MODEL = 4,
                 ST_SKIP = 5, ST_ABORTED = 6 };
enum : int32_t { FL_ABORT = 0, FL_OVERFLOW = 1, FL_SPILL = 2, FL_N = 4 };
enum : int32_t { SS_FIN = 0, SS_CAND = 1, SS_FOUT = 2, SS_SNEW = 3, SS_SPILL = 4, SS_PHASES = 5,
                 SS_STEPS = 6, SS_N = 8 };

struct RegEntry {  // cas-register config: [hist | state | mask] packed in 63 bits
  uint64_t key;
};
struct CntEntry {  // counter config: key [hist | mask]; the value is a function of the mask
  uint64_t key;
  int64_t st;
};

// Two-level arrival counters (8 groups of workgroups, then a top counter) and the release
// generation, each on its own 128-B line.
struct GridBar {
  unsigned gen;
  unsigned pad0[31];
  unsigned top;
  unsigned pad1[31];
  unsigned grp[8][32];
};
constexpr int SENT_LOG = 11;  // LDS filter of candidates already routed this phase

struct SearchParams {
  int32_t n_hist, nwg;
  int32_t mask_bits, state_shift, hist_shift;  // key layout
  int32_t cell_cap, f_cap, spill_log;
  int32_t max_t;  // run steps t < max_t (failure-frontier dumps); INT32_MAX otherwise
  int32_t model;
  // failure report (one history, lc_failure_configs): > 0 puts a 6-bit tag at this key bit =
  // the step (mod 64) whose closure emitted the config, kept when a config is carried through a
  // RETURN; frontier entries then differ by tag too (Knossos's per-config :last-op [ext]).
  // hist_shift sits above the tag (n_hist == 1). 0: off.
  int32_t tag_shift;
  // read-only encoded history (see encode.hpp)
  const int32_t* step_beg;   // [n_hist] first global step of each history
  const int32_t* step_end;   // [n_hist] one past its last step
  const uint8_t* step_slot;  // [total_steps]
  const int64_t* inv_off;    // [total_steps+1]
  const uint8_t* inv_slot;
  const uint8_t* inv_kind;
  const int64_t* inv_a;
  const int64_t* inv_b;
  const int64_t* init_st;  // [n_hist] initial state id (register) / value (counter)
  // per-history state
  uint64_t* live;      // [2][n_hist] live-slot masks (double-buffered by step parity)
  uint8_t* op_kind;    // [2][n_hist][64]
  int64_t* op_a;       // [2][n_hist][64]
  int64_t* op_b;       // [2][n_hist][64]
  int32_t* status;     // [n_hist]
  int32_t* fail_step;  // [n_hist]
  uint32_t* nonempty;  // [2][n_hist]
  unsigned long long* explored;  // [n_hist]
  // per-owner storage
  void* flist;         // [2][nwg][f_cap] frontier entries owned by each workgroup
  uint32_t* fcount;    // [2][nwg] (written at exit)
  void* cells;         // [2][nwg dst][nwg src][cell_cap] candidate shuffle cells
  uint32_t* cell_cnt;  // [2][nwg dst][nwg src]
  void* ovf;           // [2][nwg dst][ovf_cap] per-destination overflow of full cells
  uint32_t* ovf_cnt;   // [2][nwg dst] (global atomic reservation; rare path)
  int64_t ovf_cap;
  uint64_t* spill;     // [nwg][1 << spill_log] HBM overflow of the LDS tables
  uint32_t* spill_pos; // [nwg][1 << spill_log] used positions (for clearing)
  // grid sync and counters
  GridBar* bar;
  unsigned long long* produced;  // [4] items routed per phase (phase slot)
  unsigned* running;             // [4] histories active per step (step slot)
  int32_t* flags;                // [FL_N]
  unsigned long long* stats;     // [SS_N]
  unsigned long long* stamps;    // [nwg][8] phase cycle stamps (debug; may be null)
};

// Host launcher (search.hip). Returns hipSuccess or the launch error.
hipError_t launch_search(const SearchParams& p, hipStream_t stream);
// Occupancy-checked grid size for the cooperative launch on the current device.
int search_grid_size(int model);

}  // namespace lc
