// keys.hpp — parameters of the per-history ("keys") search kernel.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace lc {

constexpr int KB = 1024;     // threads per workgroup
constexpr int KS_LOG = 13;   // LDS closure-set table, max 8192 x 8 B
constexpr int KO_LOG = 12;   // LDS frontier-out table, max 4096 x 8 B
constexpr int K_PROBES = 24; // LDS probes before the HBM spill table

struct KeysParams {
  int32_t n_hist, model;
  const int8_t* kshift;  // [n_hist] key layout [state | mask]: mask bits = state shift
  const int8_t* kbits;   // [n_hist] register state bits
  int64_t fcap, lcap;              // per-workgroup frontier / level capacities (entries)
  int32_t spill_log;
  const int32_t* step_beg;
  const int32_t* step_end;
  const uint8_t* step_slot;
  const int64_t* inv_off;
  const uint8_t* inv_slot;
  const uint8_t* inv_kind;
  const int64_t* inv_a;
  const int64_t* inv_b;
  const int64_t* init_st;
  const int32_t* order;  // processing order (heaviest first)
  int32_t* queue;        // next position in `order`
  int32_t* status;
  int32_t* fail_step;
  unsigned long long* explored;
  void* scratch;         // per workgroup: F[2][fcap] then L[2][lcap]
  uint64_t* spill;       // per workgroup: 1 << spill_log
  uint32_t* spill_pos;   // per workgroup: 1 << spill_log
  unsigned long long* stats;  // SS_* counters (search.hpp)
};

hipError_t launch_keys(const KeysParams& p, int nwg, hipStream_t stream);
int keys_grid_size(int model);

}  // namespace lc
