// dense.hpp — closure-table search for narrow cas-register histories.
//
// A history whose live pending slots never exceed DENSE_LMAX and whose register takes at
// most 8 distinct values keeps its whole frontier as a table A[mask] of 8-bit state sets
// (bit s = "a config with model state id s and linearized-slot set `mask` exists") in LDS.
// The closure of one RETURN (knossos.linear/analysis [ext]) is then a
// subset DP over popcount layers — no hashing, no HBM candidate traffic — and the explored
// count is the sum of |R[mask]| over the produced sets, identical to the sparse search's
// set semantics.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace lc {

constexpr int DENSE_BLOCK = 1024;   // threads per workgroup
constexpr int DENSE_LMAX = 17;      // widest history the block-team table holds (128 KiB)
constexpr int DENSE_WAVE_LMAX = 12; // histories this narrow run one per wave (4 KiB each)
constexpr int DENSE_MAX_STATES = 8; // state sets are bytes

// Step stream (host-built, one u32 word stream per history):
//   header  live[0:22) | j[22:27) | ninv[27:32)   live = pending slots after this step's
//                                                 invocations (includes the returning j)
//   ninv op words: slot[0:8) | amask[8:16) | bmask[16:24)
// register step on a state set S: x = S & amask; bmask ? (x ? bmask : 0) : x
struct DenseParams {
  int32_t n;                   // histories in this launch (entries of order)
  const int32_t* order;        // plan-local history ids, heaviest first
  const int64_t* sbeg;         // [n_hist] first word of each history's stream
  const int32_t* nsteps;       // [n_hist]
  const int8_t* lmax;          // [n_hist] table width (bits)
  const uint32_t* stream;
  int64_t stream_words;
  int32_t* queue;              // dequeue counter (zeroed before launch)
  int32_t* status;             // [n_hist] ST_VALID / ST_INVALID
  int32_t* fail_step;          // [n_hist]
  unsigned long long* explored;// [n_hist]
  unsigned long long* stats;   // [SS_N] frontier-in, candidates, frontier-out, steps
};

hipError_t launch_dense(const DenseParams& p, bool wave_teams, int grid, hipStream_t stream);
int dense_grid_size(bool wave_teams);

}  // namespace lc
