// dense.hpp — closure-table search for narrow cas-register histories.
//
// A history whose live pending slots never exceed DENSE_WIDE_LMAX and whose register takes
// at most DENSE_MAX_STATES distinct values keeps its whole frontier as a byte-sliced table:
// u64 word w covers the 8 masks (w << 3) | p, and its byte s is register state s's bitmap
// over them (bit p = "config (s, mask) exists"). The closure of one RETURN
// (knossos.linear/analysis [ext]) is a subset DP over popcount layers of
// the word index — no hashing, no candidate lists — and the explored count is the number of
// bits the DP produces, identical to the sparse search's set semantics.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace lc {

constexpr int DENSE_LMAX = 17;       // widest table a workgroup holds in LDS (128 KiB)
constexpr int DENSE_WAVE_LMAX = 11;  // histories this narrow run one per wave
constexpr int DENSE_WIDE_LMAX = 22;  // widest table a team of workgroups keeps in HBM (4 MiB)
constexpr int DENSE_MAX_STATES = 8;  // register values (state ids) per history
constexpr int DENSE_WORD_BITS = DENSE_WIDE_LMAX - 3;  // bits of the sorted word list

// Step stream (host-built, one u32 word stream per history):
//   header  live[0:22) | j[22:27) | ninv[27:32)   live = pending slots after this step's
//                                                 invocations (includes the returning j)
//   ninv op words: slot[0:8) | amask[8:16) | bmask[16:24)
// register step on a state set S: x = S & amask; bmask ? (x ? bmask : 0) : x
struct DenseParams {
  int32_t n;                    // histories in this launch (entries of order)
  const int32_t* order;         // plan-local history ids, heaviest first
  const int64_t* sbeg;          // [n_hist] first word of each history's stream
  const int32_t* nsteps;        // [n_hist]
  const int8_t* lmax;           // [n_hist] table width (bits)
  const uint32_t* words;        // DENSE_WORD_BITS-bit word indices sorted by (popcount, value)
  const uint32_t* stream;
  int64_t stream_words;
  int32_t* queue;               // dequeue counter (zeroed before launch)
  int32_t* status;              // [n_hist] ST_VALID / ST_INVALID
  int32_t* fail_step;           // [n_hist]
  unsigned long long* explored; // [n_hist] (wide teams add into it: zeroed before launch)
  unsigned long long* stats;    // [SS_N] frontier-out, steps
  unsigned long long* stamps;   // [n_hist][2] start / end (s_memrealtime, 100 MHz); may be null
  // wide teams only
  int32_t team_size;            // workgroups per team
  uint64_t* gtab;               // [teams][2^DENSE_WORD_BITS] HBM tables
  void* ctl;                    // [teams] TeamCtl (zeroed before launch)
  int32_t* abort;               // set when a team barrier times out
};

// Team kinds: WAVE = 256-thread workgroups, one history per wave (width <= DENSE_WAVE_LMAX);
// BLOCK = 1024-thread workgroup per history, LDS table (width <= DENSE_LMAX);
// WIDE = team_size 1024-thread workgroups per history: steps of width <= DENSE_LMAX run on
// the leader's LDS table, wider steps on an HBM table shared by the team.
enum DenseTeam { DENSE_WAVE = 0, DENSE_BLOCK = 1, DENSE_WIDE = 2 };
hipError_t launch_dense(const DenseParams& p, DenseTeam kind, int grid, hipStream_t stream);
int dense_grid_size(DenseTeam kind);
size_t dense_ctl_bytes();  // per team
// The sorted word list (host-built, uploaded once): words of `bits` bits in colex order by
// popcount layer; the words of popcount q below 2^H (H <= bits) are a prefix of layer q.
void dense_word_list(int bits, uint32_t* out);

}  // namespace lc
