// wide.hpp — closure tables in HBM for cas-register histories wider than the LDS tile teams
// hold: live width DENSE_WIDE_LMAX < L <= WIDE_LMAX.
//
// The same table and the same subset DP as dense.hpp (byte-sliced u64 words, one word per 8
// masks; a RETURN step is its popcount layers in order), but the two tables (step t on t & 1)
// live in HBM and the whole GPU works on one history: one persistent launch, every workgroup
// takes a share of each popcount layer, a grid barrier ends the layer. Words are written with
// sc1 (write-through) stores and read with sc1 (L1-bypassing) loads, so the barrier needs no
// fences (the search kernel's level-phase protocol, MI355X_MICROARCH "Valid forms" row 1).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace lc {

constexpr int WIDE_LMAX = 36;       // widest history: 2 tables of 2^33 words (128 GiB of the 288 GB HBM)
constexpr int WIDE_SLAB_BITS = 32;  // a slab holds at most 2^32 words (its local index is 32-bit)
constexpr int WIDE_MAX_SPLIT = 3;   // at most 2^3 slabs (LC_WIDE_SPLIT, the rank split of §3.10)
constexpr int WIDE_NOPIPE_LMAX = 31;  // the one-step-at-a-time kernel's layer prefix tables stop here
constexpr int WIDE_OPS = 37;        // op-table entries per step (slots 0..35, + the pull loop's reads)
constexpr int WIDE_MAX_NINV = 60;   // invocations per step (3 header words + 60 in a 64-lane read;
                                    // never binding: a step's invocations are live, <= WIDE_LMAX)
constexpr int WIDE_LOW_BITS = 19;   // a layer's words = high part x low part from the sorted list

// Step stream of a wide history (host-built, its own buffer):
//   header word 0  live slots 0..30, bit 31 clear
//   header word 1  live slots 31..61 (bit k - 31), bit 31 clear
//   header word 2  j (the returning slot), bit 31 clear
//   op words, one per invocation since the previous step (<= DENSE_MAX_NINV), bit 31 set:
//                  slot[0:8) | amask[8:16) | bmask[16:24) | DENSE_OPW
//   a 0 word after the last step
struct WideParams {
  int32_t n;                  // wide histories in this launch (run one after another)
  const int64_t* sbeg;        // [n] first word of each history's stream in `stream`
  const int32_t* nsteps;      // [n]
  const int8_t* lmax;         // [n] table width (slots)
  const uint32_t* stream;
  const uint32_t* words;      // the DENSE_WORD_BITS-bit sorted word list (dense_word_list)
  uint64_t* tab;              // 2 tables of tab_words words each
  int64_t tab_words;
  // the pipelined kernel's slabs: the top `split` hi bits of a word pick one of 2^split slabs of
  // tab_words >> split words (<= 2^32), ranked inside the slab over the remaining hi bits
  int32_t split;
  int32_t* status;            // [n] ST_VALID / ST_INVALID
  int32_t* fail_step;         // [n] the failing RETURN step (-1: none)
  unsigned long long* explored;  // [n] (zeroed before launch)
  unsigned long long* any;    // [n] latest step (+1) whose frontier held a config (zeroed)
  unsigned* bar;              // grid barrier words (zeroed before launch)
  int32_t* abort;             // a barrier watchdog fired
  unsigned long long* stats;  // [4] frontier-out configs, steps, words visited, words stored nonzero
  int32_t pipe;               // 1: pipelined steps (wide_pipe_kernel), 0: one step at a time
  uint32_t* anyv;             // pipelined: per history, bit t = some X of step t was nonzero (zeroed)
  uint64_t watchdog;          // s_memrealtime ticks (100 MHz) a grid barrier may wait before *abort
  const int64_t* anyv_off;    // [n] word offset of each history's bits (ns / 32 + 1 words)
  // test hook (LC_WIDE_STALL=h:wg, tests only; stall = null otherwise): workgroup stall_wg
  // arms *stall as it starts history stall_hist and then skips its next barrier arrival
  int32_t* stall;
  int32_t stall_hist, stall_wg;
};

// failure reports (lc_failure_configs): the frontier before step t, read from tab = step t - 1's
// table through its returning slot jp, over the post-return live slots lv; configs (mask, state)
// in any order, at most cap of them, *count = all of them
struct WideDumpParams {
  const uint64_t* tab;
  int32_t ranked;  // the pipelined kernel's layout (colex_rank), else word w at index w
  int32_t Hm;      // the table holds 2^Hm words
  int32_t split;   // in 2^split slabs (ranked layout only)
  uint64_t lv;
  int32_t jp;
  int64_t cap;
  uint64_t* masks;
  uint8_t* states;
  unsigned long long* count;
};

hipError_t launch_wide(const WideParams& p, int grid, hipStream_t stream);
hipError_t launch_wide_dump(const WideDumpParams& d, hipStream_t stream);
// out[i] = the word of tab (as d: layout, Hm) at hi-bit word hw[i]
hipError_t launch_wide_gather(const WideDumpParams& d, const uint64_t* hw, uint64_t* out, int n, hipStream_t stream);
int wide_grid_size(bool pipe);
// counter histories on the HBM tables (wctr_pipe_kernel): live width up to
// WCTR_LMAX, the stream in wide.hip's counter format, tab_words = 2^(lmax - 6)
constexpr int WCTR_LMAX = 38;      // 2 tables of 2^32 words (64 GiB): the word index stays 32-bit
constexpr int WCTR_MAX_NINV = 30;  // invocations per step (3 header words + 2 per invocation in 64 lanes)
hipError_t launch_wctr(const WideParams& p, int grid, hipStream_t stream);
// failure reports: the configs (masks) of tab (ranked over Hm hi bits, 64 masks per word) through jp
hipError_t launch_wctr_dump(const WideDumpParams& d, hipStream_t stream);
int wctr_grid_size();
size_t wide_bar_bytes();

}  // namespace lc
