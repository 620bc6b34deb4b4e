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
constexpr int DENSE_MID_LMAX = 14;   // ... this narrow one per 256-thread workgroup (16 KiB table)
constexpr int DENSE_WIDE_LMAX = 24;  // widest history a tile team holds (<= 2^7 LDS tiles)
constexpr int DENSE_MAX_STATES = 8;  // register values (state ids) per history
constexpr int DENSE_WORD_BITS = 19;  // bits of the sorted word list (a tile's words use <= 14)
constexpr int DENSE_MAX_NINV = 30;   // invocations per step (a step must fit a 32-word window)
constexpr int DENSE_MRING = 64;      // mirror slots per tile (pipelined tile teams)
constexpr int DENSE_TEAM_MAXB = 8;   // team bits of a pipelined tile team (packed segments)
constexpr int DENSE_TEAM_MAXB_SERIAL = 5;  // ... with serial segments
constexpr int DENSE_PIPE_SERIAL_SEGS = 32;  // DenseParams.pipe bit 5: one pass per segment
constexpr int DENSE_PIPE_DBL = 512;         // DenseParams.pipe bit 9: double-buffered tables

// Step stream (host-built, one u32 word stream per history):
//   header  live[0:24) | j[24:29), bit 31 clear   live = pending slots after this step's
//                                                 invocations (includes the returning j)
//   op words, one per invocation since the previous step (<= DENSE_MAX_NINV), bit 31 set:
//           slot[0:8) | amask[8:16) | bmask[16:24) | DENSE_OPW
//   (a decoder counts a step's op words with one ballot over the words that follow it)
constexpr uint32_t DENSE_LIVE_MASK = 0xffffffu, DENSE_OPW = 1u << 31;
constexpr int DENSE_J_SHIFT = 24;
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
  int32_t n2;                   // BLOCK teams: a second queue drained after the first (the MID
  const int32_t* order2;        // histories, so a CU whose BLOCK work is done helps there)
  int32_t* queue2;
  int32_t* status;              // [n_hist] ST_VALID / ST_INVALID
  int32_t* fail_step;           // [n_hist]
  unsigned long long* explored; // [n_hist] (wide teams add into it: zeroed before launch)
  unsigned long long* stats;    // [SS_N] frontier-out, steps
  unsigned long long* stamps;   // [n_hist][4] start, end, team-step time (s_memrealtime, 100 MHz),
                                // team steps; may be null
  // tile teams (big kernel): workgroups [0, n_team_wgs) form the teams, the rest run the
  // BLOCK histories of order[0..n)
  int32_t n_team_wgs;
  const int32_t* wg_team;       // [n_team_wgs] team of each workgroup
  const int32_t* team_base;     // [teams] first workgroup
  const int8_t* team_bits;      // [teams] t: 2^t workgroups, history width <= lb + t
  const int8_t* team_lbits;     // [teams] lb: local slots per tile (<= DENSE_LMAX)
  const int32_t* team_hist;     // [teams] history id
  uint64_t* mirror;             // [n_team_wgs][DENSE_MRING][2^(DENSE_LMAX-3)] published tile words
                                // (one slot per step in flight when pipelined, else slot 0)
  unsigned long long* flags;    // [n_team_wgs] layer tokens (zeroed before launch)
  void* ctl;                    // [teams] TeamCtl (zeroed before launch)
  int32_t* abort;               // set when a team barrier / token wait times out
  unsigned long long* tstamps;  // [n_team_wgs][8] LC_DEBUG phase cycles of each tile workgroup
  unsigned long long* lhist;    // LC_DEBUG [2 teams (wave, block)][32 widths][LH_N]; may be null
                                // (per-step loop only)
  uint32_t* team_any;           // pipelined teams: per team, bit t = some tile read a nonzero
  const int32_t* team_any_off;  // frontier in step t (step ns: the last return); word offsets
  unsigned long long* done;      // [n_team_wgs] team steps finished (LC_PIPE bit 3)
  int32_t n_w;                  // big kernel: WAVE histories its waves run after the BLOCK
  const int32_t* order_w;       // queue (0: dense_wave_kernel runs them)
  int32_t* queue_w;
  uint32_t mirror_tag;          // tagged mirrors (LC_PIPE bit 8): this launch's tag base
  int32_t mid_first;            // big kernel, LC_PIPE bit 7: BLOCK-pool workgroups (just below the
                                // WAVE-first ones) that start on the MID queue
  int32_t pipe;                 // bit 3: tile teams without per-step team barriers;
                                // bit 0: BLOCK, bit 1: WAVE, bit 2: TILE teams overlap
                                // consecutive steps (history_pipe / team_pipe); default 11
};

// Kernels: WAVE = 256-thread workgroups, one history per wave (width <= DENSE_WAVE_LMAX);
// BIG = 1024-thread workgroups: tile teams (one history of width 18..DENSE_WIDE_LMAX each,
// one workgroup per 17-bit LDS tile) and BLOCK histories (width <= DENSE_LMAX, one
// workgroup each, LDS table) in the same launch.
// LC_DEBUG per-width step profile: steps, step time (100 MHz), nonzero words before the
// closure, nonzero words after it, configs explored
constexpr int LH_N = 5;
enum DenseTeam { DENSE_WAVE = 0, DENSE_BIG = 1, DENSE_MID = 2 };
hipError_t launch_dense(const DenseParams& p, DenseTeam kind, int grid, hipStream_t stream);
int dense_grid_size(DenseTeam kind);
size_t dense_ctl_bytes();  // per team
// The sorted word list (host-built, uploaded once): words of `bits` bits in colex order by
// popcount layer; the words of popcount q below 2^H (H <= bits) are a prefix of layer q.
void dense_word_list(int bits, uint32_t* out);

}  // namespace lc
