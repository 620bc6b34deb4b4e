// ctab.hpp — closure-table search for counter histories.
//
// The reference checks a counter run as ONE whole-history knossos.linear search with
// CounterModel (src/jepsen/jgroups/workload/counter.clj:100-137). A counter
// config's value is a function of its linearized set: every config at a RETURN step has
// linearized the ops returned so far (base = the sum of their deltas) plus a subset m of the
// pending slots, so value(m) = init + base + S(m), S(m) = the sum of m's deltas. The frontier is
// therefore a bitmap over masks — one bit per config, no state bytes — and a step of op k from
// mask m is consistent iff k is unconstrained (:add, :decr, a read of nil, a crashed
// *-and-get) or S(m) equals k's requirement (a read of v: v - init - base; an :ok *-and-get
// [d new]: new -/+ d - init - base).
//
// Layout: u64 word w covers the 64 masks (w << 6) | p; slots 0..5 are inside the word, slots
// >= 6 index words. A RETURN is the subset DP over the popcount layers of the word index that
// the register tables run (dense.hpp), with each op's consistency as a per-position gate:
// S((w, p)) = S_hi(w) + S_lo(p), and the positions p of one word whose low sum equals a value
// come from a 64-entry table EQ[v - lo_min] rebuilt per step.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace lc {

constexpr int CTAB_LO = 6;          // slots inside a table word
constexpr int CTAB_LMAX = 20;       // widest table a workgroup holds in LDS (2^20 bits = 128 KiB)
constexpr int CTAB_TEAM_LMAX = 24;  // widest table a tile team holds (the step header's 24 live bits;
                                    // 64 tiles of 18 local slots)
constexpr int CTAB_MAX_NINV = 31;   // invocations per step (2 stream words each, a 128-word window;
                                    // never binding: a step's invocations are live, <= CTAB_LMAX)
constexpr int CTAB_DMAX = 10;       // |delta| of every op (EQ tables of 64 entries over 6 slots)
constexpr int32_t CTAB_REQ_BIAS = 1 << 29;  // stream requirement bias (|req| < 2^29, else never)
constexpr int64_t CTAB_SUM_MAX = 1 << 27;   // sum of |delta| over a history (bounds every config value)

// Step stream (host-built, one u32 stream per history):
//   header  live[0:24) | j[24:29), bit 31 clear (as dense.hpp)
//   per invocation since the previous step, two words with bit 31 (DENSE_OPW) set:
//     w0 = slot[0:8) | flags[8:16) | (uint8_t)delta[16:24)       flags: CT_UNC, CT_NEVER
//     w1 = (req + CTAB_REQ_BIAS) & 0x3fffffff                   req: the value relative to the
//          initial one the counter must hold before the op (when neither flag is set)
constexpr uint32_t CT_UNC = 1u, CT_NEVER = 2u;

struct CtabParams {
  int32_t n;                     // histories in this launch (entries of order)
  const int32_t* order;          // plan-local history ids, heaviest first
  const int64_t* sbeg;           // [n_hist] first word of each history's stream
  const int32_t* nsteps;         // [n_hist]
  const int8_t* lmax;            // [n_hist] table width (bits)
  const uint32_t* words;         // the sorted word list (dense_word_list, DENSE_WORD_BITS bits)
  const uint32_t* stream;
  int64_t stream_words;
  int32_t* queue;                // dequeue counter (zeroed before launch)
  int32_t* status;               // [n_hist] ST_VALID / ST_INVALID
  int32_t* fail_step;            // [n_hist]
  unsigned long long* explored;  // [n_hist]
  unsigned long long* stats;     // [2] frontier configs out, steps
  unsigned long long* stamps;    // [n_hist][2] start, end (s_memrealtime, 100 MHz); may be null
  unsigned long long* prof;      // LC_DEBUG [16 waves][8]: super-layer phase cycles, super-layers, words closed
                                 // (ring view, words, decode + start, barrier) and super-layers
  int32_t pipe;                  // bit 0: double-buffered tables when two fit (default on)
};

hipError_t launch_ctab(const CtabParams& p, int grid, hipStream_t stream);
int ctab_grid_size();

// Counter tile teams: ONE counter history's table split
// over 2^T workgroups by its top T slots (the team slots lb..lb+T-1, lb = lmax - T). Tile r holds
// the masks whose team slots spell r, over its lb local slots, in LDS; a pull over a team slot
// reads tile r \ b's word from that tile's mirror in HBM (sc1 stores, drained, then a token =
// super-layers finished), and so does the X of a step after a team-slot return (tile r | jp).
// The super-layer schedule is the LDS kernel's, skewed per tile: tile r runs its local layer q
// of step t at super-layer start_t + q + |r| (|r| = its live team slots), so whatever it pulls
// from another tile was finished one super-layer earlier. One cooperative launch: every team's
// workgroups are resident together.
constexpr int CT_MRING = 64;  // mirror slots per tile (steps)
constexpr int CTAB_TEAM_MAXB = 6;  // team slots (64 tiles)
struct CtabTeamParams {
  CtabParams c;                  // sbeg, nsteps, lmax, words, stream, status, fail_step, explored, stats, stamps
  int32_t n_teams;
  const int32_t* wg_team;        // [grid] the team of each workgroup
  const int32_t* team_base;      // [n_teams] its first workgroup
  const int8_t* team_bits;       // [n_teams] T (2^T tiles)
  const int32_t* team_hist;      // [n_teams] plan-local history id
  const int32_t* team_any_off;   // [n_teams] first word of the team's per-step survivor bits
  unsigned long long* flags;     // [grid] tokens: super-layers the tile has finished (zeroed)
  uint64_t* mirror;              // [grid][CT_MRING][2^mshift] published words
  int32_t mshift;
  uint32_t* anyv;                // per team, bit t: a tile read a nonzero frontier in step t (zeroed)
  unsigned* ctl;                 // per team 64 words: barrier arrivals [0], generation [32] (zeroed)
  int32_t* abort;                // a watchdog fired (zeroed)
  uint64_t watchdog;             // s_memrealtime ticks a wait may last before *abort
};
hipError_t launch_ctab_team(const CtabTeamParams& p, int grid, hipStream_t stream);
int ctab_team_max_wgs();  // workgroups one cooperative team launch may hold

}  // namespace lc
