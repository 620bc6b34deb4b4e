// encode.hpp — host-side history preprocessing for the GPU search (product code).
//
// Restates, for the device layout, what Knossos does before its search [ext]:
//   knossos.history: pair each :invoke with the next completion of the same process;
//     :ok folds its value into the invocation; :fail drops the pair; :info (or no
//     completion) leaves the invocation pending forever.
//   knossos.model.memo: map a cas-register's reachable values to dense state ids and the
//     history's ops to transition operands (§8(a) a8; model register.clj:110).
// and compiles the event stream into RETURN steps: step t = (slot of the returning op,
// the invocations that happened since step t-1 with the slots they occupy). Slots are
// reused after a return; a crashed op keeps its slot forever.
#pragma once
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

namespace lc {

// register op operands: a = expected state id (-1 any, -2 never), b = new state id (-1 keep)
constexpr int64_t R_ANY = -1, R_NEVER = -2, R_KEEP = -1;
// counter op kind bits: PRE_EQ (state == a), POST_EQ (state +/- d == a), SUB (d subtracted)
constexpr uint8_t C_PRE_EQ = 1, C_POST_EQ = 2, C_SUB = 4;
// LeaderModel op (leader.clj:63-75), on the counter's config layout (the state is a function of
// the linearized set): consistent iff (state & a) == 0, state |= b; a = the other contested pairs
// of the op's term, b = its own contested pair (both 0 for a term with one leader)
constexpr uint8_t C_LEADER = 8;
constexpr int LEADER_MAX_PAIRS = 64;
constexpr int MAX_SLOTS = 63;

struct HistArrays {
  int64_t n;
  const int64_t* index;  // may be null
  const int32_t* process;
  const int8_t* type;
  const int8_t* f;
  const int64_t* v0;
  const int64_t* v1;
  const int8_t* vflags;
};

// A vector whose resize leaves new elements uninitialised: the encoder writes every element it
// sizes, and an Encoded reused across calls (lc_check's cached plan) keeps its capacity, so a
// call neither zero-fills (serially) nor page-faults tens of MB of outputs.
template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInitAlloc<U>;
  };
  NoInitAlloc() = default;
  template <class U>
  NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
  template <class U>
  void construct(U* p) noexcept {
    ::new (static_cast<void*>(p)) U;  // default-initialise: nothing for scalars
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
};
template <class T>
using nvec = std::vector<T, NoInitAlloc<T>>;

struct Encoded {
  int model = 0;
  int n_hist = 0;
  int64_t init_value = 0;
  // per history
  std::vector<int32_t> step_off;   // n_hist+1, into per-step arrays
  std::vector<int32_t> err;        // LC_H_* (0 ok)
  std::vector<std::string> errmsg;
  std::vector<int32_t> live_max;   // max concurrently live slots
  std::vector<int32_t> n_states;   // register: distinct states (id 0 = nil)
  std::vector<int64_t> state_off;  // n_hist+1 into state_val (register id -> value, id>=1)
  nvec<int64_t> state_val;
  std::vector<int64_t> n_ops;      // invocations (before :fail removal)
  // per step (all histories concatenated)
  nvec<uint8_t> step_slot;     // slot of the returning op
  nvec<int64_t> inv_off;       // total_steps+1, into per-invoke arrays
  nvec<int64_t> step_cmp_idx;  // :index of the :ok completion
  nvec<int64_t> step_inv_idx;  // :index of its invocation
  // per invoke assignment
  nvec<uint8_t> inv_slot;
  nvec<uint8_t> inv_kind;
  nvec<int64_t> inv_a, inv_b;
  nvec<int64_t> inv_index;  // :index of the invocation (failure reports)

  int64_t total_steps() const { return (int64_t)step_slot.size(); }
  int32_t n_steps(int h) const { return step_off[h + 1] - step_off[h]; }
};

// One encoded history as encode() has just built it (valid during the sink call only):
// RETURN steps (returning slot, invocations since the previous step) and the invocations'
// slots and register operands, in step order.
struct HistView {
  int32_t err, live_max, n_states;
  int64_t n_steps;
  const uint8_t* step_slot;
  const int64_t* step_ninv;
  const uint8_t* inv_slot;
  const int64_t* inv_a;
  const int64_t* inv_b;
  const uint8_t* inv_kind;  // counter / leader op kind bits (C_*)
};
// Called by the worker that encoded history h, right after it (its data still in cache).
// Returns true when the caller has taken everything it needs of h's invocations: `out` then
// keeps h's RETURN steps (slots, :index values) but not its per-invocation arrays (inv_off does
// not advance over h's steps).
using HistSink = std::function<bool(int, const HistView&)>;

// model: 1 cas-register, 2 counter, 3 leader. Never throws; per-history problems land in err/errmsg.
// `out` may be reused across calls (its buffers keep their capacity). `sink` (optional) sees
// every history as soon as it is encoded (lc_plan builds its dense step streams there).
void encode(int model, int64_t init_value, int n_hist, const int64_t* hist_off,
            const HistArrays& a, Encoded& out, const HistSink* sink = nullptr);

// The histories hs of `all` (encoded without a sink: every invocation array kept) as an Encoded
// of their own, in that order: lc_check(n_gpus > 1) encodes a batch once and gives each shard
// its histories this way (a parallel copy, no second encode).
void encoded_subset(const Encoded& all, const std::vector<int>& hs, Encoded& out,
                    const HistSink* sink = nullptr);
// sink(h, view) for every history of enc, the views built from enc's arrays (on the pool)
void sink_encoded(const Encoded& enc, const HistSink& sink);
// Frees the calling thread's encoder buffers (kept between calls for speed; lc_release).
void encode_trim();

}  // namespace lc
