// encode.cpp — see encode.hpp. Product host code (independent of oracle/).
#include "encode.hpp"

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <unordered_map>

#include "../../include/lincheck.h"
#include "pool.hpp"

namespace lc {
namespace {

enum { T_INVOKE = 0, T_OK = 1, T_FAIL = 2, T_INFO = 3 };
enum { F_READ = 0, F_WRITE = 1, F_CAS = 2, F_ADD = 3, F_DECR = 4, F_AAG = 5, F_DAG = 6, F_INSPECT = 7 };
enum { V_NIL = 0, V_SCALAR = 1, V_PAIR = 2 };

struct OneOut {
  int32_t err = 0;
  std::string msg;
  int32_t live_max = 0;
  int32_t n_states = 1;
  int64_t n_ops = 0;
  std::vector<int64_t> state_val;
  std::vector<uint8_t> step_slot;
  std::vector<int64_t> step_ninv;
  std::vector<int64_t> step_cmp_idx, step_inv_idx;
  std::vector<uint8_t> inv_slot, inv_kind;
  std::vector<int64_t> inv_a, inv_b, inv_index;
};

struct Op {
  int64_t inv_pos;
  int64_t v0, v1;
  int8_t status;  // -1 pending forever, else completion type
  int8_t f, vflags;
  uint8_t slot;
  uint8_t inword;  // slot policy: chosen for an in-word slot (0..2; a counter's 0..5)
  uint8_t kind;    // model operands (computed once, before the assignment pass)
  int64_t oa, ob;
};

// per-thread scratch, kept across histories (no allocation per history once warm)
struct Scratch {
  std::vector<Op> ops;
  std::vector<int32_t> op_of;  // entry -> its op, -1 none
  std::vector<int32_t> pkey;
  std::vector<int32_t> pval;   // -2 empty slot, -1 no outstanding op, else op
  std::unordered_map<int64_t, int32_t> sid;
};

// model operands of one op (cas-register: knossos.model/CASRegister [ext]; counter:
// CounterModel.step, counter.clj:102-127); 0 or an LC_H_MODEL message
template <class Find>
const char* operands(int model, const Op& op, Find&& find_id, uint8_t& kind, int64_t& oa,
                     int64_t& ob) {
  kind = 0;
  oa = ob = 0;
  if (model == LC_MODEL_CAS_REGISTER) {
    auto lookup = [&](int64_t v) -> int64_t {
      const int32_t f = find_id(v);
      return f ? f : R_NEVER;
    };
    switch (op.f) {
      case F_WRITE:  // write v -> v
        if (op.vflags == V_PAIR) return "write with a pair value";
        oa = R_ANY;
        ob = op.vflags == V_NIL ? 0 : find_id(op.v0);
        return nullptr;
      case F_CAS:  // cas [cur new] -> new iff cur = value
        if (op.vflags != V_PAIR) return "cas without [cur new]";
        oa = lookup(op.v0);
        ob = find_id(op.v1);
        return nullptr;
      case F_READ:  // read v -> ok iff v nil or v = value
        if (op.vflags == V_PAIR) return "read with a pair value";
        oa = op.vflags == V_NIL ? R_ANY : lookup(op.v0);
        ob = R_KEEP;
        return nullptr;
      default:
        return "unknown :f for cas-register";
    }
  }
  if (model == LC_MODEL_LEADER) {  // operands set by the contested-pair pass (encode_one)
    if (op.f != F_INSPECT) return "unknown :f for LeaderModel";
    if (op.vflags == V_SCALAR) return ":inspect value is not [leader term]";
    kind = C_LEADER;
    return nullptr;
  }
  switch (op.f) {
    case F_ADD:
    case F_DECR:
      if (op.vflags != V_SCALAR) return ":add/:decr need a scalar delta";
      kind = op.f == F_DECR ? C_SUB : 0;
      ob = op.v0;
      return nullptr;
    case F_READ:
      if (op.vflags == V_PAIR) return ":read with a pair value";
      kind = op.vflags == V_NIL ? 0 : C_PRE_EQ;
      oa = op.v0;
      return nullptr;
    case F_AAG:
    case F_DAG:
      if (op.vflags == V_NIL) return "*-and-get without a delta";
      kind = (op.f == F_DAG ? C_SUB : 0) | (op.vflags == V_PAIR ? C_POST_EQ : 0);
      ob = op.v0;
      oa = op.vflags == V_PAIR ? op.v1 : 0;
      return nullptr;
    default:
      return "unknown :f for CounterModel";
  }
}

// Three passes per history: (1) pairing (knossos.history [ext]) with the slot policy's greedy
// at each :ok completion, (2) over the ops: the memo (cas-register state ids) and every op's
// model operands, (3) over the entries: slot assignment and the RETURN steps.
void encode_one(int model, const HistArrays& a, int64_t b, int64_t e, OneOut& o) {
  thread_local Scratch sc;
  auto IDX = [&](int64_t pos) { return a.index ? a.index[pos] : pos - b; };
  std::vector<Op>& ops = sc.ops;
  auto fail = [&](int code, const char* m) {
    o.err = code;
    o.msg = m;
    o.n_ops = (int64_t)ops.size();
  };
  // ---- slot policy. Slot labels are arbitrary (a config's mask is a set), so the search's
  // answers never depend on them, but the dense tables keep slots 0..2 inside a table word: a
  // RETURN of one of them lets the next step start one super-layer after it, not two (DESIGN
  // §3.2). The ops that return soonest go there: the most :ok intervals three "machines" can
  // hold (greedy by completion, best fit), chosen as the completions arrive in the pairing
  // pass. Assignment below keeps the widths of lowest-free-first (an unchosen op takes an
  // in-word slot whenever the lowest free other slot would widen the table). LC_SLOTS=lff:
  // lowest free first only.
  static const bool slots_lff = [] {
    const char* e = getenv("LC_SLOTS");
    return e && strcmp(e, "lff") == 0;
  }();
  // in-word slots: 3 for the register tables' words (8 masks x 8 states), 6 for the counter
  // tables' (64 masks, ctab.hpp)
  const int n_iw = model == LC_MODEL_COUNTER ? 6 : 3;
  int64_t mfree[6] = {-1, -1, -1, -1, -1, -1};
  // ---- pairing (knossos.history [ext])
  ops.clear();
  std::vector<int32_t>& op_of = sc.op_of;
  op_of.resize(e - b);
  // process -> its outstanding op (-1: none): a direct table over [pmin, pmax] when the process
  // ids are dense (Jepsen's are small integers), else open addressing over a power-of-two table
  // (processes are arbitrary int32; a history has at most one per entry)
  int32_t pmin = INT32_MAX, pmax = INT32_MIN;
  for (int64_t i = b; i < e; ++i) pmin = std::min(pmin, a.process[i]), pmax = std::max(pmax, a.process[i]);
  int64_t n_ok = 0;
  const char* bad = nullptr;
  auto pair_all = [&](auto&& slot_of) {
    for (int64_t i = b; i < e; ++i) {
      const int8_t t = a.type[i];
      int32_t& cur = slot_of(a.process[i]);
      if (t == T_INVOKE) {
        if (cur >= 0) return void(bad = "process invoked while an op was outstanding");
        cur = (int32_t)ops.size();
        op_of[i - b] = cur;
        ops.push_back(Op{i, a.v0[i], a.v1[i], -1, a.f[i], a.vflags[i], 0, 0, 0, 0, 0});
      } else if (t == T_OK || t == T_FAIL || t == T_INFO) {
        if (cur < 0) return void(bad = "completion without an outstanding invocation");
        Op& op = ops[cur];
        op.status = t;
        if (t == T_OK) {  // fold the completion's value into the invocation
          op.vflags = a.vflags[i];
          op.v0 = a.v0[i];
          op.v1 = a.v1[i];
          n_ok++;
          int best = -1;  // slot policy: the machine free latest before this op's invocation
          for (int m = 0; m < n_iw; ++m)
            if (mfree[m] < op.inv_pos && (best < 0 || mfree[m] > mfree[best])) best = m;
          if (best >= 0) op.inword = 1, mfree[best] = i;
        }
        op_of[i - b] = cur;
        cur = -1;
      } else {
        return void(bad = "unknown :type");
      }
    }
  };
  if (e > b && (int64_t)pmax - pmin < 4 * (e - b) + 1024) {
    sc.pval.assign((size_t)((int64_t)pmax - pmin + 1), -1);
    int32_t* pval = sc.pval.data();
    pair_all([&](int32_t proc) -> int32_t& { return pval[(int64_t)proc - pmin]; });
  } else {
    const size_t cap = (size_t)1 << (64 - __builtin_clzll((unsigned long long)(e - b) | 15));
    const size_t pmask = cap * 2 - 1;
    sc.pkey.resize(cap * 2);
    sc.pval.assign(cap * 2, -2);  // -2: empty slot
    int32_t* pkey = sc.pkey.data();
    int32_t* pval = sc.pval.data();
    pair_all([&](int32_t proc) -> int32_t& {
      size_t k = ((uint32_t)proc * 0x9E3779B1u) & pmask;
      while (pval[k] != -2 && pkey[k] != proc) k = (k + 1) & pmask;
      if (pval[k] == -2) pkey[k] = proc, pval[k] = -1;
      return pval[k];
    });
  }
  if (bad) return fail(LC_H_MALFORMED, bad);
  if (slots_lff)
    for (Op& op : ops) op.inword = 0;
  o.n_ops = (int64_t)ops.size();
  // ---- cas-register memo: value -> state id (id 0 = nil), ids in first-appearance order over
  // the values the register can hold (ops in invocation order). Values in [0, 64) (Jepsen's
  // usual domain) through a direct table, others by a linear scan while the register has taken
  // few values, then a map.
  std::unordered_map<int64_t, int32_t>& sid = sc.sid;
  sid.clear();
  int32_t small_id[64];
  std::memset(small_id, 0, sizeof(small_id));
  auto find_id = [&](int64_t v) -> int32_t {  // 0 = not seen
    if ((uint64_t)v < 64) return small_id[v];
    if (o.state_val.size() <= 32) {
      for (size_t k = 0; k < o.state_val.size(); ++k)
        if (o.state_val[k] == v) return (int32_t)k + 1;
      return 0;
    }
    auto it = sid.find(v);
    return it == sid.end() ? 0 : it->second;
  };
  if (model == LC_MODEL_CAS_REGISTER) {
    for (const Op& op : ops) {
      if (op.status == T_FAIL) continue;
      int64_t v;
      if (op.f == F_WRITE && op.vflags == V_SCALAR) v = op.v0;
      else if (op.f == F_CAS && op.vflags == V_PAIR) v = op.v1;
      else continue;
      if (find_id(v)) continue;
      o.state_val.push_back(v);
      const int32_t id = (int32_t)o.state_val.size();
      if ((uint64_t)v < 64) small_id[v] = id;
      if (id == 33)  // switch to the map: index every value seen so far
        for (size_t k = 0; k < o.state_val.size(); ++k) sid.emplace(o.state_val[k], (int32_t)k + 1);
      else if (id > 33)
        sid.emplace(v, id);
    }
  }
  // every op's operands, in invocation order (the first model error, in that order, wins)
  for (Op& op : ops) {
    if (op.status == T_FAIL) continue;  // failed ops never enter the search
    int64_t oa, ob;
    if (const char* m = operands(model, op, find_id, op.kind, oa, ob)) {
      o.live_max = 0;
      return fail(LC_H_MODEL, m);
    }
    op.oa = oa, op.ob = ob;
  }
  // LeaderModel (leader.clj:63-75): the state is the set of (term, leader) pairs of the
  // linearized ops, and a step is inconsistent iff the state holds the op's term with another
  // leader. Only a term that carries two or more leaders in this history can ever conflict: its
  // pairs ("contested") get state bits in first-appearance order; every other op steps with
  // a = b = 0 (always consistent; its pair changes no later decision). A nil value is (leader
  // nil = id -1, term nil).
  if (model == LC_MODEL_LEADER) {
    struct Term { int64_t term, first_leader; bool nil, contested; };
    struct Pair { int64_t term, leader; bool nil; };
    std::vector<Term> terms;
    std::unordered_map<int64_t, int32_t> term_at;  // integer term -> terms[]
    int32_t nil_term = -1;
    auto key_of = [](const Op& op, int64_t& t, int64_t& l, bool& nil) {
      nil = op.vflags == V_NIL;
      t = nil ? 0 : op.v1;
      l = nil ? -1 : op.v0;
    };
    auto find_term = [&](int64_t t, bool nil) -> int32_t {
      if (nil) return nil_term;
      auto it = term_at.find(t);
      return it == term_at.end() ? -1 : it->second;
    };
    for (const Op& op : ops) {
      if (op.status == T_FAIL) continue;
      int64_t t, l;
      bool nil;
      key_of(op, t, l, nil);
      const int32_t k = find_term(t, nil);
      if (k < 0) {
        if (nil) nil_term = (int32_t)terms.size();
        else term_at.emplace(t, (int32_t)terms.size());
        terms.push_back(Term{t, l, nil, false});
      } else if (terms[k].first_leader != l) {
        terms[k].contested = true;
      }
    }
    std::vector<Pair> pairs;
    std::vector<int32_t> pair_term;
    for (Op& op : ops) {
      if (op.status == T_FAIL) continue;
      int64_t t, l;
      bool nil;
      key_of(op, t, l, nil);
      const int32_t k = find_term(t, nil);
      op.oa = op.ob = 0;
      if (!terms[k].contested) continue;
      int bit = -1;
      for (size_t q = 0; q < pairs.size(); ++q)
        if (pair_term[q] == k && pairs[q].leader == l) bit = (int)q;
      if (bit < 0) {
        if ((int)pairs.size() == LEADER_MAX_PAIRS) {
          o.live_max = 0;
          return fail(LC_H_CAPACITY, "more than 64 contested (term, leader) pairs");
        }
        bit = (int)pairs.size();
        pairs.push_back(Pair{t, l, nil});
        pair_term.push_back(k);
      }
      op.ob = (int64_t)(1ull << bit);
    }
    for (Op& op : ops) {  // a = the op term's other pairs
      if (op.status == T_FAIL || !op.ob) continue;
      const int bit = __builtin_ctzll((uint64_t)op.ob);
      uint64_t a = 0;
      for (size_t q = 0; q < pairs.size(); ++q)
        if (pair_term[q] == pair_term[bit] && (int)q != bit) a |= 1ull << q;
      op.oa = (int64_t)a;
    }
  }

  // ---- RETURN steps with slot assignment (the policy above, else lowest free slot first).
  // Error precedence: a model error anywhere (above), then > 65535 register values, then > 63
  // pending ops.
  o.step_slot.resize(n_ok);
  o.step_ninv.resize(n_ok);
  o.step_cmp_idx.resize(n_ok);
  o.step_inv_idx.resize(n_ok);
  o.inv_slot.resize(ops.size());
  o.inv_kind.resize(ops.size());
  o.inv_a.resize(ops.size());
  o.inv_b.resize(ops.size());
  o.inv_index.resize(ops.size());
  uint8_t* const s_slot = o.step_slot.data();
  int64_t* const s_ninv = o.step_ninv.data();
  int64_t* const s_cmp = o.step_cmp_idx.data();
  int64_t* const s_inv = o.step_inv_idx.data();
  uint8_t* const i_slot = o.inv_slot.data();
  uint8_t* const i_kind = o.inv_kind.data();
  int64_t* const i_a = o.inv_a.data();
  int64_t* const i_b = o.inv_b.data();
  int64_t* const i_index = o.inv_index.data();
  int64_t ns = 0, ni = 0;
  const char* wide = nullptr;
  uint64_t used = 0;
  int64_t ninv_cur = 0;
  int live_max = 0;
  for (int64_t i = b; i < e && !wide; ++i) {
    const int32_t k = op_of[i - b];
    Op& op = ops[k];  // (every entry belongs to an op once pairing succeeded)
    const int8_t t = a.type[i];
    if (t == T_INVOKE) {
      if (op.status == T_FAIL) continue;  // failed ops never enter the search
      if (used == ~0ull >> (64 - MAX_SLOTS)) {
        wide = "more than 63 pending ops";
        break;
      }
      int sl = __builtin_ctzll(~used);
      if (sl < n_iw && !op.inword && !slots_lff) {
        const int hi = __builtin_ctzll(~(used | ((1ull << n_iw) - 1)));  // the lowest free slot >= n_iw
        const int npend = __builtin_popcountll(used) + 1;
        if (hi < std::max(npend, n_iw)) sl = hi;  // (no wider than lowest-free-first)
      }
      used |= 1ull << sl;
      op.slot = (uint8_t)sl;
      live_max = std::max(live_max, 64 - __builtin_clzll(used));
      i_slot[ni] = (uint8_t)sl;
      i_kind[ni] = op.kind;
      i_a[ni] = op.oa;
      i_b[ni] = op.ob;
      i_index[ni] = IDX(i);  // (the invocation entry itself)
      ++ni;
      ninv_cur++;
    } else if (t == T_OK) {
      s_slot[ns] = op.slot;
      s_ninv[ns] = ninv_cur;
      s_cmp[ns] = IDX(i);
      s_inv[ns] = IDX(op.inv_pos);
      ++ns;
      ninv_cur = 0;
      used &= ~(1ull << op.slot);
    }
  }
  o.live_max = live_max;
  o.step_slot.resize(ns);
  o.step_ninv.resize(ns);
  o.step_cmp_idx.resize(ns);
  o.step_inv_idx.resize(ns);
  o.inv_slot.resize(ni);  // (trimmed below to the invocations before the last RETURN)
  if (model == LC_MODEL_CAS_REGISTER) {
    o.n_states = (int32_t)o.state_val.size() + 1;
    if (o.n_states > 65535) {
      o.live_max = 0;
      return fail(LC_H_WIDE, "more than 65535 distinct register values");
    }
  }
  if (wide) return fail(LC_H_WIDE, wide);
  // invocations after the last RETURN never matter: drop them
  size_t keep = o.inv_slot.size() - (size_t)ninv_cur;
  o.inv_slot.resize(keep);
  o.inv_kind.resize(keep);
  o.inv_a.resize(keep);
  o.inv_b.resize(keep);
  o.inv_index.resize(keep);
}

std::vector<OneOut>& parts_of_thread() {
  thread_local std::vector<OneOut> parts;
  return parts;
}

}  // namespace

void encode_trim() { std::vector<OneOut>().swap(parts_of_thread()); }

// the sink's view of history h of enc (built from enc's concatenated arrays); ninv = scratch
static HistView view_of(const Encoded& enc, int h, std::vector<int64_t>& ninv) {
  const int64_t g0 = enc.step_off[h], m = enc.step_off[h + 1] - g0;
  ninv.resize((size_t)m);
  for (int64_t s = 0; s < m; ++s) ninv[s] = enc.inv_off[g0 + s + 1] - enc.inv_off[g0 + s];
  const int64_t q0 = m > 0 ? enc.inv_off[g0] : 0;
  return HistView{enc.err[h], enc.live_max[h], enc.n_states[h], enc.err[h] ? 0 : m, enc.step_slot.data() + g0,
                  ninv.data(), enc.inv_slot.data() + q0, enc.inv_a.data() + q0, enc.inv_b.data() + q0,
                  enc.inv_kind.data() + q0};
}

void encoded_subset(const Encoded& all, const std::vector<int>& hs, Encoded& out, const HistSink* sink) {
  const int n = (int)hs.size();
  out.model = all.model;
  out.n_hist = n;
  out.init_value = all.init_value;
  out.step_off.assign(n + 1, 0);
  out.state_off.assign(n + 1, 0);
  out.err.resize(n);
  out.errmsg.resize(n);
  out.live_max.resize(n);
  out.n_states.resize(n);
  out.n_ops.resize(n);
  // the sink sees each history straight from `all`; the per-invocation arrays of a history it
  // takes (its step stream is built) are not copied, as encode() leaves them out
  std::vector<char> taken(n, 0);
  if (sink)
    Pool::get().run(n, all.total_steps() < 100000 ? 1 : 16, [&](int i) {
      thread_local std::vector<int64_t> ninv;
      taken[i] = (*sink)(i, view_of(all, hs[i], ninv));
    });
  std::vector<int64_t> inv_base(n + 1, 0);
  for (int i = 0; i < n; ++i) {
    const int h = hs[i];
    out.err[i] = all.err[h];
    out.errmsg[i] = all.errmsg[h];
    out.live_max[i] = all.live_max[h];
    out.n_states[i] = all.n_states[h];
    out.n_ops[i] = all.n_ops[h];
    const int32_t g0 = all.step_off[h], g1 = all.step_off[h + 1];
    out.step_off[i + 1] = out.step_off[i] + (g1 - g0);
    out.state_off[i + 1] = out.state_off[i] + (all.state_off[h + 1] - all.state_off[h]);
    inv_base[i + 1] = inv_base[i] + (taken[i] ? 0 : all.inv_off[g1] - all.inv_off[g0]);
  }
  const int64_t ns = out.step_off[n], ni = inv_base[n];
  out.state_val.resize(out.state_off[n]);
  out.step_slot.resize(ns);
  out.step_cmp_idx.resize(ns);
  out.step_inv_idx.resize(ns);
  out.inv_off.resize(ns + 1);
  out.inv_off[0] = 0;
  out.inv_slot.resize(ni);
  out.inv_kind.resize(ni);
  out.inv_a.resize(ni);
  out.inv_b.resize(ni);
  out.inv_index.resize(ni);
  Pool::get().run(n, ns < 100000 ? 1 : 16, [&](int i) {
    const int h = hs[i];
    const int64_t g0 = all.step_off[h], m = all.step_off[h + 1] - g0, s0 = out.step_off[i];
    std::copy_n(all.state_val.begin() + all.state_off[h], all.state_off[h + 1] - all.state_off[h],
                out.state_val.begin() + out.state_off[i]);
    std::copy_n(all.step_slot.begin() + g0, m, out.step_slot.begin() + s0);
    std::copy_n(all.step_cmp_idx.begin() + g0, m, out.step_cmp_idx.begin() + s0);
    std::copy_n(all.step_inv_idx.begin() + g0, m, out.step_inv_idx.begin() + s0);
    const int64_t o0 = inv_base[i];
    if (taken[i]) {
      for (int64_t s = 0; s < m; ++s) out.inv_off[s0 + s + 1] = o0;
      return;
    }
    const int64_t q0 = all.inv_off[g0], qn = all.inv_off[g0 + m] - q0;
    for (int64_t s = 0; s < m; ++s) out.inv_off[s0 + s + 1] = o0 + (all.inv_off[g0 + s + 1] - q0);
    std::copy_n(all.inv_slot.begin() + q0, qn, out.inv_slot.begin() + o0);
    std::copy_n(all.inv_kind.begin() + q0, qn, out.inv_kind.begin() + o0);
    std::copy_n(all.inv_a.begin() + q0, qn, out.inv_a.begin() + o0);
    std::copy_n(all.inv_b.begin() + q0, qn, out.inv_b.begin() + o0);
    std::copy_n(all.inv_index.begin() + q0, qn, out.inv_index.begin() + o0);
  });
}

void sink_encoded(const Encoded& enc, const HistSink& sink) {
  const int64_t ns = enc.total_steps();
  Pool::get().run(enc.n_hist, ns < 100000 ? 1 : 16, [&](int h) {
    thread_local std::vector<int64_t> ninv;
    sink(h, view_of(enc, h, ninv));
  });
}

void encode(int model, int64_t init_value, int n_hist, const int64_t* hist_off,
            const HistArrays& a, Encoded& out, const HistSink* sink) {
  out.model = model;
  out.n_hist = n_hist;
  out.init_value = init_value;
  // per-history parts, kept per calling thread across calls (their buffers keep capacity;
  // encode_trim frees them)
  std::vector<OneOut>& parts_tl = parts_of_thread();
  if ((int)parts_tl.size() < n_hist) parts_tl.resize(n_hist);
  for (int h = 0; h < n_hist; ++h) {
    OneOut& o = parts_tl[h];
    o.err = 0, o.msg.clear(), o.live_max = 0, o.n_states = 1, o.n_ops = 0;
    o.state_val.clear();
  }
  std::vector<OneOut>& parts = parts_tl;
  // the process's worker pool (pool.hpp): its threads persist, so their scratch stays warm
  const int nt = hist_off[n_hist] - hist_off[0] < 200000 ? 1 : 16;
  auto run = [&](auto&& fn) {  // fn(h) over every history
    Pool::get().run(n_hist, nt, std::function<void(int)>(fn));
  };
  thread_local std::vector<char> taken_tl;
  taken_tl.assign(n_hist, 0);
  std::vector<char>& taken = taken_tl;
  run([&](int h) {
    OneOut& o = parts[h];
    encode_one(model, a, hist_off[h], hist_off[h + 1], o);
    if (sink)
      taken[h] = (*sink)(h, HistView{o.err, o.live_max, o.n_states, o.err ? 0 : (int64_t)o.step_slot.size(),
                                     o.step_slot.data(), o.step_ninv.data(), o.inv_slot.data(), o.inv_a.data(),
                                     o.inv_b.data(), o.inv_kind.data()});
  });

  // concatenate: offsets first, then every history's part copied in parallel
  out.step_off.assign(n_hist + 1, 0);
  out.state_off.assign(n_hist + 1, 0);
  std::vector<int64_t> inv_base(n_hist + 1, 0);
  out.err.resize(n_hist);
  out.errmsg.resize(n_hist);
  out.live_max.resize(n_hist);
  out.n_states.resize(n_hist);
  out.n_ops.resize(n_hist);
  for (int h = 0; h < n_hist; ++h) {
    OneOut& o = parts[h];
    if (o.err) {  // a failed history contributes no steps
      o.step_slot.clear();
      o.step_ninv.clear();
      o.inv_slot.clear();
    }
    out.err[h] = o.err;
    out.errmsg[h] = std::move(o.msg);
    out.live_max[h] = o.live_max;
    out.n_states[h] = o.n_states;
    out.n_ops[h] = o.n_ops;
    out.step_off[h + 1] = out.step_off[h] + (int32_t)o.step_slot.size();
    out.state_off[h + 1] = out.state_off[h] + (int64_t)o.state_val.size();
    inv_base[h + 1] = inv_base[h] + (o.err || taken[h] ? 0 : (int64_t)o.inv_slot.size());
  }
  const int64_t ns = out.step_off[n_hist], ni = inv_base[n_hist];
  out.state_val.resize(out.state_off[n_hist]);
  out.step_slot.resize(ns);
  out.step_cmp_idx.resize(ns);
  out.step_inv_idx.resize(ns);
  out.inv_off.resize(ns + 1);
  out.inv_off[0] = 0;
  out.inv_slot.resize(ni);
  out.inv_kind.resize(ni);
  out.inv_a.resize(ni);
  out.inv_b.resize(ni);
  out.inv_index.resize(ni);
  run([&](int h) {
    const OneOut& o = parts[h];
    std::copy(o.state_val.begin(), o.state_val.end(), out.state_val.begin() + out.state_off[h]);
    const int64_t s0 = out.step_off[h];
    int64_t ib = inv_base[h];
    const bool keep_inv = !o.err && !taken[h];
    for (size_t s = 0; s < o.step_slot.size(); ++s) {
      out.step_slot[s0 + s] = o.step_slot[s];
      out.step_cmp_idx[s0 + s] = o.step_cmp_idx[s];
      out.step_inv_idx[s0 + s] = o.step_inv_idx[s];
      if (keep_inv) ib += o.step_ninv[s];
      out.inv_off[s0 + s + 1] = ib;
    }
    if (keep_inv) {
      const int64_t q0 = inv_base[h];
      std::copy(o.inv_slot.begin(), o.inv_slot.end(), out.inv_slot.begin() + q0);
      std::copy(o.inv_kind.begin(), o.inv_kind.end(), out.inv_kind.begin() + q0);
      std::copy(o.inv_a.begin(), o.inv_a.end(), out.inv_a.begin() + q0);
      std::copy(o.inv_b.begin(), o.inv_b.end(), out.inv_b.begin() + q0);
      std::copy(o.inv_index.begin(), o.inv_index.end(), out.inv_index.begin() + q0);
    }
  });
}

}  // namespace lc
