// ctab.hip — counter closure tables (see ctab.hpp): knossos.linear/analysis [ext] (SURVEY §8(a)
// a5) with CounterModel.step (a7, src/jepsen/jgroups/workload/counter.clj:100-127) applied to
// whole bitmaps of configs, one history per 1024-thread workgroup, the table in LDS.
//
// One RETURN step of slot j on table B (bit (w, p) = "the config with mask (w << 6) | p exists";
// R = configs produced by a consistent step, X = the frontier before the step):
//   for hi-layer q = 0..H (words w of popcount q over the live slots >= 6), in parallel:
//     j hi and j ∈ w : R = B[w \ j] & G_j(w \ j)           (configs holding j are never expanded)
//     otherwise      : R = ∪_{b ∈ w} B[w \ b] & G_b(w \ b)   (pulls from finished words)
//                      then the in-word closure over the live low slots k != j (each op's gated
//                      transfer (X | R) & G_k moved up by 2^k, repeated until nothing changes)
//                      and, when j is a low slot, one final j transfer
//     explored += popcount(R);  B[w] = X | R
//   return j: B'[m] = B[m ∪ j] for m ∌ j                   B' empty => invalid at this RETURN
// G_k(v) = the positions p of word v whose config may step op k: every position for an
// unconstrained op, else those with S_lo(p) = req_k - base - S_hi(v) (an EQ lookup), minus the
// positions holding k (and j: configs holding the returning op are never expanded).
// Every config reachable by linearizing pending calls is produced at exactly its own mask,
// whose predecessors are final earlier, so R is the sparse search's closure set and
// popcount(R) its explored count, bit-exact with the oracle.
//
// Steps are pipelined as the register tables' history_pipe (dense.hip): step t's
// layer q runs in the same super-layer as step t-1's layer q + 2 (q + 1 after an in-word return
// on double-buffered tables); one workgroup barrier ends a super-layer; step t reads its
// frontier X through step t-1's returning slot from step t-1's table, so the return is never
// applied in place. A ring of decoded steps holds each step's per-slot requirements, its EQ
// table and its hi-slot delta sums.
#include "ctab.hpp"
#include "dense.hpp"
#include "search.hpp"
#include "dense_ops.hpp"
#include "device_common.hpp"

namespace lc {
namespace {

constexpr int CT_TEAM = 1024;  // (r4i: 512 threads, two passes per super-layer, 30.7 -> 41.4 ms on C2c)
constexpr int CT_RING = 16;
constexpr int CT_CAPW = 1 << (CTAB_LMAX - CTAB_LO);  // LDS table words (128 KiB)
constexpr int CT_BINOM = 24;
constexpr int32_t CQ_UNC = 0x3fffffff;   // cq sentinel: the op steps from any config
constexpr int32_t CQ_NEVER = -0x3fffffff;  // ... from none (out of the EQ range whatever the sum)
constexpr int CT_PIPE_DBL = 1;
constexpr int CT_PIPE_DYN = 2;  // LC_CTAB_PIPE bit 1: multi-pass super-layers' chunks from an LDS counter

struct __attribute__((aligned(16))) CStep {
  uint32_t live, fresh, anyx;
  int32_t base;              // sum of the deltas of the ops returned before this step
  int32_t j, jp, H, start;   // returning slot, previous step's, layers - 1, first super-layer
  int32_t pstart, hpl, Hl, tb;  // tile teams: the previous step's start and local layers - 1, this
                                // step's local layers - 1 and live team bits (ctab_team_kernel)
  uint64_t keep_lo;          // positions without a fresh low slot
  int32_t req[32];           // per slot: requirement relative to init (CQ_UNC / CQ_NEVER)
  int32_t cq[32];            // per slot: EQ index base (k < 6: req - base - lo_min; k >= 6: + d_k)
  int8_t d[32];              // per slot: delta
  int16_t sh[3][128];        // sums of the hi slots' deltas: slots 6..12 by w & 127, 13..19 by
                             // (w >> 7) & 127, 20..26 by w >> 14 (tile teams, to CTAB_TEAM_LMAX)
  uint64_t eq[64];           // EQ[v]: positions p with S_lo(p) - lo_min = v
};

__device__ __forceinline__ int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }
template <typename T>
__device__ __forceinline__ T rdl(T v, int l) {
  return (T)__builtin_amdgcn_readlane((int)v, l);
}

// positions (of 64) whose mask lacks low slot k
__device__ __forceinline__ uint64_t keep6(int k) {
  switch (k) {
    case 0: return 0x5555555555555555ull;
    case 1: return 0x3333333333333333ull;
    case 2: return 0x0f0f0f0f0f0f0f0full;
    case 3: return 0x00ff00ff00ff00ffull;
    case 4: return 0x0000ffff0000ffffull;
    default: return 0x00000000ffffffffull;
  }
}

__device__ __forceinline__ uint64_t gate(const CStep* st, int32_t c, int s) {
  if (c == CQ_UNC) return ~0ull;
  const uint32_t i = (uint32_t)(c - s);
  return i < 64u ? st->eq[i] : 0ull;
}

// per-wave window of 128 words over a history's step stream: lane i holds words base + i and
// base + 64 + i (a step is at most 1 + 2 * CTAB_MAX_NINV = 63 words)
struct StreamWin {
  int64_t base = -(1ll << 40);
  uint32_t w0 = 0, w1 = 0;
  __device__ __forceinline__ void need(const CtabParams& p, int64_t pos, int lane) {
    if (pos + 64 > base + 128) {
      base = pos;
      w0 = (base + lane < p.stream_words) ? p.stream[base + lane] : 0u;
      w1 = (base + 64 + lane < p.stream_words) ? p.stream[base + 64 + lane] : 0u;
    }
  }
  __device__ __forceinline__ uint32_t at(int64_t pos) const {
    const int off = (int)(pos - base);
    const uint32_t a = (uint32_t)__shfl((int)w0, off & 63, 64), b = (uint32_t)__shfl((int)w1, off & 63, 64);
    return off < 64 ? a : b;
  }
};

// Decode the step at pos into dst (one whole wave): the per-slot requirements and deltas are
// the previous step's plus this step's invocations; then the derived tables (cq, EQ, hi sums).
__device__ __forceinline__ void ct_decode(const CtabParams& p, StreamWin& sw, int64_t& pos, int lane, CStep* dst,
                                          const CStep* prev) {
  sw.need(p, pos, lane);
  const uint32_t H0 = (uint32_t)rfl((int)sw.at(pos));
  const uint32_t wd = sw.at(pos + 1 + lane);
  const int nw = (int)__builtin_ctzll(~__ballot(lane < 2 * CTAB_MAX_NINV && (wd & DENSE_OPW)));
  const int ninv = nw >> 1;
  const uint32_t w0 = sw.at(pos + 1 + 2 * lane), w1 = sw.at(pos + 2 + 2 * lane);
  // lane k < 32: slot k's requirement and delta after this step's invocations
  int32_t req = prev && lane < 32 ? prev->req[lane] : CQ_UNC;
  int32_t d = prev && lane < 32 ? (int32_t)prev->d[lane] : 0;
  for (int i = 0; i < ninv; ++i) {
    const uint32_t a = (uint32_t)rdl((int)w0, i), b = (uint32_t)rdl((int)w1, i);
    if (lane == (int)(a & 31u)) {
      const uint32_t fl = (a >> 8) & 0xffu;
      d = (int32_t)(int8_t)(uint8_t)((a >> 16) & 0xffu);
      req = (fl & CT_UNC) ? CQ_UNC : (fl & CT_NEVER) ? CQ_NEVER : (int32_t)(b & 0x3fffffffu) - CTAB_REQ_BIAS;
    }
  }
  const uint32_t plive = prev ? (uint32_t)rfl((int)prev->live) : 0u;
  const int pj = prev ? rfl(prev->j) : -1;
  const int32_t base = prev ? rfl(prev->base) + (int32_t)prev->d[pj] : 0;
  // low sums: lane p = the sum of the deltas of p's slots; lo_min = the smallest
  int32_t slo = 0, lo_min = 0;
#pragma unroll
  for (int k = 0; k < CTAB_LO; ++k) {
    const int32_t dk = rdl(d, k);
    if ((lane >> k) & 1) slo += dk;
    lo_min += dk < 0 ? dk : 0;
  }
  if (lane < 32) {
    dst->req[lane] = req;
    dst->d[lane] = (int8_t)d;
    dst->cq[lane] = req == CQ_UNC || req == CQ_NEVER ? req : req - base - lo_min + (lane >= CTAB_LO ? d : 0);
  }
  dst->eq[lane] = 0;
  // (one wave's LDS operations stay in order: the zeroing lands before the ORs)
  __hip_atomic_fetch_or(&dst->eq[slo - lo_min], 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  // hi sums: entries lane and lane + 64 of both halves
#pragma unroll
  for (int half = 0; half < 3; ++half)
#pragma unroll
    for (int e2 = 0; e2 < 2; ++e2) {
      const int e = lane + 64 * e2;
      int32_t s = 0;
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        const int32_t dk = CTAB_LO + 7 * half + k < 32 ? rdl(d, CTAB_LO + 7 * half + k) : 0;
        if ((e >> k) & 1) s += dk;
      }
      dst->sh[half][e] = (int16_t)s;
    }
  if (lane == 0) {
    const uint32_t live = H0 & DENSE_LIVE_MASK;
    const int L = live ? 32 - __clz((int)live) : 0;
    const uint32_t fresh = prev ? live & ~(plive & ~(1u << pj)) : live;
    uint64_t kl = ~0ull;
    for (int k = 0; k < CTAB_LO; ++k)
      if (fresh & (1u << k)) kl &= keep6(k);
    dst->live = live;
    dst->fresh = fresh;
    dst->anyx = 0;
    dst->base = base;
    dst->j = (int)((H0 >> DENSE_J_SHIFT) & 31u);
    dst->jp = pj;
    dst->H = L > CTAB_LO ? L - CTAB_LO : 0;
    dst->start = 1 << 30;  // not started
    dst->keep_lo = kl;
  }
  pos += 1 + nw;
}

// word w's frontier before step (fresh, jp): step jp's post-return table, read in place
__device__ __forceinline__ uint64_t ct_x(const uint64_t* B, uint32_t w, uint32_t fresh_hi, int jp, uint64_t keep_lo) {
  if (w & fresh_hi) return 0;
  uint64_t v;
  if (jp >= CTAB_LO) v = B[w | (1u << (jp - CTAB_LO))];
  else if (jp >= 0) v = (B[w] & ~keep6(jp)) >> (1 << jp);
  else v = B[w];
  return v & keep_lo;
}

// One step's closure of word w (its frontier X): the hi pulls and the in-word closure. Returns R.
// pf (builds with LC_CT_WORDPROF and LC_DEBUG, else null): cycles to the hi sums, the pulls, the
// gates, the closure; closure sweeps. (Compiled out by default: the checks alone cost C2c 3 %.)
// wg: the word's hi bits over the whole table (a tile team's tile holds the words w | rank << lb),
// which set its delta sum; R0: pulls already made from other tiles (gated).
__device__ __forceinline__ uint64_t ct_word(const uint64_t* Bt, uint32_t w, const CStep* st, uint32_t live, int j,
                                            uint64_t X, uint32_t wg, uint64_t R0,
                                            unsigned long long* pf = nullptr) {
#ifdef LC_CT_WORDPROF
  unsigned long long tp = pf ? __builtin_amdgcn_s_memtime() : 0;
  auto pmark = [&](int k) {
    if (pf) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const unsigned long long tn = __builtin_amdgcn_s_memtime();
      pf[k] += tn - tp;
      tp = tn;
    }
  };
#else
  auto pmark = [](int) {};
#endif
  const int s_hi = (int)st->sh[0][wg & 127u] + (int)st->sh[1][(wg >> 7) & 127u] + (int)st->sh[2][(wg >> 14) & 127u];
  pmark(0);
  const bool jhi = j >= CTAB_LO;
  // (a tile team's j above the tile's local slots gives jh 0 here: that tile pulls it remotely)
  const uint32_t jh = jhi && j - CTAB_LO < 32 ? 1u << (j - CTAB_LO) : 0u;
  uint32_t m = (w & jh) ? jh : w;
  uint64_t R = R0;
  while (m) {  // the word's set hi bits, two at a time (their loads issued together; r4b A/B: a batch
               // of four with every EQ lookup issued at once was 3 % slower on C2c)
    int b[2];
    uint64_t v[2];
    int32_t c[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      b[u] = m ? __builtin_ctz(m) : -1;
      m &= m - 1;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      v[u] = b[u] >= 0 ? Bt[w ^ (1u << b[u])] : 0ull;
      c[u] = b[u] >= 0 ? st->cq[CTAB_LO + b[u]] : CQ_NEVER;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) R |= v[u] & gate(st, c[u], s_hi);
  }
  pmark(1);
  if (w & jh) return R;  // a word holding j (hi) is produced by linearizing j last only
  const uint64_t notj = jhi ? ~0ull : keep6(j);
  R &= notj;
  const uint32_t lo = live & 63u & ~(jhi ? 0u : 1u << j);
  uint64_t G[CTAB_LO];
#ifdef LC_CT_GATES_BATCH
  {  // the low slots' EQ bases (one broadcast read each), then their six EQ words, all issued at once
    int32_t cl[CTAB_LO];
    uint64_t el[CTAB_LO];
#pragma unroll
    for (int k = 0; k < CTAB_LO; ++k) cl[k] = st->cq[k];
#pragma unroll
    for (int k = 0; k < CTAB_LO; ++k) el[k] = st->eq[(uint32_t)(cl[k] - s_hi) & 63u];
#pragma unroll
    for (int k = 0; k < CTAB_LO; ++k) {
      const uint32_t i = (uint32_t)(cl[k] - s_hi);
      const uint64_t g = cl[k] == CQ_UNC ? ~0ull : i < 64u ? el[k] : 0ull;
      G[k] = ((live >> k) & 1u) ? g & keep6(k) & notj : 0ull;
    }
  }
#else
#pragma unroll
  for (int k = 0; k < CTAB_LO; ++k) G[k] = ((live >> k) & 1u) ? gate(st, st->cq[k], s_hi) & keep6(k) & notj : 0ull;
#endif
  pmark(2);
  for (;;) {  // the in-word closure: gated transfers until nothing changes
    const uint64_t R0 = R;
#pragma unroll
    for (int k = 0; k < CTAB_LO; ++k)
      if ((lo >> k) & 1u) R |= ((X | R) & G[k]) << (1 << k);
#ifdef LC_CT_WORDPROF
    if (pf) pf[4] += 1;
#endif
    if (R == R0) break;
  }
  pmark(3);
  if (!jhi) {  // the returning op, linearized last
#pragma unroll
    for (int k = 0; k < CTAB_LO; ++k)
      if (k == j) R |= ((X | R) & G[k]) << (1 << k);
  }
  return R;
}

__device__ __forceinline__ void init_binom(uint32_t* binom, int tid, int nthreads) {
  for (int i = tid; i < CT_BINOM * CT_BINOM; i += nthreads) {
    const int n = i / CT_BINOM, k = i % CT_BINOM;
    uint32_t c = 0;
    if (k <= n) {
      uint64_t v = 1;
      for (int q = 1; q <= k; ++q) v = v * (uint64_t)(n - k + q) / (uint64_t)q;
      c = (uint32_t)v;
    }
    binom[i] = c;
  }
}

__global__ void __launch_bounds__(CT_TEAM) ctab_kernel(CtabParams p) {
  __shared__ uint64_t sTab[CT_CAPW];
  __shared__ CStep sRing[CT_RING];
  __shared__ uint32_t sBinom[CT_BINOM * CT_BINOM];
  __shared__ uint32_t sWOff[CT_BINOM + 2];
  __shared__ int sQ;
  __shared__ unsigned long long sExpl;
  __shared__ uint32_t sChunk[2];  // CT_PIPE_DYN: the super-layers' chunk counters (by parity)
  const int tt = threadIdx.x, lane = tt & 63;
  const bool decoder = tt >= CT_TEAM - 64;  // the last wave: packed passes fill the low threads first
  init_binom(sBinom, tt, CT_TEAM);
  if (tt <= DENSE_WORD_BITS + 1) {  // offsets of the global list's popcount layers
    uint32_t o = 0;
    for (int q = 0; q < tt; ++q) {
      uint64_t v = 1;
      for (int i = 1; i <= q; ++i) v = v * (uint64_t)(DENSE_WORD_BITS - q + i) / (uint64_t)i;
      o += (uint32_t)v;
    }
    sWOff[tt] = o;
  }
  __syncthreads();
  unsigned long long st_fout = 0, st_steps = 0;
  for (;;) {
    if (tt == 0) sQ = atomicAdd(p.queue, 1), sExpl = 0;
    __syncthreads();
    const int qi = sQ;
    if (qi >= p.n) break;
    const int h = p.order[qi];
    if (p.stamps && tt == 0) p.stamps[2 * h] = __builtin_amdgcn_s_memrealtime();
    const int lmax = p.lmax[h];
    const int ns = p.nsteps[h];
    const int Hh = lmax > CTAB_LO ? lmax - CTAB_LO : 0;
    const int NW = 1 << Hh;
    const bool dbl = (p.pipe & CT_PIPE_DBL) && 2 * NW <= CT_CAPW;
    uint64_t* const B = sTab;
    uint64_t* const B2 = dbl ? sTab + NW : sTab;
    auto tab = [&](int t) { return (t & 1) ? B2 : B; };
    const int ntab = dbl ? 2 * NW : NW;
    for (int i = tt; i < ntab; i += CT_TEAM) sTab[i] = 0;
    // the word list in the LDS left beside the tables (layers of the Hh-bit words), else global
    const uint32_t* words = p.words;
    const uint32_t* wofs = sWOff;
    uint32_t* const lw = reinterpret_cast<uint32_t*>(sTab + ntab);
    uint32_t* const lo = lw + NW;
    const bool lds_list = Hh > 0 && ntab + NW / 2 + 16 <= CT_CAPW;
    if (lds_list) {
      if (tt <= Hh + 1) {
        uint32_t o = 0;
        for (int q = 0; q < tt; ++q) o += sBinom[Hh * CT_BINOM + q];
        lo[tt] = o;
      }
      __syncthreads();
      for (int q = 0; q <= Hh; ++q) {
        const uint32_t nq = sBinom[Hh * CT_BINOM + q], og = sWOff[q], ol = lo[q];
        for (uint32_t r = (uint32_t)tt; r < nq; r += (uint32_t)CT_TEAM) lw[ol + r] = p.words[og + r];
      }
      words = lw, wofs = lo;
    }
    __syncthreads();
    if (tt == 0) B2[0] = 1;  // the initial config: nothing linearized (step 0 reads tab(-1))
    if (tt < 2) sChunk[tt] = 0u;
    StreamWin sw;
    int64_t pos = p.sbeg[h];
    if (ns > 0 && decoder) {
      ct_decode(p, sw, pos, lane, &sRing[0], nullptr);
      if (lane == 0) sRing[0].start = 0;
    }
    __syncthreads();
    unsigned long long expl = 0;
    int fail_t = -1;
    int t_dec = ns > 0 ? 1 : 0, t_run = t_dec, t_ret = 0;  // decoded, started, retired
    // LC_DEBUG: super-layer phase cycles of every wave (s_memtime) and the words it closed
    const bool prof = p.prof != nullptr;
    unsigned long long ph[4] = {0, 0, 0, 0}, tp = prof ? __builtin_amdgcn_s_memtime() : 0, nsl = 0, nwd = 0;
    unsigned long long pw[6] = {0, 0, 0, 0, 0, 0};  // a word's phases (ct_word's pf), + to the word
    auto mark = [&](int k) {
      if (prof) {
        const unsigned long long tnow = __builtin_amdgcn_s_memtime();
        ph[k] += tnow - tp;
        tp = tnow;
      }
    };
    for (int s = 0; t_ret < ns; ++s) {
      // ---- ring view: lane i = step t_ret + i (decoded steps only)
      const int tl = t_ret + lane;
      const bool dec_l = lane < CT_RING && tl < t_dec;
      uint4 h0 = {0u, 0u, 0u, 0u};
      int4 h1 = {0, 0, 0, 1 << 30};
      if (dec_l) {
        const CStep* st = &sRing[tl % CT_RING];
        h0 = *reinterpret_cast<const uint4*>(&st->live);  // live, fresh, anyx, base
        h1 = *reinterpret_cast<const int4*>(&st->j);      // j, jp, H, start
      }
      const bool run_l = dec_l && tl < t_run;
      // retire the steps whose last layer ran in an earlier super-layer, in order
      const bool fin_l = run_l && h1.w + h1.z < s;
      const uint64_t fin = __ballot(fin_l);
      const int lead = (int)__builtin_ctzll(~fin);
      const uint64_t lead_mask = lead >= 64 ? ~0ull : (1ull << lead) - 1;
      const uint64_t bad = __ballot(fin_l && tl > 0 && h0.z == 0u) & lead_mask;
      if (bad) {  // step (first such) - 1 returned an empty frontier
        fail_t = t_ret + (int)__builtin_ctzll(bad) - 1;
        break;
      }
      const int t_ret_old = t_ret;
      t_ret += lead;
      if (t_ret >= ns) break;
      // ---- segments: running steps in their layer q = s - start <= H
      const int q_l = s - h1.w;
      const bool seg_l = run_l && q_l >= 0 && q_l <= h1.z;
      uint32_t nq_l = 0, o_l = 0;
      if (seg_l) nq_l = sBinom[h1.z * CT_BINOM + q_l], o_l = wofs[q_l];
      const uint64_t segm = __ballot(seg_l);
      mark(0);
      ++nsl;
      // the segments' words packed over the team, each padded to whole waves (every wave works
      // on a single step: its parameters are wave-uniform)
      uint32_t total = 0;
      for (uint64_t m = segm; m; m &= m - 1) total += (rdl(nq_l, (int)__builtin_ctzll(m)) + 63u) & ~63u;
      // CT_PIPE_DYN: a super-layer of more words than threads hands its 64-word chunks out from an
      // LDS counter (the next chunk fetched while this one runs), so the waves that lose issue
      // arbitration under load take fewer chunks instead of ending the super-layer last
      const bool dyn = (p.pipe & CT_PIPE_DYN) && total > (uint32_t)CT_TEAM;
      if (tt == 0) sChunk[(s + 1) & 1] = 0u;  // the next super-layer's counter (unused in this one)
      auto fetch = [&]() -> uint32_t {
        uint32_t c = 0;
        if (lane == 0) c = atomicAdd(&sChunk[s & 1], 1u);
        return 64u * (uint32_t)__builtin_amdgcn_readfirstlane((int)c);
      };
      // chunk f's segment (wave-uniform) and this lane's word of it (~0u past the segment's end);
      // the next chunk's word is loaded while this one runs (the word list of a 14-hi-bit table
      // is in global memory)
      auto chunk_word = [&](uint32_t f, int& seg) -> uint32_t {
        int i = 0;
        uint32_t e = 0, acc = 0;
        for (uint64_t m = segm; m; m &= m - 1) {
          const int k = (int)__builtin_ctzll(m);
          if (f >= acc) i = k, e = acc;
          acc += (rdl(nq_l, k) + 63u) & ~63u;
        }
        seg = i;
        const uint32_t r = f - e + (uint32_t)lane;
        return r < rdl(nq_l, i) ? words[rdl(o_l, i) + r] : ~0u;
      };
      uint32_t f0 = dyn ? fetch() : (uint32_t)(tt & ~63);
      int seg_n = 0;
      uint32_t w_n = f0 < total ? chunk_word(f0, seg_n) : ~0u;
      for (; f0 < total;) {
        const uint32_t f_next = dyn ? fetch() : f0 + (uint32_t)CT_TEAM;
        f0 = f_next;
#ifdef LC_CT_WORDPROF
        const unsigned long long tpw = prof ? __builtin_amdgcn_s_memtime() : 0;
#endif
        const int i = seg_n;
        const uint32_t w = w_n;
        if (f_next < total) w_n = chunk_word(f_next, seg_n);
        const uint32_t live = rdl(h0.x, i), fresh = rdl(h0.y, i);
        const int j = rdl(h1.x, i), jp = rdl(h1.y, i);
        const int t = t_ret_old + i;
        if (w & ~(live >> CTAB_LO)) continue;  // (~0u: past the segment's end)
        CStep* st = &sRing[t % CT_RING];
        uint64_t* const Bt = tab(t);
#ifdef LC_CT_WORDPROF
        if (prof) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          const unsigned long long tn = __builtin_amdgcn_s_memtime();
          pw[5] += tn - tpw;  // to the word (segment lookup, word index, X)
        }
#endif
        const uint64_t X = ct_x(tab(t - 1), w, fresh >> CTAB_LO, jp, st->keep_lo);
        // (r4k: wave-uniform control flow in the word, every lane through every pull round and
        // closure sweep with masked loads, was 8 % slower on C2c4: the divergent form is kept)
        #ifdef LC_CT_WORDPROF
        const uint64_t R = ct_word(Bt, w, st, live, j, X, w, 0ull, prof ? pw : nullptr);
#else
        const uint64_t R = ct_word(Bt, w, st, live, j, X, w, 0ull);
#endif
        Bt[w] = X | R;
        expl += (uint32_t)__popcll(R);
        if (t > 0) st_fout += (uint32_t)__popcll(X);
        if (X) st->anyx = 1;
        if (prof) ++nwd;
      }
      mark(1);
      // ---- decode ahead into a slot nobody read in this super-layer
      const int t_dec_old = t_dec;
      if (t_dec < ns && t_dec - t_ret_old < CT_RING) {
        if (decoder) ct_decode(p, sw, pos, lane, &sRing[t_dec % CT_RING], &sRing[(t_dec - 1) % CT_RING]);
        ++t_dec;
      }
      // ---- start the next decoded step at s + 1: two super-layers after its predecessor (one
      // if that has a single layer, or returned an in-word slot on double-buffered tables), or
      // at once if the predecessor retired
      if (t_run < t_dec_old) {
        const int lp = t_run - 1 - t_ret_old;  // the predecessor's lane (< 0: retired)
        bool ok;
        if (lp < 0 || lp < lead) {
          ok = true;
        } else {
          const bool pred_hi = rdl(h1.x, lp) >= CTAB_LO;
          const int gap = (dbl && !pred_hi) ? 1 : 2;
          ok = s + 1 - rdl(h1.w, lp) >= min(gap, rdl(h1.z, lp) + 1);
        }
        if (ok) {
          if (tt == 0) sRing[t_run % CT_RING].start = s + 1;
          ++t_run;
        }
      }
      mark(2);
      __syncthreads();
      mark(3);
    }
    if (prof) {
      for (int off = 32; off > 0; off >>= 1) nwd += __shfl_down(nwd, off, 64);
      if (lane == 0) {
        unsigned long long* q = p.prof + 8 * (tt >> 6);
        for (int k = 0; k < 4; ++k) atomicAdd(&q[k], ph[k]);
        atomicAdd(&q[4], nsl);
        atomicAdd(&q[5], nwd);
        atomicAdd(&q[6], pw[0] + pw[1]);  // hi sums + pulls
        atomicAdd(&q[7], pw[2]);          // gates
        unsigned long long* r = p.prof + 128 + 4 * (tt >> 6);
        atomicAdd(&r[0], pw[3]);  // closure
        atomicAdd(&r[1], pw[5]);  // to the word
        atomicAdd(&r[2], pw[4]);  // closure sweeps (lane 0's)
        atomicAdd(&r[3], pw[1]);  // pulls alone
      }
    }
    if (fail_t < 0 && ns > 0) {  // the last step's return
      const CStep* st = &sRing[(ns - 1) % CT_RING];
      const int jl = rfl(st->j);
      const uint32_t live = (uint32_t)rfl((int)st->live) & ~(1u << jl);
      const int L = live ? 32 - __clz((int)live) : 0;
      const int nwt = 1 << (L > CTAB_LO ? L - CTAB_LO : 0);
      uint64_t nzx = 0;
      for (int w = tt; w < nwt; w += CT_TEAM) {
        if ((uint32_t)w & ~(live >> CTAB_LO)) continue;
        const uint64_t X = ct_x(tab(ns - 1), (uint32_t)w, 0u, jl, ~0ull);
        st_fout += (uint32_t)__popcll(X);
        nzx |= X;
      }
      if (!__syncthreads_or(nzx != 0)) fail_t = ns - 1;
    }
    if (tt == 0) st_steps += fail_t >= 0 ? fail_t + 1 : ns;
    for (int off = 32; off > 0; off >>= 1) expl += __shfl_down(expl, off, 64);
    if (lane == 0 && expl) atomicAdd(&sExpl, expl);
    __syncthreads();
    if (tt == 0) {
      p.explored[h] = sExpl;
      p.fail_step[h] = fail_t;
      p.status[h] = fail_t >= 0 ? ST_INVALID : ST_VALID;
      if (p.stamps) p.stamps[2 * h + 1] = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
  }
  for (int off = 32; off > 0; off >>= 1) {
    st_fout += __shfl_down(st_fout, off, 64);
    st_steps += __shfl_down(st_steps, off, 64);
  }
  if (lane == 0 && st_fout) atomicAdd(&p.stats[0], st_fout);
  if (lane == 0 && st_steps) atomicAdd(&p.stats[1], st_steps);
}

// ---- counter tile teams (ctab.hpp CtabTeamParams) ----------------------------
// One history per team of G = 2^T workgroups: tile r holds the masks whose team slots (lb..lb+T-1)
// spell r, its table over the lb local slots in LDS (2^(lb-6) words, double-buffered when two
// fit). Every tile walks the step stream itself and runs the LDS kernel's pipelined schedule over
// its local layers, shifted by its live team slots (tile r's layer q of step t at super-layer
// start_t + q + |r|), so a step spans Hl + tb + 1 super-layers. Hand-offs (the schedule of
// dense.hip's pipelined tile teams with global layers, r2):
//  * a wide step's words (some team slot live) are stored sc1 into the tile's mirror slot for the
//    step, in layer order (cum[Hl][q] + the word's index in its layer); after its super-layer each
//    tile drains its stores and stores its token = super-layers finished;
//  * a pull over team slot b reads tile r \ b's mirror word, finished one super-layer earlier
//    (token >= s); a tile holding the returning team slot j takes only T_j of tile r \ j;
//  * after a team-slot return jp the X of tile r is tile r | jp's word of the previous step,
//    finished at pstart + q + |r| + 1 (token >= pstart + q + |r| + 2);
//  * every CTT_CW super-layers a tile waits until no tile is more than CTT_CW behind, so a
//    mirror slot (reused CT_MRING steps later) is never rewritten while a reader lags.
// Failures: a tile that read a nonzero X in step t sets the team's bit t; after the last step
// (and its return, checked tile by tile) the first missing bit t names step t - 1. An empty
// frontier stays empty, so the explored count of the steps after a failure is 0.
constexpr int CTT_RING = 24;
constexpr int CTT_CAPW = 1 << 13;  // LDS table words of a tile (64 KiB: two tables of <= 2^12 words)
constexpr int CTT_CW = 8;          // credit window (super-layers)

__device__ __forceinline__ bool ct_poll(const CtabTeamParams& tp, const unsigned long long* f,
                                        unsigned long long need, uint64_t t0, long& spins) {
  if (ld_agent(f) >= need) return true;
  __builtin_amdgcn_s_sleep(1);
  if ((++spins & 255) == 0 && (__builtin_amdgcn_s_memrealtime() - t0 > tp.watchdog || ld_agent(tp.abort))) {
    st_agent(tp.abort, 1);
    return true;  // gives up: the caller sees the abort word
  }
  return false;
}

// all G workgroups of a team: every wave's stores drained, one arrival each, the last one bumps
// the generation (ctl[32]) the others poll; false when a watchdog fired
__device__ __forceinline__ bool ct_team_bar(const CtabTeamParams& tp, unsigned* ctl, int G, int* sAbort) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = ld_agent(&ctl[32]);
    if (__hip_atomic_fetch_add(&ctl[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)G - 1) {
      st_agent(&ctl[0], 0u);
      __hip_atomic_store(&ctl[32], g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      long spins = 0;
      while (ld_agent(&ctl[32]) == g) {
        __builtin_amdgcn_s_sleep(1);
        if ((++spins & 255) == 0 && (__builtin_amdgcn_s_memrealtime() - t0 > tp.watchdog || ld_agent(tp.abort))) {
          st_agent(tp.abort, 1);
          break;
        }
      }
    }
    *sAbort = ld_agent(tp.abort);
  }
  __syncthreads();
  return *sAbort == 0;
}

__global__ void __launch_bounds__(CT_TEAM) ctab_team_kernel(CtabTeamParams tp) {
  const CtabParams& p = tp.c;
  __shared__ uint64_t sTab[CTT_CAPW];
  __shared__ CStep sRing[CTT_RING];
  __shared__ uint32_t sBinom[CT_BINOM * CT_BINOM];
  __shared__ uint32_t sCum[CT_BINOM * CT_BINOM];  // cum[H][q] = sum_{p < q} C(H, p): layer q's first index
  __shared__ uint32_t sWOff[CT_BINOM + 2];
  __shared__ int sAbort, sFail;
  __shared__ unsigned long long sExpl;
  const int tt = threadIdx.x, lane = tt & 63;
  const bool decoder = tt < 64;
  const int team = tp.wg_team[blockIdx.x];
  const int base = tp.team_base[team], rank = (int)blockIdx.x - base, T = tp.team_bits[team], G = 1 << T;
  const int h = tp.team_hist[team];
  init_binom(sBinom, tt, CT_TEAM);
  if (tt <= DENSE_WORD_BITS + 1) {  // offsets of the global list's popcount layers
    uint32_t o = 0;
    for (int q = 0; q < tt; ++q) {
      uint64_t v = 1;
      for (int i = 1; i <= q; ++i) v = v * (uint64_t)(DENSE_WORD_BITS - q + i) / (uint64_t)i;
      o += (uint32_t)v;
    }
    sWOff[tt] = o;
  }
  if (tt == 0) sAbort = 0, sExpl = 0, sFail = INT32_MAX;
  __syncthreads();
  if (tt < CT_BINOM * CT_BINOM) {
    const int n = tt / CT_BINOM, q = tt % CT_BINOM;
    uint32_t c = 0;
    for (int r = 0; r < q; ++r) c += sBinom[n * CT_BINOM + r];
    sCum[tt] = c;
  }
  const int lmax = p.lmax[h], ns = p.nsteps[h];
  const int lb = lmax - T, Hm = lb > CTAB_LO ? lb - CTAB_LO : 0;
  const uint32_t lmask = (1u << lb) - 1u;
  const int NW = 1 << Hm;
  const bool dbl = (p.pipe & CT_PIPE_DBL) && 2 * NW <= CTT_CAPW;
  uint64_t* const B = sTab;
  uint64_t* const B2 = dbl ? sTab + NW : sTab;
  auto tab = [&](int t) { return (t & 1) ? B2 : B; };
  const int ntab = dbl ? 2 * NW : NW;
  for (int i = tt; i < ntab; i += CT_TEAM) sTab[i] = 0;
  const uint32_t* words = p.words;
  const uint32_t* wofs = sWOff;
  uint32_t* const lw = reinterpret_cast<uint32_t*>(sTab + ntab);
  uint32_t* const lo = lw + NW;
  const bool lds_list = Hm > 0 && ntab + NW / 2 + 16 <= CTT_CAPW;
  __syncthreads();
  if (lds_list) {
    if (tt <= Hm + 1) lo[tt] = sCum[Hm * CT_BINOM + tt];
    for (int q = 0; q <= Hm; ++q) {
      const uint32_t nq = sBinom[Hm * CT_BINOM + q], og = sWOff[q], ol = sCum[Hm * CT_BINOM + q];
      for (uint32_t r = (uint32_t)tt; r < nq; r += (uint32_t)CT_TEAM) lw[ol + r] = p.words[og + r];
    }
    words = lw, wofs = lo;
  }
  unsigned long long* const flags = tp.flags + base;
  uint32_t* const anyv = tp.anyv + tp.team_any_off[team];
  auto mirror = [&](int r, int t) {
    return tp.mirror + (((size_t)(base + r) * CT_MRING + (size_t)(t % CT_MRING)) << tp.mshift);
  };
  if (p.stamps && rank == 0 && tt == 0) p.stamps[2 * h] = __builtin_amdgcn_s_memrealtime();
  __syncthreads();
  if (rank == 0 && tt == 0) B2[0] = 1;  // the initial config (step 0 reads tab(-1))
  StreamWin sw;
  int64_t pos = p.sbeg[h];
  // decode a step, then its tile-team fields (local layers - 1, live team slots, the previous
  // step's local layers - 1)
  auto decode = [&](int t) {
    CStep* dst = &sRing[t % CTT_RING];
    const CStep* prev = t > 0 ? &sRing[(t - 1) % CTT_RING] : nullptr;
    ct_decode(p, sw, pos, lane, dst, prev);
    if (lane == 0) {
      const uint32_t live = dst->live;
      const int L = live ? 32 - __clz((int)live) : 0;
      const int Ll = L < lb ? L : lb;
      dst->Hl = Ll > CTAB_LO ? Ll - CTAB_LO : 0;
      dst->tb = __popc(live >> lb);
      dst->hpl = prev ? prev->Hl : 0;
      dst->pstart = 0;
    }
  };
  if (ns > 0 && decoder) {
    decode(0);
    if (lane == 0) sRing[0].start = 0;
  }
  __syncthreads();
  unsigned long long expl = 0, st_fout = 0;
  int t_dec = ns > 0 ? 1 : 0, t_run = t_dec, t_ret = 0, last_start = 0;
  int s = 0;
  for (; t_ret < ns; ++s) {
    if (s >= CTT_CW && (s % CTT_CW) == 0) {  // credit: nobody more than CTT_CW super-layers behind
      if (decoder) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        long spins = 0;
        while (!__all(lane >= G || ct_poll(tp, &flags[lane < G ? lane : 0], (unsigned long long)(s - CTT_CW), t0, spins)))
          ;
        if (lane == 0) sAbort = ld_agent(tp.abort);
      }
      __syncthreads();
      if (sAbort) break;
    }
    // ---- ring view: lane i = step t_ret + i
    const int tl = t_ret + lane;
    const bool dec_l = lane < CTT_RING && tl < t_dec;
    uint4 h0 = {0u, 0u, 0u, 0u};
    int4 h1 = {0, 0, 0, 1 << 30}, h2 = {0, 0, 0, 0};
    if (dec_l) {
      const CStep* st = &sRing[tl % CTT_RING];
      h0 = *reinterpret_cast<const uint4*>(&st->live);    // live, fresh, anyx, base
      h1 = *reinterpret_cast<const int4*>(&st->j);        // j, jp, H, start
      h2 = *reinterpret_cast<const int4*>(&st->pstart);   // pstart, hpl, Hl, tb
    }
    const bool run_l = dec_l && tl < t_run;
    const bool fin_l = run_l && h1.w + h2.z + h2.w < s;
    const uint64_t fin = __ballot(fin_l);
    const int lead = (int)__builtin_ctzll(~fin);
    if (decoder && lane < lead && tl > 0 && h0.z)  // retired: this tile read a config in step tl
      __hip_atomic_fetch_or(&anyv[tl >> 5], 1u << (tl & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int t_ret_old = t_ret;
    t_ret += lead;
    if (t_ret >= ns) break;
    // ---- this tile's segments: running steps whose live team slots cover the tile
    const uint32_t lteam_l = h0.x >> lb;
    const int dr_l = __popc((uint32_t)rank & lteam_l);
    const int q_l = s - h1.w - dr_l;
    const bool seg_l = run_l && ((uint32_t)rank & ~lteam_l) == 0 && q_l >= 0 && q_l <= h2.z;
    uint32_t nq_l = 0, o_l = 0, mo_l = 0, mp_l = 0, pm_l = 0;
    int xs_l = -1;
    if (seg_l) {
      nq_l = sBinom[h2.z * CT_BINOM + q_l], o_l = wofs[q_l], mo_l = sCum[h2.z * CT_BINOM + q_l];
      mp_l = sCum[h2.y * CT_BINOM + min(q_l, h2.y)];
      const int jt = h1.x >= lb ? h1.x - lb : -1;
      const bool tile_j = jt >= 0 && ((rank >> jt) & 1);
      pm_l = lteam_l == 0 ? 0u : tile_j ? (1u << jt) : ((uint32_t)rank & lteam_l);
      if (h1.y >= lb && !((uint32_t)rank & (h0.y >> lb))) xs_l = rank | (1 << (h1.y - lb));
    }
    if (__any(pm_l != 0 || xs_l >= 0)) {  // wait for the tiles this super-layer reads
      if (decoder) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        long spins = 0;
        for (;;) {
          bool ok = true;
          for (uint32_t m = pm_l; m && ok; m &= m - 1)
            ok = ct_poll(tp, &flags[rank ^ (1 << __builtin_ctz(m))], (unsigned long long)s, t0, spins);
          if (ok && xs_l >= 0)
            ok = ct_poll(tp, &flags[xs_l], (unsigned long long)(h2.x + q_l + dr_l + 2), t0, spins);
          if (__all(ok)) break;
        }
        if (lane == 0) sAbort = ld_agent(tp.abort);
      }
      __syncthreads();
      if (sAbort) break;
    }
    const uint64_t segm = __ballot(seg_l);
    const bool wide_any = __ballot(seg_l && lteam_l != 0) != 0;
    uint32_t total = 0;
    for (uint64_t m = segm; m; m &= m - 1) total += (rdl(nq_l, (int)__builtin_ctzll(m)) + 63u) & ~63u;
    for (uint32_t f0 = (uint32_t)(tt & ~63); f0 < total; f0 += (uint32_t)CT_TEAM) {
      int i = 0;
      uint32_t e = 0, acc = 0;
      for (uint64_t m = segm; m; m &= m - 1) {
        const int k = (int)__builtin_ctzll(m);
        if (f0 >= acc) i = k, e = acc;
        acc += (rdl(nq_l, k) + 63u) & ~63u;
      }
      const uint32_t nq = rdl(nq_l, i), r = f0 - e + (uint32_t)lane;
      const uint32_t mo = rdl(mo_l, i), mp = rdl(mp_l, i), pmask = rdl(pm_l, i), o = rdl(o_l, i);
      const uint32_t live = rdl(h0.x, i), fresh = rdl(h0.y, i);
      const int j = rdl(h1.x, i), jp = rdl(h1.y, i), xs = rdl(xs_l, i);
      const int t = t_ret_old + i;
      if (r >= nq) continue;
      const uint32_t w = words[o + r];
      const uint32_t live_loc = live & lmask, lteam = live >> lb;
      if (w & ~(live_loc >> CTAB_LO)) continue;
      const bool wide = lteam != 0;
      const int jt = j >= lb ? j - lb : -1;
      const bool tile_j = jt >= 0 && ((rank >> jt) & 1);
      const bool jloc_hi = j >= CTAB_LO && j < lb;
      const bool tile_fresh = ((uint32_t)rank & (fresh >> lb)) != 0;
      const uint32_t fresh_hi = (fresh & lmask) >> CTAB_LO;
      CStep* st = &sRing[t % CTT_RING];
      uint64_t* const Bt = tab(t);
      const uint32_t wg = w | ((uint32_t)rank << Hm);  // the word's hi bits over the whole table
      const uint64_t keep_lo = st->keep_lo;
      const bool fx = !tile_fresh && !(w & fresh_hi);
      // HBM loads first (X from tile xs, the pulls from the tiles one team slot below), used after
      uint64_t X = 0, pv[CTAB_TEAM_MAXB];
      if (fx && xs >= 0) X = HbmTab::ld(mirror(xs, t - 1) + mp + r);
      const bool pl = tile_j || !(jloc_hi && ((w >> (j - CTAB_LO)) & 1u));
#pragma unroll
      for (int b = 0; b < CTAB_TEAM_MAXB; ++b)
        pv[b] = (pl && ((pmask >> b) & 1u)) ? HbmTab::ld(mirror(rank ^ (1 << b), t) + mo + r) : 0ull;
      if (xs >= 0) X &= keep_lo;
      else if (fx) X = ct_x(tab(t - 1), w, 0u, jp, keep_lo);
      const int s_hi = (int)st->sh[0][wg & 127u] + (int)st->sh[1][(wg >> 7) & 127u] + (int)st->sh[2][(wg >> 14) & 127u];
      uint64_t R0 = 0;
#pragma unroll
      for (int b = 0; b < CTAB_TEAM_MAXB; ++b)
        if ((pmask >> b) & 1u) R0 |= pv[b] & gate(st, st->cq[CTAB_LO + Hm + b], s_hi);
      const uint64_t R = tile_j ? R0 : ct_word(Bt, w, st, live, j, X, wg, R0);
      const uint64_t nv = X | R;
      Bt[w] = nv;
      if (wide) HbmTab::st(mirror(rank, t) + mo + r, nv);
      expl += (uint32_t)__popcll(R);
      if (t > 0) st_fout += (uint32_t)__popcll(X);
      if (X) st->anyx = 1;
    }
    // ---- decode ahead into a slot nobody read in this super-layer
    const int t_dec_old = t_dec;
    if (t_dec < ns && t_dec - t_ret_old < CTT_RING) {
      if (decoder) decode(t_dec);
      ++t_dec;
    }
    // ---- start the next decoded step at s + 1: two super-layers after its predecessor (one after
    // an in-word return on double-buffered tables, or the predecessor's whole span if shorter),
    // at once if the predecessor retired
    if (t_run < t_dec_old) {
      const int lp = t_run - 1 - t_ret_old;
      bool ok = lp < 0 || lp < lead;
      if (!ok) {
        const int gap = (dbl && rdl(h1.x, lp) < CTAB_LO) ? 1 : 2;
        ok = s + 1 - rdl(h1.w, lp) >= min(gap, rdl(h2.z, lp) + rdl(h2.w, lp) + 1);
      }
      if (ok) {
        if (tt == 0) sRing[t_run % CTT_RING].start = s + 1, sRing[t_run % CTT_RING].pstart = last_start;
        last_start = s + 1;
        ++t_run;
      }
    }
    if (wide_any) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
    __syncthreads();
    if (tt == 0) st_agent(&flags[rank], (unsigned long long)(s + 1));
  }
  unsigned* const ctl = tp.ctl + 64 * team;
  // the last step's return, tile by tile, once every tile has finished
  if (ct_team_bar(tp, ctl, G, &sAbort) && ns > 0) {
    const CStep* st = &sRing[(ns - 1) % CTT_RING];
    const int jl = rfl(st->j);
    const uint32_t live = (uint32_t)rfl((int)st->live);
    const uint32_t lteam = live >> lb;
    const int jt = jl >= lb ? jl - lb : -1;
    // a team-slot j: the post-return frontier of tile r \ j is tile r's own words (its masks hold j)
    const bool mine = jt >= 0 ? (((uint32_t)rank & ~lteam) == 0 && ((rank >> jt) & 1))
                              : ((uint32_t)rank & ~lteam) == 0;
    uint64_t nzx = 0;
    if (mine) {
      const uint32_t lhi = ((live & ~(jt >= 0 ? 0u : 1u << jl)) & lmask) >> CTAB_LO;
      const int nwt = 1 << Hm;
      for (int w = tt; w < nwt; w += CT_TEAM) {
        if ((uint32_t)w & ~lhi) continue;
        const uint64_t X = jt >= 0 ? tab(ns - 1)[w] : ct_x(tab(ns - 1), (uint32_t)w, 0u, jl, ~0ull);
        st_fout += (uint32_t)__popcll(X);
        nzx |= X;
      }
    }
    if (__syncthreads_or(nzx != 0) && tt == 0)
      __hip_atomic_fetch_or(&anyv[ns >> 5], 1u << (ns & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int off = 32; off > 0; off >>= 1) expl += __shfl_down(expl, off, 64);
  if (lane == 0 && expl) atomicAdd(&sExpl, expl);
  __syncthreads();
  if (tt == 0 && sExpl) atomicAdd(&p.explored[h], sExpl);
  const bool done = ct_team_bar(tp, ctl, G, &sAbort);
  if (done && rank == 0) {  // the first step whose frontier was empty everywhere
    for (int wd = tt; wd <= (ns >> 5); wd += CT_TEAM) {
      uint32_t v = ld_agent(&anyv[wd]);
      if (wd == 0) v |= 1u;  // (step 0 reads the initial config)
      const int top = ns - 32 * wd;  // bits 0..min(31, top) are steps
      const uint32_t need = top >= 31 ? ~0u : ((1u << (top + 1)) - 1u);
      const uint32_t miss = ~v & need;
      if (miss) atomicMin(&sFail, 32 * wd + __builtin_ctz(miss));
    }
    __syncthreads();
    if (tt == 0) {
      const int fail_t = sFail == INT32_MAX ? -1 : sFail - 1;
      p.fail_step[h] = fail_t;
      p.status[h] = fail_t >= 0 ? ST_INVALID : ST_VALID;
      if (p.stamps) p.stamps[2 * h + 1] = __builtin_amdgcn_s_memrealtime();
      atomicAdd(&p.stats[1], (unsigned long long)(fail_t >= 0 ? fail_t + 1 : ns));
    }
  }
  for (int off = 32; off > 0; off >>= 1) st_fout += __shfl_down(st_fout, off, 64);
  if (lane == 0 && st_fout) atomicAdd(&p.stats[0], st_fout);
}

}  // namespace

int ctab_grid_size() {
  int dev = 0, ncu = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, ctab_kernel, CT_TEAM, 0) != hipSuccess) return 0;
  return ncu * per;
}

int ctab_team_max_wgs() {
  int dev = 0, ncu = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, ctab_team_kernel, CT_TEAM, 0) != hipSuccess) return 0;
  return ncu * per;
}

hipError_t launch_ctab_team(const CtabTeamParams& p, int grid, hipStream_t stream) {
  CtabTeamParams q = p;
  void* args[] = {&q};
  return hipLaunchCooperativeKernel((const void*)ctab_team_kernel, dim3(grid), dim3(CT_TEAM), args, 0, stream);
}

hipError_t launch_ctab(const CtabParams& p, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(ctab_kernel, dim3(grid), dim3(CT_TEAM), 0, stream, p);
  return hipGetLastError();
}

}  // namespace lc
