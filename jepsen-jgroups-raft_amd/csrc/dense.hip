// dense.hip — byte-sliced closure-table search (see dense.hpp) for cas-register histories
// whose live slot width is at most DENSE_WIDE_LMAX: knossos.linear/analysis [ext] (SURVEY
// §8(a) a5) with CASRegister.step (a6, register.clj:110) applied to whole bitmaps.
//
// Table: one u64 per word w; byte s of B[w] is register state s's bitmap over the 8 masks
// (w << 3) | p, p < 8. One RETURN step of slot j (R = configs produced by a consistent step,
// X = table before):
//   for hi-layer q = 0..H (words w with popcount(w) = q, H = width - 3), in parallel:
//     j hi and j ∈ w : R = T_j(B[w \ j])                 (configs holding j are never expanded)
//     otherwise      : R = ∪_{k ∈ w} T_k(B[w \ k])        (pulls from finalized words)
//                      then the in-word closure over the low 3 bits: the live low ops k ≠ j
//                      in a sequence holding every ordering of them as a subsequence
//                      (R |= T_k((X | R) at positions without k, j) moved up by 2^k), and,
//                      when j is a low bit, one final j pass into the j positions
//     explored += popcount(R);  B[w] = X | R
//   return j: B'[m] = B[m ∪ j] for m ∌ j, B'[m ∪ j] = 0   (post-return frontier)
//   B' empty => not linearizable at this RETURN.
// An op moves bytes: write b: OR of all bytes -> byte b; cas a b: byte a -> byte b;
// read a: byte a -> byte a; read nil: every byte stays; an op naming a value the register
// never holds moves nothing. Shifts by wave-uniform amounts, no per-state branching.
// Every config reachable by linearizing pending calls is produced at exactly its own mask,
// whose predecessors (one bit fewer) are final earlier, so R is the closure set of the
// sparse search and popcount(R) its explored count, bit-exact.
//
// Teams:
//   WAVE  one wave, LDS table, widths <= 11 (256-thread workgroups beside the big kernel)
//   BLOCK one 1024-thread workgroup, LDS table, widths 12..17 (dequeued heaviest first)
//   TILE  2^t workgroups for one history of width 17 + t, each holding one 17-bit tile of
//         the table in LDS; cross-tile pulls go through per-tile HBM mirrors written sc1
//         (write-through) and read sc1 (L1-bypassing), published by a per-layer token that
//         every storing wave drained before (cdna_hip_programming.md Guideline 16,
//         MI355X_MICROARCH.md "Valid forms" row 1), so no fences are needed.
#include "dense.hpp"
#include "dense_ops.hpp"
#include "device_common.hpp"
#include "search.hpp"

namespace lc {
namespace {

constexpr int BINOM_N = 24;
constexpr int CMD_STEP = 1, CMD_EXIT = 2;


// Per-team control block (zeroed before every launch): barrier words and the leader's
// command for the next team step, each group on its own 128-B line.
struct TeamCtl {
  unsigned count;
  unsigned pad0[31];
  unsigned gen;
  unsigned pad1[31];
  int cmd, h;
  long long pos;
  unsigned any;
  unsigned pad2[27];
  unsigned ops[64];  // the leader's op table (OpSel lo, hi per slot)
};



// Tagged mirror words (LC_PIPE bit 8): word i of a mirror slot is two 8-byte granules
// {data half, tag}, each single-copy atomic, so a reader polls the data itself until both tags
// name the step it wants (MI355X_MICROARCH "handoff-1to1": data-tagged 8-byte granules). The
// producer then needs neither a store drain nor a token on the hand-off path.
struct TagTab {
  static __device__ __forceinline__ void st(uint64_t* slot, uint32_t i, uint64_t v, uint32_t tag) {
    HbmTab::st(&slot[2 * i], ((uint64_t)tag << 32) | (uint32_t)v);
    HbmTab::st(&slot[2 * i + 1], ((uint64_t)tag << 32) | (uint32_t)(v >> 32));
  }
  // both granules of word i once they carry `tag`; a 20 s watchdog raises *abort (then 0)
  static __device__ __forceinline__ uint64_t ld(const uint64_t* slot, uint32_t i, uint32_t tag, int32_t* abort) {
    uint64_t a = HbmTab::ld(&slot[2 * i]), b = HbmTab::ld(&slot[2 * i + 1]);
    if ((uint32_t)(a >> 32) == tag && (uint32_t)(b >> 32) == tag) return (uint32_t)a | (b << 32);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (long spins = 1;; ++spins) {
      __builtin_amdgcn_s_sleep(1);
      a = HbmTab::ld(&slot[2 * i]);
      b = HbmTab::ld(&slot[2 * i + 1]);
      if ((uint32_t)(a >> 32) == tag && (uint32_t)(b >> 32) == tag) return (uint32_t)a | (b << 32);
      if ((spins & 255) == 0 && (__builtin_amdgcn_s_memrealtime() - t0 > 2000000000ull || ld_agent(abort))) {
        st_agent(abort, 1);
        return 0;
      }
    }
  }
};


// Pulls of word w over its hi bits from the finalized words one hi bit below (LDS table B):
// the bulk of a word's closure, needing nothing from other tiles. BATCH bits at a time: the
// loads of a batch are issued together (lanes without the bit read a zero word instead of
// taking a branch), then the batch's ops are applied. Bits >= H read the zero word (w < 2^H).
// ops: the team's LDS op table (slot k); foldm: its write slots (wave-uniform).
template <int BATCH>
__device__ __forceinline__ uint64_t pull_hi(const uint64_t* B, const uint64_t* zero, uint32_t w, int j, int H,
                                           const OpSel* ops, uint32_t foldm) {
  const uint32_t jh = j < 3 ? 0u : 1u << (j - 3);
  const uint32_t pm = (w & jh) ? jh : w;  // bits this word pulls over (only j when it holds j)
  uint64_t R = 0;
  // the batch's four ops (slots b0+3 .. b0+6) come in two 16-B reads: slot 3 + 4i of an op
  // table is 16-B aligned (OP_PAD)
  static_assert(BATCH == 4, "op reads are two 16-B pairs");
  for (int b0 = 0; b0 < H; b0 += BATCH) {
    const uint4* op4 = reinterpret_cast<const uint4*>(__builtin_assume_aligned(&ops[b0 + 3], 16));
    const uint4 s01 = op4[0], s23 = op4[1];
    uint64_t v[BATCH];
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const uint32_t bit = 1u << (b0 + u);
      v[u] = *((pm & bit) ? &B[w ^ bit] : zero);
    }
    // the selectors are needed here, after the data loads issued: keeps the compiler from
    // sinking half of them into the branches below (one more LDS round trip per op)
    asm volatile("" ::"v"(s01.x), "v"(s01.y), "v"(s01.z), "v"(s01.w), "v"(s23.x), "v"(s23.y), "v"(s23.z),
                 "v"(s23.w));
    const OpSel sel[4] = {{s01.x, s01.y}, {s01.z, s01.w}, {s23.x, s23.y}, {s23.z, s23.w}};
#pragma unroll
    for (int u = 0; u < BATCH; ++u) R |= transfer(sel[u], (foldm >> (b0 + u + 3)) & 1u, v[u]);
  }
  return R;
}

// pull_hi over the set bits of the word only (the pipelined teams' pull): a word of popcount q
// pulls over its q bits, two at a time (each lane its own bits: the ops are gathered per lane
// from the LDS table), instead of over all H bits with zero words for the absent ones (half the
// loads and transfers of a layer's words on average; C3 12.2 -> 11.0 ms, C2 32.5 -> 29.1). The
// same R as pull_hi.
__device__ __forceinline__ uint64_t pull_set(const uint64_t* B, uint32_t w, int j, const OpSel* ops,
                                            uint32_t foldm) {
  const uint32_t jh = j < 3 ? 0u : 1u << (j - 3);
  uint32_t m = (w & jh) ? jh : w;
  uint64_t R = 0;
#ifdef LC_PULL_BF
  // branch-free pairs: a lane without a second bit reads its own word and slot 3's op, masked after
  while (m) {
    int b[2];
    uint64_t v[2];
    OpSel o[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      b[u] = m ? __builtin_ctz(m) : -1;
      m &= m - 1;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      v[u] = B[w ^ (b[u] >= 0 ? 1u << b[u] : 0u)];
      o[u] = ops[(b[u] >= 0 ? b[u] : 0) + 3];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint64_t x = transfer(o[u], (foldm >> ((b[u] >= 0 ? b[u] : 0) + 3)) & 1u, v[u]);
      R |= b[u] >= 0 ? x : 0ull;
    }
  }
  return R;
#endif
  while (m) {  // (a lane's trip count is ceil(popcount / 2); a layer's words share the popcount;
               // pairs, not quads: quads spill registers in the big kernel, r2h3: C3 11.5 vs 11.0 ms)
    int b[2];
    uint64_t v[2];
    OpSel o[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      b[u] = m ? __builtin_ctz(m) : -1;
      m &= m - 1;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      v[u] = b[u] >= 0 ? B[w ^ (1u << b[u])] : 0ull;
      o[u] = b[u] >= 0 ? ops[b[u] + 3] : OpSel{SEL_NONE, SEL_NONE};
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (b[u] >= 0) R |= transfer(o[u], (foldm >> (b[u] + 3)) & 1u, v[u]);
  }
  return R;
}

// pull_hi over the batches b0 = bfirst, bfirst + bstep, ... only: a word's pulls split over
// the lanes of a group (run_layers' narrow layers), OR-combined by the caller.
__device__ __forceinline__ uint64_t pull_hi_part(const uint64_t* B, const uint64_t* zero, uint32_t w, int j, int H,
                                                const OpSel* ops, uint32_t foldm, int bfirst, int bstep) {
  const uint32_t jh = j < 3 ? 0u : 1u << (j - 3);
  const uint32_t pm = (w & jh) ? jh : w;
  uint64_t R = 0;
  for (int b0 = bfirst; b0 < H; b0 += bstep) {
    const uint4* op4 = reinterpret_cast<const uint4*>(__builtin_assume_aligned(&ops[b0 + 3], 16));
    const uint4 s01 = op4[0], s23 = op4[1];
    uint64_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t bit = 1u << (b0 + u);
      v[u] = *((pm & bit) ? &B[w ^ bit] : zero);
    }
    asm volatile("" ::"v"(s01.x), "v"(s01.y), "v"(s01.z), "v"(s01.w), "v"(s23.x), "v"(s23.y), "v"(s23.z),
                 "v"(s23.w));
    const OpSel sel[4] = {{s01.x, s01.y}, {s01.z, s01.w}, {s23.x, s23.y}, {s23.z, s23.w}};
#pragma unroll
    for (int u = 0; u < 4; ++u) R |= transfer(sel[u], (foldm >> (b0 + u + 3)) & 1u, v[u]);
  }
  return R;
}


__device__ __forceinline__ uint32_t finish_word(uint64_t* B, uint32_t w, uint32_t live, int j, const OpSel* ops,
                                               uint32_t foldm, uint64_t R, uint64_t* out) {
  const uint64_t X = B[w];
  R = close_in_word(X, w, live, j, ops, foldm, R);
  if (R) B[w] = X | R;
  *out = X | R;
  return (uint32_t)__popcll(R);
}

// One step's closure of word w: R0 (pulls from other tiles, computed by the caller) plus the
// hi-bit pulls and the in-word closure.
template <int HMAX, int BATCH>
__device__ __forceinline__ uint32_t close_word(uint64_t* B, const uint64_t* zero, uint32_t w, uint32_t live, int j,
                                              int H, const OpSel* ops, uint32_t foldm, uint64_t R0,
                                              uint64_t* out) {
  return finish_word(B, w, live, j, ops, foldm, R0 | pull_hi<BATCH>(B, zero, w, j, H, ops, foldm), out);
}

// The closure layers of one step on an LDS table, words split over the team's threads
// tt = 0..nt-1; sync() ends every layer (the last one too: the return that follows reads
// the last layer's words).
template <int HMAX, int BATCH, class Sync>
__device__ __forceinline__ unsigned long long run_layers(uint64_t* B, const uint64_t* zero, const uint32_t* words,
                                                        const uint32_t* wofs, const uint32_t* binom, uint32_t live,
                                                        int j, const OpSel* ops, uint32_t foldm, int tt, int nt,
                                                        Sync&& sync) {
  const int L = 32 - __clz((int)live);
  const int H = L > 3 ? L - 3 : 0;
  const uint32_t live_hi = live >> 3;
  unsigned long long expl = 0;
  // words of popcount q below 2^H: a prefix of layer q of the sorted list. Each thread loads
  // its next word index one word ahead (the next layer's first before the barrier), so the
  // list load's latency hides behind a word's closure.
  uint32_t nq = __builtin_amdgcn_readfirstlane(binom[H * BINOM_N]);
  uint32_t o = __builtin_amdgcn_readfirstlane(wofs[0]);
  uint32_t wn = (uint32_t)tt < nq ? words[o + tt] : 0u;
  for (int q = 0; q <= H; ++q) {
    // a layer of at most nt/2 (nt/4) words with two or more pull batches: each word's batches
    // go to a group of 2 (4) lanes, OR-combined by shuffles, and the group's first lane
    // finishes the word (every lane reaches the shuffles: inactive sources read 0)
    const int split = H <= 4 ? 1 : (int)nq * 4 <= nt ? 4 : (int)nq * 2 <= nt ? 2 : 1;
    if (split > 1) {
      const int sub = tt & (split - 1);
      const uint32_t r = (uint32_t)tt / (uint32_t)split;
      const uint32_t w = r < nq ? words[o + r] : ~0u;
      const bool act = r < nq && !(w & ~live_hi);
      uint64_t R = act ? pull_hi_part(B, zero, w, j, H, ops, foldm, 4 * sub, 4 * split) : 0ull;
      R |= (uint64_t)__shfl_xor((unsigned long long)R, 1, 64);
      if (split == 4) R |= (uint64_t)__shfl_xor((unsigned long long)R, 2, 64);
      if (act && sub == 0) {
        uint64_t nv;
        expl += finish_word(B, w, live, j, ops, foldm, R, &nv);
      }
    } else {
      for (uint32_t r = (uint32_t)tt; r < nq; r += (uint32_t)nt) {
        const uint32_t w = wn;
        if (r + nt < nq) wn = words[o + r + nt];
        if (w & ~live_hi) continue;
        uint64_t nv;
        expl += close_word<HMAX, BATCH>(B, zero, w, live, j, H, ops, foldm, 0ull, &nv);
      }
    }
    if (q < H) {
      nq = __builtin_amdgcn_readfirstlane(binom[H * BINOM_N + q + 1]);
      o = __builtin_amdgcn_readfirstlane(wofs[q + 1]);
      wn = (uint32_t)tt < nq ? words[o + tt] : 0u;
    }
    sync();
  }
  return expl;
}

// Return slot j < 17 on an LDS table: the post-return frontier moves down to the masks
// without j. Returns the OR of this thread's new words (nonzero = some config survived).
__device__ __forceinline__ uint64_t return_slot(uint64_t* B, uint32_t live, int j, int tt, int nt,
                                               unsigned long long& fout) {
  const int L = 32 - __clz((int)live);
  const int nwt = 1 << (L > 3 ? L - 3 : 0);
  uint64_t anyv = 0;
  if (j < 3) {
    const uint64_t with_j = ~keep64(j);
    const int sh = 1 << j;
    for (int w = tt; w < nwt; w += nt) {
      const uint64_t v = (B[w] & with_j) >> sh;
      B[w] = v;
      anyv |= v;
      fout += __popcll(v);
    }
  } else {
    const int jb = 1 << (j - 3);
    const int half = nwt >> 1;
    for (int x = tt; x < half; x += nt) {
      const int lo = x & (jb - 1);
      const int w = ((x ^ lo) << 1) | lo;
      const uint64_t v = B[w | jb];
      B[w] = v;
      B[w | jb] = 0;
      anyv |= v;
      fout += __popcll(v);
    }
  }
  return anyv;
}

template <int TEAM>
__device__ __forceinline__ void team_sync() {
  if constexpr (TEAM >= 256) {
    __syncthreads();
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

template <int TEAM>
__device__ __forceinline__ int team_any(int v) {
  if constexpr (TEAM >= 256) return __syncthreads_or(v);
  else return __any(v);
}

// Barrier of the TEAM/64 waves of a sub-workgroup team: one lane per wave arrives on an LDS
// counter (qb[0]), the last arriver bumps the generation (qb[1]) the others poll.
template <int TEAM>
__device__ __forceinline__ void sub_sync(unsigned* qb) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63) == 0) {
    const unsigned g = __hip_atomic_load(&qb[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (__hip_atomic_fetch_add(&qb[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) == TEAM / 64 - 1) {
      __hip_atomic_store(&qb[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_store(&qb[1], g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
      while (__hip_atomic_load(&qb[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == g)
        __builtin_amdgcn_s_sleep(1);
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// binomials and the first entry of each popcount layer of the `lbits`-bit word list
__device__ __forceinline__ void init_tables(uint32_t* binom, uint32_t* wofs, int lbits, int nthreads) {
  const int tid = threadIdx.x;
  for (int i = tid; i < BINOM_N * BINOM_N; i += nthreads) {
    const int n = i / BINOM_N, k = i % BINOM_N;
    uint32_t c = 0;
    if (k <= n) {  // C(n, k), exact in 64 bits for n < 24
      uint64_t v = 1;
      for (int q = 1; q <= k; ++q) v = v * (uint64_t)(n - k + q) / (uint64_t)q;
      c = (uint32_t)v;
    }
    binom[i] = c;
  }
  __syncthreads();
  if (tid <= lbits + 1) {
    uint32_t o = 0;
    for (int q = 0; q < tid; ++q) o += binom[lbits * BINOM_N + q];
    wofs[tid] = o;
  }
  __syncthreads();
}

// per-wave window over a history's step stream: lane i holds word base + i
struct StreamWin {
  int64_t base = -(1ll << 40);
  uint32_t win = 0;
  __device__ __forceinline__ void need(const DenseParams& p, int64_t pos, int lane) {
    if (pos + 32 > base + 64) {  // a step is at most 32 words
      base = pos;
      win = (base + lane < p.stream_words) ? p.stream[base + lane] : 0u;
    }
  }
  __device__ __forceinline__ uint32_t at(int64_t pos) const {
    return (uint32_t)__shfl((int)win, (int)((pos - base) & 63), 64);
  }
};

// decode the step header at pos; lanes < ninv of the calling wave store their op words
__device__ __forceinline__ uint32_t read_step(const StreamWin& sw, int64_t pos, int lane, bool writer,
                                             OpSel* opt, int* ninv_out) {
  const uint32_t H0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)sw.at(pos));  // wave-uniform
  const uint32_t w = sw.at(pos + 1 + lane);
  const int ninv = (int)__builtin_ctzll(~__ballot(lane <= DENSE_MAX_NINV && (w & DENSE_OPW)));
  if (writer && lane < ninv) opt[w & 31u] = decode_op((w >> 8) & 0xffu, (w >> 16) & 0xffu);
  *ninv_out = ninv;
  return H0;
}

// Histories dequeued one at a time by a team of TEAM threads (a wave or a workgroup) that
// keeps the whole table in LDS (B, 2^(TLOG-3) words).
template <int TEAM, int TLOG>
__device__ __forceinline__ void history_loop(const DenseParams& p, uint64_t* B, const uint64_t* zero, OpSel* opt,
                                             int* sQ,
                                             unsigned long long* sExpl, const uint32_t* words,
                                             const uint32_t* wofs, const uint32_t* binom, int tt,
                                             unsigned long long& st_fout, unsigned long long& st_steps) {
  constexpr int HMAX = TLOG - 3;
  const int lane = threadIdx.x & 63;
  for (;;) {
    if (tt == 0) *sQ = atomicAdd(p.queue, 1);
    team_sync<TEAM>();
    const int qi = *sQ;
    if (tt == 0) *sExpl = 0;
    team_sync<TEAM>();
    if (qi >= p.n) break;
    const int h = p.order[qi];
    if (p.stamps && tt == 0) p.stamps[4 * h] = __builtin_amdgcn_s_memrealtime();
    const int lmax = p.lmax[h];
    const int NW = lmax > 3 ? 1 << (lmax - 3) : 1;
    const int ns = p.nsteps[h];
    for (int i = tt; i < NW; i += TEAM) B[i] = 0;
    team_sync<TEAM>();
    if (tt == 0) B[0] = 1;  // (cas-register) starts at nil: state id 0, nothing linearized
    StreamWin sw;
    int64_t pos = p.sbeg[h];
    unsigned long long expl = 0;
    int fail_t = -1;
    for (int t = 0; t < ns; ++t) {
      sw.need(p, pos, lane);
      int ninv;
      const uint32_t H0 = read_step(sw, pos, lane, tt < 64, opt, &ninv);
      pos += 1 + ninv;
      team_sync<TEAM>();
      const uint32_t live = H0 & DENSE_LIVE_MASK;
      const int j = (int)((H0 >> DENSE_J_SHIFT) & 31u);
      const uint32_t foldm = fold_mask(opt);
      const int Lw = 32 - __clz((int)live);
      const int nwt = 1 << (Lw > 3 ? Lw - 3 : 0);
      unsigned long long t0 = 0, nzx = 0, e0 = expl;
      if (p.lhist) {
        for (int i = tt; i < nwt; i += TEAM) nzx += B[i] != 0;
        t0 = __builtin_amdgcn_s_memrealtime();
      }
      expl += run_layers<HMAX, 4>(B, zero, words, wofs, binom, live, j, opt, foldm, tt, TEAM,
                                  [] { team_sync<TEAM>(); });
      if (p.lhist) {
        const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;
        unsigned long long nza = 0;
        for (int i = tt; i < nwt; i += TEAM) nza += B[i] != 0;
        unsigned long long* lh = p.lhist + ((TEAM >= 256 ? 32 : 0) + Lw) * LH_N;
        if (tt == 0) atomicAdd(&lh[0], 1ull), atomicAdd(&lh[1], dt);
        if (nzx) atomicAdd(&lh[2], nzx);
        if (nza) atomicAdd(&lh[3], nza);
        if (expl - e0) atomicAdd(&lh[4], expl - e0);
        team_sync<TEAM>();
      }
      const uint64_t anyv = return_slot(B, live, j, tt, TEAM, st_fout);
      ++st_steps;
      if (!team_any<TEAM>(anyv != 0)) {
        fail_t = t;
        break;
      }
    }
    // explored: team reduction
    for (int off = 32; off > 0; off >>= 1) expl += __shfl_down(expl, off, 64);
    if constexpr (TEAM >= 256) {
      if (lane == 0 && expl) atomicAdd(sExpl, expl);
      __syncthreads();
      expl = *sExpl;
    } else {
      expl = __shfl(expl, 0, 64);
    }
    if (tt == 0) {
      p.explored[h] = expl;
      p.fail_step[h] = fail_t;
      p.status[h] = fail_t >= 0 ? ST_INVALID : ST_VALID;
      if (p.stamps) p.stamps[4 * h + 1] = __builtin_amdgcn_s_memrealtime();
    }
    team_sync<TEAM>();
  }
}

// ---- REG histories (LC_PIPE bit 10): a WAVE history at most DENSE_REG_LMAX slots wide keeps its
// whole table in the wave's registers, word w in lane w (2^6 words), and runs history_loop's
// per-step schedule with lane shuffles for the pulls: no LDS round trip on a word's chain (C1's
// histories are 5..7 slots wide: ~16 words, a few shuffles per layer).
constexpr int PIPE_REG = 1024;
constexpr int PIPE_REG_FIX = 2048;  // REG histories: the closure as a whole-table fixpoint
// ... for steps at most this wide: a fixpoint iteration costs a fraction of a layer, but a
// step needs up to L + 1 of them against H + 1 = L - 2 layers (r3c: C1's 5..7-slot histories
// 0.498 -> 0.379 ms of kernel time with it on every REG step; C3, whose REG keys reach 9 slots,
// 11.39 -> 11.60 ms)
constexpr int REG_FIX_MAXL = 7;
constexpr int REG_LMAX = 9;

// Lane i <- lane i ^ 2^b of a 64-bit value, b a compile-time constant (REG histories: word w in
// lane w). b <= 3 stays inside a 16-lane row and is a DPP move (quad_perm for 1 and 2,
// row_half_mirror then quad_perm 3 for 4, row_ror 8 for 8): a VALU op instead of ds_bpermute's LDS
// round trip on every fixpoint iteration; wider distances keep the shuffle.
template <int B>
__device__ __forceinline__ uint64_t lane_xor(uint64_t v) {
  auto dpp = [](uint32_t x) -> uint32_t {
    if constexpr (B == 0) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);
    else if constexpr (B == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);
    else if constexpr (B == 2)
      return (uint32_t)__builtin_amdgcn_update_dpp(
          0, __builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false), 0x1B, 0xF, 0xF, false);
    else return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xF, 0xF, false);
  };
  if constexpr (B <= 3) return ((uint64_t)dpp((uint32_t)(v >> 32)) << 32) | dpp((uint32_t)v);
  else return (uint64_t)__shfl_xor((unsigned long long)v, 1 << B, 64);
}
template <int B>
__device__ __forceinline__ uint64_t lane_xor_dyn(uint64_t v, int b) {  // b == B..REG_LMAX-4, unrolled
  if constexpr (B >= 6) return v;
  else return b == B ? lane_xor<B>(v) : lane_xor_dyn<B + 1>(v, b);
}

// close_in_word with the in-word ops and the returning op's passed by value (no indexed array)
__device__ __forceinline__ uint64_t close_in_word_r(uint64_t X, uint32_t w, uint32_t live, int j, OpSel o0,
                                                   OpSel o1, OpSel o2, uint32_t foldm, uint64_t R) {
  const OpSel lo[3] = {o0, o1, o2};
  const bool j_lo = j < 3;
  const uint32_t jh = j_lo ? 0u : 1u << (j - 3);
  if (w & jh) return R;
  const uint32_t notj = j_lo ? keep8(j) : 0xffu;
  const uint64_t notj64 = j_lo ? keep64(j) : ~0ull;
  R &= notj64;
  const uint32_t lo_ops = live & 7u & ~(j_lo ? (1u << j) : 0u);
  const int nlo = __popc(lo_ops);
  auto lo_step = [&](int k) {
    if (lo_ops & (1u << k))
      R |= transfer_lo(lo[k], (foldm >> k) & 1u, X | R, keep8(k) & notj, keep64(k) & notj64, 1 << k);
  };
  lo_step(0);
  lo_step(1);
  lo_step(2);
  if (nlo == 3) {
    lo_step(0);
    lo_step(1);
    lo_step(0);
    lo_step(2);
  } else if (nlo == 2) {
    if (lo_ops & 1u) lo_step(0);
    else lo_step(1);
  }
  if (j_lo) {
    const OpSel oj = j == 0 ? o0 : j == 1 ? o1 : o2;
    R |= transfer_lo(oj, (foldm >> j) & 1u, X | R, notj, notj64, 1 << j);
  }
  return R;
}

// One REG history h on the calling wave (opt: an LDS op table of the wave, slot k at opt[k]).
__device__ __forceinline__ void run_regs(const DenseParams& p, int h, OpSel* opt, unsigned long long& st_fout,
                                         unsigned long long& st_steps) {
  const int lane = threadIdx.x & 63;
  const int ns = p.nsteps[h];
  if (lane < 16) opt[lane] = OpSel{SEL_NONE, SEL_NONE};
  uint64_t Bw = lane == 0 ? 1ull : 0ull;  // (cas-register) starts at nil, nothing linearized
  StreamWin sw;
  int64_t pos = p.sbeg[h];
  unsigned long long expl = 0;
  int fail_t = -1;
  for (int t = 0; t < ns; ++t) {
    sw.need(p, pos, lane);
    int ninv;
    const uint32_t H0 = read_step(sw, pos, lane, true, opt, &ninv);
    pos += 1 + ninv;
    const uint32_t live = H0 & DENSE_LIVE_MASK;
    const int j = (int)((H0 >> DENSE_J_SHIFT) & 31u);
    const uint32_t foldm = fold_mask(opt);
    const int L = 32 - __clz((int)live);
    const int H = L > 3 ? L - 3 : 0;
    const OpSel o0 = opt[0], o1 = opt[1], o2 = opt[2];
    OpSel oh[REG_LMAX - 3];
#pragma unroll
    for (int b = 0; b < REG_LMAX - 3; ++b) oh[b] = opt[3 + b];
    const uint32_t w = (uint32_t)lane;
    const uint32_t jh = j < 3 ? 0u : 1u << (j - 3);
    const uint32_t pm = (w & jh) ? jh : w;  // bits this word pulls over (only j when it holds j)
    const bool valid = w < (1u << H) && !(w & ~(live >> 3));
    const int pc = __popc(w);
    const bool fix = (p.pipe & PIPE_REG_FIX) && L <= REG_FIX_MAXL;
    if (fix) {
      // ---- the closure as a fixpoint over the whole table at once (LC_PIPE bit 11): every word
      // recomputes what its predecessors produce (hi pulls by lane shuffles, the low ops inside
      // the word) from the current table until no word changes. The layer DP above visits the
      // H + 1 popcount layers in order, each a dependent chain of up to 8 low-op transfers;
      // here an iteration's transfers are independent, and a step needs as many iterations as
      // its longest chain of linearizations (+1 to see no change). Same least fixpoint, so the
      // same produced set R and explored count.
      const bool j_lo = j < 3;
      const uint64_t notj64 = j_lo ? keep64(j) : ~0ull;
      const uint32_t notj = j_lo ? keep8(j) : 0xffu;
      const uint32_t lo_ops = live & 7u & ~(j_lo ? (1u << j) : 0u);
      const bool holds_j = (w & jh) != 0;
      const OpSel olo[3] = {o0, o1, o2};
      const uint64_t X = valid ? Bw : 0ull;
      uint64_t R = 0;
      for (int it = 0; it <= L + 1; ++it) {
        const uint64_t B = X | R;
        uint64_t Rn = 0;
#pragma unroll
        for (int b = 0; b < REG_LMAX - 3; ++b) {
          if (b >= H) break;
          const uint64_t v = lane_xor_dyn<0>(B, b) & notj64;
          if ((pm >> b) & 1u) Rn |= transfer(oh[b], (foldm >> (b + 3)) & 1u, v);
        }
        if (!holds_j) {
#pragma unroll
          for (int k = 0; k < 3; ++k)
            if (lo_ops & (1u << k))
              Rn |= transfer_lo(olo[k], (foldm >> k) & 1u, B, keep8(k) & notj, keep64(k) & notj64, 1 << k);
          if (j_lo) Rn |= transfer_lo(olo[j], (foldm >> j) & 1u, B, notj, notj64, 1 << j);
        }
        Rn = valid ? Rn : 0ull;
        const bool grew = __any(Rn != R);  // (R only grows)
        R = Rn;
        if (!grew) break;
      }
      expl += (uint32_t)__popcll(R);
      Bw = X | R;
    }
    for (int q = 0; q <= H && !fix; ++q) {
      uint64_t R = 0;
#pragma unroll
      for (int b = 0; b < REG_LMAX - 3; ++b) {
        if (b >= H) break;
        const uint64_t v = lane_xor_dyn<0>(Bw, b);
        if ((pm >> b) & 1u) R |= transfer(oh[b], (foldm >> (b + 3)) & 1u, v);
      }
      R = close_in_word_r(Bw, w, live, j, o0, o1, o2, foldm, R);
      if (valid && pc == q) {
        expl += (uint32_t)__popcll(R);
        Bw |= R;
      }
    }
    // return j: B'[m] = B[m | j], B'[m | j] = 0
    uint64_t nb;
    if (j >= 3) {
      const uint64_t v = (uint64_t)__shfl_xor((unsigned long long)Bw, (int)jh, 64);
      nb = (w & jh) ? 0ull : v;
    } else {
      nb = (Bw & ~keep64(j)) >> (1 << j);
    }
    Bw = valid ? nb : 0ull;
    st_fout += (uint32_t)__popcll(Bw);
    ++st_steps;
    if (!__any(Bw != 0)) {
      fail_t = t;
      break;
    }
  }
  for (int off = 32; off > 0; off >>= 1) expl += __shfl_down(expl, off, 64);
  if (lane == 0) {
    p.explored[h] = expl;
    p.fail_step[h] = fail_t;
    p.status[h] = fail_t >= 0 ? ST_INVALID : ST_VALID;
  }
}

// ---- pipelined steps (WAVE and BLOCK teams) ---------------------------------------------
//
// Consecutive RETURN steps of one history overlap. Step t+1's layer q reads only words of
// popcount <= q + 1 of step t's table (its own X, through the return map below) and writes
// words of popcount q, which step t last reads in its layer q + 1. So step t+1 may run its
// layer q in the same super-layer as step t's layer q + 2: a step starts two super-layers
// after its predecessor (one if the predecessor has a single layer), every running step
// advances one layer per super-layer, and one team barrier ends each super-layer. Up to
// (H + 1) / 2 steps are in flight; the barrier count per step falls from H + 1 to about 2.
//
// The return is never applied in place. Step t reads its frontier through step t-1's
// returning slot jp: X(w) = B[w | jp] (jp a word bit), (B[w] & with_jp) >> 2^jp (jp a low
// bit), and 0 for masks holding a slot invoked since that return ("fresh": those configs do
// not exist yet, whatever stale words their index holds). It stores every visited word, so
// the next step finds X | R at the word's own index. The OR of the X a step reads is step
// t-1's post-return frontier: zero means step t-1 is the failing RETURN. An empty frontier
// stays empty, so the steps started after a failure add no explored configs.
constexpr int PIPE_SERIAL_SEGS = DENSE_PIPE_SERIAL_SEGS;
// DenseParams.pipe bit 9: double-buffered tables. Step t works on table t & 1 and reads its X
// from the other one, so the WAR hazard that makes a step wait two super-layers for its
// predecessor disappears when the predecessor returned an in-word slot (jp < 3): step t's layer
// q then needs only step t-1's layer q (the same words), and may run one super-layer after it.
constexpr int PIPE_DBL = DENSE_PIPE_DBL;
constexpr int PIPE_OPN = 26;  // op-table entries per step: OP_PAD + slots 0..24 (team slots), + the pull batches' tail
struct __attribute__((aligned(16))) PipeStep {
  OpSel ops[PIPE_OPN];  // slot k at ops[OP_PAD + k]; every entry initialised
  uint32_t live, fresh, foldm, anyx;
  int32_t j, jp, H, start;  // H: layers - 1 over the LOCAL slots (all slots outside tile teams)
  int32_t pstart, hp, pad0, pad1;  // tile teams: the previous step's start and H
#ifndef LC_RING_NOPAD
  // 272 B, not 256: a ring view's lanes read consecutive entries' headers (16 B each), which at a
  // 256-B stride all fall into the same four LDS banks (a 16-way conflict per read); at 272 B
  // (68 dwords) sixteen entries cover all 64 banks once
  uint32_t bank_pad[4];
#endif
};
static_assert(sizeof(PipeStep) % 16 == 0, "ring entries stay 16-B aligned (the pull batches' op pairs)");

__device__ __forceinline__ int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Decode the step header at pos into dst (one whole wave): the op table is the previous
// step's plus this step's invocations; the fresh slots are the live ones the previous step
// did not leave pending.
__device__ __forceinline__ void pipe_decode(const DenseParams& p, StreamWin& sw, int64_t& pos, int lane,
                                            PipeStep* dst, const PipeStep* prev, uint32_t lmask = ~0u) {
  sw.need(p, pos, lane);
  const uint32_t H0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)sw.at(pos));
  const uint32_t wd = sw.at(pos + 1 + lane);
  const int ninv = (int)__builtin_ctzll(~__ballot(lane <= DENSE_MAX_NINV && (wd & DENSE_OPW)));
  const uint32_t plive = prev ? (uint32_t)rfl((int)prev->live) : 0u;
  const int pj = prev ? rfl(prev->j) : -1;
  if (lane < PIPE_OPN) dst->ops[lane] = prev ? prev->ops[lane] : OpSel{SEL_NONE, SEL_NONE};
  if (lane < ninv) dst->ops[OP_PAD + (wd & 31u)] = decode_op((wd >> 8) & 0xffu, (wd >> 16) & 0xffu);
  // after the stores (one wave's LDS ops stay in order)
  const uint32_t foldm =
      (uint32_t)__ballot(lane < PIPE_OPN - OP_PAD && dst->ops[OP_PAD + lane].hi == OPS_FOLD);
  if (lane == 0) {
    const uint32_t live = H0 & DENSE_LIVE_MASK, lloc = live & lmask;
    const int L = lloc ? 32 - __clz((int)lloc) : 0;
    dst->live = live;
    dst->fresh = prev ? live & ~(plive & ~(1u << pj)) : live;
    dst->foldm = foldm;
    dst->anyx = 0;
    dst->j = (int)((H0 >> DENSE_J_SHIFT) & 31u);
    dst->jp = pj;
    dst->H = L > 3 ? L - 3 : 0;
    dst->start = 1 << 30;  // not started
    dst->hp = prev ? prev->H : 0;
  }
  pos += 1 + ninv;
}

// word w's frontier before step (fresh, jp): step jp's post-return table, read in place
__device__ __forceinline__ uint64_t pipe_x(const uint64_t* B, uint32_t w, uint32_t fresh_hi, int jp,
                                           uint64_t keep_lo) {
  if (w & fresh_hi) return 0;
  uint64_t v;
  if (jp >= 3) v = B[w | (1u << (jp - 3))];
  else if (jp >= 0) v = (B[w] & ~keep64(jp)) >> (1 << jp);
  else v = B[w];
  return v & keep_lo;
}

// LC_PIPE bit 12 (double-buffered tables): a step after a hi-slot return starts ONE super-layer
// after its predecessor, not two. Step t's frontier word X_t(w) = B_{t-1}(w | j) (j = step t-1's
// returning slot, a hi bit) is a word of popcount q + 1 that step t-1 finishes in the same
// super-layer as step t's layer q. But step t-1 computes that word as X_{t-1}(w | j) |
// T_j(B_{t-1}(w)) (configs holding j are only produced by linearizing j last, never expanded),
// and both parts are ready a super-layer earlier: B_{t-1}(w) has popcount q, and X_{t-1}(w | j)
// is a read of step t-2's finished table (popcount q + 1, or q + 2 through a hi return of step
// t-2). So step t computes its X itself from them; the start rule then only needs step t-2 to
// be 2 (3) super-layers ahead. Same X, so the same tables, explored counts and verdicts.
// Off by default: measured (r3e, 8-way rank 0 share) it cuts the super-layers of the WAVE /
// BLOCK / MID teams by 18 / 23 / 16 %, but each super-layer then holds more steps' words and a
// longer X chain (two dependent LDS reads), and costs 25-30 % more: the pools end 3-10 % later
// (C3 11.46 -> 11.46 ms, rank shares unchanged within noise). Bit-exact either way (GPU tests
// run LC_PIPE 8143).
constexpr int PIPE_XHI = 4096;

// X_t(w) of a step whose predecessor (ring entry pv, table Bp; its own predecessor's table Bpp)
// returned hi slot jp: X_{t-1}(w | jp) | T_jp(B_{t-1}(w)). The caller masks fresh masks / slots.
__device__ __forceinline__ uint64_t pipe_x_hi(const uint64_t* Bpp, const uint64_t* Bp, const PipeStep* pv,
                                              uint32_t w, int jp) {
  const uint32_t pf = pv->fresh;
  uint64_t pk = ~0ull;
#pragma unroll
  for (int k = 0; k < 3; ++k)
    if (pf & (1u << k)) pk &= keep64(k);
  const uint64_t xp = pipe_x(Bpp, w | (1u << (jp - 3)), pf >> 3, pv->jp, pk);
  return xp | transfer(pv->ops[OP_PAD + jp], (pv->foldm >> jp) & 1u, Bp[w]);
}

template <typename T>
__device__ __forceinline__ T rdl(T v, int l) {
  return (T)__builtin_amdgcn_readlane((int)v, l);
}

// Control state is wave-uniform and identical in every wave of the team. Each super-layer
// starts after a barrier with ONE lane-parallel read of the ring: lane i holds the header of
// step t_ret + i. Retirement (in order, with the failure test), the running steps' layers
// ("segments") and the next start all come from that view by ballots and readlanes.
// SUB: the team is TEAM/64 waves of a larger workgroup (big_mid_mode), synchronised through
// its own LDS barrier words qb (s_barrier would stop every wave of the workgroup).
template <int TEAM, int TLOG, int RING, bool SUB = false, int CAPW = (1 << (TLOG - 3))>
__device__ __forceinline__ void history_pipe(const DenseParams& p, uint64_t* B, const uint64_t* zero,
                                             PipeStep* ring, int* sQ, unsigned long long* sExpl,
                                             const uint32_t* words_g, const uint32_t* wofs_g, const uint32_t* binom,
                                             int tt, unsigned long long& st_fout, unsigned long long& st_steps,
                                             unsigned* qb = nullptr) {
  auto tsync = [&]() {
    if constexpr (SUB) sub_sync<TEAM>(qb);
    else team_sync<TEAM>();
  };
  // pull batches read entries up to OP_PAD + b0 + 6 (b0 < H, a multiple of 4); slots < TLOG
  static_assert(OP_PAD + ((TLOG - 4) / 4) * 4 + 6 < PIPE_OPN && OP_PAD + TLOG <= PIPE_OPN, "op table too small");
  static_assert(RING <= 64, "one lane per ring entry");
  const int lane = threadIdx.x & 63;
  // the team's last wave decodes the step headers: packed passes fill the low threads first,
  // so it has the fewest words of a super-layer
  const bool decoder = tt >= TEAM - 64;
  for (;;) {
    if (tt == 0) *sQ = atomicAdd(p.queue, 1);
    tsync();
    const int qi = *sQ;
    if (tt == 0) *sExpl = 0;
    tsync();
    if (qi >= p.n) break;
    const int h = p.order[qi];
    if (p.stamps && tt == 0) p.stamps[4 * h] = __builtin_amdgcn_s_memrealtime();
    const int lmax = p.lmax[h];
    if constexpr (TEAM == 64) {
      if ((p.pipe & PIPE_REG) && lmax <= REG_LMAX) {  // the table fits the wave's registers
        unsigned long long sf = 0, ss = 0;
        run_regs(p, h, ring[0].ops + OP_PAD, sf, ss);
        if (tt == 0) st_steps += ss;
        st_fout += sf;
        if (p.stamps && tt == 0) p.stamps[4 * h + 1] = __builtin_amdgcn_s_memrealtime();
        continue;
      }
    }
    const int NW = lmax > 3 ? 1 << (lmax - 3) : 1;
    const int ns = p.nsteps[h];
    // double-buffered tables (PIPE_DBL) when two fit the team's LDS: step t on tab(t)
    const bool dbl = (p.pipe & PIPE_DBL) && 2 * NW <= CAPW;
    const bool xhi = dbl && (p.pipe & PIPE_XHI);  // (needs step t-2's table intact: two tables)
    uint64_t* const B2 = dbl ? B + NW : B;
    auto tab = [&](int t) { return (t & 1) ? B2 : B; };
    const int ntab = dbl ? 2 * NW : NW;
    for (int i = tt; i < ntab; i += TEAM) B[i] = 0;
    // a BLOCK history of width <= 16 leaves room in the LDS table for its own word list (the
    // 2^(lmax-3) words below the table's width, by popcount layer) and the layers' offsets:
    // the word index of a packed pass then comes from LDS, not from the global list
    const uint32_t* words = words_g;
    const uint32_t* wofs = wofs_g;
    if constexpr (TLOG == DENSE_LMAX && TEAM >= 256) {
      if (lmax <= DENSE_LMAX - 1 && lmax > 3 && ntab + NW / 2 + 16 <= CAPW) {
        const int Hh = lmax - 3;
        uint32_t* lw = reinterpret_cast<uint32_t*>(B + ntab);
        uint32_t* lo = lw + NW;
        if (tt <= Hh + 1) {
          uint32_t o = 0;
          for (int q = 0; q < tt; ++q) o += binom[Hh * BINOM_N + q];
          lo[tt] = o;
        }
        tsync();
        for (int q = 0; q <= Hh; ++q) {
          const uint32_t nq = binom[Hh * BINOM_N + q], og = wofs_g[q], ol = lo[q];
          for (uint32_t r = (uint32_t)tt; r < nq; r += (uint32_t)TEAM) lw[ol + r] = words_g[og + r];
        }
        words = lw, wofs = lo;
      }
    }
    tsync();
    // (cas-register) starts at nil: state id 0, nothing linearized; step 0 reads tab(-1)
    if (tt == 0) B2[0] = 1;
    StreamWin sw;
    int64_t pos = p.sbeg[h];
    if (ns > 0 && decoder) {
      pipe_decode(p, sw, pos, lane, &ring[0], nullptr);
      if (lane == 0) ring[0].start = 0;  // (the decoder wave, after its own stores)
    }
    tsync();
    unsigned long long expl = 0;
    int fail_t = -1;
    int t_dec = ns > 0 ? 1 : 0, t_run = t_dec, t_ret = 0;  // decoded, started, retired
    // LC_DEBUG: super-layer phase cycles of wave 0 and of the decoder wave (ring view + retire,
    // segments, decode + start, barrier), s_memtime
    const bool prof = p.lhist != nullptr && (tt == 0 || tt == TEAM - 64);
    unsigned long long ph[4] = {0, 0, 0, 0}, tp = prof ? __builtin_amdgcn_s_memtime() : 0, nsl = 0;
    auto mark = [&](int k) {
      if (prof) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        ph[k] += t - tp;
        tp = t;
      }
    };
    for (int s = 0; t_ret < ns; ++s) {
      // ---- ring view: lane i = step t_ret + i (decoded steps only)
      const int tl = t_ret + lane;
      const bool dec_l = lane < RING && tl < t_dec;
      uint4 h0 = {0u, 0u, 0u, 0u};
      int4 h1 = {0, 0, 0, 1 << 30};
      if (dec_l) {
        const PipeStep* st = &ring[tl % RING];
        h0 = *reinterpret_cast<const uint4*>(&st->live);  // live, fresh, foldm, anyx
        h1 = *reinterpret_cast<const int4*>(&st->j);      // j, jp, H, start
      }
      const bool run_l = dec_l && tl < t_run;
      // retire the steps whose last layer ran in an earlier super-layer, in order
      const bool fin_l = run_l && h1.w + h1.z < s;
      const uint64_t fin = __ballot(fin_l);
      const int lead = (int)__builtin_ctzll(~fin);
      const uint64_t lead_mask = lead >= 64 ? ~0ull : (1ull << lead) - 1;
      const uint64_t bad = __ballot(fin_l && tl > 0 && h0.w == 0u) & lead_mask;
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
      if (seg_l) nq_l = binom[h1.z * BINOM_N + q_l], o_l = wofs[q_l];
      uint64_t segm = __ballot(seg_l);
      mark(0);
      ++nsl;
      if (TEAM == 64 && !(p.pipe & PIPE_SERIAL_SEGS)) {
        // one wave: the segments' words packed lane by lane (a wave team's layers are small),
        // each lane with its own step's parameters from the ring entry
        uint32_t total = 0;
        for (uint64_t m = segm; m; m &= m - 1) total += rdl(nq_l, (int)__builtin_ctzll(m));
        for (uint32_t f0 = 0; f0 < total; f0 += 64u) {
          const uint32_t f = f0 + (uint32_t)lane;
          int i = 0;
          uint32_t e = 0, acc = 0, o = 0;
          for (uint64_t m = segm; m; m &= m - 1) {
            const int k = (int)__builtin_ctzll(m);
            if (f >= acc) i = k, e = acc, o = rdl(o_l, k);
            acc += rdl(nq_l, k);
          }
          if (f >= total) continue;
          const uint32_t w = words[o + (f - e)];
          const int t = t_ret_old + i;
          PipeStep* st = &ring[t % RING];
          const uint4 a = *reinterpret_cast<const uint4*>(&st->live);  // live, fresh, foldm, anyx
          const int4 c = *reinterpret_cast<const int4*>(&st->j);       // j, jp, H, start
          const uint32_t live = a.x, fresh = a.y, foldm = a.z;
          if (w & ~(live >> 3)) continue;
          uint64_t keep_lo = ~0ull;
#pragma unroll
          for (int k = 0; k < 3; ++k)
            if (fresh & (1u << k)) keep_lo &= keep64(k);
          const OpSel* ops = st->ops + OP_PAD;
          uint64_t* const Bt = tab(t);
          const uint64_t X = (xhi && c.y >= 3 && t > 0)
                                 ? ((w & (fresh >> 3)) ? 0ull
                                                       : pipe_x_hi(tab(t - 2), tab(t - 1), &ring[(t - 1) % RING], w, c.y) &
                                                             keep_lo)
                                 : pipe_x(tab(t - 1), w, fresh >> 3, c.y, keep_lo);
          uint64_t R = pull_set(Bt, w, c.x, ops, foldm);
          R = close_in_word(X, w, live, c.x, ops, foldm, R);
          Bt[w] = X | R;
          expl += (uint32_t)__popcll(R);
          if (t > 0) st_fout += (uint32_t)__popcll(X);
          if (X) st->anyx = 1;
        }
        segm = 0;
      }
      if (!(p.pipe & PIPE_SERIAL_SEGS)) {
        // packed: the running segments' words form one flat index over the whole team, each
        // segment padded to whole waves (segment i at [e_i, e_i + roundup(nq_i, 64))), so a
        // super-layer of several small layers is ONE pass of the team instead of one pass per
        // segment, and every wave works on a single step: its parameters are wave-uniform
        // (readlanes of the ring view), its op branches scalar
        uint32_t total = 0;
        for (uint64_t m = segm; m; m &= m - 1) total += (rdl(nq_l, (int)__builtin_ctzll(m)) + 63u) & ~63u;
        for (uint32_t f0 = (uint32_t)(tt & ~63); f0 < total; f0 += (uint32_t)TEAM) {
          int i = 0;
          uint32_t e = 0, acc = 0;
          for (uint64_t m = segm; m; m &= m - 1) {
            const int k = (int)__builtin_ctzll(m);
            if (f0 >= acc) i = k, e = acc;
            acc += (rdl(nq_l, k) + 63u) & ~63u;
          }
          const uint32_t nq = rdl(nq_l, i), r = f0 - e + (uint32_t)lane;
          const uint32_t live = rdl(h0.x, i), fresh = rdl(h0.y, i), foldm = rdl(h0.z, i);
          const int j = rdl(h1.x, i), jp = rdl(h1.y, i), H = rdl(h1.z, i);
          const int t = t_ret_old + i;
          if (r >= nq) continue;
          const uint32_t w = words[rdl(o_l, i) + r];
          if (w & ~(live >> 3)) continue;
          uint64_t keep_lo = ~0ull;
#pragma unroll
          for (int k = 0; k < 3; ++k)
            if (fresh & (1u << k)) keep_lo &= keep64(k);
          PipeStep* st = &ring[t % RING];
          const OpSel* ops = st->ops + OP_PAD;
          uint64_t* const Bt = tab(t);
          const uint64_t X = (xhi && jp >= 3 && t > 0)
                                 ? ((w & (fresh >> 3)) ? 0ull
                                                       : pipe_x_hi(tab(t - 2), tab(t - 1), &ring[(t - 1) % RING], w, jp) &
                                                             keep_lo)
                                 : pipe_x(tab(t - 1), w, fresh >> 3, jp, keep_lo);
          uint64_t R = pull_set(Bt, w, j, ops, foldm);
          R = close_in_word(X, w, live, j, ops, foldm, R);
          Bt[w] = X | R;
          expl += (uint32_t)__popcll(R);
          if (t > 0) st_fout += (uint32_t)__popcll(X);
          if (X) st->anyx = 1;
        }
        segm = 0;
      }
      int i = segm ? (int)__builtin_ctzll(segm) : -1;
      uint32_t wn = 0;
      if (i >= 0 && (uint32_t)tt < rdl(nq_l, i)) wn = words[rdl(o_l, i) + tt];
      while (i >= 0) {  // serial segments (PIPE_SERIAL_SEGS): one pass per segment
        segm &= segm - 1;
        const int i2 = segm ? (int)__builtin_ctzll(segm) : -1;
        uint32_t wn2 = 0;  // the next segment's first word, loaded ahead
        if (i2 >= 0 && (uint32_t)tt < rdl(nq_l, i2)) wn2 = words[rdl(o_l, i2) + tt];
        const uint32_t nq = rdl(nq_l, i), o = rdl(o_l, i);
        const uint32_t live = rdl(h0.x, i), fresh = rdl(h0.y, i), foldm = rdl(h0.z, i);
        const int j = rdl(h1.x, i), jp = rdl(h1.y, i), H = rdl(h1.z, i);
        const int t = t_ret_old + i;
        uint64_t keep_lo = ~0ull;
#pragma unroll
        for (int k = 0; k < 3; ++k)
          if (fresh & (1u << k)) keep_lo &= keep64(k);
        const uint32_t live_hi = live >> 3, fresh_hi = fresh >> 3;
        PipeStep* st = &ring[t % RING];
        const OpSel* ops = st->ops + OP_PAD;
        uint64_t* const Bt = tab(t);
        const uint64_t* const Bp = tab(t - 1);
        uint64_t nzx = 0;
        for (uint32_t r = (uint32_t)tt; r < nq; r += (uint32_t)TEAM) {
          const uint32_t w = wn;
          if (r + TEAM < nq) wn = words[o + r + TEAM];
          if (w & ~live_hi) continue;
          const uint64_t X = (xhi && jp >= 3 && t > 0)
                                 ? ((w & fresh_hi) ? 0ull
                                                   : pipe_x_hi(tab(t - 2), Bp, &ring[(t - 1) % RING], w, jp) & keep_lo)
                                 : pipe_x(Bp, w, fresh_hi, jp, keep_lo);
          uint64_t R = pull_set(Bt, w, j, ops, foldm);
          R = close_in_word(X, w, live, j, ops, foldm, R);
          Bt[w] = X | R;
          expl += (uint32_t)__popcll(R);
          if (t > 0) st_fout += (uint32_t)__popcll(X);
          nzx |= X;
        }
        if (nzx) st->anyx = 1;
        i = i2, wn = wn2;
      }
      mark(1);
      // ---- decode ahead into a slot nobody read in this super-layer
      const int t_dec_old = t_dec;
      // (with xhi a running step reads its predecessor's ring entry: one slot stays reserved)
      if (t_dec < ns && t_dec - t_ret_old < RING - (xhi ? 1 : 0)) {
        if (decoder) pipe_decode(p, sw, pos, lane, &ring[t_dec % RING], &ring[(t_dec - 1) % RING]);
        ++t_dec;
      }
      // ---- start the next decoded step at s + 1: two super-layers after its predecessor
      // (one if that has a single layer, or returned an in-word slot on double-buffered
      // tables; with xhi also after a hi return, when the predecessor's predecessor is 2 (3 after
      // its own hi return) super-layers ahead), or at once if the predecessor retired
      if (t_run < t_dec_old) {
        const int lp = t_run - 1 - t_ret_old;  // the predecessor's lane (< 0: retired)
        const int lpp = lp - 1;
        const bool pred_hi = lp >= 0 && rdl(h1.x, lp) >= 3;
        bool ok;
        if (lp < 0 || lp < lead) {
          ok = true;
        } else if (xhi && pred_hi) {
          ok = lpp < 0 || lpp < lead || t_run < 2 ||
               s + 1 - rdl(h1.w, lpp) >= min(rdl(h1.x, lpp) < 3 ? 2 : 3, rdl(h1.z, lpp) + 1);
        } else {
          const int gap = (dbl && !pred_hi) ? 1 : 2;
          ok = s + 1 - rdl(h1.w, lp) >= min(gap, rdl(h1.z, lp) + 1);
        }
        if (ok) {
          if (tt == 0) ring[t_run % RING].start = s + 1;
          ++t_run;
        }
      }
      mark(2);
      tsync();
      mark(3);
    }
    if (prof) {
      unsigned long long* q = p.lhist + 64 * LH_N + (TEAM == 64 ? 0 : TEAM >= 1024 ? 10 : 20) + (tt == 0 ? 0 : 5);
      for (int k = 0; k < 4; ++k) atomicAdd(&q[k], ph[k]);
      atomicAdd(&q[4], nsl);
    }
    if (fail_t < 0 && ns > 0) {  // the last step's return
      const PipeStep* st = &ring[(ns - 1) % RING];
      const int jl = rfl(st->j);
      const uint32_t live = (uint32_t)rfl((int)st->live) & ~(1u << jl);
      const int L = live ? 32 - __clz((int)live) : 0;
      const int nwt = 1 << (L > 3 ? L - 3 : 0);
      uint64_t nzx = 0;
      for (int w = tt; w < nwt; w += TEAM) {
        if ((uint32_t)w & ~(live >> 3)) continue;
        const uint64_t X = pipe_x(tab(ns - 1), (uint32_t)w, 0u, jl, ~0ull);
        st_fout += (uint32_t)__popcll(X);
        nzx |= X;
      }
      if constexpr (SUB) {
        const bool anyw = __any(nzx != 0);  // (every lane votes)
        if ((tt & 63) == 0 && anyw) atomicOr(&qb[2], 1u);
        tsync();
        if (!qb[2]) fail_t = ns - 1;
        tsync();
        if (tt == 0) qb[2] = 0;
      } else if (!team_any<TEAM>(nzx != 0)) {
        fail_t = ns - 1;
      }
    }
    if (tt == 0) st_steps += fail_t >= 0 ? fail_t + 1 : ns;
    for (int off = 32; off > 0; off >>= 1) expl += __shfl_down(expl, off, 64);
    if constexpr (TEAM >= 256) {
      if (lane == 0 && expl) atomicAdd(sExpl, expl);
      tsync();
      expl = *sExpl;
    } else {
      expl = __shfl(expl, 0, 64);
    }
    if (tt == 0) {
      p.explored[h] = expl;
      p.fail_step[h] = fail_t;
      p.status[h] = fail_t >= 0 ? ST_INVALID : ST_VALID;
      if (p.stamps) p.stamps[4 * h + 1] = __builtin_amdgcn_s_memrealtime();
    }
    tsync();
  }
}

// launch statistics (per wave, one atomic each)
// (st_steps is held by each team's first thread, zero elsewhere: summed over every wave)
__device__ __forceinline__ void flush_stats(const DenseParams& p, unsigned long long st_fout,
                                            unsigned long long st_steps, bool /*step_owner*/) {
  for (int off = 32; off > 0; off >>= 1) {
    st_fout += __shfl_down(st_fout, off, 64);
    st_steps += __shfl_down(st_steps, off, 64);
  }
  if ((threadIdx.x & 63) == 0 && st_fout) atomicAdd(&p.stats[SS_FOUT], st_fout);
  if ((threadIdx.x & 63) == 0 && st_steps) atomicAdd(&p.stats[SS_STEPS], st_steps);
}

constexpr int WAVE_WG = 256;
// pipeline rings: running steps <= (H + 1) / 2, plus one decoded ahead and one retire margin
constexpr int WAVE_RING = 8, BLOCK_RING = 16;
// tile teams: steps decoded ahead + in flight. With global layers (PIPE_GLAY) a step spans
// H + T + 1 super-layers, so at one start per ~1.2-1.8 super-layers 16 entries ran out (r3g:
// rotated C3 share 1190 -> 1339 super-layers)
constexpr int TEAM_RING = 32;

// WAVE teams: one history per wave, 4 waves per workgroup, tables of 2^DENSE_WAVE_LMAX masks.
__global__ void __launch_bounds__(WAVE_WG) dense_wave_kernel(DenseParams p) {
  constexpr int NTEAM = WAVE_WG / 64;
  constexpr int HMAX = DENSE_WAVE_LMAX - 3;
  __shared__ uint64_t sTab[NTEAM << HMAX];
  __shared__ uint32_t sWords[1 << HMAX];  // words sorted by (popcount, value)
  __shared__ uint32_t sWOff[HMAX + 2];
  __shared__ uint32_t sBinom[BINOM_N * BINOM_N];
  __shared__ __attribute__((aligned(16))) OpSel sOp[NTEAM][OP_TAB];
  __shared__ int sQ[NTEAM];
  __shared__ uint64_t sZero;  // the word pulls of absent bits read
  __shared__ unsigned long long sExpl[NTEAM];
  __shared__ PipeStep sRing[NTEAM][WAVE_RING];
  const int tid = threadIdx.x, team = tid / 64, tt = tid % 64;
  init_tables(sBinom, sWOff, HMAX, WAVE_WG);
  if (tid == 0) sZero = 0;
  // every op-table entry moves nothing until its slot is invoked (v_perm selector bytes
  // 13..15 would make 0xff out of a zero word)
  for (int i = tid; i < NTEAM * OP_TAB; i += WAVE_WG) (&sOp[0][0])[i] = OpSel{SEL_NONE, SEL_NONE};
  for (int v = tid; v < (1 << HMAX); v += WAVE_WG) {  // colex rank within its popcount layer
    uint32_t rank = 0;
    int i = 0;
    for (uint32_t x = (uint32_t)v; x; x &= x - 1, ++i) rank += sBinom[__builtin_ctz(x) * BINOM_N + i + 1];
    sWords[sWOff[__popc(v)] + rank] = (uint32_t)v;
  }
  __syncthreads();
  unsigned long long st_fout = 0, st_steps = 0;
  if (p.pipe & 2)
    history_pipe<64, DENSE_WAVE_LMAX, WAVE_RING>(p, &sTab[team << HMAX], &sZero, sRing[team], &sQ[team], &sExpl[team],
                                                 sWords, sWOff, sBinom, tt, st_fout, st_steps);
  else
    history_loop<64, DENSE_WAVE_LMAX>(p, &sTab[team << HMAX], &sZero, sOp[team] + OP_PAD, &sQ[team], &sExpl[team],
                                      sWords, sWOff, sBinom, tt, st_fout, st_steps);
  flush_stats(p, st_fout, st_steps, tt == 0);
}

// MID teams: one history per 256-thread workgroup, tables of 2^DENSE_MID_LMAX masks (16 KiB),
// pipelined steps; several workgroups share a CU (BLOCK histories of widths 12..14, whose
// steps are mostly narrow and latency-bound, no longer hold a whole CU each).
constexpr int MID_WG = 256, MID_RING = 6;  // LDS <= the wave kernel's (both fit beside a big workgroup)
__global__ void __launch_bounds__(MID_WG) dense_mid_kernel(DenseParams p) {
  constexpr int HMAX = DENSE_MID_LMAX - 3;
  __shared__ uint64_t sTab[1 << HMAX];
  __shared__ uint32_t sWOff[DENSE_WORD_BITS + 2];
  __shared__ uint32_t sBinom[BINOM_N * BINOM_N];
  __shared__ PipeStep sRing[MID_RING];
  __shared__ int sQ;
  __shared__ unsigned long long sRed;
  __shared__ uint64_t sZero;
  const int tid = threadIdx.x;
  init_tables(sBinom, sWOff, DENSE_WORD_BITS, MID_WG);
  if (tid == 0) sZero = 0;
  __syncthreads();
  unsigned long long st_fout = 0, st_steps = 0;
  history_pipe<MID_WG, DENSE_MID_LMAX, MID_RING>(p, sTab, &sZero, sRing, &sQ, &sRed, p.words, sWOff, sBinom, tid,
                                                 st_fout, st_steps);
  flush_stats(p, st_fout, st_steps, tid == 0);
}

// Team barrier over a tile team's G workgroups: every wave drains its (sc1) stores, one lane
// per workgroup adds to the arrival counter, the last arriver bumps the generation the
// others poll (relaxed sc1 loads + s_sleep). A 20 s watchdog raises p.abort instead of
// hanging. Returns false once aborted.
__device__ __forceinline__ bool team_bar(TeamCtl* c, int G, int32_t* abort_flag, int* s_abort) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = ld_agent(&c->gen);
    const unsigned a = __hip_atomic_fetch_add(&c->count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a == (unsigned)G - 1) {
      st_agent(&c->count, 0u);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      st_agent(&c->gen, g + 1);
    } else {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      long spins = 0;
      while (ld_agent(&c->gen) == g) {
        __builtin_amdgcn_s_sleep(2);
        if ((++spins & 255) == 0) {
          if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000000ull) {
            st_agent(abort_flag, 1);
            break;
          }
          if (ld_agent(abort_flag)) break;
        }
      }
    }
    *s_abort = ld_agent(abort_flag);
  }
  __syncthreads();
  return *s_abort == 0;
}

// thread 0 waits until every flag of `mask` (bit b -> flags[rank ^ (1 << b)]) reaches
// token, then the workgroup proceeds (sc1 polls, s_sleep, 20 s watchdog).
__device__ __forceinline__ void wait_flags(const DenseParams& p, unsigned long long* flags, int rank,
                                           uint32_t mask, unsigned long long token, int* s_abort) {
  if (threadIdx.x == 0 && mask) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    long spins = 0;
    for (uint32_t m = mask; m;) {
      const int b = __builtin_ctz(m);
      if (ld_agent(&flags[rank ^ (1 << b)]) >= token) {
        m &= m - 1;
        continue;
      }
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 255) == 0) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000000ull) {
          st_agent(p.abort, 1);
          *s_abort = 1;
          break;
        }
        if (ld_agent(p.abort)) {
          *s_abort = 1;
          break;
        }
      }
    }
  }
  __syncthreads();
}

__device__ __forceinline__ unsigned long long block_sum(unsigned long long v, unsigned long long* s) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  if (threadIdx.x == 0) *s = 0;
  __syncthreads();
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(s, v);
  __syncthreads();
  const unsigned long long r = *s;
  __syncthreads();
  return r;
}

// ---- pipelined tile team (DenseParams.pipe bit 2) ----------------------------------------
//
// Every tile walks the step stream itself and runs the pipelined schedule of history_pipe
// (layers over its LOCAL slots, identical on every tile, so all tiles agree on every
// super-layer's segments). A step whose live slots include team slots is "wide": its
// words are published to the tile's mirror slot for that step (MRING slots per tile, in
// word-list order) and successors pull them. Per super-layer a tile waits, before any work,
// until (1) every predecessor it pulls from (tile r \ b, or r \ j for a tile holding the
// returning j) has finished the same super-layer, and (2) for a step whose previous step
// returned a team slot jp, tile r | jp (which holds that step's post-return frontier for
// r's masks) has finished the previous step's same layer, i.e. super-layer pstart + q.
// Then it works, drains its sc1 mirror stores, and stores its token = super-layers done.
// Dependencies (1) point to tiles with fewer team bits and (2) to the previous step two
// super-layers back, so the team runs as a skewed pipeline. Every 8 super-layers each tile
// waits until all tokens are within 8 super-layers of its own, so a mirror slot is reused
// only after all its readers passed it (MRING = 64 > 16 + the widest step's 15 + 8 super-layers).
// Failures are decided after the last step: each tile ORs "read a nonzero X in step t"
// into the team's bit t in HBM; the leader's first missing bit t names step t - 1.
constexpr int MRING = DENSE_MRING;
// LC_PIPE bit 13 (PIPE_GLAY): super-layers index a wide step's GLOBAL popcount layers. Tile r
// runs its local layer q at super-layer start + q + |r| (|r| = its live team bits), so a pull
// from tile r \ b reads what that tile finished one super-layer earlier: no tile waits inside
// a super-layer for another tile's same super-layer, a super-layer costs one hand-off instead of
// a chain of up to T, and a step spans H + T + 1 super-layers. The start rule, the retire rule
// and the token waits count the T; the previous step's X (tile r | jp) is read at least two
// super-layers after it was written, as before. Mirror slots: a step's words are read up to
// H + T super-layers after its start, plus the 16-super-layer credit lag (MRING = 64).
constexpr int PIPE_GLAY = 8192;
constexpr int PIPE_XCD = 16384;  // XCD-compact workgroup roles in the big kernel (dense_big_kernel)
// tile teams: credit tokens pre-polled a super-layer early (r3n A/B, 2 runs each: C2 30.08 ->
// 29.92 ms, 8-way shares 0/1 7.14 -> 7.12 / 7.03 -> 6.97, C3 11.46 -> 11.44)
constexpr int PIPE_CPRE = 65536;
constexpr int PIPE_CW16 = 131072;  // tile teams: a credit window of 16 super-layers (else 8)
constexpr int PIPE_WSPREAD = 262144;  // big kernel: WAVE histories one per workgroup (big_wave_mode)

__device__ __forceinline__ bool poll_until(const DenseParams& p, const unsigned long long* f,
                                           unsigned long long need, uint64_t t0, long& spins) {
  if (ld_agent(f) >= need) return true;
  __builtin_amdgcn_s_sleep(1);
  if ((++spins & 255) == 0 && (__builtin_amdgcn_s_memrealtime() - t0 > 2000000000ull || ld_agent(p.abort))) {
    st_agent(p.abort, 1);
    return true;  // gives up: the caller sees the abort flag
  }
  return false;
}

__device__ __forceinline__ void team_pipe(const DenseParams& p, uint64_t* B, const uint64_t* zero, PipeStep* ring,
                                          const uint32_t* cum, const uint32_t* binom, const uint32_t* wofs,
                                          int team, int base, int rank, int G, int h, int lb, int* sAbort,
                                          unsigned long long& expl, unsigned long long& st_fout) {
  constexpr int HSOLO = DENSE_LMAX - 3;
  constexpr int RING = TEAM_RING;
  const int tid = threadIdx.x, lane = tid & 63;
  const bool decoder = tid < 64;
  const uint32_t lmask = (1u << lb) - 1;
  // double-buffered tile tables (PIPE_DBL) when two fit the LDS table (lb <= 16)
  const bool dbl = (p.pipe & PIPE_DBL) && lb <= DENSE_LMAX - 1;
  uint64_t* const B2 = dbl ? B + (1 << (lb - 3)) : B;
  auto tab = [&](int t) { return (t & 1) ? B2 : B; };
  // the tile's word list (2^(lb-3) words by popcount layer; a step of H < lb - 3 hi bits uses
  // each layer's first C(H, q): colex order) in LDS beside the table(s) when it fits, as BLOCK
  // histories do: a word's index is then an LDS read, not a global load, on every word's chain
  const uint32_t* words = p.words;
  const uint32_t* wof = wofs;
  {
    const int Hm = lb - 3, ntab = (dbl ? 2 : 1) << Hm;
    if (Hm >= 1 && ntab + (1 << Hm) / 2 + 16 <= (1 << HSOLO)) {
      uint32_t* lw = reinterpret_cast<uint32_t*>(B + ntab);
      uint32_t* lo = lw + (1 << Hm);
      if (tid <= Hm + 1) {
        uint32_t o = 0;
        for (int q = 0; q < tid; ++q) o += binom[Hm * BINOM_N + q];
        lo[tid] = o;
      }
      __syncthreads();
      for (int q = 0; q <= Hm; ++q) {
        const uint32_t nq = binom[Hm * BINOM_N + q], og = wofs[q], ol = lo[q];
        for (uint32_t r = (uint32_t)tid; r < nq; r += 1024u) lw[ol + r] = p.words[og + r];
      }
      __syncthreads();
      words = lw, wof = lo;
    }
  }
  unsigned long long* const flags = p.flags + base;
  uint32_t* const anyv = p.team_any + p.team_any_off[team];
  // LC_PIPE bit 8: tagged mirror words (two granules per word, TagTab): readers poll the data,
  // no token waits before a super-layer, no store drain after it (tokens remain for credits)
  const bool tagged = (p.pipe & 256) != 0;
  const bool glay = (p.pipe & PIPE_GLAY) != 0;
  const int mshift = HSOLO + (tagged ? 1 : 0);
  auto mirror = [&](int r, int t) {
    return p.mirror + (((size_t)(base + r) * MRING + (size_t)(t % MRING)) << mshift);
  };
  auto tag_of = [&](int t) { return p.mirror_tag + (uint32_t)t + 1u; };
  const int ns = p.nsteps[h];
  // LC_DEBUG phase cycles: pred/X waits, segments, publish + token, credit waits, -, super-layers
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};
  auto now = []() { return __builtin_amdgcn_s_memrealtime(); };
  const bool timed = p.tstamps != nullptr;
  if (p.stamps && rank == 0 && tid == 0) p.stamps[4 * h] = now();
  if (rank == 0 && tid == 0) B2[0] = 1;  // (cas-register) starts at nil: state id 0 (step 0 reads tab(-1))
  StreamWin sw;
  int64_t pos = p.sbeg[h];
  if (ns > 0 && decoder) {
    pipe_decode(p, sw, pos, lane, &ring[0], nullptr, lmask);
    if (tid == 0) ring[0].start = 0, ring[0].pstart = 0;
  }
  __syncthreads();
  int t_dec = ns > 0 ? 1 : 0, t_run = t_dec, t_ret = 0, last_start = 0;
  // credit pre-poll: the decoder lanes load every tile's token one super-layer before a credit
  // check (lane = tile, 64 tiles per register), so the check's first poll costs no HBM round
  // trip when nobody lags (tokens only grow: an early value that suffices stays valid)
  unsigned long long cpre[4] = {0, 0, 0, 0};
  // the credit window (super-layers a tile may run ahead of the slowest): 8, or 16 with
  // PIPE_CW16 (a mirror slot is a step's, reused 64 steps later: >= 64 super-layers, more than
  // the window's lag of 2 x 16 plus a step's span of at most H + T + 1 <= 25)
  const int cw = (p.pipe & PIPE_CW16) ? 16 : 8;
  static_assert((1 << DENSE_TEAM_MAXB) <= 4 * 64, "credit pre-poll registers");
  for (int s = 0; t_ret < ns; ++s) {
    unsigned long long tp = timed ? now() : 0;
    if (s >= cw && (s & (cw - 1)) == 0) {  // credit: nobody more than cw super-layers behind
      if (decoder) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        long spins = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // one lane per tile, 64 tiles at a time
          const int r = 64 * k + lane;
          if (64 * k >= G) break;
          const bool pre_ok = r >= G || cpre[k] >= (unsigned long long)(s - cw);
          while (!__all(pre_ok || poll_until(p, &flags[r < G ? r : 0], (unsigned long long)(s - cw), t0, spins)))
            ;
        }
        if (lane == 0) *sAbort = ld_agent(p.abort);
      }
      __syncthreads();
      if (*sAbort) break;
      if (timed) ph[3] += now() - tp, tp = now();
    }
    if (decoder && (p.pipe & PIPE_CPRE) && s >= cw - 1 && (s & (cw - 1)) == cw - 1) {  // the next check's tokens, loaded now
#pragma unroll
      for (int k = 0; k < 4; ++k)
        cpre[k] = 64 * k + lane < G ? ld_agent(&flags[64 * k + lane]) : 0ull;
    }
    // ---- ring view: lane i = step t_ret + i
    const int tl = t_ret + lane;
    const bool dec_l = lane < RING && tl < t_dec;
    uint4 h0 = {0u, 0u, 0u, 0u};
    int4 h1 = {0, 0, 0, 1 << 30}, h2 = {0, 0, 0, 0};
    if (dec_l) {
      const PipeStep* st = &ring[tl % RING];
      h0 = *reinterpret_cast<const uint4*>(&st->live);  // live, fresh, foldm, anyx
      h1 = *reinterpret_cast<const int4*>(&st->j);      // j, jp, H, start
      h2 = *reinterpret_cast<const int4*>(&st->pstart); // pstart, hp
    }
    const bool run_l = dec_l && tl < t_run;
    const uint32_t lteam_l = h0.x >> lb;
    // PIPE_GLAY: a wide step's tile r runs local layer q at super-layer start + q + |r|, so it
    // spans H + T + 1 super-layers (T = its live team bits)
    const int tb_l = glay ? __popc(lteam_l) : 0;
    const bool fin_l = run_l && h1.w + h1.z + tb_l < s;
    const uint64_t fin = __ballot(fin_l);
    const int lead = (int)__builtin_ctzll(~fin);
    // retired steps: this tile read a nonzero frontier in step tl => step tl - 1 survived here
    if (decoder && lane < lead && tl > 0 && h0.w)
      __hip_atomic_fetch_or(&anyv[tl >> 5], 1u << (tl & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int t_ret_old = t_ret;
    t_ret += lead;
    if (t_ret >= ns) break;
    // ---- segments of this tile: running steps whose team slots cover the tile
    const int dr_l = glay ? __popc((uint32_t)rank & lteam_l) : 0;  // the tile's layer delay
    const int q_l = s - h1.w - dr_l;
    const bool seg_l = run_l && (rank & ~lteam_l) == 0 && q_l >= 0 && q_l <= h1.z;
    uint32_t nq_l = 0, o_l = 0, mo_l = 0, mp_l = 0;
    uint32_t pm_l = 0;  // team bits b: pull from tile rank ^ b at this super-layer
    int xs_l = -1;      // tile holding this step's X (previous step returned a team slot)
    if (seg_l) {
      nq_l = binom[h1.z * BINOM_N + q_l], o_l = wof[q_l], mo_l = cum[h1.z * BINOM_N + q_l];
      mp_l = cum[h2.y * BINOM_N + min(q_l, h2.y)];
      const int jt = h1.x >= lb ? h1.x - lb : -1;
      const bool tile_j = jt >= 0 && ((rank >> jt) & 1);
      pm_l = lteam_l == 0 ? 0u : tile_j ? (1u << jt) : ((uint32_t)rank & lteam_l);
      if (h1.y >= lb && !((uint32_t)rank & (h0.y >> lb))) xs_l = rank | (1 << (h1.y - lb));
    }
    if (!tagged && __any(pm_l != 0 || xs_l >= 0)) {  // wait for the tiles this super-layer reads
      if (decoder) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        long spins = 0;
        for (;;) {
          bool ok = true;
          for (uint32_t m = pm_l; m && ok; m &= m - 1)
            ok = poll_until(p, &flags[rank ^ (1 << __builtin_ctz(m))], (unsigned long long)(glay ? s : s + 1), t0,
                            spins);
          // (PIPE_GLAY: tile xs = r | jp ran the previous step's layer q at pstart + q + |r| + 1)
          if (ok && xs_l >= 0)
            ok = poll_until(p, &flags[xs_l], (unsigned long long)(h2.x + q_l + (glay ? dr_l + 2 : 1)), t0, spins);
          if (__all(ok)) break;
        }
      }
      __syncthreads();
      if (timed) ph[0] += now() - tp, tp = now();
    }
    uint64_t segm = __ballot(seg_l);
    const bool wide_any = __ballot(seg_l && lteam_l != 0) != 0;
    constexpr int TW = 2, TB = DENSE_TEAM_MAXB_SERIAL;
    if (!(p.pipe & PIPE_SERIAL_SEGS)) {
      constexpr int TB = DENSE_TEAM_MAXB;
      // packed (as in history_pipe): one flat index over every running segment's words, each
      // segment padded to whole waves, so every wave works on one step with wave-uniform
      // parameters (readlanes of the ring view and of this tile's per-segment values)
      uint32_t total = 0;
      for (uint64_t m = segm; m; m &= m - 1) total += (rdl(nq_l, (int)__builtin_ctzll(m)) + 63u) & ~63u;
      for (uint32_t f0 = (uint32_t)(tid & ~63); f0 < total; f0 += 1024u) {
        int i = 0;
        uint32_t e = 0, acc = 0;
        for (uint64_t m = segm; m; m &= m - 1) {
          const int k = (int)__builtin_ctzll(m);
          if (f0 >= acc) i = k, e = acc;
          acc += (rdl(nq_l, k) + 63u) & ~63u;
        }
        const uint32_t nq = rdl(nq_l, i), r = f0 - e + (uint32_t)lane;
        const uint32_t mo = rdl(mo_l, i), mp = rdl(mp_l, i), pmask = rdl(pm_l, i), o = rdl(o_l, i);
        const uint32_t live = rdl(h0.x, i), fresh = rdl(h0.y, i), foldm = rdl(h0.z, i);
        const int j = rdl(h1.x, i), jp = rdl(h1.y, i), H = rdl(h1.z, i), xs = rdl(xs_l, i);
        const int t = t_ret_old + i;
        if (r >= nq) continue;
        const uint32_t w = words[o + r];
        const uint32_t live_loc = live & lmask, lteam = live >> lb;
        if (w & ~(live_loc >> 3)) continue;
        const bool wide = lteam != 0;
        const int jt = j >= lb ? j - lb : -1;
        const bool tile_j = jt >= 0 && ((rank >> jt) & 1);
        const bool jloc_hi = j >= 3 && j < lb;
        const bool tile_fresh = ((uint32_t)rank & (fresh >> lb)) != 0;  // the tile's masks start empty
        uint64_t keep_lo = ~0ull;
#pragma unroll
        for (int k = 0; k < 3; ++k)
          if (fresh & (1u << k)) keep_lo &= keep64(k);
        const uint32_t fresh_hi = (fresh & lmask) >> 3;
        PipeStep* st = &ring[t % RING];
        const OpSel* ops = st->ops + OP_PAD;
        uint64_t* const Bt = tab(t);
        if (!wide && xs < 0) {  // a step on this tile alone (then tile 0, jp local): LDS only
          const uint64_t X = pipe_x(tab(t - 1), w, fresh_hi, jp, keep_lo);
          uint64_t R = pull_set(Bt, w, j, ops, foldm);
          R = close_in_word(X, w, live_loc, j, ops, foldm, R);
          Bt[w] = X | R;
          expl += (uint32_t)__popcll(R);
          if (t > 0) st_fout += (uint32_t)__popcll(X);
          if (X) st->anyx = 1;
          continue;
        }
        const bool fx = !tile_fresh && !(w & fresh_hi);
        // HBM loads first (X from tile xs, one pull per predecessor tile), used after
        uint64_t xv = 0, pv[TB];
        // pulls from the tiles one team bit below: none for masks holding a local j (never
        // expanded); a tile holding j takes only T_j of r \ j
        const bool pl = tile_j || !(jloc_hi && ((w >> (j - 3)) & 1u));
        if (tagged) {
          if (fx && xs >= 0) xv = TagTab::ld(mirror(xs, t - 1), mp + r, tag_of(t - 1), p.abort);
#pragma unroll
          for (int b = 0; b < TB; ++b)
            pv[b] = (pl && ((pmask >> b) & 1u)) ? TagTab::ld(mirror(rank ^ (1 << b), t), mo + r, tag_of(t), p.abort)
                                                 : 0ull;
        } else {
          if (fx && xs >= 0) xv = HbmTab::ld(mirror(xs, t - 1) + mp + r);
#pragma unroll
          for (int b = 0; b < TB; ++b)
            pv[b] = (pl && ((pmask >> b) & 1u)) ? HbmTab::ld(mirror(rank ^ (1 << b), t) + mo + r) : 0ull;
        }
        uint64_t X = xs >= 0 ? (xv & keep_lo) : (fx && jp < lb) ? pipe_x(tab(t - 1), w, 0u, jp, keep_lo) : 0ull;
        uint64_t R = tile_j ? 0ull : pull_set(Bt, w, j, ops, foldm);
#pragma unroll
        for (int b = 0; b < TB; ++b)
          if ((pmask >> b) & 1u) R |= transfer(ops[lb + b], (foldm >> (lb + b)) & 1u, pv[b]);
        if (!tile_j) R = close_in_word(X, w, live_loc, j, ops, foldm, R);
        const uint64_t nv = X | R;
        Bt[w] = nv;
        if (wide) {
          if (tagged) TagTab::st(mirror(rank, t), mo + r, nv, tag_of(t));
          else HbmTab::st(mirror(rank, t) + mo + r, nv);
        }
        expl += (uint32_t)__popcll(R);
        if (t > 0) st_fout += (uint32_t)__popcll(X);
        if (X) st->anyx = 1;
      }
      segm = 0;
    }
    // serial segments (PIPE_SERIAL_SEGS): TW words per thread at a time, each chunk's word
    // indices loaded one chunk ahead (the next segment's first chunk while this segment runs)
    int i = segm ? (int)__builtin_ctzll(segm) : -1;
    uint32_t wn[TW];
#pragma unroll
    for (int k = 0; k < TW; ++k) {
      const uint32_t r = (uint32_t)tid + 1024u * k;
      wn[k] = (i >= 0 && r < rdl(nq_l, i)) ? words[rdl(o_l, i) + r] : ~0u;
    }
    while (i >= 0) {
      segm &= segm - 1;
      const int i2 = segm ? (int)__builtin_ctzll(segm) : -1;
      uint32_t wn2[TW];
#pragma unroll
      for (int k = 0; k < TW; ++k) {
        const uint32_t r = (uint32_t)tid + 1024u * k;
        wn2[k] = (i2 >= 0 && r < rdl(nq_l, i2)) ? words[rdl(o_l, i2) + r] : ~0u;
      }
      const uint32_t nq = rdl(nq_l, i), mo = rdl(mo_l, i), mp = rdl(mp_l, i), pmask = rdl(pm_l, i);
      const uint32_t o = rdl(o_l, i);
      const uint32_t live = rdl(h0.x, i), fresh = rdl(h0.y, i), foldm = rdl(h0.z, i);
      const int j = rdl(h1.x, i), jp = rdl(h1.y, i), H = rdl(h1.z, i), xs = rdl(xs_l, i);
      const int t = t_ret_old + i;
      const uint32_t live_loc = live & lmask, lteam = live >> lb;
      const bool wide = lteam != 0;
      const int jt = j >= lb ? j - lb : -1;
      const bool tile_j = jt >= 0 && ((rank >> jt) & 1);
      const bool jloc_hi = j >= 3 && j < lb;
      const bool tile_fresh = ((uint32_t)rank & (fresh >> lb)) != 0;  // the tile's masks start empty
      uint64_t keep_lo = ~0ull;
#pragma unroll
      for (int k = 0; k < 3; ++k)
        if (fresh & (1u << k)) keep_lo &= keep64(k);
      const uint32_t live_hi = live_loc >> 3, fresh_hi = (fresh & lmask) >> 3;
      PipeStep* st = &ring[t % RING];
      const OpSel* ops = st->ops + OP_PAD;
      uint64_t* const Bt = tab(t);
      const uint64_t* const Bp = tab(t - 1);
      const uint64_t* xsrc = xs >= 0 ? mirror(xs, t - 1) + mp : nullptr;
      uint64_t* mine = mirror(rank, t) + mo;
      uint64_t nzx = 0;
      if (!wide && !xsrc) {  // a step on this tile alone: the BLOCK loop (LDS only)
        for (uint32_t r0 = (uint32_t)tid; r0 < nq; r0 += 1024u * TW) {
#pragma unroll
          for (int k = 0; k < TW; ++k) {
            const uint32_t r = r0 + 1024u * k, rn = r + 1024u * TW;
            const uint32_t w = wn[k];
            wn[k] = rn < nq ? words[o + rn] : ~0u;
            if (r >= nq || (w & ~live_hi)) continue;
            const uint64_t X = tile_fresh ? 0ull : pipe_x(Bp, w, fresh_hi, jp, keep_lo);
            uint64_t R = pull_set(Bt, w, j, ops, foldm);
            R = close_in_word(X, w, live_loc, j, ops, foldm, R);
            Bt[w] = X | R;
            expl += (uint32_t)__popcll(R);
            if (t > 0) st_fout += (uint32_t)__popcll(X);
            nzx |= X;
          }
        }
      } else
      // every HBM load of a chunk (X from tile xs, one pull per predecessor tile) is issued
      // before any is used
      for (uint32_t r0 = (uint32_t)tid; r0 < nq; r0 += 1024u * TW) {
        uint32_t wl[TW];
        bool ok[TW];
        uint64_t xv[TW], pv[TW][TB];
#pragma unroll
        for (int k = 0; k < TW; ++k) {
          const uint32_t r = r0 + 1024u * k, rn = r + 1024u * TW;
          wl[k] = wn[k];
          wn[k] = rn < nq ? words[o + rn] : ~0u;
          ok[k] = r < nq && !(wl[k] & ~live_hi);
        }
#pragma unroll
        for (int k = 0; k < TW; ++k) {
          const uint32_t r = r0 + 1024u * k;
          const bool fx = ok[k] && !tile_fresh && !(wl[k] & fresh_hi);
          xv[k] = (fx && xsrc) ? HbmTab::ld(xsrc + r) : 0ull;
          // pulls from the tiles one team bit below: none for masks holding a local j (never
          // expanded); a tile holding j takes only T_j of r \ j
          const bool pl = ok[k] && (tile_j || !(jloc_hi && ((wl[k] >> (j - 3)) & 1u)));
#pragma unroll
          for (int b = 0; b < TB; ++b)
            pv[k][b] = (pl && ((pmask >> b) & 1u)) ? HbmTab::ld(mirror(rank ^ (1 << b), t) + mo + r) : 0ull;
        }
#pragma unroll
        for (int k = 0; k < TW; ++k) {
          if (!ok[k]) continue;
          const uint32_t w = wl[k], r = r0 + 1024u * k;
          uint64_t X = xv[k] & keep_lo;
          if (!xsrc && !tile_fresh && !(w & fresh_hi) && jp < lb) X = pipe_x(Bp, w, 0u, jp, keep_lo);
          uint64_t R = tile_j ? 0ull : pull_set(Bt, w, j, ops, foldm);
#pragma unroll
          for (int b = 0; b < TB; ++b)
            if ((pmask >> b) & 1u) R |= transfer(ops[lb + b], (foldm >> (lb + b)) & 1u, pv[k][b]);
          if (!tile_j) R = close_in_word(X, w, live_loc, j, ops, foldm, R);
          const uint64_t nv = X | R;
          Bt[w] = nv;
          if (wide) HbmTab::st(mine + r, nv);
          expl += (uint32_t)__popcll(R);
          if (t > 0) st_fout += (uint32_t)__popcll(X);
          nzx |= X;
        }
      }
      if (nzx) st->anyx = 1;
      i = i2;
#pragma unroll
      for (int k = 0; k < TW; ++k) wn[k] = wn2[k];
    }
    const int t_dec_old = t_dec;
    if (t_dec < ns && t_dec - t_ret_old < RING) {
      if (decoder) pipe_decode(p, sw, pos, lane, &ring[t_dec % RING], &ring[(t_dec - 1) % RING], lmask);
      ++t_dec;
    }
    if (t_run < t_dec_old) {
      const int lp = t_run - 1 - t_ret_old;
      const int gap = (dbl && lp >= 0 && rdl(h1.x, lp) < 3) ? 1 : 2;  // as in history_pipe
      // (r3n: a gap of 3 after team-slot returns, so that a tile's X is another tile's word of two
      // super-layers back, cost more super-layers than it saved: C2 30.1 -> 31.0 ms)
      const bool ok = lp < 0 || lp < lead || s + 1 - rdl(h1.w, lp) >= min(gap, rdl(h1.z, lp) + rdl(tb_l, lp) + 1);
      if (ok) {
        if (tid == 0) ring[t_run % RING].start = s + 1, ring[t_run % RING].pstart = last_start;
        last_start = s + 1;
        ++t_run;
      }
    }
    if (timed) ph[1] += now() - tp, tp = now();
    if (wide_any && !tagged) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
    __syncthreads();
    if (tid == 0) st_agent(&flags[rank], (unsigned long long)(s + 1));
    if (timed) ph[2] += now() - tp, ph[5] += 1;
  }
  if (timed && tid == 0)
    for (int k = 0; k < 6; ++k) p.tstamps[(base + rank) * 8 + k] = ph[k];
  // make sure the last token is out before the team barrier's readers look (the barrier orders it)
  if (ns > 0) {  // the last step's return, over this tile, once every tile has finished
    team_bar((TeamCtl*)p.ctl + team, G, p.abort, sAbort);
    const PipeStep* st = &ring[(ns - 1) % RING];
    const int jl = rfl(st->j), H = rfl(st->H);
    const uint32_t live = (uint32_t)rfl((int)st->live) & ~(1u << jl);
    const uint32_t live_hi = (live & lmask) >> 3;
    uint64_t nzx = 0;
    if (((uint32_t)rank & ~(live >> lb)) == 0) {
      const uint64_t* xsrc = jl >= lb ? mirror(rank | (1 << (jl - lb)), ns - 1) : nullptr;
      for (int q = 0; q <= H; ++q) {
        const uint32_t nq = binom[H * BINOM_N + q], o = wof[q], mo = cum[H * BINOM_N + q];
        for (uint32_t r = (uint32_t)tid; r < nq; r += 1024u) {
          const uint32_t w = words[o + r];
          if (w & ~live_hi) continue;
          const uint64_t X = !xsrc ? pipe_x(tab(ns - 1), w, 0u, jl, ~0ull)
                             : tagged ? TagTab::ld(xsrc, mo + r, tag_of(ns - 1), p.abort)
                                      : HbmTab::ld(xsrc + mo + r);
          st_fout += (uint32_t)__popcll(X);
          nzx |= X;
        }
      }
    }
    if (__syncthreads_or(nzx != 0) && tid == 0)
      __hip_atomic_fetch_or(&anyv[ns >> 5], 1u << (ns & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// WAVE histories inside a big workgroup (DenseParams.n_w > 0, host knob LC_WAVE_IN_BIG): each
// of its 16 waves is a WAVE team (history_pipe<64>, as in dense_wave_kernel) on its own 2 KiB
// slice of the workgroup's LDS table, dequeuing from the WAVE queue. Running them here instead
// of in dense_wave_kernel keeps that kernel's workgroups off the CUs: beside a big workgroup
// of the pipelined-team instantiation (121 VGPRs, 4 waves per SIMD) no other wave fits, so
// every CU a wave workgroup held was closed to the big kernel until the wave pool ended.
__device__ __forceinline__ void big_wave_mode(const DenseParams& p, uint64_t* sTab, const uint64_t* zero,
                                              const uint32_t* binom, int tid, unsigned long long& st_fout,
                                              unsigned long long& st_steps) {
  // each wave's slice holds two tables of TABW words (PIPE_DBL)
  constexpr int NWV = 16, HW = DENSE_WAVE_LMAX - 3, TABW = 1 << HW, SLW = 2 * TABW;
  uint64_t* const tabs = sTab;                                         // NWV slices of SLW words
  PipeStep* const rings = reinterpret_cast<PipeStep*>(sTab + NWV * SLW);  // NWV rings
  uint32_t* const words = reinterpret_cast<uint32_t*>(rings + NWV * WAVE_RING);  // HW-bit word list
  uint32_t* const wofs = words + TABW;                                 // its layer offsets
  int* const sQw = reinterpret_cast<int*>(wofs + 16);
  unsigned long long* const sEx = reinterpret_cast<unsigned long long*>(sQw + NWV);
  static_assert((NWV * SLW) * 8 + NWV * WAVE_RING * sizeof(PipeStep) + TABW * 4 + 16 * 4 + NWV * 4 + NWV * 8 <=
                (1 << (DENSE_LMAX - 3)) * 8, "wave mode fits the big table");
  __syncthreads();  // the table's previous users are done
  if (tid <= HW + 1) {
    uint32_t o = 0;
    for (int q = 0; q < tid; ++q) o += binom[HW * BINOM_N + q];
    wofs[tid] = o;
  }
  __syncthreads();
  for (int v = tid; v < TABW; v += 1024) {  // colex rank within its popcount layer
    uint32_t rank = 0;
    int i = 0;
    for (uint32_t x = (uint32_t)v; x; x &= x - 1, ++i) rank += binom[__builtin_ctz(x) * BINOM_N + i + 1];
    words[wofs[__popc(v)] + rank] = (uint32_t)v;
  }
  __syncthreads();
  DenseParams q = p;
  q.n = p.n_w, q.order = p.order_w, q.queue = p.queue_w;
  const int w = tid / 64;
  // LC_PIPE bit 18 (PIPE_WSPREAD, a plan of few WAVE histories): one wave per workgroup dequeues,
  // so each history's wave has a CU to itself (a REG history's step is VALU/shuffle work that
  // 16 waves on one CU would share)
  if (!(p.pipe & PIPE_WSPREAD) || w == 0)
  history_pipe<64, DENSE_WAVE_LMAX, WAVE_RING, false, SLW>(q, tabs + w * SLW, zero, rings + w * WAVE_RING, &sQw[w],
                                                          &sEx[w], words, wofs, binom, tid & 63, st_fout, st_steps);
  __syncthreads();
}

// MID histories (widths 12..DENSE_MID_LMAX) inside a big workgroup (LC_PIPE bit 7): its 16
// waves are 4 MID teams of 4 waves (history_pipe<256, SUB>), each on a 16 KiB quarter of the
// LDS table with a ring of its own and its own LDS barrier, dequeuing from the MID queue. A
// BLOCK team's narrow steps keep only a few of its 16 waves busy (a width-12 super-layer is
// ~256 words), so four histories share the CU instead of one.
constexpr int QUAD_RING = 8;
__device__ __forceinline__ void big_mid_mode(const DenseParams& p, uint64_t* sTab, const uint64_t* zero,
                                             const uint32_t* binom, int tid, unsigned long long& st_fout,
                                             unsigned long long& st_steps) {
  constexpr int NQ = 4, HQ = DENSE_MID_LMAX - 3, TABQ = 1 << HQ;
  uint64_t* const tabs = sTab;                                             // NQ tables of TABQ words
  PipeStep* const rings = reinterpret_cast<PipeStep*>(sTab + NQ * TABQ);  // NQ rings
  unsigned long long* const sEx = reinterpret_cast<unsigned long long*>(rings + NQ * QUAD_RING);
  uint32_t* const words = reinterpret_cast<uint32_t*>(sEx + NQ);          // HQ-bit word list
  uint32_t* const wofs = words + TABQ;                                     // its layer offsets
  int* const sQq = reinterpret_cast<int*>(wofs + 16);
  unsigned* const qbar = reinterpret_cast<unsigned*>(sQq + NQ);           // per team: count, gen, any
  static_assert((NQ * TABQ) * 8 + NQ * QUAD_RING * sizeof(PipeStep) + NQ * 8 + TABQ * 4 + 16 * 4 + NQ * 4 +
                        NQ * 4 * 4 <= (1 << (DENSE_LMAX - 3)) * 8,
                "MID mode fits the big table");
  __syncthreads();  // the table's previous users are done
  if (tid <= HQ + 1) {
    uint32_t o = 0;
    for (int q = 0; q < tid; ++q) o += binom[HQ * BINOM_N + q];
    wofs[tid] = o;
  }
  if (tid < NQ * 4) qbar[tid] = 0;
  __syncthreads();
  for (int v = tid; v < TABQ; v += 1024) {  // colex rank within its popcount layer
    uint32_t rank = 0;
    int i = 0;
    for (uint32_t x = (uint32_t)v; x; x &= x - 1, ++i) rank += binom[__builtin_ctz(x) * BINOM_N + i + 1];
    words[wofs[__popc(v)] + rank] = (uint32_t)v;
  }
  __syncthreads();
  DenseParams q = p;
  q.n = p.n2, q.order = p.order2, q.queue = p.queue2;
  const int team = tid / 256;
  history_pipe<256, DENSE_MID_LMAX, QUAD_RING, true>(q, tabs + team * TABQ, zero, rings + team * QUAD_RING,
                                                     &sQq[team], &sEx[team], words, wofs, binom, tid & 255,
                                                     st_fout, st_steps, qbar + team * 4);
  __syncthreads();
}

// BLOCK histories and TILE teams in one launch (same 1024-thread, 128 KiB-LDS workgroups, so
// every workgroup is resident: the grid never exceeds one workgroup per CU).
//
// A TILE team checks one history of width 17 + t with G = 2^t workgroups. Workgroup r holds
// tile r: the masks whose slots 17..17+t-1 spell r, over the low 17 slots, in its LDS. The
// leader (r = 0) runs every step of width <= 17 alone (the other tiles are empty then);
// wider steps run on every tile. Tile r's word w pulls from its own words (local bits) and
// from word w of tiles r \ b (bits b of r), which are final once tile r \ b finished the
// same local layer: each tile publishes every finished word to its HBM mirror (sc1 stores,
// in word-list order, so a wave's stores and a successor's loads are contiguous) and then
// its layer token (flags[r] = step << 5 | layer + 1), and successors poll the
// tokens of their predecessors — point-to-point, one hop per team bit, instead of a team
// barrier per layer. Returning a team slot j: tiles without j take tile r | j's mirror.
template <bool TEAM_PIPE>
__global__ void __launch_bounds__(1024) dense_big_kernel(DenseParams p) {
  constexpr int HSOLO = DENSE_LMAX - 3;
  __shared__ uint64_t sTab[1 << HSOLO];
  __shared__ uint32_t sWOff[DENSE_WORD_BITS + 2];
  __shared__ uint32_t sBinom[BINOM_N * BINOM_N];
  __shared__ __attribute__((aligned(16))) OpSel sOpT[OP_TAB];
  OpSel* const sOp = sOpT + OP_PAD;
  __shared__ int sQ, sCmd, sAbort;
  __shared__ long long sPos;
  __shared__ unsigned sAny;
  __shared__ unsigned long long sRed;
  __shared__ uint64_t sZero;
  __shared__ PipeStep sRing[TEAM_RING > BLOCK_RING ? TEAM_RING : BLOCK_RING];
  __shared__ uint32_t sCum[BINOM_N * BINOM_N];  // sCum[n][k] = sum of C(n, q) for q < k

  const int tid = threadIdx.x, lane = tid & 63;
  // LC_DEBUG: the workgroup's shader-clock and 100-MHz-clock spans (their ratio: the core clock
  // the chains ran at), summed over workgroups
  const unsigned long long clk0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
  auto note_clock = [&]() {
    if (p.lhist && tid == 0) {
      atomicAdd(&p.lhist[64 * LH_N + 30], __builtin_amdgcn_s_memtime() - clk0);
      atomicAdd(&p.lhist[64 * LH_N + 31], __builtin_amdgcn_s_memrealtime() - rt0);
    }
  };
  init_tables(sBinom, sWOff, DENSE_WORD_BITS, 1024);
  for (int i = tid; i < BINOM_N * BINOM_N; i += 1024) {
    uint32_t c = 0;
    for (int q = 0; q < i % BINOM_N; ++q) c += sBinom[(i / BINOM_N) * BINOM_N + q];
    sCum[i] = c;
  }
  if (tid == 0) sAbort = 0, sZero = 0;
  if (tid < OP_TAB) sOpT[tid] = OpSel{SEL_NONE, SEL_NONE};  // (see dense_wave_kernel)
  __syncthreads();
  unsigned long long st_fout = 0, st_steps = 0;

  // LC_PIPE bit 14 (PIPE_XCD): workgroup roles by an XCD-compact index. Blocks are dealt
  // round-robin over the 8 XCDs (MI355X_MICROARCH "Workgroup dispatch": b and b + 8 share one), so
  // index (b % 8) * (grid / 8) + b / 8 puts consecutive team workgroups on one XCD: a team of <= 32
  // tiles hands its mirror words off inside one XCD (handoff-1to1: cross-XCD +0.1-0.3 us). Speed
  // only: the hand-off protocol (sc1 granules, tags) is the same under any placement.
  const int bid = ((p.pipe & PIPE_XCD) && (gridDim.x & 7u) == 0)
                      ? (int)((blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3))
                      : (int)blockIdx.x;
  if (bid >= p.n_team_wgs) {  // ------------------------------------------------ BLOCK histories
    // the last ceil(n_w / 16) workgroups start on the WAVE queue: a WAVE history is a long
    // latency-bound chain, and started after the BLOCK queue it would be the launch's tail
    const int wave_first = p.n_w > 0 ? ((p.pipe & PIPE_WSPREAD) ? min(p.n_w, (int)gridDim.x - p.n_team_wgs) : (p.n_w + 15) / 16) : 0;
    if (wave_first && bid >= (int)gridDim.x - wave_first)
      big_wave_mode(p, sTab, &sZero, sBinom, tid, st_fout, st_steps);
    // and the next mid_first start on the MID queue (long chains too, four per workgroup)
    else if (p.n2 > 0 && (p.pipe & 128) && bid >= (int)gridDim.x - wave_first - p.mid_first)
      big_mid_mode(p, sTab, &sZero, sBinom, tid, st_fout, st_steps);
    if (p.pipe & 1) {
      history_pipe<1024, DENSE_LMAX, BLOCK_RING>(p, sTab, &sZero, sRing, &sQ, &sRed, p.words, sWOff, sBinom, tid,
                                                 st_fout, st_steps);
      if (p.n2 > 0 && (p.pipe & 128)) {  // then the MID queue, four histories per workgroup
        big_mid_mode(p, sTab, &sZero, sBinom, tid, st_fout, st_steps);
      } else {
        DenseParams q2 = p;  // then help with the MID queue
        q2.n = p.n2, q2.order = p.order2, q2.queue = p.queue2;
        history_pipe<1024, DENSE_LMAX, BLOCK_RING>(q2, sTab, &sZero, sRing, &sQ, &sRed, p.words, sWOff, sBinom,
                                                   tid, st_fout, st_steps);
      }
    } else
      history_loop<1024, DENSE_LMAX>(p, sTab, &sZero, sOp, &sQ, &sRed, p.words, sWOff, sBinom, tid, st_fout,
                                     st_steps);
    if (p.n_w > 0) big_wave_mode(p, sTab, &sZero, sBinom, tid, st_fout, st_steps);  // then the WAVE queue
    note_clock();
    flush_stats(p, st_fout, st_steps, tid == 0);
    return;
  }

  // ------------------------------------------------------------------------- TILE team
  const int team = p.wg_team[bid];
  const int base = p.team_base[team];
  const int rank = bid - base;
  const int G = 1 << p.team_bits[team];
  const int h = p.team_hist[team];
  TeamCtl* const ctl = (TeamCtl*)p.ctl + team;
  unsigned long long* const flags = p.flags + base;
  const int lb = p.team_lbits[team];  // local slots of every tile (<= DENSE_LMAX)
  int mpar = 0;  // mirror buffer of the current team step (LC_PIPE bit 3: team-step parity)
  auto mirror = [&](int r) { return p.mirror + ((size_t)(2 * (base + r) + mpar) << HSOLO); };
  auto bar = [&]() { return team_bar(ctl, G, p.abort, &sAbort); };
  const bool nobar = (p.pipe & 8) != 0;
  unsigned long long expl = 0, stepctr = 0;
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};  // LC_DEBUG phase cycles (wait, compute, publish, return, barrier, steps)
  auto now = []() { return __builtin_amdgcn_s_memrealtime(); };

  for (int i = tid; i < (1 << HSOLO); i += 1024) sTab[i] = 0;
  __syncthreads();
  if (rank == 0 && tid == 0) sTab[0] = 1;  // (cas-register) starts at nil: state id 0

  if constexpr (TEAM_PIPE) {  // pipelined tile team (LC_PIPE bit 2; its own instantiation: it
    // needs far more scalar registers than the rest, which must leave room beside the
    // wave / MID workgroups)
    team_pipe(p, sTab, &sZero, sRing, sCum, sBinom, sWOff, team, base, rank, G, h, lb, &sAbort, expl, st_fout);
    bar();  // every tile's survivor bits are in
    if (rank == 0 && tid == 0) {
      const int ns = p.nsteps[h];
      const uint32_t* anyv = p.team_any + p.team_any_off[team];
      int fail_t = -1;
      for (int t = 1; t <= ns && fail_t < 0; ++t)
        if (!((ld_agent(&anyv[t >> 5]) >> (t & 31)) & 1u)) fail_t = t - 1;
      p.fail_step[h] = fail_t;
      p.status[h] = fail_t >= 0 ? ST_INVALID : ST_VALID;
      st_steps += fail_t >= 0 ? fail_t + 1 : ns;
      if (p.stamps) p.stamps[4 * h + 1] = __builtin_amdgcn_s_memrealtime();
    }
    const unsigned long long e = block_sum(expl, &sRed);
    if (tid == 0 && e) atomicAdd(&p.explored[h], e);
    // the team is done (every tile passed its final barrier; other tiles read only this tile's
    // HBM mirror): join the BLOCK queue, then the WAVE queue
    __syncthreads();
    history_pipe<1024, DENSE_LMAX, BLOCK_RING>(p, sTab, &sZero, sRing, &sQ, &sRed, p.words, sWOff, sBinom, tid,
                                               st_fout, st_steps);
    if (p.n2 > 0 && (p.pipe & 128)) big_mid_mode(p, sTab, &sZero, sBinom, tid, st_fout, st_steps);
    if (p.n_w > 0) big_wave_mode(p, sTab, &sZero, sBinom, tid, st_fout, st_steps);
    note_clock();
    flush_stats(p, st_fout, st_steps, tid == 0);
    return;
  }

  // one step of width > 17 on every tile (the ops are in sOp); returns "survived"
  auto team_step = [&](long long hpos) -> bool {
    ++stepctr;
    const unsigned long long tok0 = stepctr << 5;
    if (nobar) {
      // double-buffered mirrors: the buffer of step stepctr - 2 is rewritten only after every
      // tile finished that step (its pulls and return copies read it)
      mpar = (int)(stepctr & 1);
      if (stepctr > 2 && tid < 64) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        long spins = 0;
        for (int r0 = 0; r0 < G; r0 += 64)
          while (!__all(r0 + lane >= G ||
                        poll_until(p, &p.done[base + (r0 + lane < G ? r0 + lane : 0)], stepctr - 2, t0, spins)))
            ;
      }
      __syncthreads();
    }
    uint64_t* const mine = mirror(rank);
    const uint32_t H0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.stream[hpos]);
    const uint32_t live = H0 & DENSE_LIVE_MASK;
    const int j = (int)((H0 >> DENSE_J_SHIFT) & 31u);
    const uint32_t foldm = fold_mask(sOp);
    const uint32_t live_loc = live & ((1u << lb) - 1), live_team = live >> lb;
    const bool active = ((uint32_t)rank & ~live_team) == 0;
    const int jt = j >= lb ? j - lb : -1;
    const bool tile_j = jt >= 0 && ((rank >> jt) & 1);
    const int Lloc = live_loc ? 32 - __clz((int)live_loc) : 0;
    const int H = Lloc > 3 ? Lloc - 3 : 0;
    const uint32_t live_hi = live_loc >> 3;
    // tiles this one pulls from: r \ b for its team bits (only r \ j when r holds j)
    const uint32_t preds = tile_j ? (1u << jt) : ((uint32_t)rank & live_team);
    const bool jloc_hi = j >= 3 && j < lb;
    uint64_t anyv = 0;
    ph[5] += 1;
    if (active) {
      // mirror position of layer q's first word: words below 2^H in (popcount, value) order,
      // so positions stay below 2^H <= 2^(lb-3) <= 2^(DENSE_LMAX-3), the mirror's size
      uint32_t mo = 0;
      for (int q = 0; q <= H; ++q) {
        unsigned long long tp = now();
        const uint32_t nq = __builtin_amdgcn_readfirstlane(sBinom[H * BINOM_N + q]);
        const uint32_t o = __builtin_amdgcn_readfirstlane(sWOff[q]);
        // this thread's words of the layer (at most TW: C(14, 7) = 3432 <= TW * 1024). Their
        // cross-tile pulls go out together per predecessor tile: one HBM round trip per
        // predecessor and layer, not one per word.
        constexpr int TW = 4;
        static_assert(TW * 1024 >= 3432, "a layer of a 17-bit tile fits TW words per thread");
        uint32_t wl[TW];
        uint64_t R0[TW];
        // a layer of at most 512 (256) words: word rr belongs to a group of 2 (4) lanes that
        // split its local pull batches (as in run_layers); the group's first lane goes on
        const int split = H <= 4 ? 1 : (int)nq * 4 <= 1024 ? 4 : (int)nq * 2 <= 1024 ? 2 : 1;
        const int sub = tid & (split - 1);
        const uint32_t rr = (uint32_t)tid / (uint32_t)split;
#pragma unroll
        for (int k = 0; k < TW; ++k) {
          const uint32_t r = rr + (uint32_t)k * 1024u;
          wl[k] = r < nq ? p.words[o + r] : ~0u;  // ~0u: no word (fails the live test)
          R0[k] = 0;
        }
        // the hi-bit pulls read only this tile's finished layers: done before waiting for the
        // predecessors' layer q (a tile holding j pulls nothing locally)
        if (split > 1) {
          uint64_t R = (!tile_j && !(wl[0] & ~live_hi))
                           ? pull_hi_part(sTab, &sZero, wl[0], j, H, sOp, foldm, 4 * sub, 4 * split)
                           : 0ull;
          R |= (uint64_t)__shfl_xor((unsigned long long)R, 1, 64);
          if (split == 4) R |= (uint64_t)__shfl_xor((unsigned long long)R, 2, 64);
          R0[0] = R;
          if (sub) wl[0] = ~0u;
        } else {
#pragma unroll
          for (int k = 0; k < TW; ++k)
            if (!tile_j && !(wl[k] & ~live_hi)) R0[k] = pull_hi<4>(sTab, &sZero, wl[k], j, H, sOp, foldm);
        }
        {
          const unsigned long long tw = now();
          wait_flags(p, flags, rank, preds, tok0 + q + 1, &sAbort);
          ph[0] += now() - tw;
          tp += now() - tw;  // (compute excludes the wait)
        }
        for (uint32_t m = preds; m; m &= m - 1) {
          const int b = __builtin_ctz(m);
          const OpSel sb = sOp[lb + b];
          const bool fb = (foldm >> (lb + b)) & 1u;
          const uint64_t* src = mirror(rank ^ (1 << b)) + mo + rr;
          uint64_t v[TW];
#pragma unroll
          for (int k = 0; k < TW; ++k) {
            const uint32_t w = wl[k];
            // pulls from the tiles one team bit below: none for masks holding a local j
            // (configs holding j are never expanded); a tile holding j takes only T_j of r \ j
            const bool pull = !(w & ~live_hi) && (tile_j || !(jloc_hi && ((w >> (j - 3)) & 1u)));
            v[k] = pull ? HbmTab::ld(src + k * 1024) : 0ull;
          }
#pragma unroll
          for (int k = 0; k < TW; ++k) R0[k] |= transfer(sb, fb, v[k]);
        }
#pragma unroll
        for (int k = 0; k < TW; ++k) {
          const uint32_t w = wl[k];
          if (w & ~live_hi) continue;
          uint64_t nv;
          if (tile_j) {  // every mask here holds j: linearized last, from tile r \ j
            const uint64_t X = sTab[w];
            nv = X | R0[k];
            if (R0[k]) sTab[w] = nv;
            expl += (uint32_t)__popcll(R0[k]);
          } else {
            expl += finish_word(sTab, w, live_loc, j, sOp, foldm, R0[k], &nv);
          }
          HbmTab::st(mine + mo + rr + k * 1024, nv);  // mirrors are in word-list order
        }
        mo += nq;
        __syncthreads();
        ph[1] += now() - tp;
        tp = now();
        // layer q published: every wave drains its sc1 stores, then one lane signals
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) st_agent(&flags[rank], tok0 + q + 1);
        ph[2] += now() - tp;
      }
      const unsigned long long tr = now();
      // return j
      if (jt < 0) {
        anyv = return_slot(sTab, live_loc, j, tid, 1024, st_fout);
      } else if (tile_j) {  // this tile's masks all hold j: they move to tile r \ j
        for (int w = tid; w < (1 << H); w += 1024) sTab[w] = 0;
      } else {  // take tile r | j (final once its last layer is published)
        wait_flags(p, flags, rank, 1u << jt, tok0 + H + 1, &sAbort);
        const uint64_t* src = mirror(rank | (1 << jt));
        // the words below 2^H are the first C(H, q) entries of every layer of the list
        uint32_t mo = 0;
        for (int q = 0; q <= H; ++q) {
          const uint32_t nq = sBinom[H * BINOM_N + q], o = sWOff[q];
          for (uint32_t r = (uint32_t)tid; r < nq; r += 1024) {
            const uint32_t w = p.words[o + r];
            const uint64_t v = (w & ~live_hi) ? 0ull : HbmTab::ld(src + mo + r);
            sTab[w] = v;
            anyv |= v;
            st_fout += __popcll(v);
          }
          mo += nq;
        }
      }
      ph[3] += now() - tr;
    }
    const unsigned long long tb = now();
    if (nobar) {  // this tile's survivors only; the verdict is decided after the last step
      const bool mine_any = __syncthreads_or(anyv != 0);
      if (tid == 0) st_agent(&p.done[base + rank], stepctr);
      ph[4] += now() - tb;
      return mine_any;
    }
    if (__syncthreads_or(anyv != 0) && tid == 0)
      __hip_atomic_fetch_or(&ctl->any, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bar();  // every tile done with this step (mirrors may be rewritten after this)
    if (tid == 0) sAny = ld_agent(&ctl->any);
    __syncthreads();
    ph[4] += now() - tb;
    return sAny != 0;
  };

  if (nobar) {  // every tile walks the stream; no team barrier per step
    const int ns = p.nsteps[h];
    uint32_t* const anyb = p.team_any + p.team_any_off[team];
    if (p.stamps && rank == 0 && tid == 0) p.stamps[4 * h] = __builtin_amdgcn_s_memrealtime();
    StreamWin sw;
    long long pos = p.sbeg[h];
    unsigned long long team_cycles = 0, team_steps = 0;
    for (int t = 0; t < ns; ++t) {
      sw.need(p, pos, lane);
      int ninv;
      const uint32_t H0 = read_step(sw, pos, lane, tid < 64, sOp, &ninv);
      const long long hpos = pos;
      pos += 1 + ninv;
      __syncthreads();
      const uint32_t live = H0 & DENSE_LIVE_MASK;
      const int j = (int)((H0 >> DENSE_J_SHIFT) & 31u);
      bool surv = false;
      if ((live >> lb) == 0) {  // narrow step: the leader alone (other tiles empty)
        if (rank == 0) {
          const uint32_t foldm = fold_mask(sOp);
          expl += run_layers<HSOLO, 4>(sTab, &sZero, p.words, sWOff, sBinom, live, j, sOp, foldm, tid, 1024,
                                       [] { __syncthreads(); });
          surv = __syncthreads_or(return_slot(sTab, live, j, tid, 1024, st_fout) != 0);
        }
      } else {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        surv = team_step(hpos);
        team_cycles += __builtin_amdgcn_s_memrealtime() - t0;
        ++team_steps;
      }
      if (surv && tid == 0)
        __hip_atomic_fetch_or(&anyb[t >> 5], 1u << (t & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();  // the next header rewrites sOp
    }
    bar();  // every tile's survivor bits are in
    if (rank == 0 && tid == 0) {
      int fail_t = -1;  // the first step after which no tile holds a config
      for (int t = 0; t < ns && fail_t < 0; ++t)
        if (!((ld_agent(&anyb[t >> 5]) >> (t & 31)) & 1u)) fail_t = t;
      p.fail_step[h] = fail_t;
      p.status[h] = fail_t >= 0 ? ST_INVALID : ST_VALID;
      st_steps += fail_t >= 0 ? fail_t + 1 : ns;
      if (p.stamps) {
        p.stamps[4 * h + 1] = __builtin_amdgcn_s_memrealtime();
        p.stamps[4 * h + 2] = team_cycles;
        p.stamps[4 * h + 3] = team_steps;
      }
    }
    const unsigned long long e = block_sum(expl, &sRed);
    if (tid == 0 && e) atomicAdd(&p.explored[h], e);
  } else if (rank == 0) {  // ------------------------------------------------- leader
    if (p.stamps && tid == 0) p.stamps[4 * h] = __builtin_amdgcn_s_memrealtime();
    const int ns = p.nsteps[h];
    unsigned long long team_cycles = 0, team_steps = 0;
    StreamWin sw;
    long long pos = p.sbeg[h];
    int fail_t = -1;
    for (int t = 0; t < ns && !sAbort; ++t) {
      sw.need(p, pos, lane);
      int ninv;
      const uint32_t H0 = read_step(sw, pos, lane, tid < 64, sOp, &ninv);
      const long long hpos = pos;
      pos += 1 + ninv;
      __syncthreads();
      const uint32_t live = H0 & DENSE_LIVE_MASK;
      const int j = (int)((H0 >> DENSE_J_SHIFT) & 31u);
      bool survived;
      if ((live >> lb) == 0) {  // narrow step: the leader alone (other tiles empty)
        const uint32_t foldm = fold_mask(sOp);
        expl += run_layers<HSOLO, 4>(sTab, &sZero, p.words, sWOff, sBinom, live, j, sOp, foldm, tid, 1024,
                                     [] { __syncthreads(); });
        survived = __syncthreads_or(return_slot(sTab, live, j, tid, 1024, st_fout) != 0);
      } else {  // wide step: every tile
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        if (tid == 0) {
          st_agent(&ctl->cmd, CMD_STEP);
          st_agent(&ctl->pos, hpos);
          st_agent(&ctl->any, 0u);
        }
        if (tid < 64) st_agent(&ctl->ops[tid], (&sOp[0].lo)[tid]);
        if (!bar()) break;
        survived = team_step(hpos);
        team_cycles += __builtin_amdgcn_s_memrealtime() - t0;
        ++team_steps;
      }
      if (tid == 0) ++st_steps;
      if (!survived) {
        fail_t = t;
        break;
      }
    }
    if (tid == 0) st_agent(&ctl->cmd, CMD_EXIT);
    bar();
    const unsigned long long e = block_sum(expl, &sRed);
    if (tid == 0) {
      if (e) atomicAdd(&p.explored[h], e);
      p.fail_step[h] = fail_t;
      p.status[h] = fail_t >= 0 ? ST_INVALID : ST_VALID;
      if (p.stamps) {
        p.stamps[4 * h + 1] = __builtin_amdgcn_s_memrealtime();
        p.stamps[4 * h + 2] = team_cycles;
        p.stamps[4 * h + 3] = team_steps;
      }
    }
  } else {  // ----------------------------------------------------------------- worker
    for (;;) {
      const bool ok = bar();
      if (tid == 0) {
        sCmd = ok ? ld_agent(&ctl->cmd) : CMD_EXIT;
        sPos = ld_agent(&ctl->pos);
      }
      if (tid < 64) (&sOp[0].lo)[tid] = ld_agent(&ctl->ops[tid]);
      __syncthreads();
      if (sCmd != CMD_STEP) break;
      team_step(sPos);
    }
    const unsigned long long e = block_sum(expl, &sRed);
    if (tid == 0 && e) atomicAdd(&p.explored[h], e);
  }
  if (p.tstamps && tid == 0)
    for (int i = 0; i < 6; ++i) p.tstamps[(base + rank) * 8 + i] = ph[i];
  if (nobar && (p.pipe & 1)) {
    // the team is done (its final barrier passed, and other tiles read only this tile's HBM
    // mirror, never its LDS): join the BLOCK queue, whose heaviest-first order leaves the
    // light tail to late joiners
    __syncthreads();
    history_pipe<1024, DENSE_LMAX, BLOCK_RING>(p, sTab, &sZero, sRing, &sQ, &sRed, p.words, sWOff, sBinom, tid,
                                               st_fout, st_steps);
    if (p.n2 > 0 && (p.pipe & 128)) {
      big_mid_mode(p, sTab, &sZero, sBinom, tid, st_fout, st_steps);
    } else {
      DenseParams q2 = p;
      q2.n = p.n2, q2.order = p.order2, q2.queue = p.queue2;
      history_pipe<1024, DENSE_LMAX, BLOCK_RING>(q2, sTab, &sZero, sRing, &sQ, &sRed, p.words, sWOff, sBinom,
                                                 tid, st_fout, st_steps);
    }
    if (p.n_w > 0) big_wave_mode(p, sTab, &sZero, sBinom, tid, st_fout, st_steps);
  }
  flush_stats(p, st_fout, st_steps, tid == 0);
}

}  // namespace

void dense_word_list(int bits, uint32_t* out) {
  int pos = 0;
  for (int q = 0; q <= bits; ++q)
    for (uint32_t v = 0; v < (1u << bits); ++v)  // numeric order within a layer = colex
      if (__builtin_popcount(v) == q) out[pos++] = v;
}

size_t dense_ctl_bytes() { return sizeof(TeamCtl); }

int dense_grid_size(DenseTeam kind) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
  int per_cu = 0;
  hipError_t e = kind == DENSE_WAVE ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dense_wave_kernel, WAVE_WG, 0)
                 : kind == DENSE_MID  ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dense_mid_kernel, MID_WG, 0)
                                      : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dense_big_kernel<false>, 1024, 0);
  if (e != hipSuccess || per_cu < 1) return 0;
  // wave teams: one workgroup per CU beside a big-kernel workgroup (whose LDS leaves room);
  // big kernel: one workgroup per CU, so every tile team is resident at once
  return prop.multiProcessorCount;
}

hipError_t launch_dense(const DenseParams& p, DenseTeam kind, int grid, hipStream_t stream) {
  if (kind == DENSE_WAVE)
    hipLaunchKernelGGL(dense_wave_kernel, dim3(grid), dim3(WAVE_WG), 0, stream, p);
  else if (kind == DENSE_MID)
    hipLaunchKernelGGL(dense_mid_kernel, dim3(grid), dim3(MID_WG), 0, stream, p);
  else if (p.pipe & 4)
    hipLaunchKernelGGL(dense_big_kernel<true>, dim3(grid), dim3(1024), 0, stream, p);
  else
    hipLaunchKernelGGL(dense_big_kernel<false>, dim3(grid), dim3(1024), 0, stream, p);
  return hipGetLastError();
}

}  // namespace lc
