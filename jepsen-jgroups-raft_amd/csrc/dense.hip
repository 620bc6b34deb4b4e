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
//                      then the in-word closure over the low 3 bits: nlo passes of every live
//                      low op k ≠ j (R |= T_k((X | R) at positions without k, j) moved up
//                      by 2^k), and, when j is a low bit, one final j pass into the j positions
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
// Teams (one history each, dequeued heaviest first from a global counter):
//   WAVE  one wave, LDS table, widths <= 11 (256-thread workgroups beside the wide teams)
//   BLOCK one 1024-thread workgroup, LDS table, widths 12..17
//   WIDE  team_size workgroups: the leader runs steps of width <= 17 on its LDS table;
//         wider steps run on an HBM table the whole team shares, one team barrier per
//         layer. Every HBM table byte is stored sc1 (write-through) and loaded sc1
//         (L1-bypassing), drained before each barrier arrival (cdna_hip_programming.md
//         Guideline 16, MI355X_MICROARCH.md "Valid forms" row 1), so no fences are needed.
#include "dense.hpp"
#include "device_common.hpp"
#include "search.hpp"

namespace lc {
namespace {

constexpr int BINOM_N = 24;
constexpr int CMD_STEP = 1, CMD_EXIT = 2;

typedef __attribute__((address_space(1))) uint64_t gu64;

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
  unsigned ops[32];
};

// decoded op, laid out for transfer(): srcsh[0:7) = 8 * source state, or OPF_FOLD (a write
// reads every state); dstsh[8:14) = 8 * destination state; OPF_IDENT (read nil: every state
// stays); OPF_NONE (the op names a value the register never holds: it moves nothing)
constexpr uint32_t OPF_FOLD = 64u, OPF_IDENT = 1u << 16, OPF_NONE = 1u << 17;
__device__ __forceinline__ uint32_t decode_op(uint32_t am, uint32_t bm) {
  if (am == 0) return OPF_NONE;  // precondition names a value the register never holds
  if (bm) {
    const uint32_t dst = ((uint32_t)__builtin_ctz(bm) * 8u) << 8;
    if (am == 0xffu) return OPF_FOLD | dst;  // write: from any state
    return (uint32_t)__builtin_ctz(am) * 8u | dst;
  }
  if (am == 0xffu) return OPF_IDENT;  // read nil: every state stays
  const uint32_t a = (uint32_t)__builtin_ctz(am) * 8u;
  return a | (a << 8);
}

// positions (of 8) whose mask lacks bit k (k < 3), one byte / replicated over 8 bytes
__device__ __forceinline__ uint32_t keep8(int k) { return k == 0 ? 0x55u : k == 1 ? 0x33u : 0x0fu; }
__device__ __forceinline__ uint64_t keep64(int k) {
  return k == 0 ? 0x5555555555555555ull : k == 1 ? 0x3333333333333333ull : 0x0f0f0f0f0f0f0f0full;
}

// op (wave-uniform) applied to word a (all 8 states), result bytes kept at positions
// `keep` (8-bit, replicated as keep_all), then moved up by `up` positions. The flag tests
// are scalar branches on a uniform value; the common MOVE path is shift, mask, shift.
__device__ __forceinline__ uint64_t transfer(uint32_t op, uint64_t a, uint32_t keep, uint64_t keep_all, int up) {
  if (op & (OPF_IDENT | OPF_NONE)) return (op & OPF_NONE) ? 0ull : (a & keep_all) << up;
  uint32_t t;
  if (op & OPF_FOLD) {
    t = (uint32_t)a | (uint32_t)(a >> 32);
    t |= t >> 16;
    t |= t >> 8;
  } else {
    t = (uint32_t)(a >> (op & 63u));
  }
  return (uint64_t)(t & keep) << (((op >> 8) & 63u) + (uint32_t)up);
}

// table access: LDS tables plainly, HBM team tables write-through sc1 / L1-bypassing sc1
struct LdsTab {
  static __device__ __forceinline__ uint64_t ld(const uint64_t* p) { return *p; }
  static __device__ __forceinline__ void st(uint64_t* p, uint64_t v) { *p = v; }
};
struct HbmTab {
  static __device__ __forceinline__ uint64_t ld(const uint64_t* p) {
    return __hip_atomic_load((const gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  static __device__ __forceinline__ void st(uint64_t* p, uint64_t v) {
    __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
};

// One step's hi pulls and in-word closure for word w; returns popcount(R).
// opv: lane k holds slot k's decoded op (read with readlane, wave-uniform).
template <int HMAX, int BATCH, class M>
__device__ __forceinline__ uint32_t close_word(uint64_t* B, uint32_t w, uint32_t live, int j, int H,
                                              uint32_t opv) {
  const uint64_t X = M::ld(B + w);
  uint64_t R = 0;
  const bool j_lo = j < 3;
  const uint32_t jh = j_lo ? 0u : 1u << (j - 3);
  const bool has_j = (w & jh) != 0;
  // ---- pulls from the finalized words one hi bit below, BATCH loads in flight
#pragma unroll
  for (int b0 = 0; b0 < HMAX; b0 += BATCH) {
    if (b0 >= H) break;
    uint64_t v[BATCH];
#pragma unroll
    for (int i = 0; i < BATCH; ++i) {
      const int b = b0 + i;
      v[i] = 0;
      if (b < H) {
        const uint32_t bit = 1u << b;
        const bool act = has_j ? (bit == jh) : ((w & bit) != 0);
        if (act) v[i] = M::ld(B + (w ^ bit));
      }
    }
#pragma unroll
    for (int i = 0; i < BATCH; ++i) {
      const int b = b0 + i;
      if (b < H) R |= transfer((uint32_t)__builtin_amdgcn_readlane((int)opv, b + 3), v[i], 0xffu, ~0ull, 0);
    }
  }
  if (!has_j) {
    const uint32_t notj = j_lo ? keep8(j) : 0xffu;
    const uint64_t notj64 = j_lo ? keep64(j) : ~0ull;
    R &= notj64;  // configs holding j come only from T_j
    // ---- in-word closure: nlo passes over the live low ops other than j
    const uint32_t lo_ops = live & 7u & ~(j_lo ? (1u << j) : 0u);
    const int nlo = __popc(lo_ops);
    for (int pass = 0; pass < nlo; ++pass) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        if (lo_ops & (1u << k))
          R |= transfer((uint32_t)__builtin_amdgcn_readlane((int)opv, k), X | R, keep8(k) & notj,
                        keep64(k) & notj64, 1 << k);
      }
    }
    if (j_lo)  // the returning op, linearized last
      R |= transfer((uint32_t)__builtin_amdgcn_readlane((int)opv, j), X | R, notj, notj64, 1 << j);
  }
  if (R) M::st(B + w, X | R);
  return (uint32_t)__popcll(R);
}

// The closure layers of one step, words split over participants gt = 0..gn-1; sync() ends
// every layer (the last one too: the return that follows reads the last layer's words).
template <int HMAX, int BATCH, class M, class Sync>
__device__ __forceinline__ unsigned long long run_layers(uint64_t* B, const uint32_t* words, const uint32_t* wofs,
                                                        const uint32_t* binom, uint32_t live, int j,
                                                        uint32_t opv, int gt, int gn, Sync&& sync) {
  const int L = 32 - __clz((int)live);
  const int H = L > 3 ? L - 3 : 0;
  const uint32_t live_hi = live >> 3;
  unsigned long long expl = 0;
  for (int q = 0; q <= H; ++q) {
    // words of popcount q below 2^H: a prefix of layer q of the sorted list
    const uint32_t nq = binom[H * BINOM_N + q], o = wofs[q];
    for (uint32_t r = (uint32_t)gt; r < nq; r += (uint32_t)gn) {
      const uint32_t w = words[o + r];
      if (w & ~live_hi) continue;
      expl += close_word<HMAX, BATCH, M>(B, w, live, j, H, opv);
    }
    sync();
  }
  return expl;
}

// Return slot j: the post-return frontier moves down to the masks without j. Returns the
// OR of this participant's new words (nonzero = some config survived).
template <class M>
__device__ __forceinline__ uint64_t return_slot(uint64_t* B, uint32_t live, int j, int gt, int gn,
                                               unsigned long long& fout) {
  const int L = 32 - __clz((int)live);
  const int nwt = 1 << (L > 3 ? L - 3 : 0);
  uint64_t anyv = 0;
  if (j < 3) {
    const uint64_t with_j = ~keep64(j);
    const int sh = 1 << j;
    for (int w = gt; w < nwt; w += gn) {
      const uint64_t v = (M::ld(B + w) & with_j) >> sh;
      M::st(B + w, v);
      anyv |= v;
      fout += __popcll(v);
    }
  } else {
    const int jb = 1 << (j - 3);
    const int half = nwt >> 1;
    for (int x = gt; x < half; x += gn) {
      const int lo = x & (jb - 1);
      const int w = ((x ^ lo) << 1) | lo;
      const uint64_t v = M::ld(B + (w | jb));
      M::st(B + w, v);
      M::st(B + (w | jb), 0);
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
                                             uint32_t* opt, int* ninv_out) {
  const uint32_t H0 = sw.at(pos);
  const int ninv = (int)(H0 >> 27);
  const uint32_t w = sw.at(pos + 1 + lane);
  if (writer && lane < ninv) opt[w & 31u] = decode_op((w >> 8) & 0xffu, (w >> 16) & 0xffu);
  *ninv_out = ninv;
  return H0;
}

template <int TEAM, int WG, int TLOG, bool GLOBAL_WORDS>
__global__ void __launch_bounds__(WG) dense_kernel(DenseParams p) {
  constexpr int NTEAM = WG / TEAM;
  constexpr int HMAX = TLOG - 3;
  constexpr int TWORDS = 1 << HMAX;  // u64 words per team
  constexpr int LBITS = GLOBAL_WORDS ? DENSE_WORD_BITS : HMAX;
  __shared__ uint64_t sTab[NTEAM * TWORDS];
  __shared__ uint32_t sWords[GLOBAL_WORDS ? 1 : (1 << HMAX)];  // words sorted by (popcount, value)
  __shared__ uint32_t sWOff[LBITS + 2];
  __shared__ uint32_t sBinom[BINOM_N * BINOM_N];
  __shared__ uint32_t sOp[NTEAM][32];  // decoded op per slot
  __shared__ int sQ[NTEAM];
  __shared__ unsigned long long sExpl[NTEAM];

  const int tid = threadIdx.x;
  const int team = tid / TEAM, tt = tid % TEAM, lane = tid & 63;
  uint64_t* const B = &sTab[team * TWORDS];
  uint32_t* const opt = sOp[team];
  const uint32_t* const words = GLOBAL_WORDS ? p.words : sWords;

  init_tables(sBinom, sWOff, LBITS, WG);
  if constexpr (!GLOBAL_WORDS) {
    for (int v = tid; v < (1 << HMAX); v += WG) {  // colex rank within its popcount layer
      uint32_t rank = 0;
      int i = 0;
      for (uint32_t x = (uint32_t)v; x; x &= x - 1, ++i) rank += sBinom[__builtin_ctz(x) * BINOM_N + i + 1];
      sWords[sWOff[__popc(v)] + rank] = (uint32_t)v;
    }
    __syncthreads();
  }

  unsigned long long st_fout = 0, st_steps = 0;
  for (;;) {
    if (tt == 0) sQ[team] = atomicAdd(p.queue, 1);
    team_sync<TEAM>();
    const int qi = sQ[team];
    if (tt == 0) sExpl[team] = 0;
    team_sync<TEAM>();
    if (qi >= p.n) break;
    const int h = p.order[qi];
    if (p.stamps && tt == 0) p.stamps[2 * h] = __builtin_amdgcn_s_memrealtime();
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
      const uint32_t live = H0 & 0x3fffffu;
      const int j = (int)((H0 >> 22) & 31u);
      const uint32_t opv = opt[lane & 31];  // lane k: slot k's op, read with readlane
      expl += run_layers<HMAX, 4, LdsTab>(B, words, sWOff, sBinom, live, j, opv, tt, TEAM,
                                          [] { team_sync<TEAM>(); });
      const uint64_t anyv = return_slot<LdsTab>(B, live, j, tt, TEAM, st_fout);
      ++st_steps;
      if (!team_any<TEAM>(anyv != 0)) {
        fail_t = t;
        break;
      }
    }
    // explored: team reduction
    for (int off = 32; off > 0; off >>= 1) expl += __shfl_down(expl, off, 64);
    if constexpr (TEAM >= 256) {
      if (lane == 0 && expl) atomicAdd(&sExpl[team], expl);
      __syncthreads();
      expl = sExpl[team];
    } else {
      expl = __shfl(expl, 0, 64);
    }
    if (tt == 0) {
      p.explored[h] = expl;
      p.fail_step[h] = fail_t;
      p.status[h] = fail_t >= 0 ? ST_INVALID : ST_VALID;
      if (p.stamps) p.stamps[2 * h + 1] = __builtin_amdgcn_s_memrealtime();
    }
    team_sync<TEAM>();
  }
  // launch statistics (per wave, one atomic each)
  for (int off = 32; off > 0; off >>= 1) st_fout += __shfl_down(st_fout, off, 64);
  if (lane == 0 && st_fout) atomicAdd(&p.stats[SS_FOUT], st_fout);
  if (tt == 0 && st_steps) atomicAdd(&p.stats[SS_STEPS], st_steps);
}

// Team barrier over the team's G workgroups: every wave drains its (sc1) stores, one lane
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

__global__ void __launch_bounds__(1024) dense_wide_kernel(DenseParams p) {
  constexpr int HSOLO = DENSE_LMAX - 3;
  constexpr int HTEAM = DENSE_WORD_BITS;
  __shared__ uint64_t sTab[1 << HSOLO];
  __shared__ uint32_t sWOff[DENSE_WORD_BITS + 2];
  __shared__ uint32_t sBinom[BINOM_N * BINOM_N];
  __shared__ uint32_t sOp[32];
  __shared__ int sQ, sCmd, sH, sAbort;
  __shared__ long long sPos;
  __shared__ unsigned sAny;
  __shared__ unsigned long long sRed;

  const int tid = threadIdx.x, lane = tid & 63;
  const int G = p.team_size;
  const int team = blockIdx.x / G, rank = blockIdx.x % G;
  TeamCtl* const ctl = (TeamCtl*)p.ctl + team;
  uint64_t* const GT = p.gtab + ((size_t)team << DENSE_WORD_BITS);
  const int gt = rank * 1024 + tid, gn = G * 1024;
  init_tables(sBinom, sWOff, DENSE_WORD_BITS, 1024);
  if (tid == 0) sAbort = 0;
  __syncthreads();
  unsigned long long expl = 0, st_fout = 0, st_steps = 0;
  auto bar = [&]() { return team_bar(ctl, G, p.abort, &sAbort); };

  // one team step on the HBM table (every rank; the ops are in sOp); returns "survived"
  auto team_step = [&](long long pos) -> bool {
    const uint32_t H0 = p.stream[pos];
    const uint32_t live = H0 & 0x3fffffu;
    const int j = (int)((H0 >> 22) & 31u);
    const uint32_t opv = sOp[lane & 31];
    expl += run_layers<HTEAM, 8, HbmTab>(GT, p.words, sWOff, sBinom, live, j, opv, gt, gn, [&] { bar(); });
    const uint64_t a = return_slot<HbmTab>(GT, live, j, gt, gn, st_fout);
    if (__syncthreads_or(a != 0) && tid == 0)
      __hip_atomic_fetch_or(&ctl->any, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bar();
    if (tid == 0) sAny = ld_agent(&ctl->any);
    __syncthreads();
    return sAny != 0;
  };

  if (rank == 0) {  // ---------------------------------------------------------- leader
    for (;;) {
      if (tid == 0) sQ = atomicAdd(p.queue, 1);
      __syncthreads();
      const int qi = sQ;
      __syncthreads();
      if (qi >= p.n || sAbort) {
        if (tid == 0) st_agent(&ctl->cmd, CMD_EXIT);
        bar();
        break;
      }
      const int h = p.order[qi];
      if (p.stamps && tid == 0) p.stamps[2 * h] = __builtin_amdgcn_s_memrealtime();
      const int ns = p.nsteps[h];
      for (int i = tid; i < (1 << HSOLO); i += 1024) sTab[i] = 0;
      for (int i = tid; i < (1 << (p.lmax[h] - 3)); i += 1024) HbmTab::st(GT + i, 0);
      __syncthreads();
      if (tid == 0) sTab[0] = 1;  // (cas-register) starts at nil: state id 0
      bool team_mode = false;
      StreamWin sw;
      long long pos = p.sbeg[h];
      int fail_t = -1;
      for (int t = 0; t < ns; ++t) {
        sw.need(p, pos, lane);
        int ninv;
        const uint32_t H0 = read_step(sw, pos, lane, tid < 64, sOp, &ninv);
        const long long hpos = pos;
        pos += 1 + ninv;
        __syncthreads();
        const uint32_t live = H0 & 0x3fffffu;
        const int j = (int)((H0 >> 22) & 31u);
        const int L = 32 - __clz((int)live);
        bool survived;
        if (L <= DENSE_LMAX) {  // narrow step: the leader alone, LDS table
          if (team_mode) {
            for (int i = tid; i < (1 << HSOLO); i += 1024) sTab[i] = HbmTab::ld(GT + i);
            __syncthreads();
            team_mode = false;
          }
          const uint32_t opv = sOp[lane & 31];
          expl += run_layers<HSOLO, 4, LdsTab>(sTab, p.words, sWOff, sBinom, live, j, opv, tid, 1024,
                                               [] { __syncthreads(); });
          survived = __syncthreads_or(return_slot<LdsTab>(sTab, live, j, tid, 1024, st_fout) != 0);
        } else {  // wide step: the whole team, HBM table
          if (!team_mode) {  // masks >= 2^17 are all empty: only the LDS part moves
            for (int i = tid; i < (1 << HSOLO); i += 1024) HbmTab::st(GT + i, sTab[i]);
            team_mode = true;
          }
          if (tid == 0) {
            st_agent(&ctl->cmd, CMD_STEP);
            st_agent(&ctl->h, h);
            st_agent(&ctl->pos, hpos);
            st_agent(&ctl->any, 0u);
          }
          if (tid < 32) st_agent(&ctl->ops[tid], sOp[tid]);
          if (!bar()) break;
          survived = team_step(hpos);
        }
        if (tid == 0) ++st_steps;
        if (!survived) {
          fail_t = t;
          break;
        }
      }
      const unsigned long long e = block_sum(expl, &sRed);
      expl = 0;
      if (tid == 0) {
        if (e) atomicAdd(&p.explored[h], e);
        p.fail_step[h] = fail_t;
        p.status[h] = fail_t >= 0 ? ST_INVALID : ST_VALID;
        if (p.stamps) p.stamps[2 * h + 1] = __builtin_amdgcn_s_memrealtime();
      }
    }
  } else {  // ----------------------------------------------------------------- worker
    int cur_h = -1;
    for (;;) {
      const bool ok = bar();
      if (tid == 0) {
        sCmd = ok ? ld_agent(&ctl->cmd) : CMD_EXIT;
        sH = ld_agent(&ctl->h);
        sPos = ld_agent(&ctl->pos);
      }
      if (tid < 32) sOp[tid] = ld_agent(&ctl->ops[tid]);
      __syncthreads();
      const int cmd = sCmd, h = sH;
      const long long pos = sPos;
      if (cmd != CMD_STEP || h != cur_h) {  // this rank's share of the previous history
        const unsigned long long e = block_sum(expl, &sRed);
        expl = 0;
        if (tid == 0 && e && cur_h >= 0) atomicAdd(&p.explored[cur_h], e);
        cur_h = h;
      }
      if (cmd != CMD_STEP) break;
      team_step(pos);
    }
  }
  for (int off = 32; off > 0; off >>= 1) st_fout += __shfl_down(st_fout, off, 64);
  if (lane == 0 && st_fout) atomicAdd(&p.stats[SS_FOUT], st_fout);
  if (tid == 0 && st_steps) atomicAdd(&p.stats[SS_STEPS], st_steps);
}

constexpr int WAVE_WG = 256;
#define WAVE_KERNEL dense_kernel<64, WAVE_WG, DENSE_WAVE_LMAX, false>
#define BLOCK_KERNEL dense_kernel<1024, 1024, DENSE_LMAX, true>

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
  hipError_t e = kind == DENSE_WAVE
      ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, WAVE_KERNEL, WAVE_WG, 0)
      : kind == DENSE_BLOCK ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, BLOCK_KERNEL, 1024, 0)
                            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dense_wide_kernel, 1024, 0);
  if (e != hipSuccess || per_cu < 1) return 0;
  // wave teams: one workgroup per CU beside a wide team (the wide team's LDS leaves room);
  // wide teams: one workgroup per CU, every workgroup of a team resident at once
  return prop.multiProcessorCount * (kind == DENSE_BLOCK ? per_cu : 1);
}

hipError_t launch_dense(const DenseParams& p, DenseTeam kind, int grid, hipStream_t stream) {
  if (kind == DENSE_WAVE)
    hipLaunchKernelGGL(WAVE_KERNEL, dim3(grid), dim3(WAVE_WG), 0, stream, p);
  else if (kind == DENSE_BLOCK)
    hipLaunchKernelGGL(BLOCK_KERNEL, dim3(grid), dim3(1024), 0, stream, p);
  else
    hipLaunchKernelGGL(dense_wide_kernel, dim3(grid), dim3(1024), 0, stream, p);
  return hipGetLastError();
}

}  // namespace lc
