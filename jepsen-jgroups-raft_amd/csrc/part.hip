// part.hip — one cas-register history searched by several ranks at once, its frontier
// partitioned by config hash (SURVEY §8(e) axis 2; knossos.linear/analysis [ext], §8(a) a5,
// model register.clj:110). The library runs the per-rank work; the caller (lincheck/
// partition.py, or any host with a collective library) moves candidates between ranks with
// one all-to-all per BFS level (RCCL over xGMI under torch.distributed "nccl").
//
// Per RETURN step of slot j (bitj = 1 << j), every rank r holds F_r, its part of the frontier
// (globally duplicate-free), and owns the configs c with owner(c & ~bitj) = r:
//   level 0 : expand F_r: a config holding j goes DIRECT to the owner of c & ~bitj (its
//             post-return image); every other config steps each pending op k not in its mask
//             (cas-register: consistent iff the op's expected state is any/equal) -> c2.
//   exchange: candidates travel to their owners (one all-to-all, counts gathered first).
//   absorb  : DIRECT -> OUT set. Else insert c2 into the closure set S; a new c2 counts as
//             explored and either holds j (linearized the returning op: its image c2 & ~bitj
//             goes to OUT, same owner by construction) or joins the next level's list.
//   level l : expand the new list (its configs never hold j), exchange, absorb ... until no
//             rank produced a candidate. Then F_r = OUT_r; sum over ranks of |F_r| = 0 =>
//             not linearizable at this RETURN.
// S and OUT are open-addressing hash sets in HBM (atomicCAS on 64-bit words, linear probing)
// whose words carry a 16-bit step epoch above the 48-bit key, so a new step needs no clear.
// Survivors are compacted with one wave ballot + one global atomic per wave and list.
// The explored count is a set cardinality per step, so it is independent of the rank count
// and of arrival order: bit-exact with the single-GPU paths and the oracle.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lincheck.h"
#include "device_common.hpp"
#include "encode.hpp"

namespace lc {
namespace {

constexpr int PW_MAX = 16;                   // ranks
constexpr int PS_MAX = 48;                   // slots (mask bits)
constexpr int KEY_BITS = 48;                 // [state | mask] below the epoch
constexpr uint64_t DIRECT = 1ull << 63;      // in transit: already returned, goes to OUT
constexpr int PT = 256;                      // threads per workgroup
constexpr uint32_t EPOCH_MAX = 0xffffu;

enum : int { PF_OVERFLOW = 1, PF_STAGE = 2, PF_ABORT = 4 };

// device counters of one rank (one D2H read per level; per chunk of steps in lc_part_run)
struct PartCtl {
  unsigned long long cnt[PW_MAX];  // candidates per destination (this level)
  unsigned long long lc[2];        // level lists (count)
  unsigned long long oc[2];        // frontier F / OUT list, by step parity (F = oc[sp ^ 1])
  unsigned long long explored;     // all steps
  unsigned long long flags;
  unsigned long long lvl[3];       // lc_part_run: candidates of level l in lvl[l % 3]
  unsigned long long listed;       // lc_part_run: configs expanded, candidates absorbed,
  unsigned long long cand;         //   BFS levels (for the algorithmic bytes / stats)
  unsigned long long levels;
};

// lc_part_run's grid barrier words, each on its own 64-B line
struct PartBar {
  unsigned grp[8][16];
  unsigned top, pad0[15];
  unsigned gen, pad1[15];
};

struct StepArgs {
  uint64_t ops[PS_MAX];  // per slot: (uint32 b << 32) | uint32 a; a: expected state id (-1 any,
                         // -2 never), b: new state id (-1 keep)
  uint64_t live, bitj;
  int32_t mask_bits, world, rank, pad;
};

__device__ __forceinline__ uint32_t owner_of(uint64_t k, uint32_t world) {
  return (uint32_t)(((mix64(k) >> 32) * (uint64_t)world) >> 32);
}

// Block-aggregated append, step 1: every wave adds its ballot count of `pred` to the LDS
// counter and gets its lanes' offsets within the block (one LDS atomic per wave).
__device__ __forceinline__ uint32_t block_slot(uint32_t* s_counter, bool pred) {
  const unsigned long long m = __ballot(pred);
  if (m == 0) return 0;
  const int lane = __lane_id();
  const int leader = __ffsll((long long)m) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(s_counter, (uint32_t)__popcll(m));
  base = __shfl(base, leader, 64);
  const unsigned long long below = lane ? (m & ((~0ull) >> (64 - lane))) : 0ull;
  return base + (uint32_t)__popcll(below);
}

// insert key (< 2^48) into an epoch-tagged open-addressing set; 1 = new, 0 = present. A probe
// run longer than PROBE_MAX (tables are sized at most half full, where linear probing's runs
// are a few dozen words) raises PF_OVERFLOW: an over-full table is reported at once instead of
// every insert scanning the whole table.
constexpr uint64_t PROBE_MAX = 4096;
__device__ __forceinline__ int set_insert(uint64_t* T, uint64_t tmask, uint64_t key, uint64_t ep,
                                          unsigned long long* flags) {
  const uint64_t v = (ep << KEY_BITS) | key;
  uint64_t i = mix64(key) & tmask;
  const uint64_t pmax = tmask < PROBE_MAX ? tmask : PROBE_MAX;
  for (uint64_t probe = 0; probe <= pmax; ++probe) {
    uint64_t cur = ld_agent(&T[i]);
    if (cur == v) return 0;
    if ((cur >> KEY_BITS) != ep) {  // free in this epoch: claim it
      const uint64_t old = atomicCAS((unsigned long long*)&T[i], (unsigned long long)cur, (unsigned long long)v);
      if (old == cur) return 1;
      if (old == v) return 0;
      if ((old >> KEY_BITS) != ep) {  // raced with a stale word's owner? (cannot happen) retry
        --probe;
        continue;
      }
    }
    i = (i + 1) & tmask;
  }
  atomicOr(flags, (unsigned long long)PF_OVERFLOW);
  return 0;
}

// One pending op k stepped from config c (cas-register), or c's DIRECT return (k = 0 only)
struct Cand {
  bool has;
  uint32_t dst;
  uint64_t out;
};
__device__ __forceinline__ Cand candidate(const StepArgs& a, uint64_t c, bool valid, int k, uint64_t mmask) {
  Cand r{false, 0u, 0ull};
  if (!valid) return r;
  uint64_t route = 0;
  if (c & a.bitj) {  // already linearized the returning op: its image goes straight to OUT
    if (k != 0) return r;
    route = c & ~a.bitj;
    r.out = route | DIRECT;
    r.has = true;
  } else if (((a.live >> k) & 1) && !((c >> k) & 1)) {
    const uint64_t op = a.ops[k];
    const int32_t ea = (int32_t)(uint32_t)op, nb = (int32_t)(uint32_t)(op >> 32);
    const int64_t st = (int64_t)(c >> a.mask_bits);
    if (ea == -1 || ea == st) {
      const uint64_t ns = nb < 0 ? (uint64_t)st : (uint64_t)nb;
      r.out = (ns << a.mask_bits) | (c & mmask) | (1ull << k);
      route = r.out & ~a.bitj;
      r.has = true;
    }
  }
  if (r.has) r.dst = owner_of(route, (uint32_t)a.world);
  return r;
}

// Expand: thread per config of the list, its candidates over the pending slots staged per
// destination ([world][seg_cap]). Positions are reserved per block (LDS counts, then one
// global atomic per destination per block pass) and handed out per wave (ballots), so the
// global counters see ~n/256 atomics, not one per wave and slot. Counts may exceed seg_cap
// (the host then grows the staging and re-runs).
__global__ void __launch_bounds__(PT) part_expand(StepArgs a, const uint64_t* __restrict__ list,
                                                  const unsigned long long* __restrict__ count, uint32_t wd,
                                                  uint64_t* __restrict__ stage, uint64_t seg_cap, PartCtl* ctl,
                                                  unsigned long long* zero_a, unsigned long long* zero_b) {
  __shared__ uint32_t s_cnt[PW_MAX];
  // counters the following absorb fills (the next list's, and OUT's at level 0): no memset
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *zero_a = 0;
    if (zero_b) *zero_b = 0;
  }
  __shared__ unsigned long long s_base[PW_MAX];
  const uint64_t n = count[0];
  const uint64_t mmask = (1ull << a.mask_bits) - 1;
  const uint64_t stride = (uint64_t)gridDim.x * PT;
  const int W = a.world;
  for (uint64_t it = (uint64_t)blockIdx.x * PT; it < n; it += stride) {  // block-uniform trip count
    const uint64_t i = it + threadIdx.x;
    const bool valid = i < n;
    const uint64_t c = valid ? list[i] : 0ull;
    if (threadIdx.x < (unsigned)W) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    // pass 1: this block's candidates per destination
    for (int k = 0; k < (int)wd; ++k) {
      const Cand q = candidate(a, c, valid, k, mmask);
      for (int d = 0; d < W; ++d) {
        const unsigned long long m = __ballot(q.has && q.dst == (uint32_t)d);
        if (m && __lane_id() == 0) atomicAdd(&s_cnt[d], (uint32_t)__popcll(m));
      }
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)W) {
      const uint32_t cnt = s_cnt[threadIdx.x];
      s_base[threadIdx.x] = cnt ? atomicAdd(&ctl->cnt[threadIdx.x], (unsigned long long)cnt) : 0ull;
      s_cnt[threadIdx.x] = 0;
    }
    __syncthreads();
    // pass 2: the same candidates, written at the block's reserved positions
    for (int k = 0; k < (int)wd; ++k) {
      const Cand q = candidate(a, c, valid, k, mmask);
      for (int d = 0; d < W; ++d) {
        const bool mine = q.has && q.dst == (uint32_t)d;
        const uint32_t off = block_slot(&s_cnt[d], mine);
        if (mine) {
          const unsigned long long pos = s_base[d] + off;
          if (pos < seg_cap) stage[(uint64_t)d * seg_cap + pos] = q.out;
        }
      }
    }
    __syncthreads();  // s_cnt / s_base are reused by the next pass
  }
}

// Absorb the candidates this rank owns: dedup into S / OUT, compact the survivors. Each thread
// takes AB items per block pass (independent hash probes in flight); list positions are
// reserved per block (LDS counts, one global atomic per list per pass).
constexpr int AB = 4;
__global__ void __launch_bounds__(PT) part_absorb(const uint64_t* __restrict__ recv, uint64_t n, uint64_t bitj,
                                                  uint64_t* S, uint64_t smask, uint64_t* O, uint64_t omask,
                                                  uint64_t ep, uint64_t* __restrict__ next,
                                                  unsigned long long* next_count, unsigned long long* out_count,
                                                  uint64_t* __restrict__ outl, uint64_t list_cap, PartCtl* ctl,
                                                  int world) {
  __shared__ uint32_t s_cnt[2];
  // the last expand's per-destination counts (already read by the host) start the next one at 0
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)world) ctl->cnt[threadIdx.x] = 0;
  __shared__ unsigned long long s_base[2];
  const uint64_t stride = (uint64_t)gridDim.x * PT * AB;
  unsigned long long expl = 0;
  for (uint64_t it = (uint64_t)blockIdx.x * PT * AB; it < n; it += stride) {
    uint64_t key[AB], okey[AB];
    bool news[AB], newo[AB];
#pragma unroll
    for (int u = 0; u < AB; ++u) {
      const uint64_t i = it + (uint64_t)u * PT + threadIdx.x;
      key[u] = i < n ? recv[i] : 0ull;
      news[u] = newo[u] = false;
      okey[u] = 0;
    }
#pragma unroll
    for (int u = 0; u < AB; ++u) {
      if (it + (uint64_t)u * PT + threadIdx.x >= n) continue;
      if (key[u] & DIRECT) {
        okey[u] = key[u] & ~DIRECT;
        newo[u] = set_insert(O, omask, okey[u], ep, &ctl->flags);
      } else {
        news[u] = set_insert(S, smask, key[u], ep, &ctl->flags);
        if (news[u] && (key[u] & bitj)) {
          okey[u] = key[u] & ~bitj;
          newo[u] = set_insert(O, omask, okey[u], ep, &ctl->flags);
        }
      }
    }
    if (threadIdx.x < 2) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    uint32_t pn[AB], po[AB];
#pragma unroll
    for (int u = 0; u < AB; ++u) {
      const bool nl = news[u] && !(key[u] & bitj);
      expl += news[u];
      pn[u] = block_slot(&s_cnt[0], nl);
      po[u] = block_slot(&s_cnt[1], newo[u]);
    }
    __syncthreads();
    if (threadIdx.x < 2) {
      const uint32_t cnt = s_cnt[threadIdx.x];
      s_base[threadIdx.x] = cnt ? atomicAdd(threadIdx.x == 0 ? next_count : out_count, (unsigned long long)cnt)
                                : 0ull;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < AB; ++u) {
      if (news[u] && !(key[u] & bitj)) {
        const unsigned long long q = s_base[0] + pn[u];
        if (q < list_cap) next[q] = key[u];
        else atomicOr(&ctl->flags, (unsigned long long)PF_OVERFLOW);
      }
      if (newo[u]) {
        const unsigned long long q = s_base[1] + po[u];
        if (q < list_cap) outl[q] = okey[u];
        else atomicOr(&ctl->flags, (unsigned long long)PF_OVERFLOW);
      }
    }
    __syncthreads();  // s_cnt / s_base are reused by the next pass
  }
  for (int off = 32; off > 0; off >>= 1) expl += __shfl_down(expl, off, 64);
  if (__lane_id() == 0 && expl) atomicAdd(&ctl->explored, expl);
}

// ---- lc_part_run (world 1): one cooperative launch per RETURN step runs all of its levels,
// separated by grid barriers; a level absorbs its candidates and expands the new configs at
// once (no level list, no host round trip). The host reads the per-step OUT counts once per
// chunk of steps.
constexpr int PL = 512;  // threads per workgroup
constexpr int PLW = PL / 64;
constexpr int PAB = 4;   // candidates per thread per pass

struct RunArgs {
  uint64_t* S;
  uint64_t* O;
  uint64_t tmask;
  const uint64_t* F;
  uint64_t* outl;
  uint64_t list_cap;
  uint64_t* stage[2];
  uint64_t seg_cap;
  PartCtl* ctl;
  PartBar* bar;
  unsigned long long* flog;  // OUT count per step of the chunk
  uint32_t flog_i;
  int32_t sp;
  uint64_t ep;
  uint32_t wd, nwg;
};

// Grid barrier: 8 group counters then a top counter, release generation polled relaxed with
// s_sleep (MI355X_MICROARCH "barrier-xcd"); the data a level hands on is sc1 stores and
// device-scope atomics, read back with sc1 loads. A 20 s watchdog raises PF_ABORT.
__device__ __forceinline__ bool run_sync(const RunArgs& r, int* s_abort) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    PartBar* bar = r.bar;
    const unsigned g = ld_agent(&bar->gen);
    const unsigned grp = blockIdx.x & 7u;
    const unsigned gsize = (r.nwg - grp + 7u) >> 3;
    const unsigned ngroups = r.nwg < 8u ? r.nwg : 8u;
    const unsigned a = __hip_atomic_fetch_add(&bar->grp[grp][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a == gsize - 1) {
      st_agent(&bar->grp[grp][0], 0u);
      const unsigned t = __hip_atomic_fetch_add(&bar->top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == ngroups - 1) {
        st_agent(&bar->top, 0u);
        __hip_atomic_store(&bar->gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    long spins = 0;
    while (ld_agent(&bar->gen) == g) {
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 255) == 0) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000000ull) {
          atomicOr(&r.ctl->flags, (unsigned long long)PF_ABORT);
          break;
        }
        if (ld_agent(&r.ctl->flags) & PF_ABORT) break;
      }
    }
    *s_abort = (ld_agent(&r.ctl->flags) & PF_ABORT) != 0;
  }
  __syncthreads();
  return *s_abort == 0;
}

// Every thread's candidates from its NU configs (ok[u]) appended to dst at positions reserved
// with one wave scan, one block prefix and one global atomic per block. Block-uniform call.
template <int NU>
__device__ __forceinline__ void emit(const StepArgs& a, const uint64_t* c, const bool* ok, uint32_t wd,
                                     uint64_t mmask, uint64_t* dst, uint64_t cap, unsigned long long* counter,
                                     PartCtl* ctl, uint32_t* s_w, unsigned long long* s_base) {
  uint32_t tc = 0;
#pragma unroll
  for (int u = 0; u < NU; ++u)
    if (ok[u])
      for (int k = 0; k < (int)wd; ++k) tc += candidate(a, c[u], true, k, mmask).has;
  const int lane = __lane_id(), w = threadIdx.x >> 6;
  uint32_t x = tc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t sum = 0;
    for (int i = 0; i < PLW; ++i) {
      const uint32_t v = s_w[i];
      s_w[i] = sum;
      sum += v;
    }
    *s_base = sum ? atomicAdd(counter, (unsigned long long)sum) : 0ull;
  }
  __syncthreads();
  uint64_t pos = *s_base + s_w[w] + (x - tc);
  bool over = false;
  if (tc) {
#pragma unroll
    for (int u = 0; u < NU; ++u)
      if (ok[u])
        for (int k = 0; k < (int)wd; ++k) {
          const Cand q = candidate(a, c[u], true, k, mmask);
          if (!q.has) continue;
          if (pos < cap) st_agent(&dst[pos], q.out);
          else over = true;
          ++pos;
        }
  }
  if (over) atomicOr(&ctl->flags, (unsigned long long)PF_STAGE);
  __syncthreads();  // s_w / s_base are reused
}

__global__ void __launch_bounds__(PL) part_step_kernel(StepArgs a, RunArgs r) {
  __shared__ uint32_t s_w[PLW];
  __shared__ unsigned long long s_base;
  __shared__ int s_abort;
  PartCtl* ctl = r.ctl;
  const uint64_t mmask = (1ull << a.mask_bits) - 1;
  unsigned long long* out_count = &ctl->oc[r.sp];
  const int tid = threadIdx.x, lane = __lane_id();
  const bool lead = blockIdx.x == 0 && tid == 0;
  // an earlier step of the chunk overflowed (or aborted): the host starts over or reports
  // LC_H_CAPACITY after the chunk, so the rest of it does no work (the flags were set by
  // earlier launches: every workgroup reads the same value)
  if (ld_agent(&ctl->flags) & (PF_OVERFLOW | PF_STAGE | PF_ABORT)) return;
  // level 0: expand the frontier into stage 0
  if (lead) st_agent(out_count, 0ull);
  const uint64_t nf = min<uint64_t>(ld_agent(&ctl->oc[r.sp ^ 1]), r.list_cap);  // (overflowed counts: never beyond the list)
  const uint64_t stride = (uint64_t)r.nwg * PL;
  for (uint64_t it = (uint64_t)blockIdx.x * PL; it < nf; it += stride) {  // block-uniform trip count
    const uint64_t i = it + tid;
    const bool ok = i < nf;
    const uint64_t c = ok ? r.F[i] : 0ull;
    emit<1>(a, &c, &ok, r.wd, mmask, r.stage[0], r.seg_cap, &ctl->lvl[0], ctl, s_w, &s_base);
  }
  if (!run_sync(r, &s_abort)) return;
  unsigned long long expl = 0, listed = 0;
  int l = 0;
  for (;; ++l) {
    const uint64_t n_raw = ld_agent(&ctl->lvl[l % 3]);
    if (n_raw == 0) break;
    const uint64_t n = n_raw < r.seg_cap ? n_raw : r.seg_cap;  // beyond: PF_STAGE was raised
    if (lead) {
      st_agent(&ctl->lvl[(l + 2) % 3], 0ull);
      atomicAdd(&ctl->cand, (unsigned long long)n);
    }
    const uint64_t* src = r.stage[l & 1];
    uint64_t* dst = r.stage[(l + 1) & 1];
    for (uint64_t it = (uint64_t)blockIdx.x * PL * PAB; it < n; it += stride * PAB) {
      uint64_t key[PAB];
      bool nl[PAB];
#pragma unroll
      for (int u = 0; u < PAB; ++u) {
        const uint64_t i = it + (uint64_t)u * PL + tid;
        key[u] = i < n ? ld_agent(&src[i]) : 0ull;
      }
#pragma unroll
      for (int u = 0; u < PAB; ++u) {
        const bool in = it + (uint64_t)u * PL + tid < n;
        bool newo = false, news = false;
        uint64_t okey = 0;
        if (in) {
          if (key[u] & DIRECT) {
            okey = key[u] & ~DIRECT;
            newo = set_insert(r.O, r.tmask, okey, r.ep, &ctl->flags);
          } else {
            news = set_insert(r.S, r.tmask, key[u], r.ep, &ctl->flags);
            if (news && (key[u] & a.bitj)) {
              okey = key[u] & ~a.bitj;
              newo = set_insert(r.O, r.tmask, okey, r.ep, &ctl->flags);
            }
          }
        }
        expl += news;
        nl[u] = news && !(key[u] & a.bitj);
        listed += nl[u];
        // OUT list append: one global atomic per wave
        const unsigned long long m = __ballot(newo);
        if (m) {
          const int leader = __ffsll((long long)m) - 1;
          unsigned long long base = 0;
          if (lane == leader) base = atomicAdd(out_count, (unsigned long long)__popcll(m));
          base = __shfl(base, leader, 64);
          if (newo) {
            const unsigned long long q = base + __popcll(m & ((1ull << lane) - 1));
            if (q < r.list_cap) st_agent(&r.outl[q], okey);
            else atomicOr(&ctl->flags, (unsigned long long)PF_OVERFLOW);
          }
        }
      }
      emit<PAB>(a, key, nl, r.wd, mmask, dst, r.seg_cap, &ctl->lvl[(l + 1) % 3], ctl, s_w, &s_base);
    }
    if (!run_sync(r, &s_abort)) return;
  }
  // every level counter is zero again for the next step (lvl[(l + 2) % 3] held level l-1's)
  if (lead) {
    st_agent(&ctl->lvl[(l + 2) % 3], 0ull);
    r.flog[r.flog_i] = ld_agent(out_count);
    atomicAdd(&ctl->levels, (unsigned long long)(l + 1));
    atomicAdd(&ctl->listed, (unsigned long long)nf);
  }
  for (int off = 32; off > 0; off >>= 1) {
    expl += __shfl_down(expl, off, 64);
    listed += __shfl_down(listed, off, 64);
  }
  if (lane == 0 && expl) atomicAdd(&ctl->explored, expl);
  if (lane == 0 && listed) atomicAdd(&ctl->listed, listed);
}

// ---- lc_part_run, flow form (world 1, the default): no BFS levels. A step's closure is a
// set (explored = |S|, the OUT set), so the order its configs are found in does not matter and
// the level barrier (every candidate of level l absorbed before level l + 1 is expanded) is not
// needed. Each workgroup works through ITEMS (configs to expand): its share of the frontier F,
// then the new configs its own passes found (an LDS ring: no global claim, no hand-off
// latency), then, when both are empty, the global overflow queue Q that children go to when a
// ring is full (tagged words: [epoch | key], polled by the consumer). A pass takes up to FL
// items with 1, 2 or 3 threads per item (flow_ft: few items at hand, several threads split an
// item's candidate batches) and expands them FB candidates per thread at a time: the S probes and, for
// candidates holding the returning op j, the O probes of their images are issued together
// (every j-holding candidate is in S, new or not, so its image belongs to OUT either way), then
// the CASes together. New OUT configs collect in an LDS buffer flushed once per step. The step
// ends when R = (children produced) - (items completed), summed over every pass, reaches
// -|F|: each workgroup adds its pass's net once, in order, after the pass, and a child pushed
// to Q is counted BEFORE it is published, so R never reaches -|F| while an item is pending.
// Then ONE grid barrier. One cooperative launch runs a chunk of steps; the host reads the
// per-step OUT counts once per chunk. Same verdict, failing step and explored count as the
// level kernel and the oracle.
constexpr int FL = 512;   // threads per workgroup
constexpr int FB = 8;     // candidates per thread per insert batch
// threads per item, per pass: 3 when few items are at hand (thread h of an item takes its
// candidate batches h, h + 3, ...: one batch each up to 24 pending ops, so the pass is one
// round of probes and one of CASes), 1 when a pass can fill every thread with an item
__device__ __forceinline__ unsigned flow_ft(unsigned long long avail) {
  return avail > 2 * (FL / 3) ? 1u : avail > FL / 3 ? 2u : 3u;
}
constexpr int LQ = 4096;  // LDS item ring per workgroup (entries)
constexpr int LO = 2048;  // LDS OUT buffer per workgroup (entries)
constexpr uint64_t KEY_MASK = (1ull << KEY_BITS) - 1;

// one step's counters, each on its own 128-B line (three sets rotate over the steps: step t
// works on sets[t % 3], reads |F| from sets[(t + 2) % 3].outc, resets sets[(t + 1) % 3])
struct FlowSet {
  unsigned long long head, pad0[15];  // overflow queue Q: claimed
  unsigned long long tail, pad1[15];  //   reserved
  unsigned long long outc, pad2[15];  // OUT list entries
  long long R, pad3[15];              // children produced - items completed
};

struct FlowArgs {
  uint64_t* S;
  uint64_t* O;
  uint64_t tmask;
  uint64_t* L[2];  // frontier / OUT lists: step t reads L[t & 1], writes L[(t + 1) & 1]
  uint64_t list_cap;
  uint64_t* Q;
  uint64_t qcap;
  const StepArgs* steps;  // [t1 - t0]; StepArgs.pad = the step's set epoch
  FlowSet* sets;
  PartCtl* ctl;
  PartBar* bar;
  unsigned long long* flog;  // OUT count per step of the chunk
  int64_t t0, t1;
  uint32_t nwg;
  int32_t mask_bits;
};

__device__ __forceinline__ bool grid_sync(PartBar* bar, uint32_t nwg, PartCtl* ctl, int* s_abort) {
  RunArgs r{};
  r.bar = bar;
  r.nwg = nwg;
  r.ctl = ctl;
  return run_sync(r, s_abort);
}

// Insert N keys (key[u] & ~clr where has[u]) into set T at once: every probe load, then
// every CAS, in flight together; a collision (another key of this epoch in the home word, or a
// lost race) falls back to set_insert's probe run. isnew[u] = a key this call added.
template <int N>
__device__ __forceinline__ void insert_batch(uint64_t* T, uint64_t tmask, const uint64_t* key, uint64_t clr,
                                             const bool* has, uint64_t ep, unsigned long long* flags, bool* isnew) {
  uint64_t cur[N];
#pragma unroll
  for (int u = 0; u < N; ++u) cur[u] = has[u] ? ld_agent(&T[mix64(key[u] & ~clr) & tmask]) : 0ull;
  uint64_t old[N];
#pragma unroll
  for (int u = 0; u < N; ++u) {
    const uint64_t v = (ep << KEY_BITS) | (key[u] & ~clr);
    const bool tried = has[u] && cur[u] != v && (cur[u] >> KEY_BITS) != ep;
    old[u] = tried ? atomicCAS((unsigned long long*)&T[mix64(key[u] & ~clr) & tmask], (unsigned long long)cur[u],
                               (unsigned long long)v)
                   : ~cur[u];  // (never equal to cur or v: "not tried")
  }
#pragma unroll
  for (int u = 0; u < N; ++u) {
    const uint64_t v = (ep << KEY_BITS) | (key[u] & ~clr);
    isnew[u] = false;
    if (!has[u] || cur[u] == v) continue;
    if (old[u] == cur[u]) isnew[u] = true;
    else if (old[u] != v) isnew[u] = set_insert(T, tmask, key[u] & ~clr, ep, flags) != 0;
  }
}

// S and O inserts of one batch at once: key[u] into S where has[u], key[u] & ~clr into O where
// hj[u]; every probe load of both, then every CAS of both, in flight together.
template <int N>
__device__ __forceinline__ void insert_batch2(uint64_t* S, uint64_t* O, uint64_t tmask, const uint64_t* key,
                                              uint64_t clr, const bool* has, const bool* hj, uint64_t ep,
                                              unsigned long long* flags, bool* snew, bool* onew) {
  uint64_t cs_[N], co[N];
#pragma unroll
  for (int u = 0; u < N; ++u) {
    cs_[u] = has[u] ? ld_agent(&S[mix64(key[u]) & tmask]) : 0ull;
    co[u] = hj[u] ? ld_agent(&O[mix64(key[u] & ~clr) & tmask]) : 0ull;
  }
  uint64_t os[N], oo[N];
#pragma unroll
  for (int u = 0; u < N; ++u) {
    const uint64_t vs = (ep << KEY_BITS) | key[u], vo = (ep << KEY_BITS) | (key[u] & ~clr);
    const bool ts = has[u] && cs_[u] != vs && (cs_[u] >> KEY_BITS) != ep;
    const bool to = hj[u] && co[u] != vo && (co[u] >> KEY_BITS) != ep;
    os[u] = ts ? atomicCAS((unsigned long long*)&S[mix64(key[u]) & tmask], (unsigned long long)cs_[u],
                           (unsigned long long)vs)
               : ~cs_[u];
    oo[u] = to ? atomicCAS((unsigned long long*)&O[mix64(key[u] & ~clr) & tmask], (unsigned long long)co[u],
                           (unsigned long long)vo)
               : ~co[u];
  }
#pragma unroll
  for (int u = 0; u < N; ++u) {
    const uint64_t vs = (ep << KEY_BITS) | key[u], vo = (ep << KEY_BITS) | (key[u] & ~clr);
    snew[u] = onew[u] = false;
    if (has[u] && cs_[u] != vs) {
      if (os[u] == cs_[u]) snew[u] = true;
      else if (os[u] != vs) snew[u] = set_insert(S, tmask, key[u], ep, flags) != 0;
    }
    if (hj[u] && co[u] != vo) {
      if (oo[u] == co[u]) onew[u] = true;
      else if (oo[u] != vo) onew[u] = set_insert(O, tmask, key[u] & ~clr, ep, flags) != 0;
    }
  }
}

// Wave-aggregated append of each lane's n items (vals[0..n)) at *counter: one atomic per wave.
// Returns false where an item fell beyond cap (the caller raised PF_OVERFLOW).
template <int N>
__device__ __forceinline__ bool wave_append(unsigned long long* counter, uint64_t* dst, uint64_t cap,
                                            const uint64_t* vals, uint64_t clr, const bool* keep, uint64_t tag) {
  uint32_t n = 0;
#pragma unroll
  for (int u = 0; u < N; ++u) n += keep[u];
  const int lane = __lane_id();
  uint32_t x = n;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  const uint32_t tot = __shfl(x, 63, 64);
  if (tot == 0) return true;
  unsigned long long base = 0;
  if (lane == 0) base = atomicAdd(counter, (unsigned long long)tot);
  base = __shfl(base, 0, 64);
  uint64_t pos = base + (x - n);
  bool ok = true;
#pragma unroll
  for (int u = 0; u < N; ++u)
    if (keep[u]) {
      if (pos < cap) st_agent(&dst[pos], (vals[u] & ~clr) | tag);
      else ok = false;
      ++pos;
    }
  return ok;
}

__global__ void __launch_bounds__(FL) part_flow_kernel(FlowArgs r) {
  __shared__ uint64_t s_q[LQ];  // item ring
  __shared__ uint64_t s_o[LO];  // OUT buffer
  __shared__ uint64_t s_ops[PS_MAX];
  __shared__ unsigned s_qh, s_qt, s_push, s_on, s_n, s_src, s_ring, s_ft;
  __shared__ unsigned long long s_f, s_fend, s_g0, s_base;
  __shared__ int s_abort, s_state;
  PartCtl* const ctl = r.ctl;
  // an earlier chunk overflowed or aborted: nothing more to do (set by earlier launches)
  if (ld_agent(&ctl->flags) & (PF_OVERFLOW | PF_STAGE | PF_ABORT)) return;
  const int tid = threadIdx.x;
  const bool lead = blockIdx.x == 0 && tid == 0;
  const uint64_t mmask = (1ull << r.mask_bits) - 1;
  unsigned long long expl = 0, listed = 0, cand = 0;
  for (int64_t t = r.t0; t < r.t1; ++t) {
    const StepArgs& a = r.steps[t - r.t0];
    FlowSet* const cs = &r.sets[t % 3];
    FlowSet* const ps = &r.sets[(t + 2) % 3];
    // |F|: the previous step's OUT count, which counts the appends that overflowed the list too
    // (PF_OVERFLOW is set then and the host discards the run): never read beyond the list
    const uint64_t nf = min<uint64_t>(ld_agent(&ps->outc), r.list_cap);
    if (nf == 0 && t > 0) break;  // step t - 1 returned an empty frontier (every workgroup sees it)
    if (lead) {  // the next step's counters (last used by step t - 2, read by step t - 1 at its start)
      FlowSet* const nx = &r.sets[(t + 1) % 3];
      st_agent(&nx->head, 0ull);
      st_agent(&nx->tail, 0ull);
      st_agent(&nx->outc, 0ull);
      st_agent(&nx->R, 0ll);
    }
    if (tid < PS_MAX) s_ops[tid] = a.ops[tid];
    if (tid == 0) {  // this workgroup's share of F, an empty ring and OUT buffer
      s_f = nf * blockIdx.x / r.nwg;
      s_fend = nf * (blockIdx.x + 1) / r.nwg;
      s_qh = s_qt = 0;
      s_on = 0;
    }
    const uint64_t live = a.live, bitj = a.bitj;
    const uint64_t ep = (uint64_t)(uint32_t)a.pad;
    const uint64_t tag = ep << KEY_BITS;
    const int wd = live ? 64 - __builtin_clzll(live) : 0;
    const uint64_t* const F = r.L[t & 1];
    uint64_t* const OUT = r.L[(t + 1) & 1];
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
    for (;;) {
      // ---- take up to FL items: F share, then the ring, then the overflow queue
      if (tid == 0) {
        s_state = 0;
        s_push = 0;
        s_ring = 0;
        if (s_f < s_fend) {
          s_src = 0;
          s_ft = flow_ft(s_fend - s_f);
          s_n = (unsigned)min<uint64_t>(FL / s_ft, s_fend - s_f);
        } else if (s_qt != s_qh) {
          s_src = 1;
          s_ft = flow_ft(s_qt - s_qh);
          s_n = min(FL / s_ft, s_qt - s_qh);
        } else {
          s_src = 2;
          s_n = 0;
          for (long k = 0;; ++k) {  // idle: claim from Q, or see the step finished
            const unsigned long long h = ld_agent(&cs->head), tl = ld_agent(&cs->tail);
            if (tl > h) {
              const unsigned ft = flow_ft(tl - h);
              const unsigned m = (unsigned)min<unsigned long long>(FL / ft, tl - h);
              if (atomicCAS(&cs->head, h, h + m) == h) {
                s_ft = ft;
                s_g0 = h;
                s_n = m;
                break;
              }
              continue;
            }
            if (ld_agent(&cs->R) == -(long long)nf) {
              s_state = 1;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
            if ((k & 255) == 255 && (__builtin_amdgcn_s_memrealtime() - t_start > 2000000000ull ||
                                     (ld_agent(&ctl->flags) & PF_ABORT))) {
              atomicOr(&ctl->flags, (unsigned long long)PF_ABORT);
              s_state = 2;
              break;
            }
          }
        }
      }
      __syncthreads();
      if (s_state) break;
      const unsigned n = s_n, src = s_src;
      const unsigned qh0 = s_qh, qt0 = s_qt;
      const unsigned long long f0 = s_f, g0 = s_g0;
      uint64_t c = 0;
      bool item = false;
      const unsigned ft = s_ft;
      const unsigned it = (unsigned)tid / ft, half = (unsigned)tid % ft;  // this thread's item, its part
      if (it < n) {
        if (src == 0) {  // written in this launch by the previous step: read past the caches
          c = ld_agent(&F[f0 + it]), item = true;
        } else if (src == 1) {
          c = s_q[(qh0 + it) & (LQ - 1)], item = true;
        } else if (g0 + it < r.qcap) {
          const uint64_t* q = &r.Q[g0 + it];
          uint64_t wv = ld_agent(q);
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          for (long k = 1; (wv & ~KEY_MASK) != tag; ++k) {  // reserved, not yet written
            __builtin_amdgcn_s_sleep(1);
            wv = ld_agent(q);
            if ((k & 255) == 0 && __builtin_amdgcn_s_memrealtime() - t0 > 2000000000ull) {
              atomicOr(&ctl->flags, (unsigned long long)PF_ABORT);
              break;
            }
          }
          c = wv & KEY_MASK, item = (wv & ~KEY_MASK) == tag;
        }  // else: beyond Q (PF_OVERFLOW was raised by its producer): dropped
      }
      __syncthreads();  // every thread has its item: the ring slots may be refilled
      if (tid == 0) {
        if (src == 0) s_f = f0 + n;
        else if (src == 1) s_qh = qh0 + n;
      }
      // ring slots free for this pass's children (the same value in every thread): children
      // reserve positions in order, so the ones that fit are a prefix of the reservations
      const unsigned qfree = (unsigned)LQ - (qt0 - (src == 1 ? qh0 + n : qh0));
      listed += item && half == 0;
      // OUT configs into the LDS buffer (the global list once it is full)
      auto emit_out = [&](uint64_t k, bool keep) {
        if (!keep) return;
        const unsigned i = atomicAdd(&s_on, 1u);
        if (i < (unsigned)LO) {
          s_o[i] = k;
        } else {
          const unsigned long long q = atomicAdd(&cs->outc, 1ull);
          if (q < r.list_cap) st_agent(&OUT[q], k);
          else atomicOr(&ctl->flags, (unsigned long long)PF_OVERFLOW);
        }
      };
      // a config holding the returning op (frontier only): its image goes to OUT
      {
        const bool dret[1] = {item && half == 0 && (c & bitj) != 0};
        bool dnew[1] = {false};
        if (__any(dret[0])) insert_batch<1>(r.O, r.tmask, &c, bitj, dret, ep, &ctl->flags, dnew);
        emit_out(c & ~bitj, dnew[0]);
      }
      // expand: each pending op not in c's mask, FB candidates at a time
      const bool expand = item && !(c & bitj);
      const int64_t st = (int64_t)(c >> r.mask_bits);
      unsigned ringc = 0;
      for (int b0 = 0; b0 < wd; b0 += (int)ft * FB) {  // (a wave-uniform trip count)
        const int k0 = b0 + (int)half * FB;
        uint64_t ks[FB];
        bool hs[FB], hj[FB], nw[FB], on[FB];
        bool anyh = false;
#pragma unroll
        for (int u = 0; u < FB; ++u) {
          const int k = k0 + u;
          hs[u] = false;
          ks[u] = 0;
          if (expand && k < wd && ((live >> k) & 1) && !((c >> k) & 1)) {
            const uint64_t op = s_ops[k];
            const int32_t ea = (int32_t)(uint32_t)op, nb = (int32_t)(uint32_t)(op >> 32);
            if (ea == -1 || ea == st) {
              const uint64_t ns = nb < 0 ? (uint64_t)st : (uint64_t)nb;
              ks[u] = (ns << r.mask_bits) | (c & mmask) | (1ull << k);
              hs[u] = true;
            }
          }
          hj[u] = hs[u] && (ks[u] & bitj);
          cand += hs[u];
          anyh |= hs[u];
        }
        if (!__any(anyh)) continue;
        // S and O together: a j-holding candidate is in S (new or not), so its image is in OUT
        insert_batch2<FB>(r.S, r.O, r.tmask, ks, bitj, hs, hj, ep, &ctl->flags, nw, on);
        bool toq[FB];
        unsigned nc = 0;
#pragma unroll
        for (int u = 0; u < FB; ++u) {
          expl += nw[u];
          toq[u] = nw[u] && !hj[u];
          nc += toq[u];
          emit_out(ks[u] & ~bitj, on[u]);
        }
        // new configs without j are this step's next items: the ring, or Q when it is full
        unsigned base = 0;
        if (nc) base = atomicAdd(&s_push, nc);
        const bool fits = base + nc <= qfree;
        if (nc && fits) {
          unsigned pos = qt0 + base;
#pragma unroll
          for (int u = 0; u < FB; ++u)
            if (toq[u]) s_q[(pos++) & (LQ - 1)] = ks[u];
          ringc += nc;
        }
        const bool ov = nc && !fits;
        if (__any(ov)) {  // count them in R first (returned), then reserve and publish
          const unsigned nl = ov ? nc : 0;
          unsigned x = nl;
          const int lane = __lane_id();
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) {
            const unsigned y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
          }
          const unsigned tot = __shfl(x, 63, 64);
          unsigned long long gb = 0;
          if (lane == 0) {
            (void)atomicAdd((unsigned long long*)&cs->R, (unsigned long long)tot);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            gb = atomicAdd(&cs->tail, (unsigned long long)tot);
          }
          gb = __shfl(gb, 0, 64);
          uint64_t pos = gb + (x - nl);
          if (ov)
#pragma unroll
            for (int u = 0; u < FB; ++u)
              if (toq[u]) {
                if (pos < r.qcap) st_agent(&r.Q[pos], ks[u] | tag);
                else atomicOr(&ctl->flags, (unsigned long long)PF_OVERFLOW);
                ++pos;
              }
        }
      }
      // the pass's net: ring children - items completed, once, after the pass (by one lane:
      // a ring child's +1 and its later -1 are that lane's atomics on one word, in order)
      unsigned rs = ringc;
      for (int off = 32; off > 0; off >>= 1) rs += __shfl_down(rs, off, 64);
      if (__lane_id() == 0 && rs) atomicAdd(&s_ring, rs);
      __syncthreads();
      if (tid == 0) {
        s_qt = qt0 + s_ring;
        atomicAdd((unsigned long long*)&cs->R, (unsigned long long)((long long)s_ring - (long long)n));
      }
      __syncthreads();
    }
    // flush the OUT buffer, then the step's grid barrier
    const unsigned no = min(s_on, (unsigned)LO);
    if (tid == 0 && no) s_base = atomicAdd(&cs->outc, (unsigned long long)no);
    __syncthreads();
    for (unsigned i = tid; i < no; i += FL) {
      const unsigned long long q = s_base + i;
      if (q < r.list_cap) st_agent(&OUT[q], s_o[i]);
      else atomicOr(&ctl->flags, (unsigned long long)PF_OVERFLOW);
    }
    if (!grid_sync(r.bar, r.nwg, ctl, &s_abort)) return;
    if (lead) r.flog[t - r.t0] = ld_agent(&cs->outc);
  }
  for (int off = 32; off > 0; off >>= 1) {
    expl += __shfl_down(expl, off, 64);
    listed += __shfl_down(listed, off, 64);
    cand += __shfl_down(cand, off, 64);
  }
  if (__lane_id() == 0) {
    if (expl) atomicAdd(&ctl->explored, expl);
    if (listed) atomicAdd(&ctl->listed, listed);
    if (cand) atomicAdd(&ctl->cand, cand);
  }
}

void set_msg(char* err, int32_t len, const char* fmt, ...) {
  if (!err || len <= 0) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(err, (size_t)len, fmt, ap);
  va_end(ap);
}

int bits_of(int64_t n) {
  int b = 0;
  while ((1ll << b) < n) ++b;
  return b;
}

}  // namespace
}  // namespace lc

using namespace lc;

struct lc_part {
  int device = 0, rank = 0, world = 1;
  Encoded enc;
  int mask_bits = 0, state_bits = 0;
  int slog = 0;               // S / OUT tables: 2^slog words
  uint64_t list_cap = 0;      // level lists, F, OUT: entries
  uint64_t seg_cap = 0;       // staging per destination
  uint64_t* S = nullptr;
  uint64_t* O = nullptr;
  uint64_t* F = nullptr;      // frontier (this rank's part)
  uint64_t* OUTL = nullptr;   // OUT list (next F)
  uint64_t* Lb[2] = {nullptr, nullptr};
  uint64_t* stage = nullptr;
  PartCtl* ctl = nullptr;
  PartCtl* hctl = nullptr;    // pinned host copy
  int grid = 1024;
  // lc_part_run (world 1): second stage buffer, barrier words, per-step OUT counts
  uint64_t* stage2 = nullptr;
  PartBar* bar = nullptr;
  unsigned long long* flog = nullptr;
  unsigned long long* hflog = nullptr;
  int run_grid = 0;
  uint64_t run_cap = 0;       // entries of stage and stage2 as lc_part_run sized them
  // lc_part_run, flow form: queue counters, item queue, per-chunk step arguments
  FlowSet* fsets = nullptr;
  uint64_t* Q = nullptr;
  StepArgs* dsteps = nullptr;
  StepArgs* hsteps = nullptr;
  int flow_grid = 0;
  // measurement: HIP events around each kernel (on the caller's stream), algorithmic bytes
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  bool absorb_pending = false;
  double kernel_ms = 0, alg_bytes = 0;
  int sp = 0;          // step parity: OUT count = ctl->oc[sp], F count = ctl->oc[sp ^ 1]
  uint64_t ub = 1;      // upper bound of the next expand's list (grid sizing): |F| or the last absorb's n
  // step state
  int64_t t = -1;
  uint32_t epoch = 0;
  StepArgs args{};
  int level = 0, cur = 0;     // level lists: read list Lb[cur] at levels >= 1
  uint32_t wd = 0;
  uint64_t live = 0;
  std::string last_error;

  ~lc_part() {
    for (void* q : {(void*)S, (void*)O, (void*)F, (void*)OUTL, (void*)Lb[0], (void*)Lb[1], (void*)stage,
                    (void*)ctl, (void*)stage2, (void*)bar, (void*)flog, (void*)fsets, (void*)Q, (void*)dsteps})
      if (q) (void)hipFree(q);
    if (hsteps) (void)hipHostFree(hsteps);
    if (hctl) (void)hipHostFree(hctl);
    if (hflog) (void)hipHostFree(hflog);
    for (hipEvent_t e : ev)
      if (e) (void)hipEventDestroy(e);
  }
};

namespace {

#define PT_TRY(expr)                                                          \
  do {                                                                        \
    hipError_t e_ = (expr);                                                   \
    if (e_ != hipSuccess) {                                                   \
      set_msg(err, err_len, "%s: %s", #expr, hipGetErrorString(e_));          \
      return e_ == hipErrorOutOfMemory ? LC_E_MEMORY : LC_E_DEVICE;           \
    }                                                                         \
  } while (0)

int part_read_ctl(lc_part* p, hipStream_t s, char* err, int32_t err_len) {
  PT_TRY(hipMemcpyAsync(p->hctl, p->ctl, sizeof(PartCtl), hipMemcpyDeviceToHost, s));
  PT_TRY(hipStreamSynchronize(s));
  if (p->absorb_pending) {  // the last absorb's kernel time
    float ms = 0;
    if (hipEventElapsedTime(&ms, p->ev[2], p->ev[3]) == hipSuccess) p->kernel_ms += ms;
    p->absorb_pending = false;
  }
  return 0;
}

// step t's invocations into the step arguments; a fresh set epoch (both sets cleared on wrap)
int part_begin(lc_part* p, int64_t t, hipStream_t s, char* err, int32_t err_len) {
  const Encoded& e = p->enc;
  for (int64_t q = e.inv_off[t]; q < e.inv_off[t + 1]; ++q) {
    const int k = e.inv_slot[q];
    p->args.ops[k] = ((uint64_t)(uint32_t)(int32_t)e.inv_b[q] << 32) | (uint64_t)(uint32_t)(int32_t)e.inv_a[q];
    p->live |= 1ull << k;
  }
  const int j = e.step_slot[t];
  p->args.live = p->live;
  p->args.bitj = 1ull << j;
  p->args.mask_bits = p->mask_bits;
  p->args.world = p->world;
  p->args.rank = p->rank;
  p->wd = (uint32_t)(64 - __builtin_clzll(p->live));
  if (++p->epoch > EPOCH_MAX) {  // epochs wrapped: clear both sets (and the flow queue) once
    PT_TRY(hipMemsetAsync(p->S, 0, sizeof(uint64_t) << p->slog, s));
    PT_TRY(hipMemsetAsync(p->O, 0, sizeof(uint64_t) << p->slog, s));
    if (p->Q) PT_TRY(hipMemsetAsync(p->Q, 0, sizeof(uint64_t) * p->list_cap, s));
    p->epoch = 1;
  }
  p->t = t;
  return 0;
}

// lc_part_run's flow form (part_flow_kernel): one cooperative launch per chunk of steps
int part_run_flow(lc_part* p, hipStream_t s, int64_t ns, int64_t* out4, char* err, int32_t err_len) {
  constexpr int64_t CHUNK = 2048;
  if (!p->fsets) {
    int occ = 0;
    PT_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, part_flow_kernel, FL, 0));
    hipDeviceProp_t prop;
    PT_TRY(hipGetDeviceProperties(&prop, p->device));
    if (occ < 1) {
      set_msg(err, err_len, "part_flow_kernel does not fit a CU");
      return LC_E_DEVICE;
    }
    p->flow_grid = prop.multiProcessorCount;  // one workgroup per CU: co-resident
    if (const char* e = getenv("LC_PART_GRID"))
      if (atoi(e) >= 1 && atoi(e) < p->flow_grid) p->flow_grid = atoi(e);
    if (!p->bar) {
      PT_TRY(hipMalloc(&p->bar, sizeof(PartBar)));
      PT_TRY(hipMemset(p->bar, 0, sizeof(PartBar)));
    }
    if (!p->flog) {
      PT_TRY(hipMalloc(&p->flog, CHUNK * sizeof(unsigned long long)));
      PT_TRY(hipHostMalloc(&p->hflog, CHUNK * sizeof(unsigned long long), hipHostMallocDefault));
    }
    PT_TRY(hipMalloc(&p->fsets, 3 * sizeof(FlowSet)));
    PT_TRY(hipMalloc(&p->Q, sizeof(uint64_t) * p->list_cap));
    PT_TRY(hipMemset(p->Q, 0, sizeof(uint64_t) * p->list_cap));
    PT_TRY(hipMalloc(&p->dsteps, CHUNK * sizeof(StepArgs)));
    PT_TRY(hipHostMalloc(&p->hsteps, CHUNK * sizeof(StepArgs), hipHostMallocDefault));
  }
  // step 0 reads |F| = 1 (the initial config, key 0, in p->F) from sets[2]
  PT_TRY(hipMemsetAsync(p->fsets, 0, 3 * sizeof(FlowSet), s));
  const unsigned long long one = 1;
  PT_TRY(hipMemcpyAsync(&p->fsets[2].outc, &one, sizeof one, hipMemcpyHostToDevice, s));
  uint64_t* const L0 = p->F;
  uint64_t* const L1 = p->OUTL;
  PT_TRY(hipEventRecord(p->ev[0], s));
  int64_t t = 0, fail = -1;
  uint64_t flags = 0;
  while (t < ns && fail < 0) {
    const int64_t c0 = t, c1 = std::min(ns, t + CHUNK);
    for (int64_t u = c0; u < c1; ++u) {
      int rc = part_begin(p, u, s, err, err_len);
      if (rc) return rc;
      p->hsteps[u - c0] = p->args;
      p->hsteps[u - c0].pad = (int32_t)p->epoch;
      p->live &= ~p->args.bitj;
    }
    PT_TRY(hipMemcpyAsync(p->dsteps, p->hsteps, sizeof(StepArgs) * (size_t)(c1 - c0), hipMemcpyHostToDevice, s));
    FlowArgs fa{};
    fa.S = p->S;
    fa.O = p->O;
    fa.tmask = (1ull << p->slog) - 1;
    fa.L[0] = L0;
    fa.L[1] = L1;
    fa.list_cap = p->list_cap;
    fa.Q = p->Q;
    fa.qcap = p->list_cap;
    fa.steps = p->dsteps;
    fa.sets = p->fsets;
    fa.ctl = p->ctl;
    fa.bar = p->bar;
    fa.flog = p->flog;
    fa.t0 = c0;
    fa.t1 = c1;
    fa.nwg = (uint32_t)p->flow_grid;
    fa.mask_bits = p->mask_bits;
    void* kargs[] = {(void*)&fa};
    PT_TRY(hipLaunchCooperativeKernel((const void*)part_flow_kernel, dim3(p->flow_grid), dim3(FL), kargs, 0, s));
    PT_TRY(hipMemcpyAsync(p->hflog, p->flog, sizeof(unsigned long long) * (size_t)(c1 - c0), hipMemcpyDeviceToHost,
                          s));
    int rc = part_read_ctl(p, s, err, err_len);
    if (rc) return rc;
    flags = p->hctl->flags;
    t = c1;
    if (flags) break;
    for (int64_t i = 0; i < c1 - c0; ++i)
      if (p->hflog[i] == 0) {
        fail = c0 + i;
        break;
      }
  }
  PT_TRY(hipEventRecord(p->ev[1], s));
  int rc = part_read_ctl(p, s, err, err_len);
  if (rc) return rc;
  flags = p->hctl->flags;
  float ms = 0;
  if (hipEventElapsedTime(&ms, p->ev[0], p->ev[1]) == hipSuccess) p->kernel_ms += ms;
  if (flags & PF_ABORT) {
    set_msg(err, err_len, "part_flow_kernel: watchdog expired");
    return LC_E_DEVICE;
  }
  if (flags & (PF_OVERFLOW | PF_STAGE)) {
    set_msg(err, err_len, "frontier exceeded the partition capacity (LC_H_CAPACITY)");
    return LC_H_CAPACITY;
  }
  // read each item (8 B), probe + CAS each candidate (16 B), write each new
  // config (8 B, at most one per candidate)
  p->alg_bytes += 8.0 * (double)p->hctl->listed + 24.0 * (double)p->hctl->cand;
  out4[0] = fail >= 0 ? fail + 1 : t;
  out4[1] = fail;
  out4[2] = 0;  // no BFS levels in the flow form
  out4[3] = (int64_t)p->hctl->explored;
  return 0;
}

}  // namespace

extern "C" {

int32_t lc_part_create(int32_t device, int32_t model_kind, int64_t init_value, int64_t n,
                       const int64_t* index, const int32_t* process, const int8_t* type, const int8_t* f,
                       const int64_t* v0, const int64_t* v1, const int8_t* vflags, int32_t rank,
                       int32_t world, int32_t capacity_log2, lc_part** out, char* err, int32_t err_len) {
  if (!out) return LC_E_ARG;
  *out = nullptr;
  if (model_kind != LC_MODEL_CAS_REGISTER) {
    set_msg(err, err_len, "the partitioned search runs cas-register histories (counter: lc_check / bounds)");
    return LC_E_ARG;
  }
  if (world < 1 || world > PW_MAX || rank < 0 || rank >= world) {
    set_msg(err, err_len, "rank %d / world %d out of range (world <= %d)", rank, world, PW_MAX);
    return LC_E_ARG;
  }
  if (n < 0 || (n > 0 && (!process || !type || !f || !v0 || !v1 || !vflags))) {
    set_msg(err, err_len, "bad history arrays");
    return LC_E_ARG;
  }
  if (capacity_log2 <= 0) capacity_log2 = 22;
  if (capacity_log2 < 10 || capacity_log2 > 26) {
    set_msg(err, err_len, "capacity_log2 %d out of [10, 26]", capacity_log2);
    return LC_E_ARG;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    set_msg(err, err_len, "no HIP device visible (the checker has no CPU fallback)");
    return LC_E_DEVICE;
  }
  if (device < 0 || device >= ndev) {
    set_msg(err, err_len, "device %d out of range", device);
    return LC_E_ARG;
  }
  auto p = std::make_unique<lc_part>();
  p->device = device;
  p->rank = rank;
  p->world = world;
  const int64_t off[2] = {0, n};
  HistArrays a{n, index, process, type, f, v0, v1, vflags};
  encode(model_kind, init_value, 1, off, a, p->enc);
  p->mask_bits = std::max(1, p->enc.live_max[0]);
  p->state_bits = bits_of(p->enc.n_states[0]);
  if (!p->enc.err[0] && (p->mask_bits > PS_MAX || p->mask_bits + p->state_bits > KEY_BITS)) {
    p->enc.err[0] = LC_H_WIDE;
    p->enc.errmsg[0] = "pending ops + state bits exceed the 48-bit partitioned key";
  }
  PT_TRY(hipSetDevice(device));
  p->slog = capacity_log2 + 1;  // tables at most half full
  p->list_cap = 1ull << capacity_log2;
  p->seg_cap = std::max<uint64_t>(1024, (p->list_cap >> 2) / (uint64_t)world);
  const size_t tb = sizeof(uint64_t) << p->slog, lb = sizeof(uint64_t) * p->list_cap;
  PT_TRY(hipMalloc(&p->S, tb));
  PT_TRY(hipMalloc(&p->O, tb));
  PT_TRY(hipMemset(p->S, 0, tb));
  PT_TRY(hipMemset(p->O, 0, tb));
  PT_TRY(hipMalloc(&p->F, lb));
  PT_TRY(hipMalloc(&p->OUTL, lb));
  PT_TRY(hipMalloc(&p->Lb[0], lb));
  PT_TRY(hipMalloc(&p->Lb[1], lb));
  PT_TRY(hipMalloc(&p->stage, sizeof(uint64_t) * p->seg_cap * (uint64_t)world));
  PT_TRY(hipMalloc(&p->ctl, sizeof(PartCtl)));
  PT_TRY(hipHostMalloc(&p->hctl, sizeof(PartCtl), hipHostMallocDefault));
  PT_TRY(hipMemset(p->ctl, 0, sizeof(PartCtl)));
  hipDeviceProp_t prop;
  PT_TRY(hipGetDeviceProperties(&prop, device));
  p->grid = prop.multiProcessorCount * 8;
  for (hipEvent_t& e : p->ev) PT_TRY(hipEventCreate(&e));
  // the initial config (nil, nothing linearized) = key 0 lives on rank 0
  if (rank == 0) {
    const uint64_t zero = 0;
    const unsigned long long one = 1;
    PT_TRY(hipMemcpy(p->F, &zero, sizeof zero, hipMemcpyHostToDevice));
    PT_TRY(hipMemcpy(&p->ctl->oc[1], &one, sizeof one, hipMemcpyHostToDevice));
  }
  *out = p.release();
  return 0;
}

/* info[0] = RETURN steps, [1] history error (LC_H_*), [2] mask bits, [3] state bits,
 * [4] invocations (ops), [5] list capacity, [6] kernel time so far (ns, HIP events),
 * [7] algorithmic HBM bytes so far */
int32_t lc_part_info(lc_part* p, int64_t* info, int32_t n) {
  if (!p || !info) return LC_E_ARG;
  const int64_t v[8] = {p->enc.n_steps(0), p->enc.err[0], p->mask_bits, p->state_bits, p->enc.n_ops[0],
                        (int64_t)p->list_cap, (int64_t)(p->kernel_ms * 1e6), (int64_t)p->alg_bytes};
  for (int i = 0; i < n && i < 8; ++i) info[i] = v[i];
  return 0;
}

/* Begin RETURN step t (steps run in order 0, 1, ...): applies its invocations and makes the
 * frontier F the level-0 list. */
int32_t lc_part_step_begin(lc_part* p, int64_t t, void* stream, char* err, int32_t err_len) {
  if (!p || t != p->t + 1 || t >= p->enc.n_steps(0) || p->enc.err[0]) {
    set_msg(err, err_len, "step %lld out of order or history not searchable", (long long)t);
    return LC_E_ARG;
  }
  PT_TRY(hipSetDevice(p->device));
  int rc = part_begin(p, t, (hipStream_t)stream, err, err_len);
  if (rc) return rc;
  p->level = 0;
  p->cur = 0;
  return 0;
}

/* Expand this rank's current level list. send_counts[d] = candidates for rank d. */
int32_t lc_part_expand(lc_part* p, void* stream, int64_t* send_counts, char* err, int32_t err_len) {
  if (!p || !send_counts || p->t < 0) return LC_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  PT_TRY(hipSetDevice(p->device));
  const uint64_t* list = p->level == 0 ? p->F : p->Lb[p->cur];
  const unsigned long long* cnt = p->level == 0 ? &p->ctl->oc[p->sp ^ 1] : &p->ctl->lc[p->cur];
  // the list the following absorb appends to (see lc_part_absorb)
  unsigned long long* next_cnt = &p->ctl->lc[p->level == 0 ? 0 : p->cur ^ 1];
  unsigned long long* out_cnt = p->level == 0 ? &p->ctl->oc[p->sp] : nullptr;
  for (int attempt = 0; attempt < 2; ++attempt) {
    if (attempt) PT_TRY(hipMemsetAsync(p->ctl->cnt, 0, sizeof(p->ctl->cnt), s));
    PT_TRY(hipEventRecord(p->ev[0], s));
    const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(p->grid, (p->ub + PT - 1) / PT));
    hipLaunchKernelGGL(part_expand, dim3(grid), dim3(PT), 0, s, p->args, list, cnt, p->wd, p->stage,
                       p->seg_cap, p->ctl, next_cnt, out_cnt);
    PT_TRY(hipGetLastError());
    PT_TRY(hipEventRecord(p->ev[1], s));
    int rc = part_read_ctl(p, s, err, err_len);
    if (rc) return rc;
    float ms = 0;
    if (hipEventElapsedTime(&ms, p->ev[0], p->ev[1]) == hipSuccess) p->kernel_ms += ms;
    uint64_t mx = 0;
    for (int d = 0; d < p->world; ++d) mx = std::max<uint64_t>(mx, p->hctl->cnt[d]);
    if (mx <= p->seg_cap) break;
    uint64_t cap = p->seg_cap;
    while (cap < mx) cap <<= 1;
    PT_TRY(hipFree(p->stage));
    p->stage = nullptr;
    PT_TRY(hipMalloc(&p->stage, sizeof(uint64_t) * cap * (uint64_t)p->world));
    p->seg_cap = cap;
  }
  if (p->hctl->flags & PF_OVERFLOW) {
    set_msg(err, err_len, "frontier exceeded the partition capacity (LC_H_CAPACITY)");
    return LC_H_CAPACITY;
  }
  const uint64_t listed = p->level == 0 ? p->hctl->oc[p->sp ^ 1] : p->hctl->lc[p->cur];
  uint64_t cand = 0;
  for (int d = 0; d < p->world; ++d) send_counts[d] = (int64_t)p->hctl->cnt[d], cand += p->hctl->cnt[d];
  // read the list (8 B / config), write each candidate (8 B)
  p->alg_bytes += 8.0 * (double)listed + 8.0 * (double)cand;
  return 0;
}

/* Copy the last expand's candidates into dst (device memory), contiguous by destination rank
 * in rank order (an all-to-all's input). dst_cap in entries. */
int32_t lc_part_pack(lc_part* p, void* stream, void* dst, int64_t dst_cap, char* err, int32_t err_len) {
  if (!p || (!dst && dst_cap > 0)) return LC_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  uint64_t tot = 0;
  for (int d = 0; d < p->world; ++d) tot += p->hctl->cnt[d];
  if ((int64_t)tot > dst_cap) {
    set_msg(err, err_len, "pack buffer holds %lld entries, %llu needed", (long long)dst_cap,
            (unsigned long long)tot);
    return LC_E_ARG;
  }
  PT_TRY(hipSetDevice(p->device));
  uint64_t o = 0;
  for (int d = 0; d < p->world; ++d) {
    const uint64_t c = p->hctl->cnt[d];
    if (c)
      PT_TRY(hipMemcpyAsync((uint64_t*)dst + o, p->stage + (uint64_t)d * p->seg_cap, c * sizeof(uint64_t),
                            hipMemcpyDeviceToDevice, s));
    o += c;
  }
  return 0;
}

/* Absorb n candidates this rank owns (device memory; NULL = this rank's own staged segment,
 * for world 1). Ends the level. */
int32_t lc_part_absorb(lc_part* p, void* stream, const void* recv, int64_t n, char* err, int32_t err_len) {
  if (!p || n < 0 || p->t < 0) return LC_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  PT_TRY(hipSetDevice(p->device));
  const uint64_t* src = (const uint64_t*)recv;
  if (!src && n > 0) {
    if (p->world != 1 || (uint64_t)n != p->hctl->cnt[0]) {
      set_msg(err, err_len, "NULL recv needs world 1 and n = the staged count");
      return LC_E_ARG;
    }
    src = p->stage;
  }
  const int nxt = p->level == 0 ? 0 : p->cur ^ 1;
  if (n == 0)  // no kernel to reset the expand counts (lc[nxt] was reset by the expand)
    PT_TRY(hipMemsetAsync(p->ctl->cnt, 0, sizeof(p->ctl->cnt), s));
  if (n > 0) {
    const uint64_t tmask = (1ull << p->slog) - 1;
    const int grid = (int)std::min<int64_t>(p->grid, (n + PT * AB - 1) / (PT * AB));
    PT_TRY(hipEventRecord(p->ev[2], s));
    hipLaunchKernelGGL(part_absorb, dim3(grid), dim3(PT), 0, s, src, (uint64_t)n, p->args.bitj, p->S, tmask, p->O,
                       tmask, (uint64_t)p->epoch, p->Lb[nxt], &p->ctl->lc[nxt], &p->ctl->oc[p->sp], p->OUTL,
                       p->list_cap, p->ctl, p->world);
    PT_TRY(hipGetLastError());
    PT_TRY(hipEventRecord(p->ev[3], s));
    p->absorb_pending = true;
    // read each candidate (8 B) and probe its hash word (8 B read + CAS); survivors are
    // counted in the next expand's list read
    p->alg_bytes += 16.0 * (double)n;
  }
  p->cur = nxt;
  p->level++;
  p->ub = (uint64_t)n;  // the next list holds at most the candidates absorbed here
  return 0;
}

/* End the step: F = OUT. *out_count = this rank's frontier size (sum over ranks = 0 =>
 * not linearizable at this step). */
int32_t lc_part_step_end(lc_part* p, void* stream, int64_t* out_count, char* err, int32_t err_len) {
  if (!p || !out_count || p->t < 0) return LC_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  PT_TRY(hipSetDevice(p->device));
  int rc = part_read_ctl(p, s, err, err_len);
  if (rc) return rc;
  if (p->hctl->flags & PF_OVERFLOW) {
    set_msg(err, err_len, "frontier exceeded the partition capacity (LC_H_CAPACITY)");
    return LC_H_CAPACITY;
  }
  std::swap(p->F, p->OUTL);
  p->live &= ~p->args.bitj;
  *out_count = (int64_t)p->hctl->oc[p->sp];
  p->ub = p->hctl->oc[p->sp];
  p->sp ^= 1;  // OUT becomes the frontier
  return 0;
}

/* This rank's explored count so far, and the :index triple of step t (failure reports):
 * out[0] explored, out[1] :index of step t's :ok completion, out[2] of its invocation,
 * out[3] of the previous step's completion (-1 at t = 0). */
int32_t lc_part_results(lc_part* p, int64_t t, void* stream, int64_t* out4, char* err, int32_t err_len) {
  if (!p || !out4) return LC_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  PT_TRY(hipSetDevice(p->device));
  int rc = part_read_ctl(p, s, err, err_len);
  if (rc) return rc;
  out4[0] = (int64_t)p->hctl->explored;
  const int64_t ns = p->enc.n_steps(0);
  out4[1] = (t >= 0 && t < ns) ? p->enc.step_cmp_idx[t] : -1;
  out4[2] = (t >= 0 && t < ns) ? p->enc.step_inv_idx[t] : -1;
  out4[3] = (t > 0 && t <= ns) ? p->enc.step_cmp_idx[t - 1] : -1;
  return 0;
}

/* World 1, device-resident: runs every RETURN step (or the first max_steps) with one
 * cooperative launch per step that loops over the step's BFS levels behind grid barriers
 * (part_step_kernel); the host reads the per-step frontier sizes once per 2,048 steps. Same
 * verdict, failing step and explored count as the level protocol above. Call on a fresh plan.
 * out4[0] steps run, [1] first failing step (-1: none), [2] BFS levels, [3] explored. */
int32_t lc_part_run(lc_part* p, void* stream, int64_t max_steps, int64_t* out4, char* err, int32_t err_len) {
  if (!p || !out4) return LC_E_ARG;
  if (p->world != 1 || p->t != -1 || p->enc.err[0]) {
    set_msg(err, err_len, "lc_part_run needs world 1, a fresh plan and a searchable history");
    return LC_E_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  PT_TRY(hipSetDevice(p->device));
  const int64_t ns_flow = max_steps >= 0 ? std::min<int64_t>(p->enc.n_steps(0), max_steps) : p->enc.n_steps(0);
  const char* fe = getenv("LC_PART_FLOW");  // 0: the level kernel (part_step_kernel)
  if (!fe || atoi(fe) != 0) return part_run_flow(p, s, ns_flow, out4, err, err_len);
  constexpr int64_t CHUNK = 2048;
  if (!p->bar) {
    PT_TRY(hipMalloc(&p->bar, sizeof(PartBar)));
    PT_TRY(hipMemset(p->bar, 0, sizeof(PartBar)));
    PT_TRY(hipMalloc(&p->flog, CHUNK * sizeof(unsigned long long)));
    PT_TRY(hipHostMalloc(&p->hflog, CHUNK * sizeof(unsigned long long), hipHostMallocDefault));
    int occ = 0;
    PT_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, part_step_kernel, PL, 0));
    hipDeviceProp_t prop;
    PT_TRY(hipGetDeviceProperties(&prop, p->device));
    if (occ < 1) {
      set_msg(err, err_len, "part_step_kernel does not fit a CU");
      return LC_E_DEVICE;
    }
    p->run_grid = prop.multiProcessorCount;  // one workgroup per CU: co-resident
    if (const char* e = getenv("LC_PART_GRID"))  // (tuning) fewer workgroups: cheaper barriers
      if (atoi(e) >= 1 && atoi(e) < p->run_grid) p->run_grid = atoi(e);
  }
  const int64_t ns_all = p->enc.n_steps(0);
  const int64_t ns = max_steps >= 0 ? std::min(ns_all, max_steps) : ns_all;
  const uint64_t tb = sizeof(uint64_t) << p->slog;
  for (int attempt = 0;; ++attempt) {
    // two stage buffers of seg_cap >= list_cap candidates (a level's candidates)
    const uint64_t want = std::max(p->seg_cap, p->list_cap);
    if (!p->stage2 || want != p->run_cap) {
      PT_TRY(hipFree(p->stage));
      if (p->stage2) PT_TRY(hipFree(p->stage2));
      p->stage = p->stage2 = nullptr;
      PT_TRY(hipMalloc(&p->stage, sizeof(uint64_t) * want));
      PT_TRY(hipMalloc(&p->stage2, sizeof(uint64_t) * want));
      p->seg_cap = p->run_cap = want;
    }
    if (attempt) {  // start over: empty sets, the initial frontier {key 0}, zero counters
      PT_TRY(hipMemsetAsync(p->S, 0, tb, s));
      PT_TRY(hipMemsetAsync(p->O, 0, tb, s));
      PT_TRY(hipMemsetAsync(p->ctl, 0, sizeof(PartCtl), s));
      PT_TRY(hipMemsetAsync(p->F, 0, sizeof(uint64_t), s));
      const unsigned long long one = 1;
      PT_TRY(hipMemcpyAsync(&p->ctl->oc[1], &one, sizeof one, hipMemcpyHostToDevice, s));
      PT_TRY(hipStreamSynchronize(s));
      p->epoch = 0;
      p->live = 0;
      p->args = StepArgs{};
      p->t = -1;
      p->sp = 0;
    }
    PT_TRY(hipEventRecord(p->ev[0], s));
    int64_t t = 0, fail = -1;
    uint64_t flags = 0;
    while (t < ns && fail < 0) {
      const int64_t c0 = t, c1 = std::min(ns, t + CHUNK);
      for (; t < c1; ++t) {
        int rc = part_begin(p, t, s, err, err_len);
        if (rc) return rc;
        RunArgs r{};
        r.S = p->S;
        r.O = p->O;
        r.tmask = (1ull << p->slog) - 1;
        r.F = p->F;
        r.outl = p->OUTL;
        r.list_cap = p->list_cap;
        r.stage[0] = p->stage;
        r.stage[1] = p->stage2;
        r.seg_cap = p->seg_cap;
        r.ctl = p->ctl;
        r.bar = p->bar;
        r.flog = p->flog;
        r.flog_i = (uint32_t)(t - c0);
        r.sp = p->sp;
        r.ep = p->epoch;
        r.wd = p->wd;
        r.nwg = (uint32_t)p->run_grid;
        void* kargs[] = {(void*)&p->args, (void*)&r};
        PT_TRY(hipLaunchCooperativeKernel((const void*)part_step_kernel, dim3(p->run_grid), dim3(PL), kargs, 0, s));
        std::swap(p->F, p->OUTL);  // OUT becomes the frontier
        p->live &= ~p->args.bitj;
        p->sp ^= 1;
      }
      PT_TRY(hipMemcpyAsync(p->hflog, p->flog, sizeof(unsigned long long) * (size_t)(c1 - c0),
                            hipMemcpyDeviceToHost, s));
      int rc = part_read_ctl(p, s, err, err_len);
      if (rc) return rc;
      flags = p->hctl->flags;
      if (flags) break;
      for (int64_t i = 0; i < c1 - c0; ++i)
        if (p->hflog[i] == 0) {
          fail = c0 + i;
          break;
        }
    }
    PT_TRY(hipEventRecord(p->ev[1], s));
    int rc = part_read_ctl(p, s, err, err_len);
    if (rc) return rc;
    flags = p->hctl->flags;
    float ms = 0;
    if (hipEventElapsedTime(&ms, p->ev[0], p->ev[1]) == hipSuccess) p->kernel_ms += ms;
    if (flags & PF_ABORT) {
      set_msg(err, err_len, "part_step_kernel: grid barrier watchdog expired");
      return LC_E_DEVICE;
    }
    if ((flags & PF_STAGE) && attempt < 3) {
      p->seg_cap *= 4;  // a level outgrew the stage: start over with 4x
      continue;
    }
    if (flags & (PF_OVERFLOW | PF_STAGE)) {
      set_msg(err, err_len, "frontier exceeded the partition capacity (LC_H_CAPACITY)");
      return LC_H_CAPACITY;
    }
    p->alg_bytes += 8.0 * (double)p->hctl->listed + 24.0 * (double)p->hctl->cand;
    out4[0] = fail >= 0 ? fail + 1 : t;
    out4[1] = fail;
    out4[2] = (int64_t)p->hctl->levels;
    out4[3] = (int64_t)p->hctl->explored;
    return 0;
  }
}

void lc_part_destroy(lc_part* p) { delete p; }

}  // extern "C"

namespace {

// A spin barrier for the rank threads of lc_part_check (a level's phases are tens of
// microseconds: a futex round trip would be a noticeable share of them). wait() returns the
// error word as the LAST arriver saw it: every rank wrote its errors before arriving, so all
// ranks leave with the same value and take the same branch (no rank is left in a barrier).
struct SpinBarrier {
  std::atomic<int> count{0};
  std::atomic<int> gen{0};
  std::atomic<int>* err = nullptr;
  int snap = 0;
  int n = 1;
  int wait() {
    const int g = gen.load(std::memory_order_acquire);
    if (count.fetch_add(1, std::memory_order_acq_rel) == n - 1) {
      count.store(0, std::memory_order_relaxed);
      snap = err->load(std::memory_order_acquire);
      gen.store(g + 1, std::memory_order_release);
      return snap;
    }
    for (int spins = 0; gen.load(std::memory_order_acquire) == g; ++spins)
      if (spins > 1024) std::this_thread::yield();
    return snap;
  }
};

}  // namespace

extern "C" {

/* One history, frontier partitioned over n_ranks ranks held by THIS process (SURVEY §8(e)
 * axis 2 without a collective library): rank r on device r % (visible devices), one host
 * thread per rank. Per BFS level the ranks' candidate counts are exchanged in host memory and
 * every receiver pulls its candidates straight out of each sender's staging segment with peer
 * copies (hipMemcpyPeerAsync: xGMI between MI355X devices; a plain device copy when two ranks
 * share a device). Same per-history outputs as lc_check. n_ranks == 1 runs lc_part_run (the
 * device-resident flow kernel); n_ranks <= 0: one rank per visible device. */
int32_t lc_part_check(int32_t model_kind, int64_t init_value, int64_t n, const int64_t* index,
                      const int32_t* process, const int8_t* type, const int8_t* f, const int64_t* v0,
                      const int64_t* v1, const int8_t* vflags, int32_t n_ranks, int32_t capacity_log2,
                      int8_t* out_valid, int64_t* out_fail_idx, int64_t* out_fail_inv, int64_t* out_prev_ok,
                      int64_t* out_explored, int32_t* out_err, char* err, int32_t err_len) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    set_msg(err, err_len, "no HIP device visible (the checker has no CPU fallback)");
    return LC_E_DEVICE;
  }
  const int W = n_ranks <= 0 ? std::min(ndev, PW_MAX) : n_ranks;
  if (W > PW_MAX) {
    set_msg(err, err_len, "n_ranks %d > %d", W, PW_MAX);
    return LC_E_ARG;
  }
  auto put = [&](int8_t v, int64_t fi, int64_t fv, int64_t po, int64_t ex, int32_t er) {
    if (out_valid) *out_valid = v;
    if (out_fail_idx) *out_fail_idx = fi;
    if (out_fail_inv) *out_fail_inv = fv;
    if (out_prev_ok) *out_prev_ok = po;
    if (out_explored) *out_explored = ex;
    if (out_err) *out_err = er;
  };
  std::vector<std::unique_ptr<lc_part, void (*)(lc_part*)>> plans;
  std::vector<hipStream_t> streams(W, nullptr);
  auto cleanup = [&]() {
    for (int r = 0; r < W; ++r)
      if (streams[r]) {
        (void)hipSetDevice(r % ndev);
        (void)hipStreamSynchronize(streams[r]);
        (void)hipStreamDestroy(streams[r]);
        streams[r] = nullptr;
      }
  };
  for (int r = 0; r < W; ++r) {
    lc_part* p = nullptr;
    const int rc = lc_part_create(r % ndev, model_kind, init_value, n, index, process, type, f, v0, v1, vflags, r,
                                  W, capacity_log2, &p, err, err_len);
    if (rc) {
      cleanup();
      return rc;
    }
    plans.emplace_back(p, lc_part_destroy);
    if (hipSetDevice(r % ndev) != hipSuccess ||
        hipStreamCreateWithFlags(&streams[r], hipStreamNonBlocking) != hipSuccess) {
      set_msg(err, err_len, "stream creation failed on device %d", r % ndev);
      cleanup();
      return LC_E_DEVICE;
    }
  }
  lc_part* const p0 = plans[0].get();
  if (p0->enc.err[0]) {  // an unsearchable history: :unknown with its code, like lc_check
    put(LC_UNKNOWN, -1, -1, -1, 0, p0->enc.err[0]);
    cleanup();
    return 0;
  }
  const int64_t ns = p0->enc.n_steps(0);
  if (W == 1) {
    int64_t o4[4], r4[4];
    int rc = lc_part_run(p0, streams[0], -1, o4, err, err_len);
    if (rc == LC_H_CAPACITY) {
      put(LC_UNKNOWN, -1, -1, -1, 0, LC_H_CAPACITY);
      cleanup();
      return 0;
    }
    if (!rc) rc = lc_part_results(p0, o4[1] >= 0 ? o4[1] : ns - 1, streams[0], r4, err, err_len);
    cleanup();
    if (rc) return rc;
    if (o4[1] >= 0) put(LC_INVALID, r4[1], r4[2], r4[3], o4[3], 0);
    else put(LC_VALID, -1, -1, -1, o4[3], 0);
    return 0;
  }
  // peer access between every pair of devices the ranks use (xGMI); already-enabled is fine
  for (int a = 0; a < std::min(W, ndev); ++a)
    for (int b = 0; b < std::min(W, ndev); ++b) {
      int can = 0;
      if (a != b && hipDeviceCanAccessPeer(&can, a, b) == hipSuccess && can) {
        (void)hipSetDevice(a);
        (void)hipDeviceEnablePeerAccess(b, 0);
        (void)hipGetLastError();
      }
    }
  // shared state: per-level counts [src][dst], per-step frontier sizes, the first error
  std::vector<int64_t> counts((size_t)W * W, 0), fsize(W, 0);
  std::atomic<int> fail_rc{0};
  std::vector<std::string> msgs(W);
  SpinBarrier bar;
  bar.n = W;
  bar.err = &fail_rc;
  int64_t fail_t = -1, steps_run = 0;
  auto rank_main = [&](int r) {
    lc_part* p = plans[r].get();
    const int dev = r % ndev;
    hipStream_t s = streams[r];
    (void)hipSetDevice(dev);
    char e[256] = {0};
    uint64_t* recv = nullptr;
    size_t recv_cap = 0;
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) fail_rc.store(LC_E_DEVICE);
    auto note = [&](int rc) {  // first error wins; every rank leaves at the next barrier
      int z = 0;
      if (rc && fail_rc.compare_exchange_strong(z, rc)) msgs[r] = e;
    };
    for (int64_t t = 0; t < ns; ++t) {
      if (!fail_rc.load()) note(lc_part_step_begin(p, t, s, e, sizeof e));
      for (;;) {
        int64_t* mine = &counts[(size_t)r * W];
        if (!fail_rc.load()) note(lc_part_expand(p, s, mine, e, sizeof e));
        if (fail_rc.load()) std::fill(mine, mine + W, 0);
        if (bar.wait()) break;  // every rank's counts are in (or some rank failed: all leave)
        int64_t total = 0, n_recv = 0;
        for (int q = 0; q < W * W; ++q) total += counts[q];
        if (total == 0) break;  // (every rank reads the same counts: all leave together)
        for (int src = 0; src < W; ++src) n_recv += counts[(size_t)src * W + r];
        int rc = 0;
        if ((size_t)n_recv > recv_cap) {
          if (recv) (void)hipFree(recv);
          recv = nullptr;
          recv_cap = std::max<size_t>((size_t)n_recv * 2, 1 << 16);
          if (hipMalloc(&recv, recv_cap * sizeof(uint64_t)) != hipSuccess) {
            snprintf(e, sizeof e, "receive buffer of %zu configs on device %d", recv_cap, dev);
            rc = LC_E_MEMORY;
          }
        }
        // pull this rank's candidates out of every sender's staging segment for it
        int64_t off = 0;
        for (int src = 0; src < W && !rc; ++src) {
          const int64_t c = counts[(size_t)src * W + r];
          if (!c) continue;
          const lc_part* q = plans[src].get();
          const uint64_t* seg = q->stage + (uint64_t)r * q->seg_cap;
          const hipError_t he = (src % ndev) == dev
              ? hipMemcpyAsync(recv + off, seg, (size_t)c * 8, hipMemcpyDeviceToDevice, s)
              : hipMemcpyPeerAsync(recv + off, dev, seg, src % ndev, (size_t)c * 8, s);
          if (he != hipSuccess) {
            snprintf(e, sizeof e, "candidate copy rank %d -> %d: %s", src, r, hipGetErrorString(he));
            rc = LC_E_DEVICE;
          }
          off += c;
        }
        if (!rc && hipEventRecord(ev, s) != hipSuccess) rc = LC_E_DEVICE;
        if (!rc) rc = lc_part_absorb(p, s, recv, n_recv, e, sizeof e);
        if (!rc && hipEventSynchronize(ev) != hipSuccess) rc = LC_E_DEVICE;  // the copies (not the absorb)
        note(rc);
        bar.wait();  // every copy out of every staging segment is done: the next expand may refill them
      }
      if (!fail_rc.load()) note(lc_part_step_end(p, s, &fsize[r], e, sizeof e));
      if (bar.wait()) break;  // every rank's frontier size is in
      int64_t tot = 0;
      for (int q = 0; q < W; ++q) tot += fsize[q];
      if (r == 0) steps_run = t + 1;
      if (tot == 0) {
        if (r == 0) fail_t = t;
        break;
      }
    }
    (void)hipStreamSynchronize(s);
    if (recv) (void)hipFree(recv);
    if (ev) (void)hipEventDestroy(ev);
  };
  {
    std::vector<std::thread> th;
    for (int r = 1; r < W; ++r) th.emplace_back(rank_main, r);
    rank_main(0);
    for (auto& x : th) x.join();
  }
  const int frc = fail_rc.load();
  if (frc == LC_H_CAPACITY) {
    put(LC_UNKNOWN, -1, -1, -1, 0, LC_H_CAPACITY);
    cleanup();
    return 0;
  }
  if (frc) {
    std::string m;
    for (auto& x : msgs)
      if (!x.empty()) m = x;
    set_msg(err, err_len, "%s", m.empty() ? "partitioned search failed" : m.c_str());
    cleanup();
    return frc;
  }
  // explored = the sum of the ranks' set cardinalities; the :index triple from any rank
  int64_t explored = 0, r4[4] = {0, -1, -1, -1};
  const int64_t tq = fail_t >= 0 ? fail_t : steps_run - 1;
  for (int r = 0; r < W; ++r) {
    int64_t o4[4];
    const int rc = lc_part_results(plans[r].get(), tq, streams[r], o4, err, err_len);
    if (rc) {
      cleanup();
      return rc;
    }
    explored += o4[0];
    if (r == 0) std::copy(o4, o4 + 4, r4);
  }
  cleanup();
  if (fail_t >= 0) put(LC_INVALID, r4[1], r4[2], r4[3], explored, 0);
  else put(LC_VALID, -1, -1, -1, explored, 0);
  return 0;
}

}  // extern "C"
