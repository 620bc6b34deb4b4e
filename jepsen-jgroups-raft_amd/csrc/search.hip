// search.hip — the just-in-time linearization search (knossos.linear/analysis [ext],
// SURVEY §8(a) a5) for cas-register (a6), CounterModel (a7, counter.clj:100-127) and LeaderModel
// (leader.clj:63-75, on the counter's config layout; encode.hpp C_LEADER) as one persistent, cooperative, level-synchronous kernel on gfx950.
//
// Layout and algorithm:
//  * A config (model state, linearized bits of the live pending slots) of history h is a
//    63-bit key [h | state | mask]; the pending-call mask itself is per history (live[h]),
//    not per config. Counter configs carry the value as payload: it is a function of the
//    mask (every step adds its delta), so the key is [h | mask].
//  * Each workgroup OWNS the configs whose routing hash maps to it; it dedups them in two
//    LDS hash tables (closure set S, post-return frontier OUT) with LDS atomicCAS, spilling
//    to a private HBM table when a probe run exceeds PROBE_LIMIT.
//  * Candidates cross owners through HBM "cells" [dst][src][cell_cap]: each source writes
//    its candidates with one LDS counter per destination (no global atomics), the owner
//    reads its column after the grid barrier. Routing uses the key with the returning
//    op's bit cleared, so a config and its post-return image have the same owner.
//  * One RETURN step for every history of the batch advances per outer iteration:
//      phase X : expand the owned frontier (configs that already linearized the
//                returning op are routed "direct" with MARK)
//      level ℓ : dedup incoming candidates into S / OUT, expand the new ones
//    until a phase routes nothing. Grid barriers separate phases.
#include "device_common.hpp"
#include "search.hpp"

#include <climits>

namespace lc {

__device__ __forceinline__ uint64_t stamp() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz

// sc1 (write-through, L1-bypassing) 8-byte hand-off of cell entries between workgroups
__device__ __forceinline__ void put_entry(RegEntry* dst, const RegEntry& e) { st_agent(&dst->key, e.key); }
__device__ __forceinline__ void put_entry(CntEntry* dst, const CntEntry& e) {
  st_agent(&dst->key, e.key);
  st_agent((uint64_t*)&dst->st, (uint64_t)e.st);
}
__device__ __forceinline__ RegEntry get_entry(const RegEntry* src) { return RegEntry{ld_agent(&src->key)}; }
__device__ __forceinline__ CntEntry get_entry(const CntEntry* src) {
  return CntEntry{ld_agent(&src->key), (int64_t)ld_agent((const uint64_t*)&src->st)};
}

__device__ __forceinline__ uint32_t owner_of(uint64_t x, uint32_t nwg) {
  return (uint32_t)(((mix64(x) >> 32) * (uint64_t)nwg) >> 32);
}

// Grid barrier: two-level arrival counters (8 groups, then the top counter) so at most 32
// arrivals serialise on one word, and a release generation polled relaxed with s_sleep
// (MI355X_MICROARCH "barrier-xcd" / "fanin"). `fenced` adds the agent-scope release/acquire
// (cdna_hip_programming.md §6 G16) for phases that publish plain stores; level phases hand
// off only sc1 (write-through) stores read back with sc1 loads, so they skip both fences.
// Bounded spin: a stuck barrier raises FL_ABORT instead of hanging the GPU.
__device__ __forceinline__ bool grid_sync(const SearchParams& p, int* s_abort, uint64_t* t_bar,
                                          bool fenced) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave drains its stores
  __syncthreads();
  const uint64_t t_arrive = stamp();
  if (threadIdx.x == 0) {
    if (fenced) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    GridBar* bar = p.bar;
    const unsigned nwg = (unsigned)p.nwg;
    const unsigned g = ld_agent(&bar->gen);
    const unsigned grp = blockIdx.x & 7u;
    const unsigned gsize = (nwg - grp + 7u) >> 3;
    const unsigned ngroups = nwg < 8u ? nwg : 8u;
    const unsigned a =
        __hip_atomic_fetch_add(&bar->grp[grp][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a == gsize - 1) {
      st_agent(&bar->grp[grp][0], 0u);
      const unsigned t =
          __hip_atomic_fetch_add(&bar->top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == ngroups - 1) {
        st_agent(&bar->top, 0u);
        __hip_atomic_store(&bar->gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    // watchdog on the 100 MHz constant clock: 20 s without a release aborts the search
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    long spins = 0;
    while (ld_agent(&bar->gen) == g) {
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 255) == 0) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000000ull) {
          st_agent(&p.flags[FL_ABORT], 1);
          break;
        }
        if (ld_agent(&p.flags[FL_ABORT])) break;
      }
    }
    if (fenced) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    *s_abort = ld_agent(&p.flags[FL_ABORT]);
  }
  __syncthreads();
  if (t_bar) *t_bar += stamp() - t_arrive;
  return *s_abort == 0;
}

template <int MODEL>
struct Traits;
template <>
struct Traits<1> {
  using E = RegEntry;
};
template <>
struct Traits<2> {
  using E = CntEntry;
};

template <int MODEL>
__global__ void __launch_bounds__(BLOCK) search_kernel(SearchParams p) {
  using E = typename Traits<MODEL>::E;
  __shared__ uint64_t sS[1 << S_LOG];
  __shared__ uint64_t sO[1 << O_LOG];
  __shared__ uint32_t sExpl[HMAX];
  __shared__ uint32_t sCnt[WGMAX];
  __shared__ uint32_t sPref[WGMAX + 1];
  __shared__ uint32_t sNE[HMAX / 32];  // nonempty[h] already published this step
  __shared__ uint32_t sFcount[2];
  __shared__ uint32_t sSpillUsed;
  __shared__ unsigned long long sStat[SS_N];
  __shared__ unsigned long long sTotal;
  __shared__ int sAbort;
  __shared__ uint64_t sSent[1 << SENT_LOG];  // candidate keys routed in this phase (lossy)

  const int tid = threadIdx.x;
  const uint32_t wg = blockIdx.x;
  const uint32_t nwg = (uint32_t)p.nwg;
  const int nh = p.n_hist;
  const uint64_t mmask = (1ull << p.mask_bits) - 1;
  const int state_top = p.tag_shift > 0 ? p.tag_shift : p.hist_shift;  // state bits end here
  const uint64_t smask = (state_top > p.state_shift) ? ((1ull << (state_top - p.state_shift)) - 1) : 0;
  const uint64_t tag_clear = p.tag_shift > 0 ? ~(63ull << p.tag_shift) : ~0ull;
  uint64_t tag_now = 0;  // report mode: this step's tag, already shifted into place
  const size_t fcap = (size_t)p.f_cap;
  const size_t ccap = (size_t)p.cell_cap;
  E* const flist = (E*)p.flist;
  E* const cells = (E*)p.cells;
  uint64_t* const spill = p.spill + ((size_t)wg << p.spill_log);
  uint32_t* const spill_pos = p.spill_pos + ((size_t)wg << p.spill_log);
  const uint32_t spill_mask = (1u << p.spill_log) - 1;
  const uint32_t spill_limit = (3u << p.spill_log) / 4;

  // ---------------------------------------------------------------- helpers
  // slot operands: register -> one word (b << 32) | a; counter -> kind, a, d
  auto set_op = [&](size_t oi, int64_t q) {
    if constexpr (MODEL == 1) {
      p.op_a[oi] = (int64_t)(((uint64_t)(uint32_t)(int32_t)p.inv_b[q] << 32) |
                             (uint64_t)(uint32_t)(int32_t)p.inv_a[q]);
    } else {
      p.op_kind[oi] = p.inv_kind[q];
      p.op_a[oi] = p.inv_a[q];
      p.op_b[oi] = p.inv_b[q];
    }
  };
  auto hist_of = [&](uint64_t key) -> int { return (int)((key & ~MARK) >> p.hist_shift); };

  // spill: WG-private open-addressing table in HBM (workgroup-scope atomics; stays on this CU)
  auto spill_insert = [&](uint64_t k) -> int {
    uint32_t i = (uint32_t)(mix64(k) >> 20) & spill_mask;
    for (uint32_t probe = 0; probe <= spill_mask; ++probe) {
      uint64_t expected = EMPTY;
      bool won = __hip_atomic_compare_exchange_strong(&spill[i], &expected, k, __ATOMIC_RELAXED,
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (won) {
        uint32_t n = atomicAdd(&sSpillUsed, 1u);
        if (n < spill_limit) spill_pos[n] = i;
        else __hip_atomic_store(&p.flags[FL_SPILL], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        atomicAdd(&sStat[SS_SPILL], 1ull);
        return 1;
      }
      if (expected == k) return 0;
      i = (i + 1) & spill_mask;
    }
    __hip_atomic_store(&p.flags[FL_SPILL], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 1;
  };
  // LDS insert with linear probing; tag marks OUT keys inside the shared spill table
  auto lds_insert = [&](uint64_t* T, int logsz, uint64_t k, uint64_t tag) -> int {
    const uint32_t m = (1u << logsz) - 1;
    uint32_t i = (uint32_t)mix64(k) & m;
    for (int probe = 0; probe < PROBE_LIMIT; ++probe) {
      uint64_t cur = T[i];
      if (cur == k) return 0;
      if (cur == EMPTY) {
        uint64_t old = atomicCAS((unsigned long long*)&T[i], (unsigned long long)EMPTY,
                                 (unsigned long long)k);
        if (old == EMPTY) return 1;
        if (old == k) return 0;
      }
      i = (i + 1) & m;
    }
    return spill_insert(k | tag);
  };

  // route one item to its owner's cell (parity par). A key already routed by this workgroup
  // in this phase is dropped at the source: the owner would discard it as a duplicate.
  // (cleared every phase; a key is written before its send, which completes in this phase)
  auto route = [&](const E& e, uint64_t rkey, int par) {
    const uint64_t hk = mix64(e.key);
    const uint32_t si = (uint32_t)(hk >> 40) & ((1u << SENT_LOG) - 1);
    if (sSent[si] == e.key) return;
    sSent[si] = e.key;  // racy overwrite is harmless: a miss only re-sends
    uint32_t dst = owner_of(rkey, nwg);
    uint32_t pos = atomicAdd(&sCnt[dst], 1u);
    if (pos < ccap) {
      put_entry(&cells[(((size_t)par * nwg + dst) * nwg + wg) * ccap + pos], e);
    } else {  // this cell is full: reserve a slot in the destination's overflow bucket
      const uint32_t r = atomicAdd(&p.ovf_cnt[(size_t)par * nwg + dst], 1u);
      if (r < (uint64_t)p.ovf_cap)
        put_entry(&((E*)p.ovf)[((size_t)par * nwg + dst) * p.ovf_cap + r], e);
      else
        st_agent(&p.flags[FL_OVERFLOW], 1);
    }
  };

  // expand config e of history h at step t: linearize each live, not-yet-linearized slot
  // expand config e of history h at step t: linearize each live, not-yet-linearized slot.
  // Slot operands for up to 8 candidates are loaded together (independent loads in flight).
  auto expand = [&](const E& e, int h, int b, uint64_t bj, int par) -> uint32_t {
    const uint64_t key = e.key;
    const size_t hb = ((size_t)b * nh + h);
    uint64_t todo = p.live[hb] & ~(key & mmask);
    uint32_t n = 0;
    constexpr int CH = 4;  // candidates whose operands load together
    while (todo) {
      int ks[CH];
#pragma unroll
      for (int q = 0; q < CH; ++q) {
        ks[q] = todo ? __builtin_ctzll(todo) : -1;
        todo &= todo - 1;
      }
      int64_t oa[CH], ob[CH];
      uint8_t okd[CH];
#pragma unroll
      for (int q = 0; q < CH; ++q) {
        if (ks[q] < 0) continue;
        const size_t oi = hb * 64 + ks[q];
        oa[q] = p.op_a[oi];
        if constexpr (MODEL == 2) {
          ob[q] = p.op_b[oi];
          okd[q] = p.op_kind[oi];
        }
      }
#pragma unroll
      for (int q = 0; q < CH; ++q) {
        const int k = ks[q];
        if (k < 0) continue;
        E ne;
        if constexpr (MODEL == 1) {
          // CASRegister.step [ext]: ok iff a = any or a = state; state := b unless keep.
          // operands packed as (b << 32) | a (int32 each)
          const int64_t a = (int32_t)(uint32_t)oa[q], nb = (int32_t)(uint32_t)((uint64_t)oa[q] >> 32);
          const int64_t s = (int64_t)((key >> p.state_shift) & smask);
          if (a != -1 && a != s) continue;
          const uint64_t s2 = (uint64_t)(nb >= 0 ? nb : s);
          ne.key = (((key & ~(smask << p.state_shift)) | (s2 << p.state_shift) | (1ull << k)) & tag_clear) | tag_now;
        } else {
          // CounterModel.step (counter.clj:102-127): v +/- d, optional pre/post equality
          const uint8_t kind = okd[q];
          const int64_t a = oa[q], d = ob[q];
          const int64_t st = e.st;
          int64_t r;
          if (kind & 8) {  // LeaderModel.step (leader.clj:69-75): a term's other leader -> inconsistent
            if (st & a) continue;
            r = st | d;
          } else {
            bool ovf = (kind & 4) ? __builtin_sub_overflow(st, d, &r) : __builtin_add_overflow(st, d, &r);
            if (ovf) {  // Clojure +/- throw -> the checker errors -> :valid? :unknown
              atomicCAS(&p.status[h], ST_RUNNING, ST_MODEL);
              continue;
            }
            if ((kind & 1) && st != a) continue;
            if ((kind & 2) && r != a) continue;
          }
          ne.key = ((key | (1ull << k)) & tag_clear) | tag_now;
          ne.st = r;
        }
        route(ne, ne.key & ~bj, par);
        ++n;
      }
    }
    return n;
  };

  // write this phase's per-destination counts, publish the routed total
  auto publish_counts = [&](int par, int phase) {
    __syncthreads();
    for (int i = tid; i < (1 << SENT_LOG); i += BLOCK) sSent[i] = EMPTY;
    unsigned long long local = 0;
    for (int d = tid; d < (int)nwg; d += BLOCK) {
      const uint32_t c = sCnt[d];
      st_agent(&p.cell_cnt[((size_t)par * nwg + d) * nwg + wg], (uint32_t)min((size_t)c, ccap));
      local += c;
      sCnt[d] = 0;
    }
    // block reduction of `local` via LDS atomics
    if (local) atomicAdd(&sTotal, local);
    __syncthreads();
    if (tid == 0) {
      const unsigned long long tot = sTotal;
      sTotal = 0;
      if (tot) atomicAdd(&p.produced[phase & 3], tot);
      if (wg == 0) st_agent(&p.produced[(phase + 2) & 3], 0ull);
      sStat[SS_CAND] += tot;
    }
  };

  // ---------------------------------------------------------------- init
  for (int i = tid; i < (1 << S_LOG); i += BLOCK) sS[i] = EMPTY;
  for (int i = tid; i < (1 << O_LOG); i += BLOCK) sO[i] = EMPTY;
  for (int i = tid; i < HMAX; i += BLOCK) sExpl[i] = 0;
  for (int i = tid; i < HMAX / 32; i += BLOCK) sNE[i] = 0;
  for (int i = tid; i < WGMAX; i += BLOCK) sCnt[i] = 0;
  for (int i = tid; i < (1 << SENT_LOG); i += BLOCK) sSent[i] = EMPTY;
  if (tid < SS_N) sStat[tid] = 0;
  if (tid == 0) {
    sFcount[0] = sFcount[1] = 0;
    sSpillUsed = 0;
    sTotal = 0;
    sAbort = 0;
  }
  __syncthreads();
  const int gtid = (int)wg * BLOCK + tid;
  uint64_t T[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // phase stamps (s_memtime cycles), thread 0 reports
  // slot tables for step 0 (buffer 0); buffer 1 starts empty (= state before step 0)
  if (gtid < nh && p.status[gtid] == ST_RUNNING) {
    const int h = gtid;
    const int ns = p.step_end[h] - p.step_beg[h];
    if (ns > 0) {
      const int64_t gs = p.step_beg[h];
      uint64_t live = 0;
      for (int64_t q = p.inv_off[gs]; q < p.inv_off[gs + 1]; ++q) {
        const int s = p.inv_slot[q];
        const size_t oi = ((size_t)0 * nh + h) * 64 + s;
        set_op(oi, q);
        live |= 1ull << s;
      }
      p.live[h] = live;
    }
  }
  // initial config of each history, owned by workgroup h % nwg
  for (int h = (int)wg + tid * (int)nwg; h < nh; h += BLOCK * (int)nwg) {
    if (p.status[h] != ST_RUNNING) continue;
    E e;
    if constexpr (MODEL == 1) {
      e.key = ((uint64_t)h << p.hist_shift) | ((uint64_t)p.init_st[h] << p.state_shift);
    } else {
      e.key = ((uint64_t)h << p.hist_shift);
      e.st = p.init_st[h];
    }
    const uint32_t pos = atomicAdd(&sFcount[0], 1u);
    if (pos < fcap) flist[((size_t)0 * nwg + wg) * fcap + pos] = e;
  }
  if (!grid_sync(p, &sAbort, nullptr, true)) goto done;

  {
    int phase = 0;
    for (int t = 0; t < p.max_t; ++t) {
      const int b = t & 1, nb = b ^ 1;
      if (p.tag_shift > 0) tag_now = (uint64_t)(t & 63) << p.tag_shift;
      // ============================================================ phase X
      uint64_t ts = stamp();
      if (tid == 0) sFcount[nb] = 0;
      if (wg == 0 && tid == 0) st_agent(&p.running[(t + 2) & 3], 0u);
      if (gtid < nh) {
        const int h = gtid;
        int st = ld_agent(&p.status[h]);
        const int ns = p.step_end[h] - p.step_beg[h];
        if (st == ST_RUNNING && t > 0 && ld_agent(&p.nonempty[(size_t)((t - 1) & 1) * nh + h]) == 0) {
          // no config survived RETURN t-1
          if (atomicCAS(&p.status[h], ST_RUNNING, ST_INVALID) == ST_RUNNING) p.fail_step[h] = t - 1;
          st = ST_INVALID;
        }
        if (st == ST_RUNNING) {
          if (t >= ns) {
            atomicCAS(&p.status[h], ST_RUNNING, ST_VALID);
          } else {
            atomicAdd(&p.running[t & 3], 1u);
            // bring buffer nb (state of step t-1) to step t+1
            const int64_t gs = p.step_beg[h] + t;
            uint64_t live = p.live[(size_t)nb * nh + h];
            if (t > 0) live &= ~(1ull << p.step_slot[gs - 1]);
            const int last = (t + 1 < ns) ? 1 : 0;
            for (int w = 0; w <= last; ++w) {
              const int64_t g2 = gs + w;
              if (w == 1) live &= ~(1ull << p.step_slot[gs]);
              for (int64_t q = p.inv_off[g2]; q < p.inv_off[g2 + 1]; ++q) {
                const int s = p.inv_slot[q];
                const size_t oi = ((size_t)nb * nh + h) * 64 + s;
                set_op(oi, q);
                live |= 1ull << s;
              }
            }
            p.live[(size_t)nb * nh + h] = live;
          }
        }
        if (t > 0) st_agent(&p.nonempty[(size_t)((t - 1) & 1) * nh + h], 0u);
      }
      __syncthreads();
      T[1] += stamp() - ts;
      ts = stamp();
      {
        const uint32_t nf = min(sFcount[b], (uint32_t)fcap);
        const E* F = flist + ((size_t)b * nwg + wg) * fcap;
        const int par = phase & 1;
        for (uint32_t i = tid; i < nf; i += BLOCK) {
          E e = F[i];
          const int h = hist_of(e.key);
          if (p.status[h] != ST_RUNNING) continue;
          const int32_t so = p.step_beg[h];
          if (t >= p.step_end[h] - so) continue;
          const uint64_t bj = 1ull << p.step_slot[so + t];
          if (e.key & bj) {  // returned directly: only its post-return image matters
            E r = e;
            r.key = (e.key & ~bj) | MARK;
            route(r, e.key & ~bj, par);
          } else {
            expand(e, h, b, bj, par);
          }
        }
        if (tid == 0) sStat[SS_FIN] += nf;
        publish_counts(par, phase);
      }
      T[2] += stamp() - ts;
      if (!grid_sync(p, &sAbort, &T[0], true)) goto done;  // publishes the slot tables
      ++phase;
      // ============================================================ levels
      for (;;) {
        const unsigned long long routed = ld_agent(&p.produced[(phase - 1) & 3]);
        if (routed == 0) break;
        const int pin = (phase - 1) & 1, pout = phase & 1;
        ts = stamp();
        // prefix over the column of cells addressed to this workgroup
        if (tid < 64) {
          const int per = ((int)nwg + 63) / 64;
          uint32_t sum = 0;
          uint32_t vals[WGMAX / 64];
          for (int q = 0; q < per; ++q) {
            const int s = tid * per + q;
            uint32_t c = 0;
            if (s < (int)nwg) c = min(ld_agent(&p.cell_cnt[((size_t)pin * nwg + wg) * nwg + s]), (uint32_t)ccap);
            vals[q] = c;
            sum += c;
          }
          uint32_t incl = sum;
          for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off, 64);
            if (tid >= off) incl += y;
          }
          uint32_t run = incl - sum;
          for (int q = 0; q < per; ++q) {
            const int s = tid * per + q;
            if (s < (int)nwg) sPref[s] = run;
            run += vals[q];
          }
          if (tid == 63) sPref[nwg] = incl;
        }
        __syncthreads();
        T[3] += stamp() - ts;
        ts = stamp();
        const uint32_t in_cells = sPref[nwg];
        const uint32_t in_ovf = (uint32_t)min((uint64_t)ld_agent(&p.ovf_cnt[(size_t)pin * nwg + wg]),
                                              (uint64_t)p.ovf_cap);
        const uint32_t total = in_cells + in_ovf;
        const E* col = cells + ((size_t)pin * nwg + wg) * nwg * ccap;
        const E* ovf_in = (const E*)p.ovf + ((size_t)pin * nwg + wg) * p.ovf_cap;
        // each thread fetches R entries before touching any (R sc1 loads in flight)
        constexpr int R = MODEL == 1 ? 4 : 2;
        for (uint32_t base = 0; base < total; base += BLOCK * R) {
          E ent[R];
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const uint32_t i = base + r * BLOCK + tid;
            ent[r].key = EMPTY;
            if (i >= total) continue;
            if (i < in_cells) {
              // source cell by binary search over the prefix
              int lo = 0, hi = (int)nwg;  // sPref[lo] <= i < sPref[hi]
              while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (sPref[mid] <= i) lo = mid; else hi = mid;
              }
              ent[r] = get_entry(&col[(size_t)lo * ccap + (i - sPref[lo])]);
            } else {
              ent[r] = get_entry(&ovf_in[i - in_cells]);
            }
          }
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const E e = ent[r];
            if (e.key == EMPTY) continue;
            const int h = hist_of(e.key);
            if (p.status[h] != ST_RUNNING) continue;
            const int32_t so = p.step_beg[h];
            const uint64_t bj = 1ull << p.step_slot[so + t];
            E o = e;
            if (e.key & MARK) {
              o.key = e.key & ~MARK;
            } else {
              if (!lds_insert(sS, S_LOG, e.key, 0)) continue;  // seen in this closure
              atomicAdd(&sExpl[h], 1u);
              if (!(e.key & bj)) {  // returning op not linearized yet: keep exploring
                expand(e, h, b, bj, pout);
                continue;
              }
              o.key = e.key & ~bj;  // linearized: return it
            }
            if (lds_insert(sO, O_LOG, o.key, MARK)) {
              const uint32_t pos = atomicAdd(&sFcount[nb], 1u);
              if (pos < fcap) flist[((size_t)nb * nwg + wg) * fcap + pos] = o;
              else __hip_atomic_store(&p.flags[FL_OVERFLOW], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              const uint32_t bit = 1u << (h & 31);
              if (!(atomicOr(&sNE[h >> 5], bit) & bit)) st_agent(&p.nonempty[(size_t)b * nh + h], 1u);
            }
          }
        }
        __syncthreads();
        if (tid == 0 && in_ovf) st_agent(&p.ovf_cnt[(size_t)pin * nwg + wg], 0u);
        T[4] += stamp() - ts;
        ts = stamp();
        publish_counts(pout, phase);
        T[5] += stamp() - ts;
        if (!grid_sync(p, &sAbort, &T[0], false)) goto done;
        ++phase;
      }
      ts = stamp();
      // ============================================================ end of step
      if (tid == 0) {
        sStat[SS_FOUT] += min(sFcount[nb], (uint32_t)fcap);
        sStat[SS_STEPS] += 1;
      }
      for (int i = tid; i < (1 << S_LOG); i += BLOCK) sS[i] = EMPTY;
      for (int i = tid; i < (1 << O_LOG); i += BLOCK) sO[i] = EMPTY;
      for (int i = tid; i < HMAX / 32; i += BLOCK) sNE[i] = 0;
      {
        const uint32_t used = sSpillUsed;
        if (used <= spill_limit) {
          for (uint32_t i = tid; i < used; i += BLOCK)
            __hip_atomic_store(&spill[spill_pos[i]], EMPTY, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
          for (uint32_t i = tid; i <= spill_mask; i += BLOCK)
            __hip_atomic_store(&spill[i], EMPTY, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      __syncthreads();
      if (tid == 0) sSpillUsed = 0;
      T[6] += stamp() - ts;
      if (ld_agent(&p.running[t & 3]) == 0) break;  // no history processed step t: all done
      __syncthreads();
    }
    if (tid == 0) sStat[SS_PHASES] += phase;
  }

done:
  __syncthreads();
  if (tid == 0 && p.stamps)
    for (int i = 0; i < 8; ++i) p.stamps[(size_t)wg * 8 + i] = T[i];
  for (int h = tid; h < nh; h += BLOCK)
    if (sExpl[h]) atomicAdd(&p.explored[h], (unsigned long long)sExpl[h]);
  if (tid == 0) {
    p.fcount[wg] = sFcount[0];
    p.fcount[nwg + wg] = sFcount[1];
  }
  if (tid < SS_N && (tid != SS_PHASES && tid != SS_STEPS ? true : wg == 0)) {
    if (sStat[tid]) atomicAdd(&p.stats[tid], sStat[tid]);
  }
}

int search_grid_size(int model) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
  int per_cu = 0;
  hipError_t e = model == 1
      ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, search_kernel<1>, BLOCK, 0)
      : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, search_kernel<2>, BLOCK, 0);
  if (e != hipSuccess || per_cu < 1) return 0;
  int n = prop.multiProcessorCount;  // one owner per CU (LDS-bound: 1 block/CU)
  return n > WGMAX ? WGMAX : n;
}

hipError_t launch_search(const SearchParams& p, hipStream_t stream) {
  SearchParams q = p;
  void* args[] = {&q};
  if (p.model == 1)
    return hipLaunchCooperativeKernel((const void*)search_kernel<1>, dim3(p.nwg), dim3(BLOCK), args, 0,
                                      stream);
  return hipLaunchCooperativeKernel((const void*)search_kernel<2>, dim3(p.nwg), dim3(BLOCK), args, 0,
                                    stream);
}

}  // namespace lc
