// keys.hip — the JIT linearization search (knossos.linear/analysis [ext])
// with one workgroup owning one history at a time: the path for jepsen.independent
// histories (register.clj:106 — many keys, SURVEY §8(e) axis 1).
//
// Each workgroup pulls histories from a queue ordered heaviest-first and runs every RETURN
// step of its history locally: the closure set S and the post-return frontier OUT are LDS
// hash tables (LDS atomicCAS, linear probing, sized per step to the frontier), spilling to a
// private HBM table only when a probe run exceeds K_PROBES; frontier and level lists stream
// through a private HBM scratch. Levels are separated by __syncthreads only — no grid-wide
// synchronisation, so a workgroup never waits for another history.
// A history whose frontier outgrows the scratch is marked ST_CAPACITY and re-run by the
// grid kernel (search.hip), which spreads one history over every CU's LDS.
#include "device_common.hpp"
#include "keys.hpp"
#include "search.hpp"

namespace lc {

template <int MODEL>
struct KTraits;
template <>
struct KTraits<1> {
  using E = RegEntry;
};
template <>
struct KTraits<2> {
  using E = CntEntry;
};

__device__ __forceinline__ int log2_ceil(uint64_t x) {
  return x <= 1 ? 0 : 64 - __builtin_clzll(x - 1);
}

template <int MODEL>
__global__ void __launch_bounds__(KB) keys_kernel(KeysParams p) {
  using E = typename KTraits<MODEL>::E;
  __shared__ uint64_t sS[1 << KS_LOG];
  __shared__ uint64_t sO[1 << KO_LOG];
  __shared__ int64_t sA[64], sB[64];
  __shared__ uint8_t sK[64];
  __shared__ uint32_t sNF, sNL, sNew, sSpill, sCand;
  __shared__ int sH, sErr;

  const int tid = threadIdx.x;
  const int wg = blockIdx.x;
  E* const base = (E*)p.scratch + (size_t)wg * (2 * p.fcap + 2 * p.lcap);
  E* const Fb[2] = {base, base + p.fcap};
  E* const Lb[2] = {base + 2 * p.fcap, base + 2 * p.fcap + p.lcap};
  uint64_t* const spill = p.spill + ((size_t)wg << p.spill_log);
  uint32_t* const spill_pos = p.spill_pos + ((size_t)wg << p.spill_log);
  const uint32_t spill_mask = (1u << p.spill_log) - 1;
  const uint32_t spill_limit = (3u << p.spill_log) / 4;

  unsigned long long st_fin = 0, st_fout = 0, st_spill = 0, st_steps = 0, st_cand = 0;

  for (int i = tid; i < (1 << KS_LOG); i += KB) sS[i] = EMPTY;
  for (int i = tid; i < (1 << KO_LOG); i += KB) sO[i] = EMPTY;
  if (tid == 0) sSpill = 0;

  // ---------------------------------------------------------------- helpers
  auto spill_insert = [&](uint64_t k) -> int {
    uint32_t i = (uint32_t)(mix64(k) >> 24) & spill_mask;
    for (uint32_t probe = 0; probe <= spill_mask; ++probe) {
      uint64_t expected = EMPTY;
      if (__hip_atomic_compare_exchange_strong(&spill[i], &expected, k, __ATOMIC_RELAXED,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
        const uint32_t n = atomicAdd(&sSpill, 1u);
        if (n < spill_limit) spill_pos[n] = i;
        else sErr = ST_CAPACITY;
        return 1;
      }
      if (expected == k) return 0;
      i = (i + 1) & spill_mask;
    }
    sErr = ST_CAPACITY;
    return 0;
  };
  auto insert = [&](uint64_t* T, int logsz, uint64_t k, uint64_t tag) -> int {
    const uint32_t m = (1u << logsz) - 1;
    uint32_t i = (uint32_t)mix64(k) & m;
    for (int probe = 0; probe < K_PROBES; ++probe) {
      const uint64_t cur = T[i];
      if (cur == k) return 0;
      if (cur == EMPTY) {
        const uint64_t old = atomicCAS((unsigned long long*)&T[i], (unsigned long long)EMPTY,
                                       (unsigned long long)k);
        if (old == EMPTY) return 1;
        if (old == k) return 0;
      }
      i = (i + 1) & m;
    }
    return spill_insert(k | tag);
  };

  for (;;) {
    if (tid == 0) {
      sH = atomicAdd(p.queue, 1);
      sErr = 0;
    }
    __syncthreads();
    const int qi = sH;
    if (qi >= p.n_hist) break;
    const int h = p.order[qi];
    if (p.status[h] != ST_RUNNING) {
      __syncthreads();
      continue;
    }
    const int32_t so = p.step_beg[h];
    const int ns = p.step_end[h] - so;
    const int sshift = p.kshift[h];
    const uint64_t mmask = (1ull << sshift) - 1;
    const uint64_t smask = (1ull << p.kbits[h]) - 1;
    // initial config (model state at its initial value, nothing linearized)
    if (tid == 0) {
      E e;
      if constexpr (MODEL == 1) {
        e.key = (uint64_t)p.init_st[h] << sshift;
      } else {
        e.key = 0;
        e.st = p.init_st[h];
      }
      Fb[0][0] = e;
    }
    uint32_t nF = 1;
    int fb = 0;
    uint64_t live = 0;
    unsigned long long explored = 0;
    int result = ST_VALID, fail_t = -1;
    __syncthreads();

    for (int t = 0; t < ns; ++t) {
      const int64_t g = so + t;
      const int j = p.step_slot[g];
      const uint64_t bj = 1ull << j;
      if (t > 0) live &= ~(1ull << p.step_slot[g - 1]);
      const int64_t q0 = p.inv_off[g], q1 = p.inv_off[g + 1];
      for (int64_t q = q0; q < q1; ++q) live |= 1ull << p.inv_slot[q];
      for (int64_t q = q0 + tid; q < q1; q += KB) {
        const int s = p.inv_slot[q];
        sA[s] = p.inv_a[q];
        sB[s] = p.inv_b[q];
        sK[s] = p.inv_kind[q];
      }
      // size this step's tables to the frontier (cleared over the same range afterwards)
      const int nlive = __popcll(live);
      const int slog = min(KS_LOG, max(9, log2_ceil((uint64_t)nF * (nlive + 1) * 2 + 64)));
      const int olog = min(KO_LOG, max(8, log2_ceil((uint64_t)nF * 2 + 64)));
      if (tid == 0) {
        sNF = 0;
        sNL = 0;
        sNew = 0;
        sCand = 0;
      }
      __syncthreads();

      // expand `list` (level 0 = the frontier itself, whose configs are not in S)
      auto level = [&](const E* list, uint32_t n, bool level0, E* out_level) {
        E* Fn = Fb[fb ^ 1];
        uint32_t cand = 0;
        for (uint32_t i = tid; i < n; i += KB) {
          const E c = list[i];
          if (level0 && (c.key & bj)) {  // already linearized: returns directly
            E r = c;
            r.key = c.key & ~bj;
            if (insert(sO, olog, r.key, MARK)) {
              const uint32_t pos = atomicAdd(&sNF, 1u);
              if (pos < p.fcap) Fn[pos] = r;
              else sErr = ST_CAPACITY;
            }
            continue;
          }
          uint64_t todo = live & ~(c.key & mmask);
          while (todo) {
            const int k = __builtin_ctzll(todo);
            todo &= todo - 1;
            E ne;
            if constexpr (MODEL == 1) {
              // knossos.model/CASRegister [ext]: ok iff a = any or a = state; state := b
              const int64_t a = sA[k], nb = sB[k];
              const int64_t s = (int64_t)((c.key >> sshift) & smask);
              if (a != -1 && a != s) continue;
              const uint64_t s2 = (uint64_t)(nb >= 0 ? nb : s);
              ne.key = (c.key & ~(smask << sshift)) | (s2 << sshift) | (1ull << k);
            } else {
              // CounterModel.step (counter.clj:102-127)
              const uint8_t kind = sK[k];
              const int64_t a = sA[k], d = sB[k];
              int64_t r;
              if (kind & 8) {  // LeaderModel.step (leader.clj:69-75): a term's other leader -> inconsistent
                if (c.st & a) continue;
                r = c.st | d;
              } else {
                const bool ovf = (kind & 4) ? __builtin_sub_overflow(c.st, d, &r)
                                            : __builtin_add_overflow(c.st, d, &r);
                if (ovf) {  // Clojure +/- throw -> checker error -> :unknown
                  sErr = ST_MODEL;
                  continue;
                }
                if ((kind & 1) && c.st != a) continue;
                if ((kind & 2) && r != a) continue;
              }
              ne.key = c.key | (1ull << k);
              ne.st = r;
            }
            ++cand;
            if (!insert(sS, slog, ne.key, 0)) continue;
            atomicAdd(&sNew, 1u);
            if (k == j) {  // the returning op is linearized: return it
              E r = ne;
              r.key = ne.key & ~bj;
              if (insert(sO, olog, r.key, MARK)) {
                const uint32_t pos = atomicAdd(&sNF, 1u);
                if (pos < p.fcap) Fn[pos] = r;
                else sErr = ST_CAPACITY;
              }
            } else {
              const uint32_t pos = atomicAdd(&sNL, 1u);
              if (pos < p.lcap) out_level[pos] = ne;
              else sErr = ST_CAPACITY;
            }
          }
        }
        if (cand) atomicAdd(&sCand, cand);
      };

      level(Fb[fb], nF, true, Lb[0]);
      __syncthreads();
      int lb = 0;
      for (;;) {
        const uint32_t nl = sNL;
        if (nl == 0 || sErr) break;
        __syncthreads();  // everyone has read sNL
        if (tid == 0) sNL = 0;
        __syncthreads();
        level(Lb[lb], min(nl, (uint32_t)p.lcap), false, Lb[lb ^ 1]);
        lb ^= 1;
        __syncthreads();
      }
      const uint32_t nf2 = sNF;
      explored += sNew;
      st_fin += nF;
      st_fout += min(nf2, (uint32_t)p.fcap);
      st_cand += sCand;
      st_steps += 1;
      const int err = sErr;
      // clear this step's tables and spilled keys
      for (int i = tid; i < (1 << slog); i += KB) sS[i] = EMPTY;
      for (int i = tid; i < (1 << olog); i += KB) sO[i] = EMPTY;
      {
        const uint32_t used = sSpill;
        if (used <= spill_limit) {
          for (uint32_t i = tid; i < used; i += KB)
            __hip_atomic_store(&spill[spill_pos[i]], EMPTY, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {  // positions past the list were not recorded: wipe the whole table
          for (uint32_t i = tid; i <= spill_mask; i += KB)
            __hip_atomic_store(&spill[i], EMPTY, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        st_spill += used;
      }
      __syncthreads();
      if (tid == 0) sSpill = 0;
      if (err) {
        result = err;
        break;
      }
      if (nf2 == 0) {  // no configuration survives this RETURN: not linearizable here
        result = ST_INVALID;
        fail_t = t;
        break;
      }
      nF = min(nf2, (uint32_t)p.fcap);
      fb ^= 1;
    }
    if (tid == 0) {
      p.status[h] = result;
      p.fail_step[h] = fail_t;
      p.explored[h] = explored;
    }
    __syncthreads();
  }
  if (tid == 0) {
    atomicAdd(&p.stats[SS_FIN], st_fin);
    atomicAdd(&p.stats[SS_FOUT], st_fout);
    atomicAdd(&p.stats[SS_CAND], st_cand);
    atomicAdd(&p.stats[SS_SPILL], st_spill);
    atomicAdd(&p.stats[SS_STEPS], st_steps);
  }
}

int keys_grid_size(int model) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
  int per_cu = 0;
  hipError_t e = model == 1
      ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, keys_kernel<1>, KB, 0)
      : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, keys_kernel<2>, KB, 0);
  if (e != hipSuccess || per_cu < 1) return 0;
  return prop.multiProcessorCount * per_cu;
}

hipError_t launch_keys(const KeysParams& p, int nwg, hipStream_t stream) {
  if (p.model == 1)
    hipLaunchKernelGGL(keys_kernel<1>, dim3(nwg), dim3(KB), 0, stream, p);
  else
    hipLaunchKernelGGL(keys_kernel<2>, dim3(nwg), dim3(KB), 0, stream, p);
  return hipGetLastError();
}

}  // namespace lc
