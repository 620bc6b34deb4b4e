// dense.hip — closure-table search (see dense.hpp) for cas-register histories whose live
// slot width is at most DENSE_LMAX: knossos.linear/analysis [ext] with
// CASRegister.step (a6, register.clj:110) applied to whole state sets.
//
// One RETURN step of slot j on the table A[mask] (state set per linearized-slot mask, all
// masks ⊆ live):
//   layer p = 1..L (masks of popcount p, in parallel; layers are barriers):
//     j ∈ m : R[m] = T_j(A[m \ j])                 configs holding j are never expanded
//     j ∉ m : R[m] = ∪_{k ∈ m} T_k(A[m \ k])
//     explored += |R[m]|;  A[m] |= R[m]
//   return j:  A'[m] = A[m ∪ j] for m ∌ j, A'[m ∪ j] = 0   (the post-return frontier)
//   A' empty => not linearizable at this RETURN.
// Every config reachable by linearizing pending calls is R of exactly one mask, and a mask's
// predecessors (one bit fewer) are final one layer earlier, so R is the closure set of the
// sparse search and |R| its explored count, bit-exact.
//
// Teams: a whole workgroup per history for widths 13..17 (128 KiB table), or one wave per
// history for widths <= 12 (16 tables of 4 KiB per workgroup). Histories are dequeued
// heaviest first from a global counter.
#include "dense.hpp"
#include "search.hpp"

namespace lc {
namespace {

constexpr int BINOM_N = 24;

__device__ __forceinline__ uint32_t reg_step(uint32_t op, uint32_t s) {
  const uint32_t x = s & (op & 0xffu);
  const uint32_t b = (op >> 8) & 0xffu;
  return b ? (x ? b : 0u) : x;
}

template <int TEAM>
__device__ __forceinline__ void team_sync() {
  if constexpr (TEAM == DENSE_BLOCK) {
    __syncthreads();
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

template <int TEAM>
__device__ __forceinline__ int team_any(int v) {
  if constexpr (TEAM == DENSE_BLOCK) return __syncthreads_or(v);
  else return __any(v);
}

template <int TEAM, int TLOG>
__global__ void __launch_bounds__(DENSE_BLOCK) dense_kernel(DenseParams p) {
  constexpr int NTEAM = DENSE_BLOCK / TEAM;
  __shared__ uint32_t sTab[NTEAM << (TLOG - 2)];  // byte tables, word-addressed for zeroing
  __shared__ uint32_t sOp[NTEAM][32];             // per slot: amask | bmask << 8
  __shared__ uint32_t sBinom[BINOM_N * BINOM_N];
  __shared__ int sQ[NTEAM];
  __shared__ unsigned long long sExpl[NTEAM];

  const int tid = threadIdx.x;
  const int team = tid / TEAM, tt = tid % TEAM, lane = tid & 63;
  uint8_t* const A = (uint8_t*)&sTab[team << (TLOG - 2)];
  uint32_t* const opt = sOp[team];

  for (int i = tid; i < BINOM_N * BINOM_N; i += DENSE_BLOCK) {
    const int n = i / BINOM_N, k = i % BINOM_N;
    uint32_t c = 0;
    if (k <= n) {  // C(n, k) by the multiplicative formula (exact in 64 bits for n < 24)
      uint64_t v = 1;
      for (int q = 1; q <= k; ++q) v = v * (uint64_t)(n - k + q) / (uint64_t)q;
      c = (uint32_t)v;
    }
    sBinom[i] = c;
  }
  __syncthreads();

  unsigned long long st_cand = 0, st_fout = 0, st_steps = 0;
  for (;;) {
    if (tt == 0) sQ[team] = atomicAdd(p.queue, 1);
    team_sync<TEAM>();
    const int qi = sQ[team];
    if (tt == 0) sExpl[team] = 0;
    team_sync<TEAM>();
    if (qi >= p.n) break;
    const int h = p.order[qi];
    const int lmax = p.lmax[h];
    const int ns = p.nsteps[h];
    const int64_t s0 = p.sbeg[h];
    const int twords = (1 << lmax) > 4 ? (1 << lmax) / 4 : 1;
    for (int i = tt; i < twords; i += TEAM) sTab[(team << (TLOG - 2)) + i] = 0u;
    team_sync<TEAM>();
    if (tt == 0) A[0] = 1u;  // (cas-register) starts at nil: state id 0, nothing linearized
    // per-wave window over the step stream: lane i holds word wbase + i
    int64_t wbase = -(1ll << 40), pos = s0;
    uint32_t win = 0;
    unsigned long long expl = 0;
    int fail_t = -1;
    for (int t = 0; t < ns; ++t) {
      if (pos + 32 > wbase + 64) {
        wbase = pos;
        win = (wbase + lane < p.stream_words) ? p.stream[wbase + lane] : 0u;
      }
      const uint32_t H = (uint32_t)__shfl((int)win, (int)(pos - wbase), 64);
      const uint32_t live = H & 0x3fffffu;
      const int j = (int)((H >> 22) & 31u);
      const int ninv = (int)(H >> 27);
      {
        const uint32_t w = (uint32_t)__shfl((int)win, (int)((pos + 1 + lane - wbase) & 63), 64);
        if (tt < ninv) opt[w & 31u] = w >> 8;
      }
      pos += 1 + ninv;
      team_sync<TEAM>();
      const int L = 32 - __clz((int)live);
      const uint32_t jb = 1u << j;
      const uint32_t opj = opt[j];
      // ---- closure layers
      for (int pc = 1; pc <= L; ++pc) {
        const uint32_t np = sBinom[L * BINOM_N + pc];
        const uint32_t chunk = (np + TEAM - 1) / TEAM;
        uint32_t r = (uint32_t)tt * chunk;
        if (r < np) {
          const uint32_t rend = min(r + chunk, np);
          // colex unrank of r among the C(L, pc) masks of popcount pc
          uint32_t m = 0, rr = r;
          for (int b = L - 1, k = pc; b >= 0 && k > 0; --b) {
            const uint32_t c = sBinom[b * BINOM_N + k];
            if (rr >= c) {
              m |= 1u << b;
              rr -= c;
              --k;
            }
          }
          for (; r < rend; ++r) {
            if (!(m & ~live)) {
              uint32_t res;
              if (m & jb) {
                const uint32_t s = A[m ^ jb];
                res = reg_step(opj, s);
                st_cand += __popc(s & opj & 0xffu);
              } else {
                res = 0;
                uint32_t bits = m;
                while (bits) {
                  const int k = __builtin_ctz(bits);
                  bits &= bits - 1;
                  const uint32_t op = opt[k];
                  const uint32_t s = A[m ^ (1u << k)];
                  res |= reg_step(op, s);
                  st_cand += __popc(s & op & 0xffu);
                }
              }
              if (res) {
                expl += __popc(res);
                A[m] = (uint8_t)(A[m] | res);
              }
            }
            // Gosper: next mask with the same popcount
            const uint32_t c = m & (0u - m), nx = m + c;
            m = (((nx ^ m) >> 2) >> __builtin_ctz(c)) | nx;
          }
        }
        team_sync<TEAM>();
      }
      // ---- return j: the post-return frontier moves down to the masks without j
      const uint32_t half = 1u << (L - 1);
      uint32_t anyv = 0;
      for (uint32_t i = (uint32_t)tt; i < half; i += TEAM) {
        const uint32_t lo = i & (jb - 1);
        const uint32_t m = ((i ^ lo) << 1) | lo;
        const uint32_t v = A[m | jb];
        A[m] = (uint8_t)v;
        A[m | jb] = 0;
        anyv |= v;
        st_fout += __popc(v);
      }
      ++st_steps;
      if (!team_any<TEAM>(anyv != 0)) {
        fail_t = t;
        break;
      }
    }
    // explored: team reduction
    if constexpr (TEAM == DENSE_BLOCK) {
      for (int off = 32; off > 0; off >>= 1) expl += __shfl_down(expl, off, 64);
      if (lane == 0 && expl) atomicAdd(&sExpl[team], expl);
      __syncthreads();
      expl = sExpl[team];
    } else {
      for (int off = 32; off > 0; off >>= 1) expl += __shfl_down(expl, off, 64);
      expl = __shfl(expl, 0, 64);
    }
    if (tt == 0) {
      p.explored[h] = expl;
      p.fail_step[h] = fail_t;
      p.status[h] = fail_t >= 0 ? ST_INVALID : ST_VALID;
    }
    team_sync<TEAM>();
  }
  // launch statistics (per wave, one atomic each)
  for (int off = 32; off > 0; off >>= 1) {
    st_cand += __shfl_down(st_cand, off, 64);
    st_fout += __shfl_down(st_fout, off, 64);
  }
  if (lane == 0) {
    if (st_cand) atomicAdd(&p.stats[SS_CAND], st_cand);
    if (st_fout) atomicAdd(&p.stats[SS_FOUT], st_fout);
  }
  if (tt == 0 && st_steps) atomicAdd(&p.stats[SS_STEPS], st_steps);
}

}  // namespace

int dense_grid_size(bool wave_teams) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
  int per_cu = 0;
  hipError_t e = wave_teams
      ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dense_kernel<64, DENSE_WAVE_LMAX>, DENSE_BLOCK, 0)
      : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, dense_kernel<DENSE_BLOCK, DENSE_LMAX>, DENSE_BLOCK, 0);
  if (e != hipSuccess || per_cu < 1) return 0;
  return prop.multiProcessorCount * per_cu;
}

hipError_t launch_dense(const DenseParams& p, bool wave_teams, int grid, hipStream_t stream) {
  if (wave_teams)
    hipLaunchKernelGGL((dense_kernel<64, DENSE_WAVE_LMAX>), dim3(grid), dim3(DENSE_BLOCK), 0, stream, p);
  else
    hipLaunchKernelGGL((dense_kernel<DENSE_BLOCK, DENSE_LMAX>), dim3(grid), dim3(DENSE_BLOCK), 0, stream, p);
  return hipGetLastError();
}

}  // namespace lc
