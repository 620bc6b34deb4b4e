// wide.hip — the closure-table search with its tables in HBM (wide.hpp), for
// cas-register histories of live width DENSE_WIDE_LMAX < L <= WIDE_LMAX: knossos.linear/analysis
// [ext] with CASRegister.step (a6) on whole byte-sliced words, as dense.hip,
// bit-exact with it and with the oracle.
//
// One persistent launch runs the wide histories one after another; all workgroups work on the
// same history. RETURN step t (its table T_t = tab(t & 1), the previous step's T_{t-1} intact):
//   for q = 0..H:  every word w of popcount q with w within the live hi slots, spread over the
//                  whole grid: X = T_{t-1} read through the previous return (pipe_x), the pulls
//                  T_t[w \ b] over w's set bits, the in-word closure; T_t[w] = X | R
//                  grid barrier
// so the DP is dense.hip's run_layers with the layers as grid-wide phases. A layer's words are
// (high part a, low part from the sorted word list): w = a << k | low, k = min(H, 19), the
// 2^(H-k) <= 512 high parts in a per-layer prefix table (LDS), so a thread's word comes from a
// binary search over <= 9 entries and one list load, and consecutive threads take consecutive
// low words of one high part (neighbouring table words).
// Failure: each step ORs "some X was nonzero" (step t-1's post-return frontier held a config)
// into `any` as an atomicMax of t + 1 before its last barrier; after it every workgroup reads
// the same value, so all leave together (an empty frontier stays empty).
#include "ctab.hpp"
#include "dense.hpp"
#include "dense_ops.hpp"
#include "device_common.hpp"
#include "search.hpp"
#include "wide.hpp"

#include <algorithm>

namespace lc {
namespace {

constexpr int WWG = 1024;
#ifndef LC_WIDE_MINW_EU
#define LC_WIDE_MINW_EU 5
#endif
#ifndef LC_WIDE_PWG
#define LC_WIDE_PWG 256
#endif
// the pipelined kernel's workgroup: 256 threads with <= 102 VGPRs, so 5 waves per SIMD (a
// 1024-thread workgroup holds a CU at 4)
constexpr int WPWG = LC_WIDE_PWG;
constexpr int WP_MINW = WPWG == 1024 ? 1 : LC_WIDE_MINW_EU;
constexpr int WB = 34;  // binomials C(n, k) for n <= 33 (u32: C(33, 16) = 1,166,803,110)
constexpr int WH = WIDE_LMAX - 3;  // most hi bits
constexpr int WPRE = 513;          // per layer: prefix over <= 512 high parts, + the total

struct WideBar {  // two-level arrival counters + generation, each on its own 128-B lines
  unsigned grp[8][32];
  unsigned top;
  unsigned pad0[31];
  unsigned gen;
  unsigned pad1[31];
};

// Grid barrier (search.hip's grid_sync without fences): every wave drains its sc1 stores, one
// lane per workgroup arrives on its group's counter, the last of a group on the top counter,
// the last of those bumps the generation the others poll (relaxed loads, s_sleep); p.watchdog
// (20 s by default) without a release raises *abort. The table words are sc1 stores read with sc1 loads.
__device__ __forceinline__ bool wide_sync(const WideParams& p, int* sAbort) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    WideBar* bar = reinterpret_cast<WideBar*>(p.bar);
    const unsigned nwg = gridDim.x;
    const unsigned g = ld_agent(&bar->gen);
    const unsigned grp = blockIdx.x & 7u;
    const unsigned gsize = (nwg - grp + 7u) >> 3;
    const unsigned ngroups = nwg < 8u ? nwg : 8u;
    // (test hook LC_WIDE_STALL: the armed workgroup skips this one arrival, so the barrier
    // really stalls and the watchdog has to end the launch; null in production)
    bool skip = false;
    if (p.stall && (int)blockIdx.x == p.stall_wg && ld_agent(p.stall) == 1) {
      st_agent(p.stall, 2);
      skip = true;
    }
    if (!skip && __hip_atomic_fetch_add(&bar->grp[grp][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
      st_agent(&bar->grp[grp][0], 0u);
      if (__hip_atomic_fetch_add(&bar->top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ngroups - 1) {
        st_agent(&bar->top, 0u);
        __hip_atomic_store(&bar->gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    long spins = 0;
    while (ld_agent(&bar->gen) == g) {
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 255) == 0) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > p.watchdog) {
          st_agent(p.abort, 1);
          break;
        }
        if (ld_agent(p.abort)) break;
      }
    }
    *sAbort = ld_agent(p.abort);
  }
  __syncthreads();
  return *sAbort == 0;
}

// pulls of word w from T_t over its set bits (only j's when it holds j), eight loads in flight
// per round: the loads are independent, so a round costs one HBM round trip
__device__ __forceinline__ uint64_t wide_pulls(const uint64_t* B, uint32_t w, uint32_t jh, const OpSel* ops,
                                              uint64_t foldm) {
  uint32_t m = (w & jh) ? jh : w;
  uint64_t R = 0;
  while (m) {
    int bb[8];
    uint64_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      bb[u] = m ? __builtin_ctz(m) : -1;
      m &= m - 1;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = bb[u] >= 0 ? HbmTab::ld(&B[w ^ (1u << bb[u])]) : 0ull;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (bb[u] >= 0) R |= transfer(ops[bb[u] + 3], (foldm >> (bb[u] + 3)) & 1u, v[u]);
  }
  return R;
}

// ---- the pipelined kernel's table layout: word w (hi bits of one step, all < 2^Hm) lives at
// off[|w|] + colex(w), off[q] = sum_{p < q} C(Hm, p) and colex(w) = sum_i C(pos_i, i + 1) over
// w's set bits in ascending order (i = 0, 1, ...): its index among the words of its popcount in
// ascending order. A layer's words are one contiguous span, and a run of consecutive low words
// under one high part (how the kernel hands words to threads) is a run of consecutive addresses.
// (8 set bits per round: the binomial reads of a round are independent, one LDS wait per round)
__device__ __forceinline__ uint32_t colex_rank(uint32_t w, const uint32_t* bin, uint32_t* T0 = nullptr) {
  uint32_t r = 0, t0 = 0;
  for (int i = 0; w; i += 8) {
    int bb[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      bb[u] = w ? __builtin_ctz(w) : -1;
      w &= w - 1;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (bb[u] >= 0) {
        r += bin[bb[u] * WB + i + u + 1];
        if (T0) t0 += bin[bb[u] * WB + i + u];
      }
  }
  if (T0) *T0 = t0;
  return r;
}

// wide_pulls over the ranked layout: the pull of bit b_m (the m-th set bit of w) reads
// off[|w| - 1] + sum_{i < m} C(pos_i, i + 1) + sum_{i > m} C(pos_i, i); T0 = sum_i C(pos_i, i).
// Rounds of 8 of w's set bits (up to the last pulled one): their binomials, then their pulls.
__device__ __forceinline__ uint64_t wide_pulls_ranked(const uint64_t* B, uint32_t w, uint32_t jh, const OpSel* ops,
                                                     uint64_t foldm, const uint32_t* bin, uint32_t off_dn,
                                                     uint32_t T0) {
  const uint32_t m = (w & jh) ? jh : w;
  uint32_t x = (w & jh) ? w & ((jh << 1) - 1u) : w;
  uint32_t P1 = 0, P0 = 0;
  uint64_t R = 0;
  for (int i = 0; x; i += 8) {
    int bb[8];
    uint32_t ix[8];
    uint64_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      bb[u] = x ? __builtin_ctz(x) : -1;
      x &= x - 1;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      ix[u] = 0xffffffffu;
      if (bb[u] >= 0) {
        const uint32_t c0 = bin[bb[u] * WB + i + u], c1 = bin[bb[u] * WB + i + u + 1];
        P0 += c0;
        if ((m >> bb[u]) & 1u) ix[u] = off_dn + P1 + (T0 - P0);
        P1 += c1;
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = ix[u] != 0xffffffffu ? HbmTab::ld(&B[ix[u]]) : 0ull;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (ix[u] != 0xffffffffu) R |= transfer(ops[bb[u] + 3], (foldm >> (bb[u] + 3)) & 1u, v[u]);
  }
  return R;
}

// ---- slabs (DESIGN.md §3.10 "Slabs"): the top `split` hi bits of a word w
// pick its slab s = w >> Hl, Hl = Hm - split <= 32; inside the slab w is ranked over its low Hl
// bits (wl) as above. A pull over a split bit reads the same local index in the neighbouring slab
// (index - 2^b); every other access stays inside w's slab. split 0 is the single ranked table.
__device__ __forceinline__ uint64_t slab_index(uint64_t w, int Hl, const uint32_t* bin, const uint32_t* off) {
  const uint32_t wl = (uint32_t)(w & ((1ull << Hl) - 1ull));
  return ((w >> Hl) << Hl) + off[__popc(wl)] + colex_rank(wl, bin);
}

__global__ void __launch_bounds__(WWG) wide_kernel(WideParams p) {
  __shared__ uint32_t sBin[WB * WB];
  __shared__ uint32_t sPre[(WH + 1) * WPRE];
  __shared__ uint32_t sLay[WIDE_LOW_BITS + 2];  // first entry of each popcount layer of the list
  __shared__ OpSel sOps[WIDE_OPS];               // slot k's op
  __shared__ uint64_t sHdr[4];                   // live, j, fresh, foldm
  __shared__ unsigned long long sRed;
  __shared__ int sAbort;
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < WB * WB; i += WWG) {
    const int n = i / WB, k = i % WB;
    uint64_t c = 0;
    if (k <= n) {
      c = 1;
      for (int q = 1; q <= k; ++q) c = c * (uint64_t)(n - k + q) / (uint64_t)q;
    }
    sBin[i] = (uint32_t)c;
  }
  if (tid == 0) sAbort = 0;
  __syncthreads();
  if (tid <= WIDE_LOW_BITS + 1) {
    uint32_t o = 0;
    for (int r = 0; r < tid; ++r) o += sBin[DENSE_WORD_BITS * WB + r];
    sLay[tid] = o;
  }
  const int64_t gtid = (int64_t)blockIdx.x * WWG + tid, gstride = (int64_t)gridDim.x * WWG;
  unsigned long long st_fout = 0, st_steps = 0, st_wv = 0, st_wnz = 0;
  for (int i = 0; i < p.n; ++i) {
    const int ns = p.nsteps[i];
    if (p.stall && i == p.stall_hist && (int)blockIdx.x == p.stall_wg && tid == 0) st_agent(p.stall, 1);
    uint64_t* const T0 = p.tab;
    uint64_t* const T1 = p.tab + p.tab_words;
    auto tab = [&](int t) { return (t & 1) ? T1 : T0; };
    // step 0 reads its frontier from tab(-1) = T1, at word 0 only (every slot is fresh there):
    // the initial config (register nil = state 0, nothing linearized)
    if (blockIdx.x == 0 && tid == 0) HbmTab::st(&T1[0], 1ull);
    if (tid < WIDE_OPS) sOps[tid] = OpSel{SEL_NONE, SEL_NONE};
    if (!wide_sync(p, &sAbort)) break;
    unsigned long long expl = 0;
    int fail_t = -1, cH = -1, pj = -1;
    uint64_t plive = 0;
    int64_t pos = p.sbeg[i];
    for (int t = 0; t < ns; ++t) {
      // ---- decode (wave 0 of every workgroup): 2 header words, then the op words
      if (tid < 64) {
        const uint32_t wd = p.stream[pos + lane];
        const uint64_t live = (uint64_t)(uint32_t)__shfl((int)wd, 0, 64) |
                              ((uint64_t)(uint32_t)__shfl((int)wd, 1, 64) << 31);
        const uint32_t j = (uint32_t)__shfl((int)wd, 2, 64);
        const unsigned long long ob = __ballot(lane >= 3 && lane < 3 + WIDE_MAX_NINV && (wd & DENSE_OPW));
        const int ninv = (int)__builtin_ctzll(~(ob >> 3));
        if (lane >= 3 && lane < 3 + ninv) sOps[wd & 63u] = decode_op((wd >> 8) & 0xffu, (wd >> 16) & 0xffu);
        // (after the stores: one wave's LDS ops stay in order)
        const uint64_t foldm = __ballot(lane < WIDE_OPS && sOps[lane < WIDE_OPS ? lane : 0].hi == OPS_FOLD);
        if (lane == 0) {
          sHdr[0] = live;
          sHdr[1] = j;
          sHdr[2] = t > 0 ? live & ~(plive & ~(1ull << pj)) : live;  // slots invoked since the last return
          sHdr[3] = foldm;
        }
        pos += 3 + ninv;
      }
      __syncthreads();
      const uint64_t live = sHdr[0], fresh = sHdr[2], foldm = sHdr[3];
      const int j = (int)sHdr[1], jp = pj;
      const int L = 64 - __clzll((long long)live);
      const int H = L > 3 ? L - 3 : 0;
      const int k = H < WIDE_LOW_BITS ? H : WIDE_LOW_BITS, hb = H - k;
      if (H != cH) {  // layer q's prefix over the high parts: sPre[q][a] = sum_{a' < a} C(k, q - |a'|)
        if (tid <= H) {
          uint32_t acc = 0;
          for (int a = 0; a < (1 << hb); ++a) {
            sPre[tid * WPRE + a] = acc;
            const int r = tid - __popc(a);
            if (r >= 0 && r <= k) acc += sBin[k * WB + r];
          }
          sPre[tid * WPRE + (1 << hb)] = acc;
        }
        cH = H;
        __syncthreads();
      }
      const uint32_t live_hi = (uint32_t)(live >> 3), fresh_hi = (uint32_t)(fresh >> 3);
      const uint32_t jh = j >= 3 ? 1u << (j - 3) : 0u;
      uint64_t keep_lo = ~0ull;
#pragma unroll
      for (int kk = 0; kk < 3; ++kk)
        if (fresh & (1u << kk)) keep_lo &= keep64(kk);
      uint64_t* const B = tab(t);
      const uint64_t* const Bp = tab(t - 1);
      uint64_t anyx = 0;
      bool ok = true;
      for (int q = 0; q <= H && ok; ++q) {
        const uint32_t* pre = &sPre[q * WPRE];
        const uint32_t N = pre[1 << hb];
        for (int64_t g = gtid; g < (int64_t)N; g += gstride) {
          uint32_t a = 0;  // the last high part whose prefix is <= g (it holds g: its count > 0)
          for (int bit = hb - 1; bit >= 0; --bit)
            if (pre[a | (1u << bit)] <= (uint32_t)g) a |= 1u << bit;
          const int r = q - __popc(a);
          const uint32_t w = (a << k) | p.words[sLay[r] + ((uint32_t)g - pre[a])];
          if (w & ~live_hi) continue;
          uint64_t X = 0;
          if (!(w & fresh_hi)) {  // the previous step's post-return table, read through its slot jp
            if (jp >= 3) X = HbmTab::ld(&Bp[w | (1u << (jp - 3))]);
            else if (jp >= 0) X = (HbmTab::ld(&Bp[w]) & ~keep64(jp)) >> (1 << jp);
            else X = HbmTab::ld(&Bp[w]);
            X &= keep_lo;
          }
          uint64_t R = wide_pulls(B, w, jh, sOps, foldm);
          R = close_in_word(X, w, (uint32_t)live, j, sOps, (uint32_t)foldm, R);
          HbmTab::st(&B[w], X | R);
          expl += (uint64_t)__popcll(R);
          if (t > 0) st_fout += (uint64_t)__popcll(X);
          anyx |= X;
          ++st_wv, st_wnz += (X | R) != 0;
        }
        if (q == H && __any(anyx != 0) && lane == 0)  // step t-1's post-return frontier held a config
          __hip_atomic_fetch_max(&p.any[i], (unsigned long long)(t + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = wide_sync(p, &sAbort);
      }
      if (!ok) break;
      ++st_steps;
      plive = live, pj = j;
      if (t > 0 && ld_agent(&p.any[i]) < (unsigned long long)(t + 1)) {  // the same value in every workgroup
        fail_t = t - 1;
        break;
      }
    }
    if (sAbort) break;
    if (fail_t < 0 && ns > 0) {  // the last step's return: its frontier must hold a config
      const uint64_t lv = plive & ~(1ull << pj);
      const int Lf = lv ? 64 - __clzll((long long)lv) : 0;
      const int64_t nwt = (int64_t)1 << (Lf > 3 ? Lf - 3 : 0);
      const uint64_t* const Bl = tab(ns - 1);
      uint64_t nz = 0;
      for (int64_t w = gtid; w < nwt; w += gstride) {
        if ((uint64_t)w & ~(lv >> 3)) continue;
        uint64_t X;
        if (pj >= 3) X = HbmTab::ld(&Bl[(uint32_t)w | (1u << (pj - 3))]);
        else X = (HbmTab::ld(&Bl[w]) & ~keep64(pj)) >> (1 << pj);
        st_fout += (uint64_t)__popcll(X);
        nz |= X;
      }
      if (__any(nz != 0) && lane == 0)
        __hip_atomic_fetch_max(&p.any[i], (unsigned long long)(ns + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!wide_sync(p, &sAbort)) break;
      if (ld_agent(&p.any[i]) < (unsigned long long)(ns + 1)) fail_t = ns - 1;
    }
    // explored: one add per workgroup
    for (int off = 32; off > 0; off >>= 1) expl += __shfl_down(expl, off, 64);
    if (tid == 0) sRed = 0;
    __syncthreads();
    if (lane == 0 && expl) atomicAdd(&sRed, expl);
    __syncthreads();
    if (tid == 0 && sRed) atomicAdd(&p.explored[i], sRed);
    // (the next history's first store is to T1[0]: every workgroup is past this one's reads)
    if (!wide_sync(p, &sAbort)) break;
    // the verdict only once every workgroup has added its explored count (a workgroup whose
    // watchdog fires at this barrier leaves without it, and then the history stays unfinished)
    if (blockIdx.x == 0 && tid == 0) {
      p.status[i] = fail_t >= 0 ? ST_INVALID : ST_VALID;
      p.fail_step[i] = fail_t;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    st_fout += __shfl_down(st_fout, off, 64);
    st_wv += __shfl_down(st_wv, off, 64);
    st_wnz += __shfl_down(st_wnz, off, 64);
  }
  if (lane == 0 && st_fout) atomicAdd(&p.stats[0], st_fout);
  if (blockIdx.x == 0 && tid == 0 && st_steps) atomicAdd(&p.stats[1], st_steps);
  if (lane == 0 && st_wv) atomicAdd(&p.stats[2], st_wv);
  if (lane == 0 && st_wnz) atomicAdd(&p.stats[3], st_wnz);
}

// ---- pipelined steps (WideParams.pipe): the schedule of dense.hip's history_pipe with the whole
// grid as the team. Step t+1's layer q reads step t's words of popcount <= q + 1 (its X through
// a hi return) or q (an in-word return) and writes words of popcount q on the other table, so it
// runs in the same super-layer as step t's layer q + 2 (q + 1): a step starts two super-layers
// after its predecessor (one after an in-word return; at once when the predecessor has retired)
// and a grid barrier ends each super-layer, ~1.7 per step instead of H + 1. Step t shares its
// table with step t - 2, which is at least two super-layers ahead (dense.hip §3.2's argument).
// A super-layer's words are the running steps' layers, one flat index over the grid; a layer's
// word g is (high part, low part) by popcount of the high part p (C(hb, p) highs of popcount p,
// each with C(k, q - p) lows; both parts from the sorted word list), so no per-layer tables.
// Its tables use the ranked layout (colex_rank): word w at off[|w|] + colex(w).
// Failure: a workgroup that reads a nonzero X in step t sets bit t of `anyv`; when step t retires
// (after its last layer's barrier) every workgroup reads the bit: 0 means step t - 1 returned an
// empty frontier.
#ifndef LC_WIDE_KLO
#define LC_WIDE_KLO 19
#endif
#ifndef LC_WIDE_XCD
#define LC_WIDE_XCD 1
#endif
constexpr int WRING = 16;
struct WStep {
  OpSel ops[WIDE_OPS];
  uint64_t live, fresh, foldm;
  int32_t j, jp, H, start;
};

__global__ void __launch_bounds__(WPWG, WP_MINW) wide_pipe_kernel(WideParams p) {
  __shared__ uint32_t sBin[WB * WB];
  __shared__ uint32_t sLay[WIDE_LOW_BITS + 2];
  __shared__ WStep sRing[WRING];
  __shared__ uint64_t sSeg[WRING + 1];  // running segments' first flat index (+ the total)
  __shared__ uint32_t sOff[WH + 2];     // the ranked layout's layer offsets inside a slab (colex_rank)
  __shared__ unsigned long long sRed;
  __shared__ int sAbort;
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < WB * WB; i += WPWG) {
    const int n = i / WB, k = i % WB;
    uint64_t c = 0;
    if (k <= n) {
      c = 1;
      for (int q = 1; q <= k; ++q) c = c * (uint64_t)(n - k + q) / (uint64_t)q;
    }
    sBin[i] = (uint32_t)c;
  }
  if (tid == 0) sAbort = 0;
  __syncthreads();
  if (tid <= WIDE_LOW_BITS + 1) {
    uint32_t o = 0;
    for (int r = 0; r < tid; ++r) o += sBin[DENSE_WORD_BITS * WB + r];
    sLay[tid] = o;
  }
  const int Hl = 63 - __clzll((long long)p.tab_words) - p.split;  // (tab_words = 2^Hm; a slab 2^Hl)
  const uint64_t lmask = (1ull << Hl) - 1ull;
  if (tid <= WH + 1) {
    uint32_t o = 0;  // (off[Hl + 1] = 2^Hl wraps at Hl = 32: never read)
    for (int r = 0; r < tid && r <= Hl; ++r) o += sBin[Hl * WB + r];
    sOff[tid] = o;
  }
  // XCD-aware chunks: workgroups are dealt to the 8 XCDs round robin, so logical block
  // (b mod 8) * (grid / 8) + b / 8 gives each XCD one contiguous run of a super-layer's words per
  // pass (a high part's words and their low-bit pulls stay in one L2)
  const int nb = (int)gridDim.x, bx = (int)blockIdx.x;
  const int lb = (nb & 7) == 0 && LC_WIDE_XCD ? (bx & 7) * (nb >> 3) + (bx >> 3) : bx;
  const int64_t gtid = (int64_t)lb * WPWG + tid, gstride = (int64_t)gridDim.x * WPWG;
  unsigned long long st_fout = 0, st_steps = 0, st_wv = 0, st_wnz = 0;
  for (int i = 0; i < p.n && !sAbort; ++i) {
    const int ns = p.nsteps[i];
    if (p.stall && i == p.stall_hist && (int)blockIdx.x == p.stall_wg && tid == 0) st_agent(p.stall, 1);
    uint64_t* const T0 = p.tab;
    uint64_t* const T1 = p.tab + p.tab_words;
    auto tab = [&](int t) { return (t & 1) ? T1 : T0; };
    uint32_t* const anyv = p.anyv + p.anyv_off[i];
    if (blockIdx.x == 0 && tid == 0) HbmTab::st(&T1[0], 1ull);  // the initial config, read by step 0
    int64_t pos = p.sbeg[i];
    // decode step t into its ring slot (wave 0): the previous step's ops + this step's invocations
    auto decode = [&](int t) {
      if (tid >= 64) return;
      WStep* dst = &sRing[t % WRING];
      const WStep* prev = t > 0 ? &sRing[(t - 1) % WRING] : nullptr;
      const uint32_t wd = p.stream[pos + lane];
      const uint64_t live = (uint64_t)(uint32_t)__shfl((int)wd, 0, 64) |
                            ((uint64_t)(uint32_t)__shfl((int)wd, 1, 64) << 31);
      const uint32_t j = (uint32_t)__shfl((int)wd, 2, 64);
      const unsigned long long ob = __ballot(lane >= 3 && lane < 3 + WIDE_MAX_NINV && (wd & DENSE_OPW));
      const int ninv = (int)__builtin_ctzll(~(ob >> 3));
      const uint64_t plive = prev ? prev->live : 0ull;
      const int pj = prev ? (int)prev->j : -1;
      if (lane < WIDE_OPS) dst->ops[lane] = prev ? prev->ops[lane] : OpSel{SEL_NONE, SEL_NONE};
      if (lane >= 3 && lane < 3 + ninv) dst->ops[wd & 63u] = decode_op((wd >> 8) & 0xffu, (wd >> 16) & 0xffu);
      const uint64_t foldm = __ballot(lane < WIDE_OPS && dst->ops[lane < WIDE_OPS ? lane : 0].hi == OPS_FOLD);
      if (lane == 0) {
        const int L = 64 - __clzll((long long)live);
        dst->live = live;
        dst->fresh = prev ? live & ~(plive & ~(1ull << pj)) : live;
        dst->foldm = foldm;
        dst->j = (int32_t)j;
        dst->jp = pj;
        dst->H = L > 3 ? L - 3 : 0;
        dst->start = 1 << 30;
      }
      pos += 3 + ninv;
    };
    if (ns > 0) decode(0);
    __syncthreads();
    if (ns > 0 && tid == 0) sRing[0].start = 0;
    if (!wide_sync(p, &sAbort)) break;
    unsigned long long expl = 0;
    int fail_t = -1, t_dec = ns > 0 ? 1 : 0, t_run = t_dec, t_ret = 0;
    for (int s = 0; t_ret < ns; ++s) {
      // ---- retire the steps whose last layer ran before this super-layer, in order
      while (t_ret < t_run) {
        const WStep& r = sRing[t_ret % WRING];
        if (r.start + r.H >= s) break;
        if (t_ret > 0 && !((ld_agent(&anyv[t_ret >> 5]) >> (t_ret & 31)) & 1u)) {  // same in every workgroup
          fail_t = t_ret - 1;
          break;
        }
        ++t_ret;
        ++st_steps;
      }
      if (fail_t >= 0 || t_ret >= ns) break;
      // ---- this super-layer's segments: running step t in its layer q = s - start (C(H, q) words)
      if (tid <= WRING) {
        uint64_t acc = 0;
        for (int t = t_ret; t < t_run && t - t_ret < tid; ++t) {
          const WStep& r = sRing[t % WRING];
          const int q = s - r.start;
          if (q >= 0 && q <= r.H) acc += sBin[r.H * WB + q];
        }
        sSeg[tid] = acc;
      }
      __syncthreads();
      const uint64_t total = sSeg[t_run - t_ret];
      uint32_t anyseg = 0;  // running steps (bit t - t_ret) in which this thread read a nonzero X
      for (int64_t g = gtid; g < (int64_t)total; g += gstride) {
        int si = 0;  // the segment holding g
        while (si + 1 < t_run - t_ret && sSeg[si + 1] <= (uint64_t)g) ++si;
        const int t = t_ret + si;
        const WStep& r = sRing[t % WRING];
        const int H = r.H, q = s - r.start;
        const int k = max(H < LC_WIDE_KLO ? H : LC_WIDE_KLO, H - WIDE_LOW_BITS), hb = H - k;
        uint32_t gi = (uint32_t)((uint64_t)g - sSeg[si]);  // (< C(33, 16) < 2^32)
        int pp = q - k > 0 ? q - k : 0;  // the high part's popcount: blocks of C(hb, p) C(k, q - p)
        for (;; ++pp) {
          const uint32_t blk = sBin[hb * WB + pp] * sBin[k * WB + (q - pp)];
          if (gi < blk || pp >= hb || pp >= q) break;
          gi -= blk;
        }
        const uint32_t nlo = sBin[k * WB + (q - pp)];
        const uint32_t hi_i = gi / nlo, lo_i = gi - hi_i * nlo;
        const uint64_t w = (hb ? (uint64_t)p.words[sLay[pp] + hi_i] << k : 0ull) | p.words[sLay[q - pp] + lo_i];
        const uint64_t live = r.live;
        if (w & ~(live >> 3)) continue;
        const uint64_t fresh = r.fresh, foldm = r.foldm;
        const int j = (int)r.j, jp = r.jp;
        uint64_t X = 0;
        uint32_t T0;
        // w's slab (its first word sb) and its index inside it, over the slab's hi bits wl
        const uint32_t wl = (uint32_t)(w & lmask);
        const int ql = __popc(wl);
        const uint64_t sb = w & ~lmask;
        const uint64_t iw = sb + sOff[ql] + colex_rank(wl, sBin, &T0);
        if (!(w & (fresh >> 3))) {
          const uint64_t* Bp = tab(t - 1);
          if (jp >= 3) {  // w + jp: in w's slab, or (a split bit) the same index one slab up
            const int bp = jp - 3;
            X = HbmTab::ld(&Bp[bp < Hl ? sb + sOff[ql + 1] + colex_rank(wl | (1u << bp), sBin) : iw + (1ull << bp)]);
          } else if (jp >= 0) X = (HbmTab::ld(&Bp[iw]) & ~keep64(jp)) >> (1 << jp);
          else X = HbmTab::ld(&Bp[iw]);
#pragma unroll
          for (int kk = 0; kk < 3; ++kk)
            if (fresh & (1u << kk)) X &= keep64(kk);
        }
        uint64_t* const B = tab(t);
        const int bj = j - 3;  // the returning slot's hi bit (j >= 3)
        const bool hasj = j >= 3 && ((w >> bj) & 1ull);
        uint64_t R = 0;
        if (!hasj || bj < Hl)  // pulls over the slab's own bits (only j's when w holds j)
          R = wide_pulls_ranked(B + sb, wl, hasj ? 1u << bj : 0u, r.ops, foldm, sBin, ql > 0 ? sOff[ql - 1] : 0u, T0);
        // pulls over the split bits: the same local index in the slab without bit b
        for (uint64_t sm = hasj ? (bj >= Hl ? 1ull << bj : 0ull) : w & ~lmask; sm; sm &= sm - 1) {
          const int b = __builtin_ctzll(sm);
          R |= transfer(r.ops[b + 3], (foldm >> (b + 3)) & 1u, HbmTab::ld(&B[iw - (1ull << b)]));
        }
        R = close_in_word(X, hasj ? 1u : 0u, (uint32_t)live, j >= 3 ? 3 : j, r.ops, (uint32_t)foldm, R);
        HbmTab::st(&B[iw], X | R);
        expl += (uint64_t)__popcll(R);
        if (t > 0) st_fout += (uint64_t)__popcll(X);
        if (X) anyseg |= 1u << si;
        ++st_wv, st_wnz += (X | R) != 0;
      }
      // the steps this wave saw a config in: one atomic OR per step per wave
      for (int si = 0; si < t_run - t_ret; ++si)
        if (__any((anyseg >> si) & 1u) && lane == 0) {
          const int t = t_ret + si;
          __hip_atomic_fetch_or(&anyv[t >> 5], 1u << (t & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      // ---- decode ahead into a free ring slot, and start the next step at s + 1: two
      // super-layers after its predecessor (one after an in-word return, or the predecessor's
      // H + 1 if fewer), at once if the predecessor has retired
      const int t_dec_old = t_dec;
      if (t_dec < ns && t_dec - t_ret < WRING - 1) {
        decode(t_dec);
        ++t_dec;
      }
      __syncthreads();
      if (t_run < t_dec_old) {
        bool ok = true;
        if (t_run - 1 >= t_ret) {
          const WStep& pr = sRing[(t_run - 1) % WRING];
          const int gap = pr.j < 3 ? 1 : 2;
          ok = s + 1 - pr.start >= min(gap, pr.H + 1);
        }
        if (ok) {
          if (tid == 0) sRing[t_run % WRING].start = s + 1;
          ++t_run;
        }
      }
      if (!wide_sync(p, &sAbort)) break;
    }
    if (sAbort) break;
    if (fail_t < 0 && ns > 0) {  // the last step's return: its frontier must hold a config
      const WStep& r = sRing[(ns - 1) % WRING];
      const int pj = (int)r.j;
      const uint64_t lv = r.live & ~(1ull << pj);
      const int Lf = lv ? 64 - __clzll((long long)lv) : 0;
      const int64_t nwt = (int64_t)1 << (Lf > 3 ? Lf - 3 : 0);
      const uint64_t* const Bl = tab(ns - 1);
      uint64_t nz = 0;
      for (int64_t w = gtid; w < nwt; w += gstride) {
        if ((uint64_t)w & ~(lv >> 3)) continue;
        const uint64_t wr = pj >= 3 ? (uint64_t)w | (1ull << (pj - 3)) : (uint64_t)w;
        uint64_t X = HbmTab::ld(&Bl[slab_index(wr, Hl, sBin, sOff)]);
        if (pj < 3) X = (X & ~keep64(pj)) >> (1 << pj);
        st_fout += (uint64_t)__popcll(X);
        nz |= X;
      }
      if (__any(nz != 0) && lane == 0)
        __hip_atomic_fetch_or(&anyv[ns >> 5], 1u << (ns & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!wide_sync(p, &sAbort)) break;
      if (!((ld_agent(&anyv[ns >> 5]) >> (ns & 31)) & 1u)) fail_t = ns - 1;
    }
    for (int off = 32; off > 0; off >>= 1) expl += __shfl_down(expl, off, 64);
    if (tid == 0) sRed = 0;
    __syncthreads();
    if (lane == 0 && expl) atomicAdd(&sRed, expl);
    __syncthreads();
    if (tid == 0 && sRed) atomicAdd(&p.explored[i], sRed);
    if (!wide_sync(p, &sAbort)) break;
    // the verdict only once every workgroup has added its explored count (a workgroup whose
    // watchdog fires at this barrier leaves without it, and then the history stays unfinished)
    if (blockIdx.x == 0 && tid == 0) {
      p.status[i] = fail_t >= 0 ? ST_INVALID : ST_VALID;
      p.fail_step[i] = fail_t;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    st_fout += __shfl_down(st_fout, off, 64);
    st_wv += __shfl_down(st_wv, off, 64);
    st_wnz += __shfl_down(st_wnz, off, 64);
  }
  if (lane == 0 && st_fout) atomicAdd(&p.stats[0], st_fout);
  if (blockIdx.x == 0 && tid == 0 && st_steps) atomicAdd(&p.stats[1], st_steps);
  if (lane == 0 && st_wv) atomicAdd(&p.stats[2], st_wv);
  if (lane == 0 && st_wnz) atomicAdd(&p.stats[3], st_wnz);
}

// ---- failure reports from the tables (lc_failure_configs). After a run that
// stopped after step t - 1 (WideParams nsteps = the failing step t), tab(t - 1) holds step t - 1's
// whole table; the frontier the failing RETURN saw is that table read through t - 1's returning
// slot jp (the X of step t; its fresh slots are not live yet), dumped here config by config.
__device__ __forceinline__ uint64_t dump_index(uint64_t w, const WideDumpParams& d, const uint32_t* bin,
                                               const uint32_t* off) {
  return d.ranked ? slab_index(w, d.Hm - d.split, bin, off) : w;
}

__global__ void __launch_bounds__(256) wide_dump_kernel(WideDumpParams d) {
  __shared__ uint32_t sBin[WB * WB];
  __shared__ uint32_t sOff[WH + 2];
  const int tid = threadIdx.x;
  for (int i = tid; i < WB * WB; i += 256) {
    const int n = i / WB, k = i % WB;
    uint64_t c = 0;
    if (k <= n) {
      c = 1;
      for (int q = 1; q <= k; ++q) c = c * (uint64_t)(n - k + q) / (uint64_t)q;
    }
    sBin[i] = (uint32_t)c;
  }
  __syncthreads();
  if (tid <= WH + 1) {
    uint32_t o = 0;
    for (int r = 0; r < tid && r <= d.Hm - d.split; ++r) o += sBin[(d.Hm - d.split) * WB + r];
    sOff[tid] = o;
  }
  __syncthreads();
  const int Lf = d.lv ? 64 - __clzll((long long)d.lv) : 0;
  const int64_t nwt = (int64_t)1 << (Lf > 3 ? Lf - 3 : 0);
  for (int64_t w = (int64_t)blockIdx.x * 256 + tid; w < nwt; w += (int64_t)gridDim.x * 256) {
    if ((uint64_t)w & ~(d.lv >> 3)) continue;
    const uint64_t wr = d.jp >= 3 ? (uint64_t)w | (1ull << (d.jp - 3)) : (uint64_t)w;
    uint64_t X = HbmTab::ld(&d.tab[dump_index(wr, d, sBin, sOff)]);
    if (d.jp < 3) X = (X & ~keep64(d.jp)) >> (1 << d.jp);
    if (!X) continue;
    unsigned long long at = atomicAdd(d.count, (unsigned long long)__popcll(X));
    for (; X; X &= X - 1, ++at) {
      const int b = __builtin_ctzll(X);
      if ((int64_t)at < d.cap) {
        d.masks[at] = ((uint64_t)w << 3) | (uint64_t)(b & 7);
        d.states[at] = (uint8_t)(b >> 3);
      }
    }
  }
}

// out[i] = table word at the hi-bit word hw[i] (the ranked or natural index, as dump_index)
__global__ void __launch_bounds__(256) wide_gather_kernel(WideDumpParams d, const uint64_t* hw, uint64_t* out, int n) {
  __shared__ uint32_t sBin[WB * WB];
  __shared__ uint32_t sOff[WH + 2];
  const int tid = threadIdx.x;
  for (int i = tid; i < WB * WB; i += 256) {
    const int nn = i / WB, k = i % WB;
    uint64_t c = 0;
    if (k <= nn) {
      c = 1;
      for (int q = 1; q <= k; ++q) c = c * (uint64_t)(nn - k + q) / (uint64_t)q;
    }
    sBin[i] = (uint32_t)c;
  }
  __syncthreads();
  if (tid <= WH + 1) {
    uint32_t o = 0;
    for (int r = 0; r < tid && r <= d.Hm - d.split; ++r) o += sBin[(d.Hm - d.split) * WB + r];
    sOff[tid] = o;
  }
  __syncthreads();
  for (int i = blockIdx.x * 256 + tid; i < n; i += gridDim.x * 256)
    out[i] = HbmTab::ld(&d.tab[dump_index(hw[i], d, sBin, sOff)]);
}


// ---- counter histories on the HBM tables (r5): ctab.hip's
// closure tables (one bit per mask, the value a function of the mask, consistency an EQ lookup:
// CounterModel.step, counter.clj:100-127) past the tile teams' 24 slots, to WCTR_LMAX, on the
// pipelined grid-wide schedule above. A word holds the 64 masks over slots 0..5; slots >= 6 are
// its hi bits (H = L - 6 <= 32, so one ranked table with a 32-bit index, no slabs). Per step (decoded by one wave into
// the LDS ring): the per-slot requirement relative to the config's low sum (cq), the 64-entry
// EQ table over the low sums and five 64-entry tables of hi delta sums (6 hi slots each) and one of 4 (slots 36, 37).
constexpr int32_t WC_UNC = 0x3fffffff;    // cq sentinel: the op steps from any config
constexpr int32_t WC_NEVER = -0x3fffffff;  // ... from none
constexpr int WC_LO = 6;
constexpr int WC_SLOTS = 40;  // per-slot tables (slots 0..37, padded)

struct WCStep {
  uint64_t live, fresh, keep_lo;
  int32_t j, jp, H, start, base;
  int32_t req[WC_SLOTS];
  int32_t cq[WC_SLOTS];
  int8_t d[WC_SLOTS];
  int16_t sh[5][64];  // hi slots 6 + 6g .. 11 + 6g by (w >> 6g) & 63
  int16_t sh5[4];     // hi slots 36, 37 by w >> 30
  uint64_t eq[64];    // EQ[v]: positions p (low masks) with S_lo(p) - lo_min = v
};

__device__ __forceinline__ uint64_t wc_keep6(int k) {
  switch (k) {
    case 0: return 0x5555555555555555ull;
    case 1: return 0x3333333333333333ull;
    case 2: return 0x0f0f0f0f0f0f0f0full;
    case 3: return 0x00ff00ff00ff00ffull;
    case 4: return 0x0000ffff0000ffffull;
    default: return 0x00000000ffffffffull;
  }
}

__device__ __forceinline__ uint64_t wc_gate(const WCStep& st, int32_t c, int s) {
  if (c == WC_UNC) return ~0ull;
  const uint32_t i = (uint32_t)(c - s);
  return i < 64u ? st.eq[i] : 0ull;
}

// Step stream of a wide counter history (host-built, WideParams.stream):
//   header words 0, 1, 2  live slots 0..30 | live slots 31..61 (bit k - 31) | j, bit 31 clear
//   per invocation since the previous step, ctab.hpp's two words (bit 31 set):
//     w0 = slot[0:8) | flags[8:16) | (uint8_t)delta[16:24)        flags: CT_UNC, CT_NEVER
//     w1 = (req + CTAB_REQ_BIAS) & 0x3fffffff
//   (at most WCTR_MAX_NINV invocations per step: the whole step in one 64-lane read)
//   a 0 word after the last step
__global__ void __launch_bounds__(WPWG, WP_MINW) wctr_pipe_kernel(WideParams p) {
  __shared__ uint32_t sBin[WB * WB];
  __shared__ uint32_t sLay[WIDE_LOW_BITS + 2];
  __shared__ WCStep sRing[WRING];
  __shared__ uint64_t sSeg[WRING + 1];
  __shared__ uint32_t sOff[WH + 2];
  __shared__ unsigned long long sRed;
  __shared__ int sAbort;
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < WB * WB; i += WPWG) {
    const int n = i / WB, k = i % WB;
    uint64_t c = 0;
    if (k <= n) {
      c = 1;
      for (int q = 1; q <= k; ++q) c = c * (uint64_t)(n - k + q) / (uint64_t)q;
    }
    sBin[i] = (uint32_t)c;
  }
  if (tid == 0) sAbort = 0;
  __syncthreads();
  if (tid <= WIDE_LOW_BITS + 1) {
    uint32_t o = 0;
    for (int r = 0; r < tid; ++r) o += sBin[DENSE_WORD_BITS * WB + r];
    sLay[tid] = o;
  }
  const int Hm = 63 - __clzll((long long)p.tab_words);  // (tab_words = 2^Hm, Hm <= 32)
  if (tid <= WH + 1) {
    uint32_t o = 0;
    for (int r = 0; r < tid && r <= Hm; ++r) o += sBin[Hm * WB + r];
    sOff[tid] = o;
  }
  const int nb = (int)gridDim.x, bx = (int)blockIdx.x;
  const int lb = (nb & 7) == 0 && LC_WIDE_XCD ? (bx & 7) * (nb >> 3) + (bx >> 3) : bx;
  const int64_t gtid = (int64_t)lb * WPWG + tid, gstride = (int64_t)gridDim.x * WPWG;
  unsigned long long st_fout = 0, st_steps = 0, st_wv = 0, st_wnz = 0;
  for (int i = 0; i < p.n && !sAbort; ++i) {
    const int ns = p.nsteps[i];
    uint64_t* const T0 = p.tab;
    uint64_t* const T1 = p.tab + p.tab_words;
    auto tab = [&](int t) { return (t & 1) ? T1 : T0; };
    uint32_t* const anyv = p.anyv + p.anyv_off[i];
    // the initial config: nothing linearized (mask 0 = word 0, position 0), read by step 0
    if (blockIdx.x == 0 && tid == 0) HbmTab::st(&T1[0], 1ull);
    int64_t pos = p.sbeg[i];
    auto decode = [&](int t) {  // (wave 0) ctab.hip's ct_decode with 64-bit live masks
      if (tid >= 64) return;
      WCStep* dst = &sRing[t % WRING];
      const WCStep* prev = t > 0 ? &sRing[(t - 1) % WRING] : nullptr;
      const uint32_t wd = p.stream[pos + lane];
      const uint64_t live = (uint64_t)(uint32_t)__shfl((int)wd, 0, 64) |
                            ((uint64_t)(uint32_t)__shfl((int)wd, 1, 64) << 31);
      const int j = __shfl((int)wd, 2, 64);
      const int nw = (int)__builtin_ctzll(~(__ballot(lane >= 3 && (wd & DENSE_OPW)) >> 3));
      const int ninv = nw >> 1;
      int32_t req = prev && lane < WC_SLOTS ? prev->req[lane] : WC_UNC;
      int32_t d = prev && lane < WC_SLOTS ? (int32_t)prev->d[lane] : 0;
      for (int k = 0; k < ninv; ++k) {
        const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)wd, 3 + 2 * k);
        const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)wd, 4 + 2 * k);
        if (lane == (int)(a & 63u)) {
          const uint32_t fl = (a >> 8) & 0xffu;
          d = (int32_t)(int8_t)(uint8_t)((a >> 16) & 0xffu);
          req = (fl & CT_UNC) ? WC_UNC : (fl & CT_NEVER) ? WC_NEVER : (int32_t)(b & 0x3fffffffu) - CTAB_REQ_BIAS;
        }
      }
      const uint64_t plive = prev ? prev->live : 0ull;
      const int pj = prev ? prev->j : -1;
      const int32_t base = prev ? prev->base + (int32_t)prev->d[pj] : 0;
      int32_t slo = 0, lo_min = 0;
#pragma unroll
      for (int k = 0; k < WC_LO; ++k) {
        const int32_t dk = __builtin_amdgcn_readlane(d, k);
        if ((lane >> k) & 1) slo += dk;
        lo_min += dk < 0 ? dk : 0;
      }
      if (lane < WC_SLOTS) {
        dst->req[lane] = req;
        dst->d[lane] = (int8_t)d;
        dst->cq[lane] = req == WC_UNC || req == WC_NEVER ? req : req - base - lo_min + (lane >= WC_LO ? d : 0);
      }
      dst->eq[lane] = 0;
      // (one wave's LDS operations stay in order: the zeroing lands before the ORs)
      __hip_atomic_fetch_or(&dst->eq[slo - lo_min], 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
      for (int g = 0; g < 5; ++g) {
        int32_t sm = 0;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          const int32_t dk = __builtin_amdgcn_readlane(d, WC_LO + 6 * g + k);
          if ((lane >> k) & 1) sm += dk;
        }
        dst->sh[g][lane] = (int16_t)sm;
      }
      if (lane < 4) {
        const int32_t d36 = __builtin_amdgcn_readlane(d, 36), d37 = __builtin_amdgcn_readlane(d, 37);
        dst->sh5[lane] = (int16_t)((lane & 1 ? d36 : 0) + (lane & 2 ? d37 : 0));
      }
      if (lane == 0) {
        const int L = live ? 64 - __clzll((long long)live) : 0;
        const uint64_t fresh = prev ? live & ~(plive & ~(1ull << pj)) : live;
        uint64_t kl = ~0ull;
        for (int k = 0; k < WC_LO; ++k)
          if (fresh & (1ull << k)) kl &= wc_keep6(k);
        dst->live = live;
        dst->fresh = fresh;
        dst->keep_lo = kl;
        dst->base = base;
        dst->j = j;
        dst->jp = pj;
        dst->H = L > WC_LO ? L - WC_LO : 0;
        dst->start = 1 << 30;
      }
      pos += 3 + nw;
    };
    if (ns > 0) decode(0);
    __syncthreads();
    if (ns > 0 && tid == 0) sRing[0].start = 0;
    if (!wide_sync(p, &sAbort)) break;
    unsigned long long expl = 0;
    int fail_t = -1, t_dec = ns > 0 ? 1 : 0, t_run = t_dec, t_ret = 0;
    for (int s = 0; t_ret < ns; ++s) {
      while (t_ret < t_run) {  // retire the steps whose last layer ran before this super-layer
        const WCStep& r = sRing[t_ret % WRING];
        if (r.start + r.H >= s) break;
        if (t_ret > 0 && !((ld_agent(&anyv[t_ret >> 5]) >> (t_ret & 31)) & 1u)) {
          fail_t = t_ret - 1;
          break;
        }
        ++t_ret;
        ++st_steps;
      }
      if (fail_t >= 0 || t_ret >= ns) break;
      if (tid <= WRING) {
        uint64_t acc = 0;
        for (int t = t_ret; t < t_run && t - t_ret < tid; ++t) {
          const WCStep& r = sRing[t % WRING];
          const int q = s - r.start;
          if (q >= 0 && q <= r.H) acc += sBin[r.H * WB + q];
        }
        sSeg[tid] = acc;
      }
      __syncthreads();
      const uint64_t total = sSeg[t_run - t_ret];
      uint32_t anyseg = 0;
      for (int64_t g = gtid; g < (int64_t)total; g += gstride) {
        int si = 0;
        while (si + 1 < t_run - t_ret && sSeg[si + 1] <= (uint64_t)g) ++si;
        const int t = t_ret + si;
        const WCStep& r = sRing[t % WRING];
        const int H = r.H, q = s - r.start;
        const int k = max(H < LC_WIDE_KLO ? H : LC_WIDE_KLO, H - WIDE_LOW_BITS), hb = H - k;
        uint32_t gi = (uint32_t)((uint64_t)g - sSeg[si]);
        int pp = q - k > 0 ? q - k : 0;
        for (;; ++pp) {
          const uint32_t blk = sBin[hb * WB + pp] * sBin[k * WB + (q - pp)];
          if (gi < blk || pp >= hb || pp >= q) break;
          gi -= blk;
        }
        const uint32_t nlo = sBin[k * WB + (q - pp)];
        const uint32_t hi_i = gi / nlo, lo_i = gi - hi_i * nlo;
        const uint32_t w = (hb ? (p.words[sLay[pp] + hi_i] << k) : 0u) | p.words[sLay[q - pp] + lo_i];
        const uint64_t live = r.live;
        if ((uint64_t)w & ~(live >> WC_LO)) continue;
        const int j = r.j, jp = r.jp;
        const int s_hi = (int)r.sh[0][w & 63u] + (int)r.sh[1][(w >> 6) & 63u] + (int)r.sh[2][(w >> 12) & 63u] +
                         (int)r.sh[3][(w >> 18) & 63u] + (int)r.sh[4][(w >> 24) & 63u] + (int)r.sh5[w >> 30];
        uint32_t T0w;
        const uint32_t iw = sOff[q] + colex_rank(w, sBin, &T0w);
        uint64_t X = 0;
        if (!(w & (uint32_t)(r.fresh >> WC_LO))) {  // the previous step's table through its return jp
          const uint64_t* Bp = tab(t - 1);
          if (jp >= WC_LO) X = HbmTab::ld(&Bp[sOff[q + 1] + colex_rank(w | (1u << (jp - WC_LO)), sBin)]);
          else if (jp >= 0) X = (HbmTab::ld(&Bp[iw]) & ~wc_keep6(jp)) >> (1 << jp);
          else X = HbmTab::ld(&Bp[iw]);
          X &= r.keep_lo;
        }
        uint64_t* const B = tab(t);
        // the gated pulls over w's hi bits (only j's when w holds j), ranked as wide_pulls_ranked
        const uint32_t jh = j >= WC_LO ? 1u << (j - WC_LO) : 0u;
        const uint32_t m = (w & jh) ? jh : w;
        uint32_t x = (w & jh) ? w & ((jh << 1) - 1u) : w;
        const uint32_t off_dn = q > 0 ? sOff[q - 1] : 0u;
        uint32_t P1 = 0, P0 = 0;
        uint64_t R = 0;
        for (int ii = 0; x; ii += 8) {
          int bb[8];
          uint32_t ix[8];
          uint64_t v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            bb[u] = x ? __builtin_ctz(x) : -1;
            x &= x - 1;
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            ix[u] = 0xffffffffu;
            if (bb[u] >= 0) {
              const uint32_t c0 = sBin[bb[u] * WB + ii + u], c1 = sBin[bb[u] * WB + ii + u + 1];
              P0 += c0;
              if ((m >> bb[u]) & 1u) ix[u] = off_dn + P1 + (T0w - P0);
              P1 += c1;
            }
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = ix[u] != 0xffffffffu ? HbmTab::ld(&B[ix[u]]) : 0ull;
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (ix[u] != 0xffffffffu) R |= v[u] & wc_gate(r, r.cq[WC_LO + bb[u]], s_hi);
        }
        if (!(w & jh)) {  // the in-word closure (gated transfers to a fixpoint), then j if low
          const bool jhi = j >= WC_LO;
          const uint64_t notj = jhi ? ~0ull : wc_keep6(j);
          R &= notj;
          const uint32_t lo = (uint32_t)live & 63u & ~(jhi ? 0u : 1u << j);
          uint64_t G[WC_LO];
#pragma unroll
          for (int kk = 0; kk < WC_LO; ++kk)
            G[kk] = ((live >> kk) & 1u) ? wc_gate(r, r.cq[kk], s_hi) & wc_keep6(kk) & notj : 0ull;
          for (;;) {
            const uint64_t R0 = R;
#pragma unroll
            for (int kk = 0; kk < WC_LO; ++kk)
              if ((lo >> kk) & 1u) R |= ((X | R) & G[kk]) << (1 << kk);
            if (R == R0) break;
          }
          if (!jhi) {
#pragma unroll
            for (int kk = 0; kk < WC_LO; ++kk)
              if (kk == j) R |= ((X | R) & G[kk]) << (1 << kk);
          }
        }
        HbmTab::st(&B[iw], X | R);
        expl += (uint64_t)__popcll(R);
        if (t > 0) st_fout += (uint64_t)__popcll(X);
        if (X) anyseg |= 1u << si;
        ++st_wv, st_wnz += (X | R) != 0;
      }
      for (int si = 0; si < t_run - t_ret; ++si)
        if (__any((anyseg >> si) & 1u) && lane == 0) {
          const int t = t_ret + si;
          __hip_atomic_fetch_or(&anyv[t >> 5], 1u << (t & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      const int t_dec_old = t_dec;
      if (t_dec < ns && t_dec - t_ret < WRING - 1) {
        decode(t_dec);
        ++t_dec;
      }
      __syncthreads();
      if (t_run < t_dec_old) {
        bool ok = true;
        if (t_run - 1 >= t_ret) {
          const WCStep& pr = sRing[(t_run - 1) % WRING];
          const int gap = pr.j < WC_LO ? 1 : 2;
          ok = s + 1 - pr.start >= min(gap, pr.H + 1);
        }
        if (ok) {
          if (tid == 0) sRing[t_run % WRING].start = s + 1;
          ++t_run;
        }
      }
      if (!wide_sync(p, &sAbort)) break;
    }
    if (sAbort) break;
    if (fail_t < 0 && ns > 0) {  // the last step's return: its frontier must hold a config
      const WCStep& r = sRing[(ns - 1) % WRING];
      const int pj = r.j;
      const uint64_t lv = r.live & ~(1ull << pj);
      const int Lf = lv ? 64 - __clzll((long long)lv) : 0;
      const int64_t nwt = (int64_t)1 << (Lf > WC_LO ? Lf - WC_LO : 0);
      const uint64_t* const Bl = tab(ns - 1);
      uint64_t nz = 0;
      for (int64_t w = gtid; w < nwt; w += gstride) {
        if ((uint64_t)w & ~(lv >> WC_LO)) continue;
        const uint32_t wr = pj >= WC_LO ? (uint32_t)w | (1u << (pj - WC_LO)) : (uint32_t)w;
        uint64_t X = HbmTab::ld(&Bl[sOff[__popc(wr)] + colex_rank(wr, sBin)]);
        if (pj < WC_LO) X = (X & ~wc_keep6(pj)) >> (1 << pj);
        st_fout += (uint64_t)__popcll(X);
        nz |= X;
      }
      if (__any(nz != 0) && lane == 0)
        __hip_atomic_fetch_or(&anyv[ns >> 5], 1u << (ns & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!wide_sync(p, &sAbort)) break;
      if (!((ld_agent(&anyv[ns >> 5]) >> (ns & 31)) & 1u)) fail_t = ns - 1;
    }
    for (int off = 32; off > 0; off >>= 1) expl += __shfl_down(expl, off, 64);
    if (tid == 0) sRed = 0;
    __syncthreads();
    if (lane == 0 && expl) atomicAdd(&sRed, expl);
    __syncthreads();
    if (tid == 0 && sRed) atomicAdd(&p.explored[i], sRed);
    if (!wide_sync(p, &sAbort)) break;
    if (blockIdx.x == 0 && tid == 0) {
      p.status[i] = fail_t >= 0 ? ST_INVALID : ST_VALID;
      p.fail_step[i] = fail_t;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    st_fout += __shfl_down(st_fout, off, 64);
    st_wv += __shfl_down(st_wv, off, 64);
    st_wnz += __shfl_down(st_wnz, off, 64);
  }
  if (lane == 0 && st_fout) atomicAdd(&p.stats[0], st_fout);
  if (blockIdx.x == 0 && tid == 0 && st_steps) atomicAdd(&p.stats[1], st_steps);
  if (lane == 0 && st_wv) atomicAdd(&p.stats[2], st_wv);
  if (lane == 0 && st_wnz) atomicAdd(&p.stats[3], st_wnz);
}

// failure reports of counter histories on the HBM tables: as wide_dump_kernel, configs are masks
// (the value is a function of the mask): tab = step t - 1's table (ranked over Hm hi bits, 64
// masks per word), read through its returning slot jp, over the post-return live slots lv
__global__ void __launch_bounds__(256) wctr_dump_kernel(WideDumpParams d) {
  __shared__ uint32_t sBin[WB * WB];
  __shared__ uint32_t sOff[WH + 2];
  const int tid = threadIdx.x;
  for (int i = tid; i < WB * WB; i += 256) {
    const int n = i / WB, k = i % WB;
    uint64_t c = 0;
    if (k <= n) {
      c = 1;
      for (int q = 1; q <= k; ++q) c = c * (uint64_t)(n - k + q) / (uint64_t)q;
    }
    sBin[i] = (uint32_t)c;
  }
  __syncthreads();
  if (tid <= WH + 1) {
    uint32_t o = 0;
    for (int r = 0; r < tid && r <= d.Hm; ++r) o += sBin[d.Hm * WB + r];
    sOff[tid] = o;
  }
  __syncthreads();
  const int Lf = d.lv ? 64 - __clzll((long long)d.lv) : 0;
  const int64_t nwt = (int64_t)1 << (Lf > WC_LO ? Lf - WC_LO : 0);
  for (int64_t w = (int64_t)blockIdx.x * 256 + tid; w < nwt; w += (int64_t)gridDim.x * 256) {
    if ((uint64_t)w & ~(d.lv >> WC_LO)) continue;
    const uint32_t wr = d.jp >= WC_LO ? (uint32_t)w | (1u << (d.jp - WC_LO)) : (uint32_t)w;
    uint64_t X = HbmTab::ld(&d.tab[sOff[__popc(wr)] + colex_rank(wr, sBin)]);
    if (d.jp < WC_LO) X = (X & ~wc_keep6(d.jp)) >> (1 << d.jp);
    if (!X) continue;
    unsigned long long at = atomicAdd(d.count, (unsigned long long)__popcll(X));
    for (; X; X &= X - 1, ++at)
      if ((int64_t)at < d.cap) d.masks[at] = ((uint64_t)w << WC_LO) | (uint64_t)__builtin_ctzll(X);
  }
}

}  // namespace

int wide_grid_size(bool pipe) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, pipe ? (const void*)wide_pipe_kernel
                                                                 : (const void*)wide_kernel,
                                                   pipe ? WPWG : WWG, 0) != hipSuccess ||
      per_cu < 1)
    return 0;
  // every workgroup resident (the grid barrier needs it): one 1024-thread workgroup per CU for
  // the one-step kernel, as many 256-thread ones as fit for the pipelined kernel
  return prop.multiProcessorCount * (pipe ? per_cu : 1);
}

size_t wide_bar_bytes() { return sizeof(WideBar); }

hipError_t launch_wide_dump(const WideDumpParams& d, hipStream_t stream) {
  hipLaunchKernelGGL(wide_dump_kernel, dim3(1024), dim3(256), 0, stream, d);
  return hipGetLastError();
}

hipError_t launch_wide_gather(const WideDumpParams& d, const uint64_t* hw, uint64_t* out, int n, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(wide_gather_kernel, dim3(std::min(1024, (n + 255) / 256)), dim3(256), 0, stream, d, hw, out, n);
  return hipGetLastError();
}

int wctr_grid_size() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)wctr_pipe_kernel, WPWG, 0) != hipSuccess ||
      per_cu < 1)
    return 0;
  return prop.multiProcessorCount * per_cu;
}

hipError_t launch_wctr_dump(const WideDumpParams& d, hipStream_t stream) {
  hipLaunchKernelGGL(wctr_dump_kernel, dim3(1024), dim3(256), 0, stream, d);
  return hipGetLastError();
}

hipError_t launch_wctr(const WideParams& p, int grid, hipStream_t stream) {
  WideParams q = p;
  void* args[] = {&q};
  return hipLaunchCooperativeKernel((const void*)wctr_pipe_kernel, dim3(grid), dim3(WPWG), args, 0, stream);
}

hipError_t launch_wide(const WideParams& p, int grid, hipStream_t stream) {
  WideParams q = p;
  void* args[] = {&q};
  return hipLaunchCooperativeKernel(p.pipe ? (const void*)wide_pipe_kernel : (const void*)wide_kernel, dim3(grid),
                                    dim3(p.pipe ? WPWG : WWG), args, 0, stream);
}

}  // namespace lc
