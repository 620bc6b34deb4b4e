// bounds.hip — counter bounds pre-filter as a reduce-then-scan over the history
// (CounterModel counter.clj:100-127 gives the deltas). For an observation
// O (invocation position iO, completion cO) with A = ops :ok-completed before iO and
// P = ops invoked before cO, not in A, not O:
//   lo = init + sum_A d + sum_P min(0,d),  hi = init + sum_A d + sum_P max(0,d)
// and O is rejected when its observed pre-state is outside [lo, hi]. Five exclusive prefix
// sums carry every window: CA (ok deltas), CAn/CAp (their negative/positive parts),
// IN/IP (negative/positive parts of non-failed invocation deltas).
// Sound, not complete: a rejection proves non-linearizability; a pass proves nothing.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "../../include/lincheck.h"
#include "bounds.hpp"

namespace lc {

constexpr int BT = 256;                 // threads per block
constexpr int PER = BOUNDS_TILE / BT;   // entries per thread

__device__ __forceinline__ void contrib(int64_t dok, int64_t dinv, int64_t v[5]) {
  v[0] = dok;
  v[1] = dok < 0 ? dok : 0;
  v[2] = dok > 0 ? dok : 0;
  v[3] = dinv < 0 ? dinv : 0;
  v[4] = dinv > 0 ? dinv : 0;
}

// K1: per-tile sums of the five quantities
__global__ void __launch_bounds__(BT) bounds_reduce(int64_t n, const int64_t* __restrict__ d_ok,
                                                    const int64_t* __restrict__ d_inv,
                                                    int64_t* __restrict__ partials, int nblk) {
  __shared__ int64_t red[5][BT / 64];
  const int64_t base = (int64_t)blockIdx.x * BOUNDS_TILE;
  int64_t s[5] = {0, 0, 0, 0, 0};
  for (int k = 0; k < PER; ++k) {
    const int64_t i = base + (int64_t)k * BT + threadIdx.x;  // coalesced
    if (i < n) {
      int64_t v[5];
      contrib(d_ok[i], d_inv[i], v);
      for (int q = 0; q < 5; ++q) s[q] += v[q];
    }
  }
  for (int q = 0; q < 5; ++q) {
    int64_t x = s[q];
    for (int off = 32; off; off >>= 1) x += __shfl_down(x, off, 64);
    if ((threadIdx.x & 63) == 0) red[q][threadIdx.x >> 6] = x;
  }
  __syncthreads();
  if (threadIdx.x < 5) {
    int64_t t = 0;
    for (int w = 0; w < BT / 64; ++w) t += red[threadIdx.x][w];
    partials[(size_t)threadIdx.x * (nblk + 1) + blockIdx.x] = t;
  }
}

// K2: exclusive scan of the tile sums (one block; nblk is small)
__global__ void __launch_bounds__(64) bounds_scan_partials(int64_t* partials, int nblk) {
  const int q = blockIdx.x;  // one block per quantity
  if (threadIdx.x != 0) return;
  int64_t run = 0;
  int64_t* row = partials + (size_t)q * (nblk + 1);
  for (int b = 0; b < nblk; ++b) {
    const int64_t v = row[b];
    row[b] = run;
    run += v;
  }
  row[nblk] = run;
}

// K3: exclusive prefix within each tile, offset by the tile's base
__global__ void __launch_bounds__(BT) bounds_prefix(int64_t n, const int64_t* __restrict__ d_ok,
                                                    const int64_t* __restrict__ d_inv,
                                                    const int64_t* __restrict__ partials, int nblk,
                                                    int64_t* __restrict__ prefix) {
  __shared__ int64_t wsum[5][BT / 64];
  // each thread owns PER consecutive entries of the tile
  const int64_t base = (int64_t)blockIdx.x * BOUNDS_TILE + (int64_t)threadIdx.x * PER;
  int64_t v[PER][5];
  int64_t s[5] = {0, 0, 0, 0, 0};
  for (int k = 0; k < PER; ++k) {
    const int64_t i = base + k;
    if (i < n) contrib(d_ok[i], d_inv[i], v[k]);
    else for (int q = 0; q < 5; ++q) v[k][q] = 0;
    for (int q = 0; q < 5; ++q) s[q] += v[k][q];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t excl[5];
  for (int q = 0; q < 5; ++q) {
    int64_t incl = s[q];
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t y = __shfl_up(incl, off, 64);
      if (lane >= off) incl += y;
    }
    excl[q] = incl - s[q];
    if (lane == 63) wsum[q][w] = incl;
  }
  __syncthreads();
  for (int q = 0; q < 5; ++q) {
    int64_t add = partials[(size_t)q * (nblk + 1) + blockIdx.x];
    for (int u = 0; u < w; ++u) add += wsum[q][u];
    int64_t run = excl[q] + add;
    for (int k = 0; k < PER; ++k) {
      const int64_t i = base + k;
      if (i < n) prefix[(size_t)q * (n + 1) + i] = run;
      run += v[k][q];
    }
    if (blockIdx.x == nblk - 1 && threadIdx.x == BT - 1) prefix[(size_t)q * (n + 1) + n] = run;
  }
}

// K4: check every observation against its window
__global__ void __launch_bounds__(BT) bounds_check(int64_t init, int64_t n, int64_t n_obs,
                                                   const BoundsObs* __restrict__ obs,
                                                   const int64_t* __restrict__ prefix,
                                                   unsigned long long* bad) {
  const int64_t k = (int64_t)blockIdx.x * BT + threadIdx.x;
  if (k >= n_obs) return;
  const BoundsObs o = obs[k];
  const size_t st = (size_t)n + 1;
  const int64_t CA = prefix[o.iv], CAn = prefix[st + o.iv], CAp = prefix[2 * st + o.iv];
  const int64_t IN = prefix[3 * st + o.cmp], IP = prefix[4 * st + o.cmp];
  const int64_t base = init + CA;
  const int64_t lo = base + (IN - CAn) - (o.d < 0 ? o.d : 0);
  const int64_t hi = base + (IP - CAp) - (o.d > 0 ? o.d : 0);
  if (o.x < lo || o.x > hi) atomicMin(bad, (unsigned long long)o.cmp);
}

hipError_t bounds_device(int64_t init_value, int64_t n, const int64_t* d_ok, const int64_t* d_inv,
                         int64_t n_obs, const BoundsObs* obs, int64_t* prefix, int64_t* partials,
                         unsigned long long* bad, hipStream_t stream) {
  const int nblk = (int)std::max<int64_t>(1, (n + BOUNDS_TILE - 1) / BOUNDS_TILE);
  hipError_t e = hipMemsetAsync(bad, 0xff, 8, stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(bounds_reduce, dim3(nblk), dim3(BT), 0, stream, n, d_ok, d_inv, partials, nblk);
  hipLaunchKernelGGL(bounds_scan_partials, dim3(5), dim3(64), 0, stream, partials, nblk);
  hipLaunchKernelGGL(bounds_prefix, dim3(nblk), dim3(BT), 0, stream, n, d_ok, d_inv, partials, nblk,
                     prefix);
  if (n_obs > 0)
    hipLaunchKernelGGL(bounds_check, dim3((unsigned)((n_obs + BT - 1) / BT)), dim3(BT), 0, stream,
                       init_value, n, n_obs, obs, prefix, bad);
  return hipGetLastError();
}

}  // namespace lc

using namespace lc;

namespace {
void berr(char* err, int32_t len, const char* fmt, ...) {
  if (!err || len <= 0) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(err, (size_t)len, fmt, ap);
  va_end(ap);
}
}  // namespace

extern "C" int32_t lc_counter_bounds(int64_t init_value, int32_t n_hist, const int64_t* hist_off,
                                     const int64_t* index, const int32_t* process, const int8_t* type,
                                     const int8_t* f, const int64_t* v0, const int64_t* v1,
                                     const int8_t* vflags, int8_t* out_ok, int64_t* out_bad_idx,
                                     char* err, int32_t err_len) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    berr(err, err_len, "no HIP device visible (the checker has no CPU fallback)");
    return LC_E_DEVICE;
  }
  if (!hist_off || n_hist < 0) return LC_E_ARG;
  for (int h = 0; h < n_hist; ++h) {
    const int64_t b = hist_off[h], n = hist_off[h + 1] - b;
    // pairing (knossos.history [ext]); deltas from the invocation (counter.clj:104-127)
    std::vector<int64_t> dok(n, 0), dinv(n, 0), inv_of(n, -1);
    std::vector<int8_t> status(n, 0);
    std::unordered_map<int32_t, int64_t> pend;
    for (int64_t i = 0; i < n; ++i) {
      auto it = pend.find(process[b + i]);
      if (type[b + i] == 0) {
        pend[process[b + i]] = i;
      } else if (it != pend.end() && it->second >= 0) {
        inv_of[i] = it->second;
        status[it->second] = type[b + i];
        it->second = -1;
      }
    }
    auto delta = [&](int64_t ip) -> int64_t {
      const int8_t ff = f[b + ip];
      if (ff == 3 || ff == 5) return v0[b + ip];
      if (ff == 4 || ff == 6) return -v0[b + ip];
      return 0;
    };
    std::vector<BoundsObs> obs;
    for (int64_t i = 0; i < n; ++i) {
      if (type[b + i] == 0 && status[i] != 2) dinv[i] = delta(i);
      if (type[b + i] == 1 && inv_of[i] >= 0) {
        const int64_t iv = inv_of[i];
        dok[i] = delta(iv);
        const int8_t ff = f[b + iv];
        if (ff == 0 && vflags[b + i] == 1) {
          obs.push_back({iv, i, v0[b + i], 0});
        } else if ((ff == 5 || ff == 6) && vflags[b + i] == 2) {
          const int64_t x = ff == 5 ? v1[b + i] - v0[b + i] : v1[b + i] + v0[b + i];
          obs.push_back({iv, i, x, delta(iv)});
        }
      }
    }
    const int nblk = (int)std::max<int64_t>(1, (n + BOUNDS_TILE - 1) / BOUNDS_TILE);
    void *a = nullptr, *c = nullptr, *o = nullptr, *pre = nullptr, *par = nullptr, *bad = nullptr;
    hipError_t e = hipSuccess;
    auto chk = [&](hipError_t x) { if (e == hipSuccess) e = x; };
    chk(hipMalloc(&a, std::max<int64_t>(n, 1) * 8));
    chk(hipMalloc(&c, std::max<int64_t>(n, 1) * 8));
    chk(hipMalloc(&o, std::max<size_t>(obs.size(), 1) * sizeof(BoundsObs)));
    chk(hipMalloc(&pre, 5 * (size_t)(n + 1) * 8));
    chk(hipMalloc(&par, 5 * (size_t)(nblk + 1) * 8));
    chk(hipMalloc(&bad, 8));
    if (e == hipSuccess && n) {
      chk(hipMemcpy(a, dok.data(), n * 8, hipMemcpyHostToDevice));
      chk(hipMemcpy(c, dinv.data(), n * 8, hipMemcpyHostToDevice));
    }
    if (e == hipSuccess && !obs.empty())
      chk(hipMemcpy(o, obs.data(), obs.size() * sizeof(BoundsObs), hipMemcpyHostToDevice));
    unsigned long long hb = ~0ull;
    if (e == hipSuccess) {
      chk(bounds_device(init_value, n, (int64_t*)a, (int64_t*)c, (int64_t)obs.size(), (BoundsObs*)o,
                        (int64_t*)pre, (int64_t*)par, (unsigned long long*)bad, nullptr));
      chk(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
    }
    for (void* x : {a, c, o, pre, par, bad})
      if (x) hipFree(x);
    if (e != hipSuccess) {
      berr(err, err_len, "bounds scan: %s", hipGetErrorString(e));
      return LC_E_DEVICE;
    }
    if (out_ok) out_ok[h] = hb == ~0ull ? 1 : 0;
    if (out_bad_idx)
      out_bad_idx[h] = hb == ~0ull ? -1 : (index ? index[b + (int64_t)hb] : (int64_t)hb);
  }
  return LC_OK;
}
