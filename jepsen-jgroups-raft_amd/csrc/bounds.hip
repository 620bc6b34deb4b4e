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
#include <memory>
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

// K2: exclusive scan of the tile sums, one 1024-thread block per quantity: each thread sums
// a run of consecutive tiles, the block scans the run totals (wave shuffles + LDS), then
// each thread writes its run's exclusive prefixes; row[nblk] = the total.
constexpr int SCAN_T = 1024;
__global__ void __launch_bounds__(SCAN_T) bounds_scan_partials(int64_t* partials, int nblk) {
  __shared__ int64_t wsum[SCAN_T / 64];
  int64_t* row = partials + (size_t)blockIdx.x * (nblk + 1);
  const int per = (nblk + SCAN_T - 1) / SCAN_T;
  const int b0 = min(nblk, (int)threadIdx.x * per), b1 = min(nblk, b0 + per);
  int64_t s = 0;
  for (int b = b0; b < b1; ++b) s += row[b];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t incl = s;
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int64_t run = incl - s;
  for (int u = 0; u < w; ++u) run += wsum[u];
  for (int b = b0; b < b1; ++b) {
    const int64_t v = row[b];
    row[b] = run;
    run += v;
  }
  if (threadIdx.x == SCAN_T - 1) row[nblk] = run;
}

// K3: exclusive prefixes of every tile entry, in coalesced chunks of BT entries (a block
// scan per chunk plus a running carry from the tile's base). Only the entries that are some
// observation's invocation or completion are stored: map[i] = 2k (i is observation k's
// invocation: CA, CAn, CAp) or 2k + 1 (its completion: IN, IP), -1 otherwise; rec is [5][n_obs].
__global__ void __launch_bounds__(BT) bounds_prefix(int64_t n, const int64_t* __restrict__ d_ok,
                                                    const int64_t* __restrict__ d_inv,
                                                    const int32_t* __restrict__ map,
                                                    const int64_t* __restrict__ partials, int nblk,
                                                    BoundsBase base0, int64_t n_obs,
                                                    int64_t* __restrict__ rec) {
  __shared__ int64_t wsum[2][5][BT / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t carry[5];
  for (int q = 0; q < 5; ++q) carry[q] = base0.v[q] + partials[(size_t)q * (nblk + 1) + blockIdx.x];
  const int64_t tile = (int64_t)blockIdx.x * BOUNDS_TILE;
  for (int k = 0; k < PER; ++k) {
    const int64_t i = tile + (int64_t)k * BT + threadIdx.x;
    int64_t v[5] = {0, 0, 0, 0, 0};
    int32_t m = -1;
    if (i < n) {
      contrib(d_ok[i], d_inv[i], v);
      m = map[i];
    }
    int64_t incl[5];
    for (int q = 1; q < 5; ++q) {  // CA = CAn + CAp: four scans
      incl[q] = v[q];
      for (int off = 1; off < 64; off <<= 1) {
        const int64_t y = __shfl_up(incl[q], off, 64);
        if (lane >= off) incl[q] += y;
      }
      if (lane == 63) wsum[k & 1][q][w] = incl[q];
    }
    __syncthreads();  // (wsum alternates buffers, so one barrier per chunk suffices)
    int64_t excl[5];
    for (int q = 1; q < 5; ++q) {
      int64_t before = 0, total = 0;
      for (int u = 0; u < BT / 64; ++u) {
        const int64_t x = wsum[k & 1][q][u];
        before += u < w ? x : 0;
        total += x;
      }
      excl[q] = carry[q] + before + incl[q] - v[q];
      carry[q] += total;
    }
    excl[0] = excl[1] + excl[2];  // every prefix of dok = its negative part + its positive part
    if (m >= 0) {
      const size_t kk = (size_t)(m >> 1);
      if (m & 1) {
        rec[3 * n_obs + kk] = excl[3];
        rec[4 * n_obs + kk] = excl[4];
      } else {
        rec[kk] = excl[0];
        rec[n_obs + kk] = excl[1];
        rec[2 * n_obs + kk] = excl[2];
      }
    }
  }
}

// K4: check every observation against its window
__global__ void __launch_bounds__(BT) bounds_check(int64_t init, int64_t n_obs,
                                                   const BoundsObs* __restrict__ obs,
                                                   const int64_t* __restrict__ rec,
                                                   unsigned long long* bad) {
  const int64_t k = (int64_t)blockIdx.x * BT + threadIdx.x;
  if (k >= n_obs) return;
  const BoundsObs o = obs[k];
  const int64_t CA = rec[k], CAn = rec[n_obs + k], CAp = rec[2 * n_obs + k];
  const int64_t IN = rec[3 * n_obs + k], IP = rec[4 * n_obs + k];
  const int64_t base = init + CA;
  const int64_t lo = base + (IN - CAn) - (o.d < 0 ? o.d : 0);
  const int64_t hi = base + (IP - CAp) - (o.d > 0 ? o.d : 0);
  if (o.x < lo || o.x > hi) atomicMin(bad, (unsigned long long)o.cmp);
}

hipError_t bounds_sums(int64_t n, const int64_t* d_ok, const int64_t* d_inv, int64_t* partials,
                       hipStream_t stream) {
  const int nblk = (int)std::max<int64_t>(1, (n + BOUNDS_TILE - 1) / BOUNDS_TILE);
  hipLaunchKernelGGL(bounds_reduce, dim3(nblk), dim3(BT), 0, stream, n, d_ok, d_inv, partials, nblk);
  hipLaunchKernelGGL(bounds_scan_partials, dim3(5), dim3(SCAN_T), 0, stream, partials, nblk);
  return hipGetLastError();
}

hipError_t bounds_device(int64_t init_value, int64_t n, const int64_t* d_ok, const int64_t* d_inv,
                         const int32_t* map, int64_t n_obs, const BoundsObs* obs, int64_t* rec,
                         int64_t* partials, unsigned long long* bad, hipStream_t stream,
                         const BoundsBase& base0) {
  const int nblk = (int)std::max<int64_t>(1, (n + BOUNDS_TILE - 1) / BOUNDS_TILE);
  hipError_t e = hipMemsetAsync(bad, 0xff, 8, stream);
  if (e != hipSuccess || n_obs == 0) return e;  // nothing to check
  hipLaunchKernelGGL(bounds_reduce, dim3(nblk), dim3(BT), 0, stream, n, d_ok, d_inv, partials, nblk);
  hipLaunchKernelGGL(bounds_scan_partials, dim3(5), dim3(SCAN_T), 0, stream, partials, nblk);
  hipLaunchKernelGGL(bounds_prefix, dim3(nblk), dim3(BT), 0, stream, n, d_ok, d_inv, map, partials, nblk,
                     base0, n_obs, rec);
  hipLaunchKernelGGL(bounds_check, dim3((unsigned)((n_obs + BT - 1) / BT)), dim3(BT), 0, stream, init_value,
                     n_obs, obs, rec, bad);
  return hipGetLastError();
}

// pairing (knossos.history [ext]): each invocation with its process's next completion; deltas
// from the invocation (counter.clj:104-127: add/add-and-get +d, decr/decr-and-get -d)
void bounds_prepare(int64_t n, const int32_t* process, const int8_t* type, const int8_t* f,
                    const int64_t* v0, const int64_t* v1, const int8_t* vflags, BoundsHost& out) {
  std::vector<int64_t>& dok = out.dok;
  std::vector<int64_t>& dinv = out.dinv;
  dok.assign(n, 0);
  dinv.assign(n, 0);
  out.obs.clear();
  std::vector<int64_t> inv_of(n, -1);
  std::vector<int8_t> status(n, 0);
  std::unordered_map<int32_t, int64_t> pend;
  for (int64_t i = 0; i < n; ++i) {
    auto it = pend.find(process[i]);
    if (type[i] == 0) {
      pend[process[i]] = i;
    } else if (it != pend.end() && it->second >= 0) {
      inv_of[i] = it->second;
      status[it->second] = type[i];
      it->second = -1;
    }
  }
  auto delta = [&](int64_t ip) -> int64_t {
    const int8_t ff = f[ip];
    if (ff == 3 || ff == 5) return v0[ip];
    if (ff == 4 || ff == 6) return -v0[ip];
    return 0;
  };
  for (int64_t i = 0; i < n; ++i) {
    if (type[i] == 0 && status[i] != 2) dinv[i] = delta(i);
    if (type[i] == 1 && inv_of[i] >= 0) {
      const int64_t iv = inv_of[i];
      dok[i] = delta(iv);
      const int8_t ff = f[iv];
      if (ff == 0 && vflags[i] == 1) {
        out.obs.push_back({iv, i, v0[i], 0});
      } else if ((ff == 5 || ff == 6) && vflags[i] == 2) {
        const int64_t x = ff == 5 ? v1[i] - v0[i] : v1[i] + v0[i];
        out.obs.push_back({iv, i, x, delta(iv)});
      }
    }
  }
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

// ---- device-resident bounds plans (include/lincheck.h): one counter history, or one shard of
// it, kept in HBM for repeated scans. A shard owns the observations completed in
// [own_begin, own_end) and holds the entries from the earliest owned observation's invocation
// (the halo) to own_end; the prefix sums before own_begin come from the other shards (one
// exclusive-prefix exchange of five sums per shard, SURVEY §8(e) axis 3).
struct lc_bounds_plan {
  int device = 0;
  int64_t init = 0, ext_begin = 0, own_begin = 0, own_end = 0, n_loc = 0, n_obs = 0;
  BoundsBase halo;                // sums over [ext_begin, own_begin)
  std::vector<int64_t> own_index; // :index of the owned entries
  void *a = nullptr, *c = nullptr, *map = nullptr, *o = nullptr, *rec = nullptr, *par = nullptr,
       *par2 = nullptr, *bad = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  ~lc_bounds_plan() {
    hipSetDevice(device);
    for (void* x : {a, c, map, o, rec, par, par2, bad})
      if (x) hipFree(x);
    if (e0) hipEventDestroy(e0);
    if (e1) hipEventDestroy(e1);
    if (stream) hipStreamDestroy(stream);
  }
};

extern "C" int32_t lc_bounds_plan_create(int32_t device, int64_t init_value, int64_t n, const int64_t* index,
                                         const int32_t* process, const int8_t* type, const int8_t* f,
                                         const int64_t* v0, const int64_t* v1, const int8_t* vflags,
                                         int64_t own_begin, int64_t own_end, lc_bounds_plan** out, char* err,
                                         int32_t err_len) {
  if (!out) return LC_E_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) {
    berr(err, err_len, "no HIP device %d (the checker has no CPU fallback)", device);
    return LC_E_DEVICE;
  }
  if (n < 0 || own_begin < 0 || own_end < own_begin || own_end > n ||
      (n > 0 && (!process || !type || !f || !v0 || !v1 || !vflags))) {
    berr(err, err_len, "bad history arrays or owned range [%lld, %lld) of %lld entries", (long long)own_begin,
         (long long)own_end, (long long)n);
    return LC_E_ARG;
  }
  BoundsHost bh;
  bounds_prepare(n, process, type, f, v0, v1, vflags, bh);
  auto p = std::make_unique<lc_bounds_plan>();
  p->device = device;
  p->init = init_value;
  p->own_begin = own_begin;
  p->own_end = own_end;
  std::vector<BoundsObs> mine;
  int64_t ext = own_begin;
  for (const BoundsObs& ob : bh.obs)
    if (ob.cmp >= own_begin && ob.cmp < own_end) {
      mine.push_back(ob);
      ext = std::min(ext, ob.iv);
    }
  p->ext_begin = ext;
  for (int64_t i = ext; i < own_begin; ++i) {
    const int64_t d = bh.dok[i], e = bh.dinv[i];
    p->halo.v[0] += d;
    p->halo.v[1] += d < 0 ? d : 0;
    p->halo.v[2] += d > 0 ? d : 0;
    p->halo.v[3] += e < 0 ? e : 0;
    p->halo.v[4] += e > 0 ? e : 0;
  }
  for (BoundsObs& ob : mine) ob.iv -= ext, ob.cmp -= ext;
  std::vector<int32_t> omap(own_end - ext, -1);
  for (size_t k = 0; k < mine.size(); ++k) {
    omap[mine[k].iv] = (int32_t)(2 * k);
    omap[mine[k].cmp] = (int32_t)(2 * k + 1);
  }
  p->n_loc = own_end - ext;
  p->n_obs = (int64_t)mine.size();
  p->own_index.resize(own_end - own_begin);
  for (int64_t i = own_begin; i < own_end; ++i) p->own_index[i - own_begin] = index ? index[i] : i;
  const int64_t nl = p->n_loc;
  const int nblk = (int)std::max<int64_t>(1, (nl + BOUNDS_TILE - 1) / BOUNDS_TILE);
  hipError_t e = hipSetDevice(device);
  auto chk = [&](hipError_t x) { if (e == hipSuccess) e = x; };
  chk(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
  chk(hipEventCreate(&p->e0));
  chk(hipEventCreate(&p->e1));
  chk(hipMalloc(&p->a, std::max<int64_t>(nl, 1) * 8));
  chk(hipMalloc(&p->c, std::max<int64_t>(nl, 1) * 8));
  chk(hipMalloc(&p->o, std::max<size_t>(mine.size(), 1) * sizeof(BoundsObs)));
  chk(hipMalloc(&p->map, std::max<int64_t>(nl, 1) * 4));
  chk(hipMalloc(&p->rec, 5 * std::max<size_t>(mine.size(), 1) * 8));
  chk(hipMalloc(&p->par, 5 * (size_t)(nblk + 1) * 8));
  chk(hipMalloc(&p->par2, 5 * (size_t)(nblk + 1) * 8));
  chk(hipMalloc(&p->bad, 8));
  if (e == hipSuccess && nl) {
    chk(hipMemcpy(p->a, bh.dok.data() + ext, nl * 8, hipMemcpyHostToDevice));
    chk(hipMemcpy(p->c, bh.dinv.data() + ext, nl * 8, hipMemcpyHostToDevice));
    chk(hipMemcpy(p->map, omap.data(), nl * 4, hipMemcpyHostToDevice));
  }
  if (e == hipSuccess && !mine.empty())
    chk(hipMemcpy(p->o, mine.data(), mine.size() * sizeof(BoundsObs), hipMemcpyHostToDevice));
  if (e != hipSuccess) {
    berr(err, err_len, "bounds plan: %s", hipGetErrorString(e));
    return LC_E_DEVICE;
  }
  *out = p.release();
  return LC_OK;
}

extern "C" int32_t lc_bounds_plan_sums(lc_bounds_plan* p, int64_t* out_sums, char* err, int32_t err_len) {
  if (!p || !out_sums) return LC_E_ARG;
  const int64_t h = p->own_begin - p->ext_begin, n = p->own_end - p->own_begin;
  const int nblk = (int)std::max<int64_t>(1, (n + BOUNDS_TILE - 1) / BOUNDS_TILE);
  hipError_t e = hipSetDevice(p->device);
  if (e == hipSuccess)
    e = bounds_sums(n, (const int64_t*)p->a + h, (const int64_t*)p->c + h, (int64_t*)p->par2, p->stream);
  for (int q = 0; q < 5 && e == hipSuccess; ++q)
    e = hipMemcpyAsync(&out_sums[q], (int64_t*)p->par2 + (size_t)q * (nblk + 1) + nblk, 8, hipMemcpyDeviceToHost,
                       p->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
  if (e != hipSuccess) {
    berr(err, err_len, "bounds sums: %s", hipGetErrorString(e));
    return LC_E_DEVICE;
  }
  return LC_OK;
}

extern "C" int32_t lc_bounds_plan_run(lc_bounds_plan* p, const int64_t* excl_sums, int8_t* out_ok,
                                      int64_t* out_bad_idx, double* out_ms, char* err, int32_t err_len) {
  if (!p) return LC_E_ARG;
  BoundsBase b0;
  for (int q = 0; q < 5; ++q) b0.v[q] = (excl_sums ? excl_sums[q] : 0) - p->halo.v[q];
  unsigned long long hb = ~0ull;
  float ms = 0;
  hipError_t e = hipSetDevice(p->device);
  auto chk = [&](hipError_t x) { if (e == hipSuccess) e = x; };
  chk(hipEventRecord(p->e0, p->stream));
  chk(bounds_device(p->init, p->n_loc, (int64_t*)p->a, (int64_t*)p->c, (int32_t*)p->map, p->n_obs,
                    (BoundsObs*)p->o, (int64_t*)p->rec, (int64_t*)p->par, (unsigned long long*)p->bad, p->stream,
                    b0));
  chk(hipEventRecord(p->e1, p->stream));
  chk(hipMemcpyAsync(&hb, p->bad, 8, hipMemcpyDeviceToHost, p->stream));
  chk(hipStreamSynchronize(p->stream));
  chk(hipEventElapsedTime(&ms, p->e0, p->e1));
  if (e != hipSuccess) {
    berr(err, err_len, "bounds scan: %s", hipGetErrorString(e));
    return LC_E_DEVICE;
  }
  if (out_ok) *out_ok = hb == ~0ull ? 1 : 0;
  if (out_bad_idx) *out_bad_idx = hb == ~0ull ? -1 : p->own_index[(int64_t)hb + p->ext_begin - p->own_begin];
  if (out_ms) *out_ms = ms;
  return LC_OK;
}

extern "C" void lc_bounds_plan_destroy(lc_bounds_plan* p) { delete p; }

// One-shot form: one plan per history, owning all of it.
extern "C" int32_t lc_counter_bounds(int64_t init_value, int32_t n_hist, const int64_t* hist_off,
                                     const int64_t* index, const int32_t* process, const int8_t* type,
                                     const int8_t* f, const int64_t* v0, const int64_t* v1,
                                     const int8_t* vflags, int8_t* out_ok, int64_t* out_bad_idx,
                                     char* err, int32_t err_len) {
  if (!hist_off || n_hist < 0) return LC_E_ARG;
  for (int h = 0; h < n_hist; ++h) {
    const int64_t b = hist_off[h], n = hist_off[h + 1] - b;
    lc_bounds_plan* p = nullptr;
    int32_t rc = lc_bounds_plan_create(0, init_value, n, index ? index + b : nullptr, process + b, type + b,
                                       f + b, v0 + b, v1 + b, vflags + b, 0, n, &p, err, err_len);
    if (rc) return rc;
    int8_t ok = 1;
    int64_t bad = -1;
    rc = lc_bounds_plan_run(p, nullptr, &ok, &bad, nullptr, err, err_len);
    lc_bounds_plan_destroy(p);
    if (rc) return rc;
    if (out_ok) out_ok[h] = ok;
    if (out_bad_idx) out_bad_idx[h] = bad;
  }
  return LC_OK;
}
