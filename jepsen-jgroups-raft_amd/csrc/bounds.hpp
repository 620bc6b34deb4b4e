// bounds.hpp — counter bounds pre-filter: a sound rejection
// test computed with a parallel prefix scan on the GPU (bounds.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace lc {

struct BoundsObs {  // one observation: pre-state of an :ok read / *-and-get must be x
  int64_t iv, cmp;  // positions of its invocation and completion
  int64_t x, d;     // observed pre-state, own delta (excluded from P)
};

struct BoundsBase {  // the five prefix sums before the first entry of a scanned range
  int64_t v[5] = {0, 0, 0, 0, 0};
};

// Host-side preparation of one counter history: per-entry deltas and the observations.
struct BoundsHost {
  std::vector<int64_t> dok, dinv;
  std::vector<BoundsObs> obs;
};
void bounds_prepare(int64_t n, const int32_t* process, const int8_t* type, const int8_t* f,
                    const int64_t* v0, const int64_t* v1, const int8_t* vflags, BoundsHost& out);

// Device-resident scan over one history of n entries.
//   d_ok[i]  = delta of the op completed :ok at entry i (0 otherwise)
//   d_inv[i] = delta of the op invoked at entry i if that op did not :fail (0 otherwise)
// Writes *bad = smallest completion position among out-of-window observations, or -1.
//   map[i]   = 2k / 2k + 1 when entry i is observation k's invocation / completion, else -1
// rec [5][n_obs] receives each observation's prefixes. base0: the sums before entry 0.
hipError_t bounds_device(int64_t init_value, int64_t n, const int64_t* d_ok, const int64_t* d_inv,
                         const int32_t* map, int64_t n_obs, const BoundsObs* obs, int64_t* rec,
                         int64_t* partials /*[5][nblk+1]*/, unsigned long long* bad,
                         hipStream_t stream, const BoundsBase& base0);
// The five sums over n entries: partials[q * (nblk + 1) + nblk] after the launch.
hipError_t bounds_sums(int64_t n, const int64_t* d_ok, const int64_t* d_inv, int64_t* partials,
                       hipStream_t stream);
constexpr int BOUNDS_TILE = 1024;

}  // namespace lc
