// bounds.hpp — counter bounds pre-filter: a sound rejection
// test computed with a parallel prefix scan on the GPU (bounds.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace lc {

struct BoundsObs {  // one observation: pre-state of an :ok read / *-and-get must be x
  int64_t iv, cmp;  // positions of its invocation and completion
  int64_t x, d;     // observed pre-state, own delta (excluded from P)
};

// Device-resident scan over one history of n entries.
//   d_ok[i]  = delta of the op completed :ok at entry i (0 otherwise)
//   d_inv[i] = delta of the op invoked at entry i if that op did not :fail (0 otherwise)
// Writes *bad = smallest completion position among out-of-window observations, or -1.
hipError_t bounds_device(int64_t init_value, int64_t n, const int64_t* d_ok, const int64_t* d_inv,
                         int64_t n_obs, const BoundsObs* obs, int64_t* prefix /*[5][n+1]*/,
                         int64_t* partials /*[5][nblk+1]*/, unsigned long long* bad,
                         hipStream_t stream);
constexpr int BOUNDS_TILE = 4096;

}  // namespace lc
