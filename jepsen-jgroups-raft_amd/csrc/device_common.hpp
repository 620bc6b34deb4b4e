// device_common.hpp — small device helpers shared by the search kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace lc {

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

template <typename T>
__device__ __forceinline__ T ld_agent(const T* ptr) {
  return __hip_atomic_load(ptr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_agent(T* ptr, T v) {
  __hip_atomic_store(ptr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave-aggregated append: every lane with `pred` gets a distinct slot of *counter (LDS),
// one LDS atomic per wave. Must be called by all active lanes of the wave.
__device__ __forceinline__ uint32_t wave_append(uint32_t* counter, bool pred) {
  const unsigned long long m = __ballot(pred);
  if (m == 0) return 0;
  const int lane = __lane_id();
  const int leader = __ffsll((long long)m) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
  base = __shfl(base, leader, 64);
  const unsigned long long below = lane ? (m & ((~0ull) >> (64 - lane))) : 0ull;
  return base + (uint32_t)__popcll(below);
}

}  // namespace lc
