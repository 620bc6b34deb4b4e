// dense_ops.hpp — word-level operations of the closure tables, shared by
// the LDS kernels (dense.hip) and the HBM-table kernel (wide.hip). Device code only; each
// translation unit gets its own copy (anonymous namespace).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace lc {
namespace {

typedef __attribute__((address_space(1))) uint64_t gu64;

// A decoded op is a byte permutation of the word's 8 state bytes: `lo`/`hi` are the
// v_perm_b32 selectors of the result's low and high dwords (selector byte 0..7 = the source
// state, 0x0c = nothing). cas a b: byte a -> byte b; read a: byte a -> byte a; read nil:
// identity; an op naming a value the register never holds: nothing. A write (every state ->
// byte b, an OR of the bytes, which no permutation does) is marked hi == OPS_FOLD with
// lo = 8 * b. Each team keeps its live slots' ops in an LDS table read at a uniform address,
// so the pull loop has one uniform branch (write or not) per op and no readlane.
struct OpSel {
  uint32_t lo, hi;
};
constexpr uint32_t OPS_FOLD = 0xffffffffu, SEL_NONE = 0x0c0c0c0cu;

__device__ __forceinline__ OpSel sel_move(uint32_t s, uint32_t d) {  // byte s -> byte d
  const uint32_t sh = (d & 3u) * 8u;
  const uint32_t one = (SEL_NONE & ~(0xffu << sh)) | (s << sh);
  return d < 4 ? OpSel{one, SEL_NONE} : OpSel{SEL_NONE, one};
}

__device__ __forceinline__ OpSel decode_op(uint32_t am, uint32_t bm) {
  if (am == 0) return OpSel{SEL_NONE, SEL_NONE};  // names a value the register never holds
  if (bm) {
    const uint32_t d = (uint32_t)__builtin_ctz(bm);
    if (am == 0xffu) return OpSel{d * 8u, OPS_FOLD};  // write: from any state
    return sel_move((uint32_t)__builtin_ctz(am), d);   // cas
  }
  if (am == 0xffu) return OpSel{0x03020100u, 0x07060504u};  // read nil: every state stays
  const uint32_t a = (uint32_t)__builtin_ctz(am);
  return sel_move(a, a);  // read a
}

// An op table is OP_TAB entries of LDS, 16-B aligned, used from entry OP_PAD on (slot k at
// table[OP_PAD + k]): slot 3 + 4i lands on a 16-B boundary for the pull loop's pair reads.
constexpr int OP_PAD = 1, OP_TAB = 36;

// slots whose op is a write (lanes 0..31 of the calling wave read the team's table)
__device__ __forceinline__ uint32_t fold_mask(const OpSel* ops) {
  const int lane = threadIdx.x & 63;
  return (uint32_t)__ballot(lane < 32 && ops[lane & 31].hi == OPS_FOLD);
}

// positions (of 8) whose mask lacks bit k (k < 3), one byte / replicated over 8 bytes
__device__ __forceinline__ uint32_t keep8(int k) { return k == 0 ? 0x55u : k == 1 ? 0x33u : 0x0fu; }
__device__ __forceinline__ uint64_t keep64(int k) {
  return k == 0 ? 0x5555555555555555ull : k == 1 ? 0x3333333333333333ull : 0x0f0f0f0f0f0f0f0full;
}

__device__ __forceinline__ uint64_t perm64(OpSel s, uint64_t a) {
  const uint32_t lo = (uint32_t)a, hi = (uint32_t)(a >> 32);
  return ((uint64_t)__builtin_amdgcn_perm(hi, lo, s.hi) << 32) | __builtin_amdgcn_perm(hi, lo, s.lo);
}
__device__ __forceinline__ uint32_t fold8(uint64_t a) {  // OR of the 8 state bytes, in byte 0
  uint32_t t = (uint32_t)a | (uint32_t)(a >> 32);
  t |= t >> 16;
  t |= t >> 8;
  return t & 0xffu;
}

// op applied to word a (all 8 states) for a pull over a hi bit (positions unchanged)
__device__ __forceinline__ uint64_t transfer(OpSel s, bool fold, uint64_t a) {
  return fold ? (uint64_t)fold8(a) << s.lo : perm64(s, a);
}
// op applied for an in-word step over low bit k: result positions kept by `keep` (8-bit,
// replicated as keep_all), then moved up by `up` positions
__device__ __forceinline__ uint64_t transfer_lo(OpSel s, bool fold, uint64_t a, uint32_t keep, uint64_t keep_all,
                                                int up) {
  return fold ? (uint64_t)(fold8(a) & keep) << (s.lo + (uint32_t)up) : (perm64(s, a) & keep_all) << up;
}

// HBM tile mirrors: write-through sc1 stores, L1-bypassing sc1 loads
struct HbmTab {
  static __device__ __forceinline__ uint64_t ld(const uint64_t* p) {
    return __hip_atomic_load((const gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  static __device__ __forceinline__ void st(uint64_t* p, uint64_t v) {
    __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
};

// The rest of word w's closure, given R = its pulls (hi bits and other tiles): the in-word
// closure over the 3 low bits, then the store. Returns popcount(R); *out = X | R.
__device__ __forceinline__ uint64_t close_in_word(uint64_t X, uint32_t w, uint32_t live, int j, const OpSel* ops,
                                                 uint32_t foldm, uint64_t R) {
  const bool j_lo = j < 3;
  const uint32_t jh = j_lo ? 0u : 1u << (j - 3);
  if (!(w & jh)) {
    const uint32_t notj = j_lo ? keep8(j) : 0xffu;
    const uint64_t notj64 = j_lo ? keep64(j) : ~0ull;
    R &= notj64;  // configs holding j come only from T_j
    // ---- in-word closure over the live low ops other than j. Transfers accumulate, so a
    // sequence of ops reaches every config whose chain of low ops is a subsequence of it: the
    // ops in increasing order, then (two ops a < b) a again, or (three ops) 0 1 0 2 — the
    // shortest sequences holding every ordering (3 and 7 transfers instead of 4 and 9 passes).
    const uint32_t lo_ops = live & 7u & ~(j_lo ? (1u << j) : 0u);
    const int nlo = __popc(lo_ops);
    const OpSel lo_sel[3] = {ops[0], ops[1], ops[2]};
    auto lo_step = [&](int k) {
      if (lo_ops & (1u << k))
        R |= transfer_lo(lo_sel[k], (foldm >> k) & 1u, X | R, keep8(k) & notj, keep64(k) & notj64, 1 << k);
    };
    lo_step(0);
    lo_step(1);
    lo_step(2);
    if (nlo == 3) {
      lo_step(0);
      lo_step(1);
      lo_step(0);
      lo_step(2);
    } else if (nlo == 2) {
      if (lo_ops & 1u) lo_step(0);
      else lo_step(1);
    }
    if (j_lo)  // the returning op, linearized last
      R |= transfer_lo(ops[j], (foldm >> j) & 1u, X | R, notj, notj64, 1 << j);
  }
  return R;
}

}  // namespace
}  // namespace lc
