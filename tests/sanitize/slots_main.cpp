// TEST INFRASTRUCTURE: the encoder's slot policy (csrc/encode.cpp: the soonest-returning ops take
// the in-word slots 0..2). Prints, per seeded random cas-register history, its table width
// (live_max), the RETURNs of in-word slots, and the per-step widths' table work (sum of
// 2^width); tests/test_slots.py runs it under the policy and under LC_SLOTS=lff and compares.
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#include "../../jepsen-jgroups-raft_amd/csrc/encode.hpp"
#include "../../include/lincheck.h"

// argv[1] = "counter": CounterModel histories (read / add / add-and-get), in-word slots 0..5
int main(int argc, char** argv) {
  const bool counter = argc > 1 && argv[1][0] == 'c';
  const int n_iw = counter ? 6 : 3;
  std::mt19937_64 rng(0x51075);
  for (int it = 0; it < 400; ++it) {
    // one history: nproc clients, each with one op in flight; :info makes a fresh process, :fail
    // (a cas that did not apply) drops the op
    const int nproc = 2 + (int)(rng() % 14), nops = 50 + (int)(rng() % 400);
    std::vector<int64_t> index, v0, v1;
    std::vector<int32_t> process;
    std::vector<int8_t> type, f, vflags;
    auto add = [&](int32_t p, int t, int ff, int vf, int64_t a, int64_t b) {
      index.push_back((int64_t)index.size()), process.push_back(p), type.push_back((int8_t)t);
      f.push_back((int8_t)ff), vflags.push_back((int8_t)vf), v0.push_back(a), v1.push_back(b);
    };
    std::vector<int> open(nproc, -1), pid(nproc);
    for (int p = 0; p < nproc; ++p) pid[p] = p;
    for (int k = 0; k < 2 * nops; ++k) {
      const int p = (int)(rng() % nproc);
      const int64_t a = (int64_t)(rng() % 4), b = (int64_t)(rng() % 4);
      if (open[p] < 0) {
        int ff = (int)(rng() % 3);
        if (counter) ff = ff == 0 ? 0 : ff == 1 ? 3 : 5;  // read / add / add-and-get
        add(pid[p], 0, ff, counter ? (ff == 0 ? 0 : 1) : (ff == 2 ? 2 : ff == 0 ? 0 : 1), a, b);
        open[p] = ff;
      } else {
        const int r = (int)(rng() % 20);
        const int t = r < 17 ? 1 : r < 19 ? 2 : 3;
        const int vf = counter ? (open[p] == 5 && t == 1 ? 2 : 1) : (open[p] == 2 ? 2 : 1);
        add(pid[p], t, open[p], vf, a, b);
        open[p] = -1;
        if (t == 3) pid[p] += nproc;
      }
    }
    const int64_t off[2] = {0, (int64_t)type.size()};
    lc::HistArrays h{off[1], index.data(), process.data(), type.data(), f.data(), v0.data(), v1.data(),
                     vflags.data()};
    lc::Encoded enc;
    lc::encode(counter ? LC_MODEL_COUNTER : LC_MODEL_CAS_REGISTER, 0, 1, off, h, enc);
    long inword = 0;
    double work = 0;
    uint64_t live = 0;
    for (int64_t g = enc.step_off[0]; g < enc.step_off[1]; ++g) {
      if (g > enc.step_off[0]) live &= ~(1ull << enc.step_slot[g - 1]);
      for (int64_t q = enc.inv_off[g]; q < enc.inv_off[g + 1]; ++q) live |= 1ull << enc.inv_slot[q];
      inword += enc.step_slot[g] < n_iw;
      work += (double)(1ull << (64 - __builtin_clzll(live | 1)));
    }
    std::printf("%d %d %ld %ld %.0f\n", it, enc.err[0] ? -1 : enc.live_max[0], inword,
                (long)(enc.step_off[1] - enc.step_off[0]), work);
  }
  return 0;
}
