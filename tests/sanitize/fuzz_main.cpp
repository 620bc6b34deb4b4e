// TEST INFRASTRUCTURE: host-side sanitizer run (SURVEY §5 "Race detection / sanitizers").
// Built with -fsanitize=address,undefined by tests/test_sanitize.py together with the product's
// host encoder (jepsen-jgroups-raft_amd/csrc/encode.cpp, knossos.history + memo, a4/a8) and the
// C oracle (oracle/lincheck_oracle.c). Feeds both seeded random histories — well-formed ones of
// both models, with :info/:fail ops and nil/pair values, and malformed ones (completions
// without invocations, double invocations, bad :type/:f, wrong value shapes) — and checks a few
// invariants; any memory error or undefined behaviour aborts the run.
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#include "../../jepsen-jgroups-raft_amd/csrc/encode.hpp"
#include "../../include/lincheck.h"
extern "C" {
#include "../../oracle/lincheck_oracle.h"
}

struct H {
  std::vector<int64_t> index, v0, v1;
  std::vector<int32_t> process;
  std::vector<int8_t> type, f, vflags;
  void add(int64_t i, int32_t p, int t, int ff, int vf, int64_t a, int64_t b) {
    index.push_back(i), process.push_back(p), type.push_back((int8_t)t), f.push_back((int8_t)ff);
    vflags.push_back((int8_t)vf), v0.push_back(a), v1.push_back(b);
  }
};

static H gen(std::mt19937_64& rng, int model, bool malformed) {
  H h;
  const int nproc = 1 + (int)(rng() % 6), nops = (int)(rng() % 60);
  std::vector<int> open(nproc, -1), fresh(nproc);
  for (int p = 0; p < nproc; ++p) fresh[p] = p;
  int64_t idx = 0;
  for (int k = 0; k < 2 * nops; ++k) {
    const int p = (int)(rng() % nproc);
    const int fs = model == 1 ? (int)(rng() % 3) : (int)(rng() % 7 == 0 ? 0 : 3 + rng() % 4);
    const int64_t a = (int64_t)(rng() % 5), b = (int64_t)(rng() % 5);
    if (malformed && rng() % 7 == 0) {  // anything at all
      h.add(idx++, (int32_t)(rng() % 9), (int)(rng() % 6) - 1, (int)(rng() % 9) - 1, (int)(rng() % 4), a, b);
      continue;
    }
    if (open[p] < 0) {
      const int vf = fs == 2 || ((fs == 5 || fs == 6) && rng() % 2) ? 2 : (fs == 0 ? 0 : 1);
      h.add(idx++, fresh[p], 0, fs, vf, a, b);
      open[p] = fs;
    } else {
      const int r = (int)(rng() % 10);
      const int t = r < 7 ? 1 : r < 9 ? 2 : 3;
      const int ff = open[p];
      const int vf = ff == 2 || ff >= 5 ? 2 : (ff == 0 && rng() % 3 == 0 ? 0 : 1);
      h.add(idx++, fresh[p], t, ff, vf, a, b);
      open[p] = -1;
      if (t == 3) fresh[p] += nproc;  // a fresh process after :info
    }
  }
  return h;
}

int main() {
  std::mt19937_64 rng(0x5EED5A71);
  int checked = 0, invalid = 0, errors = 0;
  for (int it = 0; it < 4000; ++it) {
    const int model = 1 + (int)(it % 2);
    const bool malformed = it % 5 == 0;
    // several histories per batch, concatenated
    const int nh = 1 + (int)(rng() % 4);
    H all;
    std::vector<int64_t> off(1, 0);
    for (int k = 0; k < nh; ++k) {
      H h = gen(rng, model, malformed);
      for (size_t i = 0; i < h.type.size(); ++i)
        all.add(h.index[i], h.process[i], h.type[i], h.f[i], h.vflags[i], h.v0[i], h.v1[i]);
      off.push_back((int64_t)all.type.size());
    }
    lc::HistArrays a{off.back(), it % 3 ? all.index.data() : nullptr, all.process.data(), all.type.data(),
                     all.f.data(), all.v0.data(), all.v1.data(), all.vflags.data()};
    lc::Encoded enc;
    lc::encode(model, 0, nh, off.data(), a, enc);
    if ((int)enc.err.size() != nh || (int)enc.step_off.size() != nh + 1) return 2;
    for (int k = 0; k < nh; ++k) {
      errors += enc.err[k] != 0;
      const int64_t b = off[k], n = off[k + 1] - b;
      oracle_result r;
      // with a failure-report buffer: the per-config :last-op tracking runs under the sanitizers
      int64_t cv[64], cl[64];
      int8_t cn[64];
      uint64_t cm[64];
      oracle_check(model, 0, n, a.index ? a.index + b : nullptr, a.process + b, a.type + b, a.f + b, a.v0 + b,
                   a.v1 + b, a.vflags + b, 0, &r, 64, cv, cn, cm, cl);
      if (r.valid < 0 || r.valid > 2) return 3;
      if ((enc.err[k] != 0) != (r.valid == 2 && r.err_code != 0) && !malformed) return 4;
      invalid += r.valid == 0;
      ++checked;
    }
  }
  std::printf("sanitize ok: %d histories, %d invalid, %d rejected by the encoder\n", checked, invalid, errors);
  return 0;
}
