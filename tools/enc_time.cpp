// enc_time.cpp — times lc::encode (the host half of lc_plan_create / lc_check) on a history
// dumped by tools/enc_time.py. Build + run: python tools/enc_time.py [workload]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../jepsen-jgroups-raft_amd/csrc/encode.hpp"

template <class T>
static std::vector<T> load(const char* dir, const char* name) {
  char p[512];
  std::snprintf(p, sizeof p, "%s/%s.bin", dir, name);
  FILE* f = std::fopen(p, "rb");
  if (!f) std::perror(p), std::exit(1);
  std::fseek(f, 0, SEEK_END);
  long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  std::vector<T> v(n / sizeof(T));
  if (std::fread(v.data(), 1, n, f) != (size_t)n) std::exit(1);
  std::fclose(f);
  return v;
}

int main(int argc, char** argv) {
  const char* dir = argv[1];
  int reps = argc > 2 ? std::atoi(argv[2]) : 5;
  auto off = load<int64_t>(dir, "off");
  auto index = load<int64_t>(dir, "index");
  auto process = load<int32_t>(dir, "process");
  auto type = load<int8_t>(dir, "type");
  auto f = load<int8_t>(dir, "f");
  auto v0 = load<int64_t>(dir, "v0");
  auto v1 = load<int64_t>(dir, "v1");
  auto vflags = load<int8_t>(dir, "vflags");
  lc::HistArrays a{(int64_t)type.size(), index.data(), process.data(), type.data(), f.data(),
                   v0.data(), v1.data(), vflags.data()};
  lc::Encoded e;  // reused across reps, as lc_check's cached plan reuses its own
  for (int r = 0; r < reps; ++r) {
    auto t0 = std::chrono::steady_clock::now();
    lc::encode(1, 0, (int)off.size() - 1, off.data(), a, e);
    auto t1 = std::chrono::steady_clock::now();
    std::printf("encode %.3f ms (%zu steps)\n",
                std::chrono::duration<double, std::milli>(t1 - t0).count(), e.step_slot.size());
  }
}
