// coop_exit.hip — standalone reproducer for the exit-time fault seen after rocprofv3 passes over
// liblincheck's cooperative kernels. Nothing of the library:
// one cooperative launch of a trivial grid-synchronising kernel, synchronize, free, exit.
//   hipcc --offload-arch=gfx950 -O2 -o tools/coop_exit tools/coop_exit.hip
//   rocprofv3 --kernel-trace --stats -d out -o run -- tools/coop_exit [coop|plain]
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

namespace cg = cooperative_groups;

__global__ void coop_kernel(unsigned* out, int rounds) {
  cg::grid_group g = cg::this_grid();
  for (int r = 0; r < rounds; ++r) {
    if (threadIdx.x == 0) atomicAdd(&out[r & 15], 1u);
    g.sync();
  }
}

int main(int argc, char** argv) {
  const bool coop = argc < 2 || strcmp(argv[1], "plain") != 0;
  int ncu = 0, per = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, coop_kernel, 256, 0);
  unsigned* d = nullptr;
  if (hipMalloc(&d, 64) != hipSuccess) return 2;
  hipMemset(d, 0, 64);
  int rounds = coop ? 64 : 1;
  void* args[] = {&d, &rounds};
  hipError_t e;
  if (coop) {
    e = hipLaunchCooperativeKernel((const void*)coop_kernel, dim3(ncu * per), dim3(256), args, 0, nullptr);
  } else {  // a plain launch of a kernel without grid syncs (the control)
    rounds = 0;
    hipLaunchKernelGGL(coop_kernel, dim3(ncu * per), dim3(256), 0, nullptr, d, rounds);
    e = hipGetLastError();
  }
  if (e != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    fprintf(stderr, "launch failed: %s\n", hipGetErrorString(e));
    return 1;
  }
  unsigned h[16];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  hipFree(d);
  printf("%s launch of %d workgroups: ok (%u)\n", coop ? "cooperative" : "plain", ncu * per, h[0]);
  return 0;
}
