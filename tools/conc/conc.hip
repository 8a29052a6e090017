// Concurrency probe: N streams each launch one kernel of W workgroups that
// spins for ~T us; wall time vs N shows how many kernels run at once.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
__global__ void spin(long long cycles, int *sink) {
  extern __shared__ int lds[];
  lds[threadIdx.x] = threadIdx.x;
  long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0 && sink) sink[blockIdx.x] = 1;
}
int main(int argc, char **argv) {
  int W = argc > 1 ? atoi(argv[1]) : 32;
  int us = argc > 2 ? atoi(argv[2]) : 1000;
  int ldsb = argc > 3 ? atoi(argv[3]) : 0;  // dynamic LDS per workgroup (bytes)
  std::vector<hipStream_t> st(32);
  for (auto &s : st) hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  long long cyc = (long long)us * 100;  // wall_clock64 is 100 MHz
  for (int N : {1, 2, 3, 4, 6, 8, 12, 16}) {
    for (int rep = 0; rep < 2; rep++) {
      hipDeviceSynchronize();
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < N; i++) hipLaunchKernelGGL(spin, dim3(W), dim3(256), ldsb, st[i], cyc, nullptr);
      hipDeviceSynchronize();
      double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (rep) printf("streams %2d x %d WGs x %d us lds %d: wall %.2f ms\n", N, W, us, ldsb, ms);
    }
  }
  return 0;
}
