// Workgroup launch-rate probe: how long a grid of near-empty 256-thread
// workgroups (K2's shape: 14 x 6144, 24 KB dynamic LDS) takes, vs fewer,
// longer workgroups doing the same total "work".
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(256) empty_k(const int *in, int *out, int iters) {
  extern __shared__ int lds[];
  int v = in[blockIdx.y];
  for (int i = 0; i < iters; i++) {
    lds[threadIdx.x] = v + i;
    __syncthreads();
    v += lds[(threadIdx.x + 1) & 255];
    __syncthreads();
  }
  if (v == 0x7fffffff) out[blockIdx.x] = v;  // never true: keeps the work
}

int main() {
  int *in, *out;
  hipMalloc(&in, 65536 * 4);
  hipMalloc(&out, 65536 * 4);
  hipMemset(in, 0, 65536 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  struct { int gx, gy, lds, iters; } cfg[] = {
      {14, 6144, 24576, 1}, {14, 6144, 24576, 8}, {7, 6144, 24576, 2}, {1, 6144, 24576, 14},
      {14, 6144, 0, 1}, {14, 6144, 8192, 1}};
  for (auto &c : cfg) {
    for (int r = 0; r < 3; r++) hipLaunchKernelGGL(empty_k, dim3(c.gx, c.gy), dim3(256), c.lds, 0, in, out, c.iters);
    hipDeviceSynchronize();
    hipEventRecord(a, 0);
    for (int r = 0; r < 10; r++) hipLaunchKernelGGL(empty_k, dim3(c.gx, c.gy), dim3(256), c.lds, 0, in, out, c.iters);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    double wgs = (double)c.gx * c.gy;
    printf("grid %dx%d lds %d iters %d: %.3f ms per launch, %.1f ns per WG, %.0f M WG/s\n", c.gx, c.gy, c.lds, c.iters,
           ms / 10, ms / 10 * 1e6 / wgs, wgs / (ms / 10 * 1e-3) / 1e6);
  }
  return 0;
}
