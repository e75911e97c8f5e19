// Workgroup dispatch ramp: when does each block of an N-block launch start?
// 512-thread blocks with a large dynamic LDS allocation (one block per CU).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

__global__ void probe(long long* t) {
  extern __shared__ float lds[];
  if (threadIdx.x == 0) {
    lds[0] = 1.f;
    t[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  }
  __syncthreads();
}

int main() {
  long long* d;
  (void)hipMalloc(&d, 4096 * 8);
  for (int lds_kb : {8, 64, 135}) {
    (void)hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    for (int n : {16, 48, 96, 177, 256}) {
      std::vector<long long> h(n);
      for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(probe, dim3(n), dim3(512), lds_kb * 1024, 0, d);
        (void)hipMemcpy(h.data(), d, n * 8, hipMemcpyDeviceToHost);
      }
      const long long t0 = *std::min_element(h.begin(), h.end());
      std::vector<long long> r(n);
      for (int i = 0; i < n; ++i) r[i] = h[i] - t0;
      printf("lds %3d KB n %3d: start of block n-1 %6lld, median %6lld, max %6lld ticks (100 MHz)\n", lds_kb, n, r[n - 1],
             r[n / 2], *std::max_element(r.begin(), r.end()));
    }
  }
  return 0;
}
