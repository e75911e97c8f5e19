// Does data written by one kernel stay in the writer XCD's L2 for the next
// kernel?  Kernel W (blocks on XCD w only) writes a buffer; kernel R (one
// block on XCD r) streams it and reports cycles.  r == w vs r != w.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void writer(float4* buf, int n4, int xcd) {
  if ((int)(blockIdx.x % 8) != xcd) return;
  const int nb = gridDim.x / 8, bi = blockIdx.x / 8;
  for (int i = bi * blockDim.x + threadIdx.x; i < n4; i += nb * blockDim.x) buf[i] = make_float4(i, 1, 2, 3);
}
__global__ void reader(const float4* buf, int n4, int xcd, long long* out, float* sink) {
  if ((int)(blockIdx.x % 8) != xcd || blockIdx.x / 8 != 0) return;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  float acc = 0.f;
  for (int i = threadIdx.x; i < n4; i += blockDim.x * 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = (i + u * blockDim.x < n4) ? buf[i + u * blockDim.x] : make_float4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u].x + v[u].w;
  }
  __syncthreads();
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  if (acc == 123.456f) sink[0] = acc;
}

int main() {
  const int bytes = 128 * 1024, n4 = bytes / 16;
  float4* buf;
  long long* out;
  float* sink;
  hipMalloc(&buf, bytes);
  hipMalloc(&out, 8);
  hipMalloc(&sink, 4);
  long long h;
  for (int rep = 0; rep < 3; ++rep)
    for (int w = 0; w < 2; ++w)
      for (int r = 0; r < 2; ++r) {
        hipLaunchKernelGGL(writer, dim3(64), dim3(256), 0, 0, buf, n4, w);
        hipLaunchKernelGGL(reader, dim3(8), dim3(512), 0, 0, buf, n4, r, out, sink);
        hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost);
        printf("rep %d writer xcd %d reader xcd %d: %lld cycles for %d KiB (%.1f B/clk)\n", rep, w, r, h,
               bytes / 1024, (double)bytes / h);
      }
  // reader twice in a row (second read: own L2 warm)
  for (int r = 0; r < 2; ++r) {
    hipLaunchKernelGGL(writer, dim3(64), dim3(256), 0, 0, buf, n4, 0);
    hipLaunchKernelGGL(reader, dim3(8), dim3(512), 0, 0, buf, n4, 1, out, sink);
    hipLaunchKernelGGL(reader, dim3(8), dim3(512), 0, 0, buf, n4, 1, out, sink);
    hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost);
    printf("second read on xcd 1: %lld cycles\n", h);
  }
  return 0;
}
