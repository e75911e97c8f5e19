// Cost of one 256x256 bf16 row-tile layer step (16 rows, 8 waves) by where its
// weights come from: held in registers (Held), streamed from a warm L2, streamed
// cold (rewritten by a previous kernel).  Uses the engine's own layer_fwd.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../soft-actor-critic_amd/csrc \
//         -I../../include held_bench.hip -o held_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include "sac_engine.h"
#include "sac_device.h"
#include "sac_phases.h"

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void fill(bf16* w, size_t n, float v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    w[i] = (bf16)(v * (float)((i * 2654435761u) % 1000) * 1e-3f);
}

#define NT 8
struct Two {
  LayerDev l[2];
};
__constant__ Two cL;  // constant memory: descriptor loads are scalar (uniform)
__global__ void __launch_bounds__(SAC_THREADS) k(long long* out, float* sink) {
  const AS_C LayerDev& L0 = *(const AS_C LayerDev*)&cL.l[0];
  const AS_C LayerDev& L1 = *(const AS_C LayerDev*)&cL.l[1];
  extern __shared__ float lds_raw[];
  lf* X = (lf*)lds_raw;
  lf* Y = X + 16 * 260;
  for (int i = threadIdx.x; i < 16 * 260; i += SAC_THREADS) X[i] = 0.01f * (i % 7);
  __syncthreads();
  Pf<bf16> pf;
  pf.tag = nullptr;
  long long t[NT];
  Held<bf16, 8> h, h1, h2;
  t[0] = __builtin_amdgcn_s_memtime();
  held_issue<bf16, 8>(h, gw_fwd(L0));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  t[1] = __builtin_amdgcn_s_memtime();  // [0] issue -> landed (cold)
  layer_fwd<bf16, 16, false, 8>(X, 260, L0, L0.bias, ACT_RELU, nullptr, 0, Y, 260, nullptr, 0, pf, gw_none(), &h);
  __syncthreads();
  t[2] = __builtin_amdgcn_s_memtime();  // [1] held layer, first run of its code
  held_issue<bf16, 8>(h1, gw_fwd(L1));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  t[3] = __builtin_amdgcn_s_memtime();  // [2] issue -> landed (second set)
  layer_fwd<bf16, 16, false, 8>(Y, 260, L1, L1.bias, ACT_RELU, nullptr, 0, X, 260, nullptr, 0, pf, gw_none(), &h1);
  __syncthreads();
  t[4] = __builtin_amdgcn_s_memtime();  // [3] held layer, same code again
  layer_fwd<bf16, 16>(X, 260, L0, L0.bias, ACT_RELU, nullptr, 0, Y, 260, nullptr, 0, pf, gw_none());
  __syncthreads();
  t[5] = __builtin_amdgcn_s_memtime();  // [4] streamed, L2-warm
  held_issue<bf16, 8>(h2, gw_fwd(L1));
  layer_fwd<bf16, 16, false, 8>(Y, 260, L1, L1.bias, ACT_RELU, nullptr, 0, X, 260, nullptr, 0, pf, gw_none(), &h2);
  __syncthreads();
  t[6] = __builtin_amdgcn_s_memtime();  // [5] held issued at use (warm)
  long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < 4; ++i) {
    layer_fwd<bf16, 16>(X, 260, L0, L0.bias, ACT_RELU, nullptr, 0, Y, 260, nullptr, 0, pf, gw_none());
    __syncthreads();
    lf* tt = X; X = Y; Y = tt;
  }
  long long r1 = __builtin_amdgcn_s_memrealtime();
  t[7] = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    for (int i = 0; i + 1 < NT; ++i) out[blockIdx.x * 16 + i] = t[i + 1] - t[i];
    out[blockIdx.x * 16 + 8] = r1 - r0;
    out[blockIdx.x * 16 + 9] = t[7] - t[6];
  }
  if (threadIdx.x < 16) sink[blockIdx.x * 16 + threadIdx.x] = X[threadIdx.x];
}

int main() {
  const int G = 16;
  bf16* W;
  float *bias, *sink;
  long long* out;
  CHK(hipMalloc(&W, (size_t)2 * 65536 * 2));
  CHK(hipMalloc(&bias, 2 * 256 * 4));
  CHK(hipMalloc(&sink, 256 * 16 * 4));
  CHK(hipMalloc(&out, 256 * 16 * 8));
  CHK(hipMemset(bias, 0, 2048));
  Two hL = {};
  for (int i = 0; i < 2; ++i) {
    hL.l[i].K = hL.l[i].N = hL.l[i].Kp = hL.l[i].Np = 256;
    hL.l[i].Wc = W + (size_t)i * 65536;
    hL.l[i].bias = bias + 256 * i;
  }
  CHK(hipMemcpyToSymbol(HIP_SYMBOL(cL), &hL, sizeof(hL)));
  size_t lds = 2 * 16 * 260 * 4;
  CHK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const char* names[] = {"held issue->landed, cold", "layer, held (1st code run)", "held issue->landed, 2nd set",
                         "layer, held (code warm)", "layer, L2-warm stream", "held issued at use", "4 warm layers"};
  std::vector<long long> h(G * 16);
  std::vector<double> acc(10, 0.0);
  const int reps = 50;
  for (int r = 0; r < reps + 5; ++r) {
    fill<<<1024, 256>>>(W, (size_t)2 * 65536, 1.0f + r);
    k<<<G, SAC_THREADS, lds>>>(out, sink);
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(h.data(), out, G * 16 * 8, hipMemcpyDeviceToHost));
    if (r < 5) continue;
    for (int b = 0; b < G; ++b)
      for (int i = 0; i < 10; ++i) acc[i] += (double)h[b * 16 + i] / G / reps;
  }
  for (int i = 0; i < 6; ++i) printf("%-26s %8.0f ticks\n", names[i], acc[i]);
  printf("%-26s %8.0f ticks = %.2f us realtime -> %.1f ticks/us\n", names[6], acc[9], acc[8] / 100.0,
         acc[9] / (acc[8] / 100.0));
  return 0;
}
