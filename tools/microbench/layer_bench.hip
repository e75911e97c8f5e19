// Per-layer cost of the row-tile MLP step on one CU (gfx950).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../soft-actor-critic_amd/csrc layer_bench.hip -o layer_bench
// Grid of G workgroups (one per CU), each runs NL dependent 256x256 bf16 layers
// on 16 rows held in LDS.  Variants: weights freshly rewritten by a previous
// kernel (distinct per layer) vs the same weights every layer (L2-resident).
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

template <int ROWS>
__global__ void __launch_bounds__(SAC_THREADS) layers(const bf16* W, const float* bias, int nl, int distinct,
                                                      long long* out, float* sink) {
  extern __shared__ float lds_raw[];
  lf* lds = (lf*)lds_raw;
  const int ld = 260;
  lf* X = lds;
  lf* Y = lds + ROWS * ld;
  for (int i = threadIdx.x; i < ROWS * ld; i += SAC_THREADS) X[i] = 0.01f * (i % 7);
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int l = 0; l < nl; ++l) {
    const bf16* Wl = W + (distinct ? (size_t)l * 256 * 256 : 0);
    layer_fwd_<bf16, ROWS>(X, ld, Wl, 256, 256, 256, 256, bias, ACT_RELU, nullptr, 0, Y, ld, nullptr, 0);
    __syncthreads();
    lf* t = X; X = Y; Y = t;
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (threadIdx.x < 16) sink[blockIdx.x * 16 + threadIdx.x] = X[threadIdx.x];
}

// fragment-packed weights: fragment (tile nt, chunk ch) = 64 lanes x 16 B contiguous
template <int ROWS>
__global__ void __launch_bounds__(SAC_THREADS) layers_packed(const bf16* W, const float* bias, int nl, int distinct,
                                                             long long* out, float* sink, float* stash, int stores) {
  extern __shared__ float lds_raw[];
  lf* lds = (lf*)lds_raw;
  constexpr int RT = ROWS / 16;
  const int ld = 260;
  lf* X = lds;
  lf* Y = lds + ROWS * ld;
  for (int i = threadIdx.x; i < ROWS * ld; i += SAC_THREADS) X[i] = 0.01f * (i % 7);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15, g = lane >> 4;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int l = 0; l < nl; ++l) {
    const AS_G bf16* Wl = GPC(bf16, W) + (distinct ? (size_t)l * 256 * 256 : 0);
    for (int nt0 = wave; nt0 < 16; nt0 += 2 * SAC_NW) {
      const int nt1 = nt0 + SAC_NW;
      f32x4 acc0[RT], acc1[RT];
      for (int rt = 0; rt < RT; ++rt) acc0[rt] = acc1[rt] = (f32x4){0, 0, 0, 0};
      bf16x8 f0[8], f1[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        f0[u] = *(const AS_G bf16x8*)(Wl + ((size_t)(nt0 * 8 + u) * 64 + lane) * 8);
        f1[u] = *(const AS_G bf16x8*)(Wl + ((size_t)(nt1 * 8 + u) * 64 + lane) * 8);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const bf16x8 a = MM<bf16>::from_lds(X + (rt * 16 + c) * ld + g * 8 + u * 32);
          MM<bf16>::mma(acc0[rt], a, f0[u]);
          MM<bf16>::mma(acc1[rt], a, f1[u]);
        }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = rt * 16 + g * 4 + i;
          Y[r * ld + nt0 * 16 + c] = fmaxf(acc0[rt][i], 0.f);
          Y[r * ld + nt1 * 16 + c] = fmaxf(acc1[rt][i], 0.f);
          if (stores) {
            GP(float, stash)[((size_t)blockIdx.x * 64 + l) * 8192 + r * 256 + nt0 * 16 + c] = acc0[rt][i];
            GP(float, stash)[((size_t)blockIdx.x * 64 + l) * 8192 + r * 256 + nt1 * 16 + c] = acc1[rt][i];
          }
        }
    }
    __syncthreads();
    lf* t = X; X = Y; Y = t;
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (threadIdx.x < 16) sink[blockIdx.x * 16 + threadIdx.x] = X[threadIdx.x];
}

int main() {
  const int NL = 10, G = 16;
  bf16* W; float *bias, *sink; long long* out;
  CHK(hipMalloc(&W, (size_t)NL * 256 * 256 * 2));
  CHK(hipMalloc(&bias, 256 * 4));
  CHK(hipMalloc(&sink, 256 * 16 * 4));
  CHK(hipMalloc(&out, 256 * 8));
  float* stash;
  CHK(hipMalloc(&stash, (size_t)256 * 64 * 8192 * 4));
  CHK(hipMemset(bias, 0, 1024));
  size_t lds = 2 * 32 * 260 * 4;
  CHK(hipFuncSetAttribute((const void*)layers<16>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CHK(hipFuncSetAttribute((const void*)layers<32>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CHK(hipFuncSetAttribute((const void*)layers_packed<16>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CHK(hipFuncSetAttribute((const void*)layers_packed<32>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  std::vector<long long> h(G);
  for (int packed : {0, 1, 2})
  for (int rows : {16, 32})
    for (int distinct : {1, 0})
      for (int fresh : {1, 0}) {
        if (packed == 0 && rows == 32) continue;
        float ms_tot = 0; double cyc = 0; int reps = 50;
        for (int r = 0; r < reps + 5; ++r) {
          if (fresh) fill<<<1024, 256>>>(W, (size_t)NL * 256 * 256, 1.0f + r);
          CHK(hipEventRecord(e0));
          if (packed) {
            if (rows == 16) layers_packed<16><<<G, SAC_THREADS, lds>>>(W, bias, NL, distinct, out, sink, stash, packed == 2);
            else layers_packed<32><<<G, SAC_THREADS, lds>>>(W, bias, NL, distinct, out, sink, stash, packed == 2);
          } else {
            if (rows == 16) layers<16><<<G, SAC_THREADS, lds>>>(W, bias, NL, distinct, out, sink);
            else layers<32><<<G, SAC_THREADS, lds>>>(W, bias, NL, distinct, out, sink);
          }
          CHK(hipEventRecord(e1));
          CHK(hipEventSynchronize(e1));
          float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
          CHK(hipMemcpy(h.data(), out, G * 8, hipMemcpyDeviceToHost));
          if (r >= 5) { ms_tot += ms; double m = 0; for (auto x : h) m += x; cyc += m / G; }
        }
        printf("packed=%d rows=%d distinct=%d fresh=%d : kernel %.2f us, in-kernel %.0f cycles/layer (%.2f us/layer @event)\n",
               packed, rows, distinct, fresh, 1000 * ms_tot / reps, cyc / reps / NL, 1000 * ms_tot / reps / NL);
      }
  return 0;
}
