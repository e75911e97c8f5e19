// Where does a held-weight 16-row 256x256 bf16 layer step spend its cycles?
// Hand-written step, 8 waves, one 2-tile pair per wave, B fragments in
// registers; variants drop one part at a time.  Cycles (s_memtime) per step,
// averaged over 8 steps (warm code) and 16 workgroups.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../soft-actor-critic_amd/csrc -I../../include \
//         layer_parts.hip -o layer_parts
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "sac_engine.h"
#include "sac_device.h"

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

// VAR bits: 1 = A fragments from LDS (fp32 + cvt), 2 = MFMA, 4 = epilogue stores, 8 = barrier,
//           16 = A fragments from a bf16 LDS image (one ds_read_b128 per fragment)
template <int VAR>
__global__ void __launch_bounds__(512) k(const bf16* W, long long* out, float* sink) {
  extern __shared__ float lds_raw[];
  lf* X = (lf*)lds_raw;
  lf* Y = X + 16 * 260;
  AS_L bf16* Xh = (AS_L bf16*)(Y + 16 * 260);  // bf16 image, row stride 264 elements
  for (int i = threadIdx.x; i < 16 * 260; i += 512) X[i] = 0.01f * (i % 7);
  for (int i = threadIdx.x; i < 16 * 264; i += 512) Xh[i] = (bf16)(0.01f * (i % 7));
  const int lane = threadIdx.x & 63, wave = wave_id(), c = lane & 15, g = lane >> 4;
  bf16x8 f0[8], f1[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    f0[u] = *(const AS_G bf16x8*)(GPC(bf16, W) + ((size_t)(wave * 8 + u) * 64 + lane) * 8);
    f1[u] = *(const AS_G bf16x8*)(GPC(bf16, W) + ((size_t)((wave + 8) * 8 + u) * 64 + lane) * 8);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 8; ++it) {
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    bf16x8 a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (VAR & 1) {
        a[u] = MM<bf16>::from_lds(X + c * 260 + g * 8 + u * 32);
      } else if (VAR & 16) {
        a[u] = *(const AS_L bf16x8*)(Xh + c * 264 + g * 8 + u * 32);
      } else {
        a[u] = f0[(u + it) & 7];
      }
    }
    if (VAR & 32) {  // B streamed from global (L2-warm): loads issued before the A reads
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        f0[u] = *(const AS_G bf16x8*)(GPC(bf16, W) + ((size_t)(wave * 8 + u) * 64 + lane) * 8);
        f1[u] = *(const AS_G bf16x8*)(GPC(bf16, W) + ((size_t)((wave + 8) * 8 + u) * 64 + lane) * 8);
      }
    }
    if (VAR & 2) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], f0[u], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], f1[u], acc1, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        acc0[u & 3] += (float)a[u][0];
        acc1[u & 3] += (float)a[u][1];
      }
    }
    if (VAR & 4) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = g * 4 + i;
        Y[r * 260 + wave * 16 + c] = fmaxf(acc0[i], 0.f);
        Y[r * 260 + (wave + 8) * 16 + c] = fmaxf(acc1[i], 0.f);
      }
    } else {
      asm volatile("" ::"v"(acc0), "v"(acc1));
    }
    if (VAR & 8) __syncthreads();
    else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[blockIdx.x * 8 + wave] = t1 - t0;
  if (threadIdx.x < 16) sink[blockIdx.x * 16 + threadIdx.x] = Y[threadIdx.x];
}

template <int VAR>
int run(const char* name, const bf16* W, long long* out, float* sink) {
  const int G = 16;
  const size_t lds = 2 * 16 * 260 * 4 + 16 * 264 * 2;
  CHK(hipFuncSetAttribute((const void*)k<VAR>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  double acc = 0;
  long long h[G * 8];
  for (int r = 0; r < 25; ++r) {
    k<VAR><<<G, 512, lds>>>(W, out, sink);
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
    if (r < 5) continue;
    long long m = 0;
    for (int i = 0; i < G * 8; ++i) m += h[i];
    acc += (double)m / (G * 8) / 20;
  }
  printf("%-44s %7.0f cycles/step\n", name, acc / 8);
  return 0;
}

int main() {
  bf16* W;
  float* sink;
  long long* out;
  CHK(hipMalloc(&W, 65536 * 2));
  CHK(hipMemset(W, 0, 65536 * 2));
  CHK(hipMalloc(&sink, 256 * 16 * 4));
  CHK(hipMalloc(&out, 256 * 8 * 8));
  run<1 | 2 | 4 | 8>("full: fp32 LDS A + MFMA + epilogue + barrier", W, out, sink);
  run<32 | 1 | 2 | 4 | 8>("full, B streamed (L2-warm)", W, out, sink);
  run<32 | 16 | 2 | 4 | 8>("full, B streamed, bf16 LDS A image", W, out, sink);
  run<16 | 2 | 4 | 8>("full, bf16 LDS A image", W, out, sink);
  run<2 | 4 | 8>("no A reads (register A)", W, out, sink);
  run<1 | 4 | 8>("no MFMA", W, out, sink);
  run<1 | 2 | 8>("no epilogue", W, out, sink);
  run<1 | 2 | 4>("no barrier", W, out, sink);
  run<1>("A reads only", W, out, sink);
  run<16>("A reads only, bf16 image", W, out, sink);
  run<2>("MFMA only", W, out, sink);
  run<4 | 8>("epilogue + barrier only", W, out, sink);
  run<8>("barrier only", W, out, sink);
  return 0;
}
