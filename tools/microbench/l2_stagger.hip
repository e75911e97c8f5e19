// Per-CU weight-stream rate of the row-tile layer step (fp32, 256x256, 16 or 32
// rows per workgroup, 8 waves, one workgroup per CU) when every CU streams the
// SAME packed weights at the same time, and how the wave -> tile-pair mapping
// changes it.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 l2_stagger.hip -o l2_stagger
// Modes:
//   0  wave w owns tile pair (w, w + 8) in every workgroup (the engine's mapping)
//   1  tile pair rotated by the workgroup id: ((w + b) & 7, ... + 8)
//   2  as 0, but each workgroup streams its own copy of the weights (b % copies)
//   3  rotation + the two 8-chunk batches issued in block-parity order
//   4  as 1, with the next batch issued before the current batch's MFMAs
//   5  as 0, every layer its own weights (8 layers, cold in L2 like the engine's
//      phase kernels, whose weights the update launches rewrote)
//   6  as 5, with the 8 layers' weights prefetched into each XCD's L2 at kernel
//      start: the 32 workgroups of an XCD each load 1/32 of them (results unused)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void fill(float* w, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    w[i] = (float)((i * 2654435761u) % 1000) * 1e-6f;
}

__device__ __forceinline__ void mma4(f32x4& acc, const f32x4& a, const f32x4& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], acc, 0, 0, 0);
}

template <int RT>
__global__ void __launch_bounds__(512) layers(const float* __restrict__ W, int nl, int mode, int copies,
                                              long long* out, float* sink) {
  __shared__ float lds[2 * RT * 16 * 260];
  const int ld = 260;
  float* X = lds;
  float* Y = lds + RT * 16 * ld;
  for (int i = threadIdx.x; i < RT * 16 * ld; i += 512) X[i] = 0.01f * (i % 7);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15, g = lane >> 4;
  const int b = blockIdx.x;
  const int t = (mode == 1 || mode == 3 || mode == 4) ? ((wave + b) & 7) : wave;
  const float* Wb = W + (mode == 2 ? (size_t)(b % copies) * 65536 : 0);
  long long t0 = __builtin_amdgcn_s_memrealtime();
  f32x4 pfx = {0.f, 0.f, 0.f, 0.f};
  if (mode == 6) {  // 8 layers x 256 KB over the XCD's 32 workgroups: 64 KB each, 8 pieces per thread
    const f32x4* base = (const f32x4*)W + (size_t)((b >> 3) & 31) * 4096;
    f32x4 q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) q[j] = base[threadIdx.x + j * 512];
#pragma unroll
    for (int j = 0; j < 8; ++j) pfx += q[j];
  }
  for (int l = 0; l < nl; ++l) {
    if (mode >= 5) Wb = W + (size_t)(l & 7) * 65536;
    const int nt0 = t, nt1 = t + 8;
    const f32x4* p0 = (const f32x4*)(Wb + (size_t)nt0 * 4096) + lane;  // tile = 16 chunks x 64 lanes x 16 B
    const f32x4* p1 = (const f32x4*)(Wb + (size_t)nt1 * 4096) + lane;
    f32x4 acc0[RT], acc1[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc0[rt] = acc1[rt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const float* arow = X + c * ld + g * 4;
    if (mode == 4) {
      f32x4 f0[8], f1[8], h0[8], h1[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) { f0[u] = p0[u * 64]; f1[u] = p1[u * 64]; }
#pragma unroll
      for (int u = 0; u < 8; ++u) { h0[u] = p0[(8 + u) * 64]; h1[u] = p1[(8 + u) * 64]; }
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const f32x4 a = *(const f32x4*)(arow + rt * 16 * ld + u * 16);
          mma4(acc0[rt], a, f0[u]);
          mma4(acc1[rt], a, f1[u]);
        }
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const f32x4 a = *(const f32x4*)(arow + rt * 16 * ld + (8 + u) * 16);
          mma4(acc0[rt], a, h0[u]);
          mma4(acc1[rt], a, h1[u]);
        }
    } else {
      for (int bb = 0; bb < 2; ++bb) {
        const int batch = mode == 3 ? (bb ^ (b & 1)) : bb;
        f32x4 f0[8], f1[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) { f0[u] = p0[(batch * 8 + u) * 64]; f1[u] = p1[(batch * 8 + u) * 64]; }
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) {
            const f32x4 a = *(const f32x4*)(arow + rt * 16 * ld + (batch * 8 + u) * 16);
            mma4(acc0[rt], a, f0[u]);
            mma4(acc1[rt], a, f1[u]);
          }
      }
    }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = rt * 16 + g * 4 + i;
        Y[r * ld + nt0 * 16 + c] = fmaxf(acc0[rt][i] * 1e-3f, 0.f);
        Y[r * ld + nt1 * 16 + c] = fmaxf(acc1[rt][i] * 1e-3f, 0.f);
      }
    __syncthreads();
    float* tmp = X; X = Y; Y = tmp;
  }
  long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (threadIdx.x < 16) sink[blockIdx.x * 16 + threadIdx.x] = X[threadIdx.x];
  if (pfx[0] == 12345.f) sink[0] = pfx[1];
}

// Twin layers (e.g. Q1t and Q2t at the same depth) on 16 rows: mode 0 runs
// them one after the other (the engine's row-tile kernels: each wave owns one
// tile pair per layer); mode 1 runs them as ONE block-diagonal GEMM (each wave
// owns pair (w, w + 8) of net a and the same pair of net b; net b's loads are
// issued before net a's MFMAs), one barrier per depth instead of two.
__global__ void __launch_bounds__(512) twin(const float* __restrict__ W, int nl, int mode, long long* out, float* sink) {
  __shared__ float lds[4 * 16 * 260];
  const int ld = 260;
  float* X[2] = {lds, lds + 16 * ld};
  float* Y[2] = {lds + 2 * 16 * ld, lds + 3 * 16 * ld};
  for (int i = threadIdx.x; i < 2 * 16 * ld; i += 512) lds[i] = 0.01f * (i % 7);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15, g = lane >> 4;
  long long t0 = __builtin_amdgcn_s_memrealtime();
  auto layer = [&](const float* Wn, const float* Xn, float* Yn, f32x4 (&f0)[16], f32x4 (&f1)[16]) {
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    const float* arow = Xn + c * ld + g * 4;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const f32x4 a = *(const f32x4*)(arow + u * 16);
      mma4(acc0, a, f0[u]);
      mma4(acc1, a, f1[u]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      Yn[(g * 4 + i) * ld + wave * 16 + c] = fmaxf(acc0[i] * 1e-3f, 0.f);
      Yn[(g * 4 + i) * ld + (wave + 8) * 16 + c] = fmaxf(acc1[i] * 1e-3f, 0.f);
    }
  };
  for (int l = 0; l < nl; ++l) {
    const float* Wa = W + (size_t)(l & 3) * 2 * 65536;
    const float* Wb = Wa + 65536;
    auto ld16 = [&](const float* Wn, f32x4 (&f0)[16], f32x4 (&f1)[16]) {
      const f32x4* p0 = (const f32x4*)(Wn + (size_t)wave * 4096) + lane;
      const f32x4* p1 = (const f32x4*)(Wn + (size_t)(wave + 8) * 4096) + lane;
#pragma unroll
      for (int u = 0; u < 16; ++u) { f0[u] = p0[u * 64]; f1[u] = p1[u * 64]; }
    };
    if (mode == 0) {
      for (int n = 0; n < 2; ++n) {
        f32x4 f0[16], f1[16];
        ld16(n ? Wb : Wa, f0, f1);
        layer(n ? Wb : Wa, X[n], Y[n], f0, f1);
        __syncthreads();
      }
    } else {  // four 8-chunk batches (a lo, a hi, b lo, b hi), each issued one batch ahead
      f32x4 p0[8], p1[8], q0[8], q1[8];
      auto ld8 = [&](const float* Wn, int ch0, f32x4 (&f0)[8], f32x4 (&f1)[8]) {
        const f32x4* r0 = (const f32x4*)(Wn + (size_t)wave * 4096) + lane;
        const f32x4* r1 = (const f32x4*)(Wn + (size_t)(wave + 8) * 4096) + lane;
#pragma unroll
        for (int u = 0; u < 8; ++u) { f0[u] = r0[(ch0 + u) * 64]; f1[u] = r1[(ch0 + u) * 64]; }
      };
      auto mm8 = [&](const float* Xn, int ch0, f32x4 (&f0)[8], f32x4 (&f1)[8], f32x4& acc0, f32x4& acc1) {
        const float* arow = Xn + c * ld + g * 4;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const f32x4 a = *(const f32x4*)(arow + (ch0 + u) * 16);
          mma4(acc0, a, f0[u]);
          mma4(acc1, a, f1[u]);
        }
      };
      f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, b0 = a0, b1 = a0;
      ld8(Wa, 0, p0, p1);
      ld8(Wa, 8, q0, q1);
      mm8(X[0], 0, p0, p1, a0, a1);
      ld8(Wb, 0, p0, p1);
      mm8(X[0], 8, q0, q1, a0, a1);
      ld8(Wb, 8, q0, q1);
      mm8(X[1], 0, p0, p1, b0, b1);
      mm8(X[1], 8, q0, q1, b0, b1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        Y[0][(g * 4 + i) * ld + wave * 16 + c] = fmaxf(a0[i] * 1e-3f, 0.f);
        Y[0][(g * 4 + i) * ld + (wave + 8) * 16 + c] = fmaxf(a1[i] * 1e-3f, 0.f);
        Y[1][(g * 4 + i) * ld + wave * 16 + c] = fmaxf(b0[i] * 1e-3f, 0.f);
        Y[1][(g * 4 + i) * ld + (wave + 8) * 16 + c] = fmaxf(b1[i] * 1e-3f, 0.f);
      }
      __syncthreads();
    }
    float* t = X[0]; X[0] = Y[0]; Y[0] = t;
    t = X[1]; X[1] = Y[1]; Y[1] = t;
  }
  long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (threadIdx.x < 16) sink[blockIdx.x * 16 + threadIdx.x] = X[0][threadIdx.x] + X[1][threadIdx.x];
}

// A whole 3-layer critic forward on 16 rows, as the row-tile kernels run it:
// layer 0 (K 32 -> 256: one 2-chunk batch per wave), layer 1 (256 -> 256),
// layer 2 (256 -> N = 1, padded to 2 tiles: waves 0 and 1, two 8-chunk
// batches each), a barrier after each layer, bias + ReLU epilogues.
__global__ void __launch_bounds__(512) mlp3(const float* __restrict__ W, int nrep, long long* out, float* sink) {
  __shared__ float lds[2 * 16 * 260];
  const int ld = 260;
  float* X = lds;
  float* Y = lds + 16 * ld;
  for (int i = threadIdx.x; i < 16 * ld; i += 512) X[i] = 0.01f * (i % 7);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15, g = lane >> 4;
  long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int rep = 0; rep < nrep; ++rep) {
    const float* W0 = W + (size_t)(rep & 3) * 3 * 65536;  // [256][32] packed
    const float* W1 = W0 + 65536;                          // [256][256]
    const float* W2 = W1 + 65536;                          // [32][256]
    {  // layer 0
      const f32x4* p0 = (const f32x4*)(W0 + (size_t)wave * 512) + lane;
      const f32x4* p1 = (const f32x4*)(W0 + (size_t)(wave + 8) * 512) + lane;
      f32x4 f0[2], f1[2], acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
      for (int u = 0; u < 2; ++u) { f0[u] = p0[u * 64]; f1[u] = p1[u * 64]; }
      const float* arow = X + c * ld + g * 4;
      for (int u = 0; u < 2; ++u) {
        const f32x4 a = *(const f32x4*)(arow + u * 16);
        mma4(acc0, a, f0[u]);
        mma4(acc1, a, f1[u]);
      }
      for (int i = 0; i < 4; ++i) {
        Y[(g * 4 + i) * ld + wave * 16 + c] = fmaxf(acc0[i] + 0.01f, 0.f);
        Y[(g * 4 + i) * ld + (wave + 8) * 16 + c] = fmaxf(acc1[i] + 0.01f, 0.f);
      }
      __syncthreads();
    }
    {  // layer 1
      const f32x4* p0 = (const f32x4*)(W1 + (size_t)wave * 4096) + lane;
      const f32x4* p1 = (const f32x4*)(W1 + (size_t)(wave + 8) * 4096) + lane;
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
      const float* arow = Y + c * ld + g * 4;
      for (int bb = 0; bb < 2; ++bb) {
        f32x4 f0[8], f1[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) { f0[u] = p0[(bb * 8 + u) * 64]; f1[u] = p1[(bb * 8 + u) * 64]; }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const f32x4 a = *(const f32x4*)(arow + (bb * 8 + u) * 16);
          mma4(acc0, a, f0[u]);
          mma4(acc1, a, f1[u]);
        }
      }
      for (int i = 0; i < 4; ++i) {
        X[(g * 4 + i) * ld + wave * 16 + c] = fmaxf(acc0[i] + 0.01f, 0.f);
        X[(g * 4 + i) * ld + (wave + 8) * 16 + c] = fmaxf(acc1[i] + 0.01f, 0.f);
      }
      __syncthreads();
    }
    if (wave < 2) {  // layer 2: tile `wave` of 2, 16 chunks
      const f32x4* p0 = (const f32x4*)(W2 + (size_t)wave * 4096) + lane;
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f};
      const float* arow = X + c * ld + g * 4;
      for (int bb = 0; bb < 2; ++bb) {
        f32x4 f0[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) f0[u] = p0[(bb * 8 + u) * 64];
#pragma unroll
        for (int u = 0; u < 8; ++u) mma4(acc0, *(const f32x4*)(arow + (bb * 8 + u) * 16), f0[u]);
      }
      for (int i = 0; i < 4; ++i) Y[(g * 4 + i) * ld + wave * 16 + c] = acc0[i];
    }
    __syncthreads();
    if (threadIdx.x < 16) X[threadIdx.x] += Y[threadIdx.x * ld] * 1e-6f;  // the head reads q
    __syncthreads();
  }
  long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (threadIdx.x < 16) sink[blockIdx.x * 16 + threadIdx.x] = X[threadIdx.x];
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? atoi(argv[1]) : 256;
  const int nl = 64;
  float* W; long long* out; float* sink;
  const int copies = 32;
  CHK(hipMalloc(&W, (size_t)copies * 65536 * 4));
  CHK(hipMalloc(&out, G * 8));
  CHK(hipMalloc(&sink, G * 64 * 4));
  fill<<<1024, 256>>>(W, (size_t)copies * 65536);
  CHK(hipDeviceSynchronize());
  std::vector<long long> h(G);
  for (int rt = 1; rt <= 2; rt *= 2)
    for (int mode = 0; mode <= 6; ++mode) {
      const int nlm = mode >= 5 ? 8 : nl;
      for (int rep = 0; rep < 3; ++rep) {
        if (mode >= 5) fill<<<1024, 256>>>(W, (size_t)8 * 65536);  // rewritten, as by the update launches
        if (rt == 1) layers<1><<<G, 512>>>(W, nlm, mode, copies, out, sink);
        else layers<2><<<G, 512>>>(W, nlm, mode, copies, out, sink);
        CHK(hipDeviceSynchronize());
      }
      CHK(hipMemcpy(h.data(), out, G * 8, hipMemcpyDeviceToHost));
      std::sort(h.begin(), h.end());
      const double med = h[G / 2] * 10.0 / nlm / 1000.0;  // us per layer (100 MHz realtime)
      const double mx = h[G - 1] * 10.0 / nlm / 1000.0;
      printf("rows %2d mode %d: per layer median %.2f us, max %.2f us -> %.1f GB/s per CU\n", rt * 16, mode, med, mx,
             262144.0 / (med * 1e3));
    }
  for (int mode = 0; mode <= 1; ++mode) {
    const int nlt = 16;
    for (int rep = 0; rep < 3; ++rep) {
      twin<<<G, 512>>>(W, nlt, mode, out, sink);
      CHK(hipDeviceSynchronize());
    }
    CHK(hipMemcpy(h.data(), out, G * 8, hipMemcpyDeviceToHost));
    std::sort(h.begin(), h.end());
    printf("twin 256x256 layers, 16 rows, %s: per depth (both nets) median %.2f us\n",
           mode ? "one block-diagonal GEMM" : "one net after the other", h[G / 2] * 10.0 / nlt / 1000.0);
  }
  {
    const int nrep = 16;
    for (int rep = 0; rep < 3; ++rep) {
      mlp3<<<G, 512>>>(W, nrep, out, sink);
      CHK(hipDeviceSynchronize());
    }
    CHK(hipMemcpy(h.data(), out, G * 8, hipMemcpyDeviceToHost));
    std::sort(h.begin(), h.end());
    printf("3-layer critic forward (24+4 -> 256 -> 256 -> 1), 16 rows: median %.2f us\n", h[G / 2] * 10.0 / nrep / 1000.0);
  }
  return 0;
}
