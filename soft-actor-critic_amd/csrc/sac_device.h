// sac_device.h — gfx950 device building blocks of the SAC update engine.
//
//   * MFMA micro-tiles for the three GEMM forms of an MLP step, all written as
//     the "NT" product C[i][j] = sum_r A[i][r] * B[j][r] with BOTH operands
//     K-contiguous rows (forward: A = activations, B = W[out][in];
//     backward dX: A = dY, B = W^T[in][out]; weight grad: A = dY^T, B = X^T),
//     on v_mfma_f32_16x16x4_f32 (exact fp32 products) or
//     v_mfma_f32_16x16x32_bf16 (fp32 accumulate);
//   * activations and their derivatives with torch's formulas
//     (reference sac/models.py:104-112);
//   * Philox4x32-10 and a Philox-keyed Feistel permutation, the device sampler
//     (distinct uniform rows = random.sample semantics, replay_buffer.py:39).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Address spaces made explicit: a generic (flat) access counts on BOTH vmcnt and
// lgkmcnt, so one flat LDS read waits for every outstanding weight load.
#define AS_G __attribute__((address_space(1)))
#define AS_L __attribute__((address_space(3)))
// Constant address space: the engine descriptor is read-only for a kernel's
// lifetime; loads through AS_C with uniform addresses become scalar (s_load)
// loads through the scalar cache instead of vector loads + vmcnt waits.
#define AS_C __attribute__((address_space(4)))
typedef AS_L float lf;
#define GP(T, p) ((AS_G T*)(p))
#define GPC(T, p) ((const AS_G T*)(p))

typedef __bf16 bf16;
typedef bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#ifndef SAC_NW
#define SAC_NW 8                // waves per row-tile workgroup
#endif
#define SAC_THREADS (64 * SAC_NW)
// Wave index as a uniform (SGPR) value: threadIdx.x >> 6 is the same for every
// lane of a wave, but the compiler's divergence analysis cannot see that, so
// branches and loop bounds on it become exec-masked and values merged after them
// land in VGPRs (a buffer descriptor merged that way needs a waterfall loop).
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }
#ifndef SAC_ROWS
#define SAC_ROWS 16             // batch rows per row-tile workgroup
#endif
#define SAC_PAD 32              // feature padding (bf16 MFMA K step)

// ----------------------------------------------------------------------------- MFMA
template <typename T> struct MM;

template <> struct MM<float> {
  static constexpr int KC = 16;  // k per 16-byte lane fragment (4 MFMAs of K=4)
  static constexpr int KL = 4;   // elements per lane per fragment
  typedef f32x4 Frag;
  static __device__ __forceinline__ Frag ld(const AS_G float* p) { return *(const AS_G f32x4*)p; }
  static __device__ __forceinline__ Frag from_lds(const lf* p) { return *(const AS_L f32x4*)p; }
  static __device__ __forceinline__ void mma(f32x4& acc, const Frag& a, const Frag& b) {
    // lane (c = l&15, g = l>>4) holds k = 4g + j for MFMA j: every k of the
    // 16-wide chunk is used once, identically for A and B.
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], acc, 0, 0, 0);
  }
  static __device__ __forceinline__ float cvt(float x) { return x; }
};

template <> struct MM<bf16> {
  static constexpr int KC = 32;  // one v_mfma_f32_16x16x32_bf16
  static constexpr int KL = 8;
  typedef bf16x8 Frag;
  static __device__ __forceinline__ Frag ld(const AS_G bf16* p) { return *(const AS_G bf16x8*)p; }
  static __device__ __forceinline__ Frag from_lds(const lf* p) {
    const f32x4 u = *(const AS_L f32x4*)p;
    const f32x4 v = *(const AS_L f32x4*)(p + 4);
    Frag f;
    f[0] = (bf16)u[0]; f[1] = (bf16)u[1]; f[2] = (bf16)u[2]; f[3] = (bf16)u[3];
    f[4] = (bf16)v[0]; f[5] = (bf16)v[1]; f[6] = (bf16)v[2]; f[7] = (bf16)v[3];
    return f;
  }
  static __device__ __forceinline__ void mma(f32x4& acc, const Frag& a, const Frag& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  }
  static __device__ __forceinline__ bf16 cvt(float x) { return (bf16)x; }
};

// Fragment-packed layout of a [rows][cols] operand matrix (cols % KC == 0,
// rows % 16 == 0): fragment (row tile t, k chunk ch) is the 64 lanes x 16 B that
// one wave loads for one MFMA step, stored contiguously in lane order, so every
// wave-level weight load is 1 KiB contiguous (8 full 128-B lines) instead of
// 16 rows x 64 B.  Element (r, k): t=r/16, c=r%16, ch=k/KC, g=(k%KC)/KL, j=k%KL.
template <typename T>
__host__ __device__ __forceinline__ size_t packed_off(int r, int k, int cols) {
  constexpr int KC = MM<T>::KC, KL = MM<T>::KL;
  const int nch = cols / KC;
  const int t = r >> 4, c = r & 15, ch = k / KC, rem = k % KC, g = rem / KL, j = rem % KL;
  return ((size_t)(t * nch + ch) * 64 + g * 16 + c) * KL + j;
}
// start of lane (c, g)'s fragment stream for row tile t: chunk ch is at + ch * 64 * KL
template <typename T>
__device__ __forceinline__ size_t packed_lane(int t, int cols, int lane) {
  return ((size_t)t * (cols / MM<T>::KC) * 64 + lane) * MM<T>::KL;
}

// ----------------------------------------------------------------------------- activations
enum Act { ACT_ID = 0, ACT_RELU = 1, ACT_TANH = 2, ACT_ELU = 3, ACT_LEAKY = 4, ACT_GELU = 5, ACT_SELU = 6 };

#define SELU_SCALE 1.0507009873554804934193349852946f
#define SELU_ALPHA 1.6732632423543772848170429916717f
#define INV_SQRT2 0.70710678118654752440f
#define INV_SQRT_2PI 0.39894228040143267794f

__device__ __forceinline__ float act_fwd(int a, float p) {
  switch (a) {
    case ACT_RELU: return p > 0.f ? p : 0.f;
    case ACT_TANH: return tanhf(p);
    case ACT_ELU: return p > 0.f ? p : expm1f(p);
    case ACT_LEAKY: return p > 0.f ? p : p * 0.01f;
    case ACT_GELU: return p * 0.5f * (1.f + erff(p * INV_SQRT2));
    case ACT_SELU: return SELU_SCALE * (p > 0.f ? p : SELU_ALPHA * expm1f(p));
    default: return p;
  }
}

// d act(p)/dp * g, torch backward formulas (threshold_backward on the result,
// tanh_backward on the result, elu/selu backward on the input, exact gelu).
__device__ __forceinline__ float act_bwd(int a, float p, float g) {
  switch (a) {
    case ACT_RELU: return p > 0.f ? g : 0.f;
    case ACT_TANH: { const float h = tanhf(p); return g * (1.f - h * h); }
    case ACT_ELU: return p > 0.f ? g : g * expf(p);
    case ACT_LEAKY: return p > 0.f ? g : g * 0.01f;
    case ACT_GELU: {
      const float cdf = 0.5f * (1.f + erff(p * INV_SQRT2));
      const float pdf = expf(-0.5f * p * p) * INV_SQRT_2PI;
      return g * (cdf + p * pdf);
    }
    case ACT_SELU: return p > 0.f ? g * SELU_SCALE : g * SELU_SCALE * SELU_ALPHA * expf(p);
    default: return g;
  }
}

// torch softplus(beta=1, threshold=20) and its derivative
__device__ __forceinline__ float softplus20(float x) { return x > 20.f ? x : log1pf(expf(x)); }
__device__ __forceinline__ float softplus20_grad(float x) {
  if (x > 20.f) return 1.f;
  const float z = expf(x);
  return z / (z + 1.f);
}

// ----------------------------------------------------------------------------- RNG
__host__ __device__ inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

// Standard normals for (row, which, pair): counter (step, row, which<<16|pair),
// key = seed; Box-Muller on the top 24 bits of the first two output words.
// which = 0: the target rsample draw, 1: the actor rsample draw (models.py:83);
// pair p gives action dims 2p, 2p+1.  Host-callable so the C ABI can export the
// same inline code (sac_debug_eps_host); oracle/sampler_oracle.py restates it.
__host__ __device__ inline void philox_normal2(uint64_t seed, uint64_t step, uint32_t row,
                                               uint32_t which, uint32_t pair, float& n0, float& n1) {
  uint32_t c[4] = {(uint32_t)step, (uint32_t)(step >> 32), row, (which << 16) | pair};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const float u1 = ((float)(c[0] >> 8) + 1.0f) * 5.9604644775390625e-8f;  // (0,1]
  const float u2 = (float)(c[1] >> 8) * 5.9604644775390625e-8f;           // [0,1)
  const float r = sqrtf(-2.0f * logf(u1));
  float s, co;
  sincosf(6.283185307179586f * u2, &s, &co);
  n0 = r * co;
  n1 = r * s;
}

__host__ __device__ inline uint32_t mix32(uint32_t x) {  // lowbias32
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

struct Feistel {
  uint32_t key[6];
  uint32_t half, mask;
};

// The round keys depend on (seed, step) only, so a launch whose step is known on
// the host takes them as kernel arguments (FeistelKeys) instead of evaluating two
// Philox blocks per lane; the width depends on the device-side buffer size.
struct FeistelKeys {
  uint32_t k[6];
};
__host__ __device__ inline FeistelKeys feistel_keys(uint64_t seed, uint64_t step) {
  uint32_t c[4] = {(uint32_t)step, (uint32_t)(step >> 32), 0xFFFFFFFFu, 0x5A3F0001u};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  uint32_t d[4] = {(uint32_t)step, (uint32_t)(step >> 32), 0xFFFFFFFFu, 0x5A3F0002u};
  philox4x32_10(d, (uint32_t)seed, (uint32_t)(seed >> 32));
  return FeistelKeys{{c[0], c[1], c[2], c[3], d[0], d[1]}};
}
__host__ __device__ inline Feistel feistel_from_keys(const FeistelKeys& k, int64_t size) {
  Feistel f;
  uint32_t bits = 2;
  while (bits < 62 && ((int64_t)1 << bits) < size) ++bits;
  if (bits & 1) ++bits;
  f.half = bits / 2;
  f.mask = (f.half >= 32) ? 0xFFFFFFFFu : ((1u << f.half) - 1u);
#pragma unroll
  for (int i = 0; i < 6; ++i) f.key[i] = k.k[i];
  return f;
}
__host__ __device__ inline Feistel feistel_make(uint64_t seed, uint64_t step, int64_t size) {
  return feistel_from_keys(feistel_keys(seed, step), size);
}

__host__ __device__ inline uint64_t feistel_perm(const Feistel& f, uint64_t x) {
  uint32_t L = (uint32_t)(x >> f.half) & f.mask, R = (uint32_t)x & f.mask;
  for (int i = 0; i < 6; ++i) {
    const uint32_t t = L ^ (mix32(R ^ f.key[i]) & f.mask);
    L = R;
    R = t;
  }
  return ((uint64_t)L << f.half) | R;
}

// b-th element of a pseudo-random permutation of [0, size): distinct for
// distinct b < size (cycle walking keeps the bijection inside [0, size)).
__host__ __device__ inline int64_t feistel_sample(const Feistel& f, int64_t b, int64_t size) {
  uint64_t y = feistel_perm(f, (uint64_t)b);
  for (int it = 0; it < 4096 && y >= (uint64_t)size; ++it) y = feistel_perm(f, y);
  return (int64_t)y;
}

// ----------------------------------------------------------------------------- replay layout
// Row strides (floats) of the replay fields (include/sac_engine.h sac_replay):
// struct-of-arrays (row_stride == 0: each field's own width) or transition
// records (every field a column of one [cap][row_stride] table).
struct RowStrides {
  int64_t obs, act, one;  // obs / next_obs, act, rew / done
};
__host__ __device__ inline RowStrides row_strides(int64_t row_stride, int obs_dim, int act_dim) {
  RowStrides r;
  r.obs = row_stride ? row_stride : obs_dim;
  r.act = row_stride ? row_stride : act_dim;
  r.one = row_stride ? row_stride : 1;
  return r;
}

// ----------------------------------------------------------------------------- block reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
