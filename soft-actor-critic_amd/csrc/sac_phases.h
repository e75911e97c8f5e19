// sac_phases.h — device state and the four phase kernels of one SAC gradient step.
// Included by sac_engine.hip only.  Reference cross-walk in sac_engine.hip.
#pragma once
#include <type_traits>
#include <utility>

#include "sac_device.h"

#define SAC_DEV_LAYERS 6  // Linear layers per network supported by the kernels

// Coherent (sc1) 16-B accesses: what a workgroup of the SAME launch on any XCD
// reads after a counter / flag hand-off (MI355X_MICROARCH.md §visibility: every
// store of the handed-off bytes sc1 + drained, every load of them sc1).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t coh_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}
template <bool COH>
__device__ __forceinline__ void coh_store16(const void* base, uint32_t byte_off, u32x4 v) {
  // uniform descriptor (base only): a per-lane bound would force a waterfall loop
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                         coh_rsrc(base, 0xFFFFFFF0u), (int)byte_off, 0, COH ? 16 : 0);
}
__device__ __forceinline__ float coh_load(const float* p) {
  return __hip_atomic_load((float*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// COH ? sc1 : plain load of a float another workgroup of the launch may have written
template <bool COH>
__device__ __forceinline__ float ldf(const float* p) {
  if constexpr (COH) return coh_load(p);
  return *GPC(float, p);
}
__device__ __forceinline__ void coh_storef(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// COH ? sc1 (write-through) : plain store of a float another workgroup of the launch reads
template <bool COH>
__device__ __forceinline__ void st_f(float* p, float v) {
  if constexpr (COH)
    coh_storef(p, v);
  else
    *GP(float, p) = v;
}
// weight-stream fragment: sc1 when the matrix was written earlier in the same launch
template <typename T, bool COH>
__device__ __forceinline__ typename MM<T>::Frag coh_frag(__amdgpu_buffer_rsrc_t rs, uint32_t byte_off) {
  return __builtin_bit_cast(typename MM<T>::Frag,
                            __builtin_amdgcn_raw_buffer_load_b128(rs, (int)byte_off, 0, COH ? 16 : 0));
}

// ============================================================================ device state
struct LayerDev {
  int K, N, Kp, Np;
  int w_off, b_off;
  void* Wc;       // [Np][Kp] compute dtype: forward B operand
  void* WTc;      // [Kp][Np] compute dtype: dX B operand (trainable nets)
  void* XT;       // [Kp][Bp] layer input, transposed (trainable nets)
  void* GT;       // [Np][Bp] d(pre-activation), transposed
  float* dbp;     // [nrt][N] bias-gradient partial sums per row tile
  float* pstash;  // pi only: pre-activations of the actor rows [Br][Np]
  uint32_t* pmask;  // pi hidden layers: ReLU masks of the actor rows [Br][Np / 32] (pair-tile kernels)
  const float* bias;  // = net P + b_off (fp32 master bias [N])
  long xt_par;        // pi only: element offset of the second (odd-step) X^T copy
};

struct NetDev {
  int L, hid_act, out_act;
  float* P;
  float* M;
  float* V;
  LayerDev l[SAC_DEV_LAYERS];
};

enum { NET_PI = 0, NET_Q1 = 1, NET_Q2 = 2, NET_Q1T = 3, NET_Q2T = 4 };

struct TileDesc;

struct EngineDev {
  int B, Bp, Br, O, A, nrt, ld, ldo;
  // Row-tile workgroups of phases A and C are blocks xs*i (the others exit at
  // once): blocks are dealt round-robin over the 8 XCDs, so xs > 1 packs the
  // tiles onto 8/xs XCDs whose L2s then share one weight stream (speed only).
  int xs;
  int role_xcd;  // phase A role kernel: a weight part's workgroups on at most two XCDs (SAC_ROLE_XCD)
  int roles;  // phases A / C split into per-network workgroups (see "role hand-offs")
  int pairs;  // phases A / C as pair-tile workgroups (sac_pairs.h)
  int gstride;     // granules per (kind, row tile): SAC_ROWS * (act_dim + 1)
  uint64_t* gran;  // [G_COUNT][nrt][gstride] data-tagged hand-off granules (gran_put)
  int upd_slots;  // update tiles: batch chunks staged per round (LDS slots, 1..2)
  // update tiles of phases B and D
  const TileDesc* tilesB;
  const TileDesc* tilesD;
  int nB, nD, nBq[2];
  int auto_entropy;
  // 0 after a reference-style load_agent: the reference rebinds log_alpha but
  // not its optimizer (sac/agent.py:550-554), so L_alpha is still computed and
  // reported while log_alpha, its Adam moments and step count stay as loaded
  int alpha_update;
  float gamma, tau, ls_min, ls_max, scale, beta1, beta2, adam_eps, target_entropy;
  double actor_lr, critic_lr, alpha_lr;
  uint64_t seed;
  NetDev net[5];
  float* s_st;     // [Br][O]   states of the batch (phase A -> C)
  float* a_st;     // [Br][A]   actor sample a~
  float* lp_st;    // [2][Br]   log pi(a~|s), by step parity
  float* head_st;  // [Br][4][A]: mu, log_std (raw), z, eps
  float* lossp;    // [2][nrt][4] per-row-tile loss partials, by step parity
  double* alpha_state;
  double* opt_steps;
  // Per-step scalars are double-buffered by step parity (rng_step & 1) so an
  // update phase of step k may run beside phase A of step k + 1.
  float* adam_sc;      // [2][3][2]: -lr/bias_correction1, sqrt(bias_correction2) (pi, q1, q2)
  double* alpha_sc;    // [2][2]: bias_correction1, bias_correction2 of the alpha optimizer
  uint64_t* rng_step;
  // [0] launch epoch, [1] hand-off timeout flag, [SYNC_*] counters (one 64-B
  // line each), [SYNC_FLAGS + 16 k] hand-off flags
  uint32_t* sync;
  float* hand;     // hand-off payloads [HK_COUNT][nrt][SAC_HAND_STRIDE]
  float* stats;
  float* seedq;    // [2][Bp] fp32 split: each critic row's dL/dq seed, applied by phase B to the unit-seed dY^T
  long long* stamps;  // optional in-kernel timestamps (SAC_STAMPS builds)
  // Next-step batch staging: phase C's stager blocks sample and gather step
  // t+1's rows per row tile into stg (header: step, replay size, replay write
  // slot, replay obs pointer; then s, s', a, r, d); phase A of step t+1 uses a
  // record whose header matches and gathers itself otherwise.
  float* stg;
  int stg_stride;  // floats per row-tile record
  int stage;       // stager blocks launched with phase C
  // hidden-split role kernels (sac_split.h): two workgroups per (role, row tile)
  int split;
  uint64_t* gran2;  // [GS_COUNT][nrt][2][gs2] split hand-off granules
  int gs2;
  int o_red;        // LDS: SAC_NW x 256 floats of k-split partial tiles
  int spin_limit;  // polls before a hand-off wait gives up and sets SYNC_TIMEOUT (~0.3 s at 1 << 22)
  // LDS layout (float offsets)
  int o_X, o_Y, o_P1[SAC_DEV_LAYERS], ldp1[SAC_DEV_LAYERS], o_P2[SAC_DEV_LAYERS], ldp2[SAC_DEV_LAYERS];
  int o_s, o_s2, o_a, o_a2, o_r, o_d, o_et, o_ea, o_out, o_outp, o_out2, o_outp2, o_lp, o_qt, o_y, o_g, o_g2,
      o_ga, o_gout, o_slot;
};

// The gradient step a phase body works on: its device RNG step (indices, eps),
// hand-off epoch (granule tags) and parity (double-buffered per-step state).
// The phase kernels read them from memory at launch.
struct StepCtx {
  uint64_t step;
  uint32_t ep;
  int par;
};

// One 32x32 weight tile of the update phases, self-contained so a block needs a
// single descriptor fetch before its first HBM load.
#define SAC_PART_STRIDE 1056  // granules per producer part: 32 x 32 partial dW, then 32 bias partials
struct TileDesc {
  const void* GT;  // row n0 of d(pre-act)^T  [.][Bp]
  const void* XT;  // row k0 of input^T       [.][Bp]
  float* W;        // master weight [N][K] (layer base)
  float* Wm;
  float* Wv;
  float* b;        // master bias [N]
  float* bm;
  float* bv;
  void* Wc;        // packed copies [Np][Kp], [Kp][Np]
  void* WTc;
  float* tW;       // Polyak target master weight / bias / packed copy (critics)
  float* tb;
  void* tWc;
  long xt_par;     // element offset of the odd-step X^T copy (pi tiles), else 0
  int K, N, Kp, Np, n0, k0, opt;
  int bp;          // batch columns this tile reduces over
  int ld, ldx;     // row strides of the GT / XT operands in elements (Bp; for a hidden-split
                   // layer 0 the parts' partial dY side by side, X duplicated)
  // A hidden-split layer-0 tile is one block per batch part (bp = Bp each, so
  // no block streams more operand bytes than a plain tile): producer parts
  // 2..nparts publish their partial dW as 1024 data-tagged granules each (part
  // + (kpart - 2) * 1024: {value, launch epoch}, one 8-B sc1 store each, no
  // drain or flag); part 1 polls them, adds them to its own (parts in order)
  // and runs Adam.  kpart 0: a whole tile.
  // A seeded tile's producer parts also publish their 32 bias-column partial
  // sums (granules 1024..1055 of the part's slot of SAC_PART_STRIDE).
  int kpart, nparts;
  uint64_t* part;
  // fp32 hidden-split layer 0, one block (kpart 0): the gsum parts' partial dY
  // column blocks (goff elements apart) are added elementwise while staging, in
  // part order, and reduced once against X -- no batch parts, no hand-off
  long goff;
  int gsum;
  // fp32 split critics (every layer): dY^T holds the unit-seed backward (phase
  // A's critic roles store it without waiting for y); every batch column b is
  // scaled by seed[b] (phase A's first target-critic half computes the seeds)
  // while staging, and the bias gradient is summed from the scaled rows here
  const float* seed;
};



#ifdef SAC_STAMPS
#define STAMP(i)                                                                               \
  do {                                                                                         \
    if (threadIdx.x == 0 && E.stamps) GP(long long, E.stamps)[blockIdx.x * 64 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
// block end with its stores drained (stamps builds only)
#define END_STAMP(i)                                   \
  do {                                                 \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   \
    __syncthreads();                                   \
    STAMP(i);                                          \
  } while (0)
// stamps from helpers that do not see the engine descriptor (stamps builds):
// the same buffer, published through a device global by sac_engine_debug_stamps.
// Reading that global waits (vmcnt) for every load the wave has in flight, so a
// probe placed after register-held weight loads serialises them: measured
// layer times there are not the real ones.
__device__ long long* sac_dbg_stamps;
#define DSTAMP(i)                                                                                          \
  do {                                                                                                     \
    if (threadIdx.x == 0 && sac_dbg_stamps) GP(long long, sac_dbg_stamps)[blockIdx.x * 64 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
// shader-clock counter next to the realtime stamps: clock rate = d(memtime) / d(realtime)
#define CLK_STAMP(i)                                                                              \
  do {                                                                                            \
    if (threadIdx.x == 0 && E.stamps) GP(long long, E.stamps)[blockIdx.x * 64 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define DSTAMP(i) \
  do {            \
  } while (0)
#define CLK_STAMP(i) \
  do {               \
  } while (0)
#define STAMP(i) \
  do {           \
  } while (0)
#define END_STAMP(i) \
  do {               \
  } while (0)
#endif

// ============================================================================ kernarg prefetch
// The ~2.8 KB EngineDev kernel argument is read field by field all through a
// phase kernel; each first touch of a 64-B line is a scalar-cache miss (~1-2K
// cycles) on the critical path.  Touch every line once at entry with
// back-to-back s_loads (one latency for the whole struct).
// All loads and their wait sit in ONE asm statement writing a declared-clobbered
// SGPR: an asm load's destination is "written" when its statement ends, so a
// per-load statement would let the compiler reuse the register while the load
// is still in flight (it corrupted addresses: illegal-address fault).
__device__ __forceinline__ void prefetch_engine(const void* p) {
  static_assert(sizeof(EngineDev) <= 4096, "extend prefetch_engine");
  const uint64_t base = (uint64_t)(uintptr_t)p;  // kernel-argument pointer: already uniform (SGPRs)
  asm volatile("s_load_dword s95, %0, 0\n\t" "s_load_dword s95, %0, 64\n\t" "s_load_dword s95, %0, 128\n\t" "s_load_dword s95, %0, 192\n\t" "s_load_dword s95, %0, 256\n\t" "s_load_dword s95, %0, 320\n\t" "s_load_dword s95, %0, 384\n\t" "s_load_dword s95, %0, 448\n\t" "s_load_dword s95, %0, 512\n\t" "s_load_dword s95, %0, 576\n\t" "s_load_dword s95, %0, 640\n\t" "s_load_dword s95, %0, 704\n\t" "s_load_dword s95, %0, 768\n\t" "s_load_dword s95, %0, 832\n\t" "s_load_dword s95, %0, 896\n\t" "s_load_dword s95, %0, 960\n\t" "s_load_dword s95, %0, 1024\n\t" "s_load_dword s95, %0, 1088\n\t" "s_load_dword s95, %0, 1152\n\t" "s_load_dword s95, %0, 1216\n\t" "s_load_dword s95, %0, 1280\n\t" "s_load_dword s95, %0, 1344\n\t" "s_load_dword s95, %0, 1408\n\t" "s_load_dword s95, %0, 1472\n\t" "s_load_dword s95, %0, 1536\n\t" "s_load_dword s95, %0, 1600\n\t" "s_load_dword s95, %0, 1664\n\t" "s_load_dword s95, %0, 1728\n\t" "s_load_dword s95, %0, 1792\n\t" "s_load_dword s95, %0, 1856\n\t" "s_load_dword s95, %0, 1920\n\t" "s_load_dword s95, %0, 1984\n\t" "s_load_dword s95, %0, 2048\n\t" "s_load_dword s95, %0, 2112\n\t" "s_load_dword s95, %0, 2176\n\t" "s_load_dword s95, %0, 2240\n\t" "s_load_dword s95, %0, 2304\n\t" "s_load_dword s95, %0, 2368\n\t" "s_load_dword s95, %0, 2432\n\t" "s_load_dword s95, %0, 2496\n\t" "s_load_dword s95, %0, 2560\n\t" "s_load_dword s95, %0, 2624\n\t" "s_load_dword s95, %0, 2688\n\t" "s_load_dword s95, %0, 2752\n\t" "s_load_dword s95, %0, 2816\n\t" "s_load_dword s95, %0, 2880\n\t" "s_load_dword s95, %0, 2944\n\t" "s_load_dword s95, %0, 3008\n\t" "s_load_dword s95, %0, 3072\n\t" "s_load_dword s95, %0, 3136\n\t" "s_load_dword s95, %0, 3200\n\t" "s_load_dword s95, %0, 3264\n\t" "s_load_dword s95, %0, 3328\n\t" "s_load_dword s95, %0, 3392\n\t" "s_load_dword s95, %0, 3456\n\t" "s_load_dword s95, %0, 3520\n\t" "s_load_dword s95, %0, 3584\n\t" "s_load_dword s95, %0, 3648\n\t" "s_load_dword s95, %0, 3712\n\t" "s_load_dword s95, %0, 3776\n\t" "s_load_dword s95, %0, 3840\n\t" "s_load_dword s95, %0, 3904\n\t" "s_load_dword s95, %0, 3968\n\t" "s_load_dword s95, %0, 4032\n\t" "s_waitcnt lgkmcnt(0)" :: "s"(base) : "s95", "memory");
}
#ifdef SAC_NO_PREFETCH
#define PREFETCH_ARG(ptr) ((void)0)
#else
#define PREFETCH_ARG(ptr) prefetch_engine(ptr)
#endif

// ============================================================================ MFMA layer steps
// A GEMM step streams a fragment-packed B matrix (weights W for a forward step,
// W^T for a dX step) against activations held in LDS.  Each wave owns output
// tile pairs (nt, nt + SAC_NW).  The weight stream is software-pipelined across
// steps: every wave keeps the first 8-chunk batch of its first tile pair of the
// NEXT step in registers (Pf), issued right after the current step's first MFMAs,
// so the load latency overlaps the epilogue, the barrier and whatever non-GEMM
// work sits between the two steps.
struct GemmW {
  const void* p;      // packed B matrix (first element of the step's first tile and chunk)
  int cols;           // reduction length of the step (multiple of SAC_PAD)
  int NT;             // 16-row tiles of the packed matrix = output tiles of the step
  const float* bias;  // forward steps: bias [N], prefetched with the weights
  int N;
  int tcols;          // column count of the whole packed matrix: a 16-row tile is 16 * tcols elements
};
__device__ __forceinline__ GemmW gw_fwd(const AS_C LayerDev& L) { return GemmW{L.Wc, L.Kp, L.Np >> 4, L.bias, L.N, L.Kp}; }
__device__ __forceinline__ GemmW gw_bwd(const AS_C LayerDev& L) { return GemmW{L.WTc, L.Np, L.Kp >> 4, nullptr, 0, L.Np}; }
__device__ __forceinline__ GemmW gw_none() { return GemmW{nullptr, 0, 0, nullptr, 0, 0}; }
// Sub-matrix view of a packed [rows][cols_full] operand: rows [row0, row0 + nrows)
// (multiples of 16) and reduction columns [col0, col0 + ncols) (multiples of the
// MFMA K chunk).  Tile t starts at t * 16 * cols_full elements and chunk ch of a
// tile at ch * 64 * KL = ch * KC * 16 elements, so the view's origin is
// row0 * cols_full + col0 * 16 (packed_off with KL / KC = 1/4 for both dtypes).
template <typename T>
__device__ __forceinline__ GemmW gw_sub(const void* p, int cols_full, int row0, int nrows, int col0, int ncols,
                                        const float* bias, int N) {
  return GemmW{(const T*)p + (size_t)row0 * cols_full + (size_t)col0 * 16, ncols, nrows >> 4, bias, N, cols_full};
}

#ifndef SAC_PF
// Cross-step register prefetch of the weight stream: chunks per tile of the
// NEXT GEMM step each wave keeps in flight, plus its first bias values (see
// gemm_step).  Measured on C2: 1 chunk (8 VGPRs) 17.3K steps/s vs 17.8K without;
// 8 chunks spill at 8 waves.  Off by default.
#define SAC_PF 0
#endif
template <typename T>
struct Pf {
#if SAC_PF
  typename MM<T>::Frag f0[SAC_PF], f1[SAC_PF];
  float b0, b1;  // bias of the lane's column in the first tile pair (forward steps)
#endif
  const void* tag;  // which B matrix the registers hold (wave-uniform)
};

// Issue batch 0 (chunks 0..7, clamped) of this wave's first tile pair of step w.
template <typename T>
__device__ __forceinline__ void pf_issue(Pf<T>& pf, const GemmW& w) {
  pf.tag = w.p;
#if SAC_PF
  constexpr int KC = MM<T>::KC, FS = 64 * MM<T>::KL;
  const int lane = threadIdx.x & 63, wave = wave_id();
  if (!w.p || wave >= w.NT) return;
  const int last = w.cols / KC - 1;
  const int nt1 = wave + SAC_NW < w.NT ? wave + SAC_NW : wave;
  const AS_G T* b0 = GPC(T, w.p) + packed_lane<T>(wave, w.tcols, lane);
  const AS_G T* b1 = GPC(T, w.p) + packed_lane<T>(nt1, w.tcols, lane);
  if (w.bias) {  // same columns as layer_fwd's first pair: n0 = 16 wave + c, n1 = n0 + 16 SAC_NW
    const int n0 = wave * 16 + (lane & 15), n1 = n0 + 16 * SAC_NW;
    pf.b0 = GPC(float, w.bias)[n0 < w.N ? n0 : w.N - 1];
    pf.b1 = GPC(float, w.bias)[n1 < w.N ? n1 : w.N - 1];
  }
#pragma unroll
  for (int u = 0; u < SAC_PF; ++u) {
    const int cu = u < last ? u : last;
    pf.f0[u] = MM<T>::ld(b0 + cu * FS);
    pf.f1[u] = MM<T>::ld(b1 + cu * FS);
  }
#endif
}

// Held weights: a role that waits on a hand-off (or on its sample) loads the
// first HC chunks of its wave's first tile pair of a later GEMM step (+ that
// pair's bias) into registers BEFORE the wait, so the step after the wait starts
// on resident fragments instead of a cold L2/HBM stream.  Numerically identical
// to streaming (same fragments, same chunk order).  HC = 8 covers a whole
// 256-deep bf16 reduction: one 256x256 layer over 8 waves = one pair per wave,
// 64 VGPRs.
// f(integral_constant<int, U>) for U = 0..N-1: compile-time indices, so arrays
// indexed inside stay SSA values (a runtime-indexed loop, even one unrolled
// later, can leave the array in scratch)
template <typename F, int... U>
__device__ __forceinline__ void static_for_(std::integer_sequence<int, U...>, F&& f) {
  (f(std::integral_constant<int, U>()), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_(std::make_integer_sequence<int, N>(), f);
}

template <typename T, int HC>
struct Held {
  typename MM<T>::Frag f0[HC], f1[HC];
  float b0, b1;
  const void* tag;  // B matrix held (wave-uniform); gemm_step ignores a mismatch
};
template <typename T, int HC, bool COH = false>
__device__ __forceinline__ void held_issue(Held<T, HC>& h, const GemmW& w) {
  constexpr uint32_t FSB = 64 * MM<T>::KL * sizeof(T);
  const int lane = threadIdx.x & 63, wave = wave_id();
  h.tag = w.p;
  if (!w.p || wave >= w.NT) return;
  const int last = w.cols / MM<T>::KC - 1;
  const int nt1 = wave + SAC_NW < w.NT ? wave + SAC_NW : wave;
  const __amdgpu_buffer_rsrc_t rs = coh_rsrc(w.p, 0xFFFFFFF0u);
  const uint32_t o0 = (uint32_t)(packed_lane<T>(wave, w.tcols, lane) * sizeof(T));
  const uint32_t o1 = (uint32_t)(packed_lane<T>(nt1, w.tcols, lane) * sizeof(T));
  if (w.bias) {  // layer_fwd's first pair: n0 = 16 wave + c, n1 = n0 + 16 SAC_NW
    const int n0 = wave * 16 + (lane & 15), n1 = n0 + 16 * SAC_NW;
    h.b0 = ldf<COH>(w.bias + (n0 < w.N ? n0 : w.N - 1));
    h.b1 = ldf<COH>(w.bias + (n1 < w.N ? n1 : w.N - 1));
  }
  static_for<HC>([&](auto uc) {
    constexpr int u = decltype(uc)::value;
    const uint32_t cu = u < last ? u : last;
    h.f0[u] = coh_frag<T, COH>(rs, o0 + cu * FSB);
    h.f1[u] = coh_frag<T, COH>(rs, o1 + cu * FSB);
  });
}

// acc{0,1} += A x B for the BM chunks [ch, ch + BM) whose B fragments are in
// f0 / f1: all BM x RT A fragments are read from LDS first (one LDS round trip
// for the batch instead of one per chunk), and the has1 test sits outside the
// MFMA sequence so it stays straight-line.
template <typename T, int RT, int BM>
__device__ __forceinline__ void mma_batch(const lf* __restrict__ arow, int lda, int ch, bool has1,
                                          const typename MM<T>::Frag (&f0)[BM], const typename MM<T>::Frag (&f1)[BM],
                                          f32x4 (&acc0)[RT], f32x4 (&acc1)[RT]) {
  constexpr int KC = MM<T>::KC;
  typename MM<T>::Frag a[BM][RT];
  static_for<BM>([&](auto uc) {
    constexpr int u = decltype(uc)::value;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) a[u][rt] = MM<T>::from_lds(arow + rt * 16 * lda + (ch + u) * KC);
  });
  if (has1) {
    static_for<BM>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        MM<T>::mma(acc0[rt], a[u][rt], f0[u]);
        MM<T>::mma(acc1[rt], a[u][rt], f1[u]);
      }
    });
  } else {
    static_for<BM>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) MM<T>::mma(acc0[rt], a[u][rt], f0[u]);
    });
  }
}

// acc{0,1} += A x B over chunks [ch0, nch) loaded here, in batches of BM chunks
// whose loads are all issued before the batch's first MFMA.  A short last batch
// loads its last chunk again for the missing slots (unconditional, so the loads
// stay back to back) and skips their MFMAs.
template <typename T, int RT, int BM>
__device__ __forceinline__ void mma_pair_from(const lf* __restrict__ arow, int lda, __amdgpu_buffer_rsrc_t rs,
                                              uint32_t o0, uint32_t o1, bool has1, int ch0, int nch,
                                              f32x4 (&acc0)[RT], f32x4 (&acc1)[RT]) {
  constexpr int KC = MM<T>::KC;
  constexpr uint32_t FSB = 64 * MM<T>::KL * sizeof(T);  // bytes per fragment
  typedef typename MM<T>::Frag F;
  for (int ch = ch0; ch < nch; ch += BM) {
    const int rem = nch - ch < BM ? nch - ch : BM;
    F f0[BM], f1[BM];
#pragma unroll
    for (int u = 0; u < BM; ++u) {
      const uint32_t cu = ch + (u < rem ? u : rem - 1);
      f0[u] = coh_frag<T, false>(rs, o0 + cu * FSB);
      f1[u] = coh_frag<T, false>(rs, o1 + cu * FSB);
    }
    if (rem == BM) {  // full batch: every A fragment read from LDS up front, then the MFMAs
      mma_batch<T, RT, BM>(arow, lda, ch, has1, f0, f1, acc0, acc1);
    } else {
#pragma unroll
      for (int u = 0; u < BM; ++u)
        if (u < rem)
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) {
            const F a = MM<T>::from_lds(arow + rt * 16 * lda + (ch + u) * KC);
            MM<T>::mma(acc0[rt], a, f0[u]);
            if (has1) MM<T>::mma(acc1[rt], a, f1[u]);
          }
    }
  }
}

// The dominant shape, specialised: exactly one tile pair per wave (N = 32
// SAC_NW columns: 256 at 8 waves) and NCH reduction chunks known at compile
// time.  Straight-line: B fragments (held, or all NCH x 2 loads issued
// together), every A fragment from LDS, the MFMAs, the two epilogues.
template <typename T, int RT, int NCH, bool COH, int HC, typename Epi>
__device__ __forceinline__ void gemm_pair_fixed(const lf* __restrict__ arow, int lda, const GemmW& w, int lane,
                                                int wave, int c, Epi& epi, const Held<T, HC ? HC : 1>* held) {
  typedef typename MM<T>::Frag F;
  constexpr int KC = MM<T>::KC;
  constexpr uint32_t FSB = 64 * MM<T>::KL * sizeof(T);
  const int nt0 = wave, nt1 = wave + SAC_NW;
  F f0[NCH], f1[NCH];
  bool have = false;
  if constexpr (HC >= NCH) {
    if (held && held->tag == w.p) {  // uniform
      static_for<NCH>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        f0[u] = held->f0[u];
        f1[u] = held->f1[u];
      });
      have = true;
    }
  }
  if (!have) {
    const __amdgpu_buffer_rsrc_t rs = coh_rsrc(w.p, 0xFFFFFFF0u);
    const uint32_t o0 = (uint32_t)(packed_lane<T>(nt0, w.tcols, lane) * sizeof(T));
    const uint32_t o1 = (uint32_t)(packed_lane<T>(nt1, w.tcols, lane) * sizeof(T));
    static_for<NCH>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      f0[u] = coh_frag<T, COH>(rs, o0 + u * FSB);
      f1[u] = coh_frag<T, COH>(rs, o1 + u * FSB);
    });
  }
  F a[NCH][RT];
  static_for<NCH>([&](auto uc) {
    constexpr int u = decltype(uc)::value;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) a[u][rt] = MM<T>::from_lds(arow + rt * 16 * lda + u * KC);
  });
  f32x4 acc0[RT], acc1[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) acc0[rt] = acc1[rt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  static_for<NCH>([&](auto uc) {
    constexpr int u = decltype(uc)::value;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      MM<T>::mma(acc0[rt], a[u][rt], f0[u]);
      MM<T>::mma(acc1[rt], a[u][rt], f1[u]);
    }
  });
  epi(0, nt0 * 16 + c, acc0, true);
  epi(1, nt1 * 16 + c, acc1, true);
}

// One GEMM step over ROWS rows: out tile (r, col) for every col < 16*w.NT,
// acc = sum_k A[r][k] B[col][k]; epi(h, col, acc[RT]) consumes each tile pair.
// Batch 0 of the first pair comes from pf; the next step's batch 0 is issued
// into pf right after those MFMAs.
template <typename T, int ROWS, int HC, typename Epi>
__device__ __forceinline__ void gemm_step(const lf* __restrict__ A, int lda, const GemmW& w, Pf<T>& pf,
                                          const GemmW& next, Epi epi, const Held<T, HC ? HC : 1>* held) {
  constexpr int RT = ROWS / 16;
  constexpr int KC = MM<T>::KC, KL = MM<T>::KL;
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int c = lane & 15, g = lane >> 4;
  const int NT = w.NT, nch = w.cols / KC;
  const lf* arow = A + c * lda + g * KL;
#if !SAC_PF
  if (w.NT == 2 * SAC_NW) {  // one pair per wave (uniform branches)
    if (nch == 8) {
      gemm_pair_fixed<T, RT, 8, false, HC>(arow, lda, w, lane, wave, c, epi, held);
      return;
    }
    if (nch == 1) {
      gemm_pair_fixed<T, RT, 1, false, HC>(arow, lda, w, lane, wave, c, epi, held);
      return;
    }
  }
#endif
  if (pf.tag != w.p) pf_issue<T>(pf, w);  // chain broken by the caller: reload (uniform)
  // weight stream: plain buffer loads through a uniform descriptor (coh_frag<T, false>)
  const __amdgpu_buffer_rsrc_t rs = coh_rsrc(w.p, 0xFFFFFFF0u);
  auto pair = [&](int nt0, bool first) __attribute__((always_inline)) {
    const int nt1 = nt0 + SAC_NW;
    const bool has1 = nt1 < NT;
    const uint32_t o0 = (uint32_t)(packed_lane<T>(nt0, w.tcols, lane) * sizeof(T));
    const uint32_t o1 = (uint32_t)(packed_lane<T>(has1 ? nt1 : nt0, w.tcols, lane) * sizeof(T));
    f32x4 acc0[RT], acc1[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc0[rt] = acc1[rt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#if SAC_PF
    int ch0 = 0;
    if (first) {
      ch0 = nch < SAC_PF ? nch : SAC_PF;
#pragma unroll
      for (int u = 0; u < SAC_PF; ++u) {
        if (u < ch0)
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) {
            const typename MM<T>::Frag a = MM<T>::from_lds(arow + rt * 16 * lda + u * KC);
            MM<T>::mma(acc0[rt], a, pf.f0[u]);
            if (has1) MM<T>::mma(acc1[rt], a, pf.f1[u]);
          }
        // bound how many A fragments the scheduler hoists (register pressure)
        if (u & 1) __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_sched_barrier(0);  // old fragments consumed before the registers are reloaded
      pf_issue<T>(pf, next);
      __builtin_amdgcn_sched_barrier(0);
    }
    mma_pair_from<T, RT, 8>(arow, lda, rs, o0, o1, has1, ch0, nch, acc0, acc1);
#else
    if (HC > 0 && first && held && held->tag == w.p) {  // resident fragments (uniform branch)
      const int hn = nch < HC ? nch : HC;
      if (hn == HC) {
        mma_batch<T, RT, (HC ? HC : 1)>(arow, lda, 0, has1, held->f0, held->f1, acc0, acc1);
      } else {
        static_for<(HC ? HC : 1)>([&](auto uc) {
          constexpr int u = decltype(uc)::value;
          if (u < hn)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
              const typename MM<T>::Frag a = MM<T>::from_lds(arow + rt * 16 * lda + u * KC);
              MM<T>::mma(acc0[rt], a, held->f0[u]);
              if (has1) MM<T>::mma(acc1[rt], a, held->f1[u]);
            }
        });
      }
      if (hn < nch) mma_pair_from<T, RT, 8>(arow, lda, rs, o0, o1, has1, hn, nch, acc0, acc1);
    } else {
      mma_pair_from<T, RT, 8>(arow, lda, rs, o0, o1, has1, 0, nch, acc0, acc1);
    }
#endif
    epi(0, nt0 * 16 + c, acc0, first);
    if (has1) epi(1, nt1 * 16 + c, acc1, first);
  };
  // one instance of the pair code (runtime `first`) keeps the kernel's code small
  bool first = true;
  for (int nt0 = wave;; nt0 += 2 * SAC_NW) {
    if (nt0 >= NT) {
      if (first) pf_issue<T>(pf, next);
      break;
    }
    pair(nt0, first);
    first = false;
  }
}

// Activations other than ReLU/identity are applied in a compact second pass by
// the lanes that wrote the tile (same (row, col) mapping as the epilogue, so no
// barrier): one act switch per GEMM step instead of one per accumulator element.
template <int ROWS>
__device__ __forceinline__ void act_pass_fwd(lf* Y, int ldy, int NT, int act) {
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int c = lane & 15, g = lane >> 4;
#pragma unroll 1
  for (int nt = wave; nt < NT; nt += SAC_NW)
#pragma unroll 1
    for (int e = 0; e < ROWS / 4; ++e) {
      const int r = (e >> 2) * 16 + g * 4 + (e & 3);
      lf* y = Y + r * ldy + nt * 16 + c;
      *y = act_fwd(act, *y);
    }
}
template <int ROWS>
__device__ __forceinline__ void act_pass_bwd(lf* G, int ldg, const lf* P, int ldp, int NT, int K, int act) {
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int c = lane & 15, g = lane >> 4;
#pragma unroll 1
  for (int nt = wave; nt < NT; nt += SAC_NW) {
    const int k = nt * 16 + c;
    if (k >= K) continue;
#pragma unroll 1
    for (int e = 0; e < ROWS / 4; ++e) {
      const int r = (e >> 2) * 16 + g * 4 + (e & 3);
      G[r * ldg + k] = act_bwd(act, P[r * ldp + k], G[r * ldg + k]);
    }
  }
}

// Forward: Y[r][n] = act(sum_k X[r][k] W[n][k] + b[n]) for n < Np (padded -> 0).
// P (optional) keeps the pre-activation; Pg (optional) stashes rows >= pg_row0.
template <typename T, int ROWS, int HC = 0>
__device__ __forceinline__ void layer_fwd(const lf* X, int ldx, const AS_C LayerDev& L, const float* bias_, int act, lf* P,
                                          int ldp, lf* Y, int ldy, float* Pg_, int pg_row0, Pf<T>& pf,
                                          const GemmW& next, const Held<T, HC ? HC : 1>* held = nullptr) {
  const AS_G float* bias = GPC(float, bias_);
  AS_G float* Pg = GP(float, Pg_);
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int g = lane >> 4;
  const int N = L.N, Np = L.Np;
  // The first pair's bias is loaded before the step: a load issued after the
  // next step's prefetch would wait for all of it (vmcnt retires in order).
  const int n0 = wave * 16 + (lane & 15), n1 = n0 + 16 * SAC_NW;
  const GemmW w = gw_fwd(L);
#if SAC_PF
  if (pf.tag != w.p) pf_issue<T>(pf, w);  // bias arrives with the prefetched weights
  const float bpre0 = pf.b0, bpre1 = pf.b1;
#else
  const bool hb = HC > 0 && held && held->tag == w.p;  // bias held with the fragments
  const float bpre0 = hb ? held->b0 : ldf<false>((const float*)bias + (n0 < N ? n0 : N - 1));
  const float bpre1 = hb ? held->b1 : ldf<false>((const float*)bias + (n1 < N ? n1 : N - 1));
#endif
  // first: the wave's first tile pair, whose columns are n0 / n1 (bias preloaded)
  gemm_step<T, ROWS, HC>(X, ldx, w, pf, next, [&](int h, int n, const f32x4* acc, bool first) {
    const bool nv = n < N;
    const float bn = first ? (h ? bpre1 : bpre0) : ldf<false>((const float*)bias + (nv ? n : N - 1));
#pragma unroll
    for (int rt = 0; rt < ROWS / 16; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = rt * 16 + g * 4 + i;
        const float p = nv ? acc[rt][i] + bn : 0.f;
        if (P) P[r * ldp + n] = p;
        Y[r * ldy + n] = act == ACT_RELU ? (p > 0.f ? p : 0.f) : p;
        if (Pg && r >= pg_row0) Pg[(size_t)(r - pg_row0) * Np + n] = p;
      }
  }, held);
  if (act != ACT_RELU && act != ACT_ID) act_pass_fwd<ROWS>(Y, ldy, Np >> 4, act);
}

// dX: Gout[r][k] = act'(Pprev[r][k]) * sum_n G[r][n] W[n][k]   (act_prev < 0: no act')
template <typename T, int ROWS, int HC = 0>
__device__ __forceinline__ void layer_bwd(const lf* G, int ldg, const AS_C LayerDev& L, const lf* Pprev, int ldp,
                                          int act_prev, lf* Gout, int ldo, Pf<T>& pf, const GemmW& next,
                                          const Held<T, HC ? HC : 1>* held = nullptr) {
  const int g = (threadIdx.x & 63) >> 4;
  const int K = L.K;
  gemm_step<T, ROWS, HC>(G, ldg, gw_bwd(L), pf, next, [&](int, int k, const f32x4* acc, bool) {
    const bool kv = k < K;
#pragma unroll
    for (int rt = 0; rt < ROWS / 16; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = rt * 16 + g * 4 + i;
        float v = kv ? acc[rt][i] : 0.f;
        if (act_prev == ACT_RELU && !(Pprev[r * ldp + k] > 0.f)) v = 0.f;
        Gout[r * ldo + k] = v;
      }
  }, held);
  if (act_prev >= 0 && act_prev != ACT_RELU && act_prev != ACT_ID)
    act_pass_bwd<ROWS>(Gout, ldo, Pprev, ldp, L.Kp >> 4, K, act_prev);
}

// dst[k][col0 + r] = x[r][k] (0 for k >= K or r >= nvalid), k < Kp, where
// x[r][k] = src[r][k] * rowscale[r] (rowscale == null: 1); with dbp != null also
// dbp[col0 / SAC_ROWS][k] = sum_{r<nvalid} x[r][k] (k < K).
template <typename T, int ROWS>
__device__ __forceinline__ void store_T(const lf* __restrict__ src, int lds_ld, int Kp, int K, void* dst_,
                                                 int Bp, int col0, int nvalid, float* dbp_,
                                                 const lf* __restrict__ rowscale = nullptr, int dbp_ld = 0) {
  AS_G T* dst = GP(T, dst_);
  AS_G float* dbp = GP(float, dbp_);
  constexpr int CH = ROWS / 8;
  const int span = (Kp * CH + 63) / 64 * 64;  // whole waves iterate together (shuffles)
  for (int i = threadIdx.x; i < span; i += SAC_THREADS) {
    const bool live = i < Kp * CH;
    const int k = i / CH, ch = i % CH;
    T v[8];
    float s = 0.f, xv[8];
    // all reads issued before any use (a branch or wait per read would serialise them)
#pragma unroll
    for (int q = 0; q < 8; ++q) xv[q] = src[(ch * 8 + q) * lds_ld + (live ? k : 0)];
    if (rowscale) {
      float sc[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) sc[q] = rowscale[ch * 8 + q];
#pragma unroll
      for (int q = 0; q < 8; ++q) xv[q] = sc[q] * xv[q];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int r = ch * 8 + q;
      const float x = (live && r < nvalid && k < K) ? xv[q] : 0.f;
      s += x;
      v[q] = MM<T>::cvt(x);
    }
    if (live) {
      AS_G T* d = dst + (size_t)k * Bp + col0 + ch * 8;
      if constexpr (sizeof(T) == 2) {
        *(AS_G u32x4*)d = *(const u32x4*)v;
      } else {
        *(AS_G u32x4*)d = *(const u32x4*)v;
        *(AS_G u32x4*)(d + 4) = *(const u32x4*)(v + 4);
      }
    }
    if (dbp) {
#pragma unroll
      for (int o = 1; o < CH; o <<= 1) s += __shfl_xor(s, o, 64);
      if (live && ch == 0 && k < K) {
        AS_G float* bp = dbp + (size_t)(col0 / SAC_ROWS) * (dbp_ld ? dbp_ld : K) + k;
        *bp = s;
      }
    }
  }
}

// Full MLP forward over ROWS rows: hidden layers ping-pong Xb/Yb (stride ld), the
// output layer writes (Pout, Yout) with stride ldo.  keepP: per-layer
// pre-activations into lds[o_P[l]] (stride ldp[l]).  storeXT: each layer's input
// transposed into L.XT (ROWS must be SAC_ROWS).  after: the GEMM step that follows.
// HELD: layers 0 and 1 start on fragments held in h0 / h1 (see Held).
template <typename T, int ROWS, bool HELD = false>
__device__ __forceinline__ void mlp_forward(const AS_C NetDev& net, lf* Xb, lf* Yb, int ld, lf* Pout, lf* Yout, int ldo,
                                            const AS_C int* o_P, const AS_C int* ldp, lf* lds, bool keepP, bool storeXT, int Bp,
                                            int col0, int nvalid, Pf<T>& pf, const GemmW& after,
                                            const Held<T, 1>* h0 = nullptr, const Held<T, 8>* h1 = nullptr) {
  lf* X = Xb;
  lf* Y = Yb;
  for (int l = 0; l < net.L; ++l) {
    const AS_C LayerDev& Ly = net.l[l];
    const bool out = l == net.L - 1;
    const GemmW next = out ? after : gw_fwd(net.l[l + 1]);
    if (storeXT) {
      if constexpr (ROWS == SAC_ROWS) store_T<T, ROWS>(X, ld, Ly.Kp, Ly.K, Ly.XT, Bp, col0, nvalid, nullptr);
    }
    const int act = out ? net.out_act : net.hid_act;
    lf* Pl = out ? Pout : (keepP ? lds + o_P[l] : nullptr);
    const int ldpl = out ? ldo : (keepP ? ldp[l] : 0);
    lf* Yl = out ? Yout : Y;
    const int ldyl = out ? ldo : ld;
    if (HELD && l == 0)
      layer_fwd<T, ROWS, 1>(X, ld, Ly, net.P + Ly.b_off, act, Pl, ldpl, Yl, ldyl, nullptr, 0, pf, next, h0);
    else if (HELD && l == 1)
      layer_fwd<T, ROWS, 8>(X, ld, Ly, net.P + Ly.b_off, act, Pl, ldpl, Yl, ldyl, nullptr, 0, pf, next, h1);
    else
      layer_fwd<T, ROWS>(X, ld, Ly, net.P + Ly.b_off, act, Pl, ldpl, Yl, ldyl, nullptr, 0, pf, next);
    __syncthreads();
    lf* t = X;
    X = Y;
    Y = t;
  }
}

// Backward from d(output pre-activation) Gout [ROWS][ldo] down to layer 0's
// pre-activation gradient.  storeGT: each layer's dY^T + bias partial sums.
// Returns the buffer (stride ld) holding d(pre-act of layer 0).
// HELD: the output layer's and layer Lh-1's dX steps start on fragments held
// in h0 / h1 (see Held).
template <typename T, int ROWS, bool HELD = false>
__device__ __forceinline__ lf* mlp_backward(const AS_C NetDev& net, const lf* Gout, int ldo, lf* Xb, lf* Yb, int ld,
                                            const AS_C int* o_P, const AS_C int* ldp, lf* lds, bool storeGT, int Bp, int col0,
                                            int nvalid, Pf<T>& pf, const GemmW& after,
                                            const Held<T, 1>* h0 = nullptr, const Held<T, 8>* h1 = nullptr) {
  const int Lh = net.L - 1;
  const AS_C LayerDev& Lo = net.l[Lh];
  if (storeGT) store_T<T, ROWS>(Gout, ldo, Lo.Np, Lo.N, Lo.GT, Bp, col0, nvalid, Lo.dbp);
  layer_bwd<T, ROWS, HELD ? 1 : 0>(Gout, ldo, Lo, lds + o_P[Lh - 1], ldp[Lh - 1], net.hid_act, Yb, ld, pf,
                                        Lh - 1 >= 1 ? gw_bwd(net.l[Lh - 1]) : after, (const Held<T, 1>*)h0);
  __syncthreads();
  lf* G = Yb;
  lf* Gn = Xb;
  for (int l = Lh - 1; l >= 0; --l) {
    const AS_C LayerDev& Ly = net.l[l];
    if (storeGT) store_T<T, ROWS>(G, ld, Ly.Np, Ly.N, Ly.GT, Bp, col0, nvalid, Ly.dbp);
    if (l == 0) break;
    if (HELD && l == Lh - 1)
      layer_bwd<T, ROWS, 8>(G, ld, Ly, lds + o_P[l - 1], ldp[l - 1], net.hid_act, Gn, ld, pf,
                                 l - 1 >= 1 ? gw_bwd(net.l[l - 1]) : after, h1);
    else
      layer_bwd<T, ROWS>(G, ld, Ly, lds + o_P[l - 1], ldp[l - 1], net.hid_act, Gn, ld, pf,
                       l - 1 >= 1 ? gw_bwd(net.l[l - 1]) : after);
    __syncthreads();
    lf* t = G;
    G = Gn;
    Gn = t;
  }
  __syncthreads();
  return G;
}

#define LOG2F 0.69314718055994530942f
#define HALF_LOG_2PI 0.91893853320467274178f

__device__ __forceinline__ float fmin_nan(float a, float b) { return (a != a) ? a : (a < b ? a : b); }

// Unit-seed backward of a critic (phase A): Gout [R][ldo] holds d(out pre-act)
// for a seed of 1 per row; writes U_l = d(pre-act of hidden layer l) for every
// hidden layer into lds + E.o_P2[l] (stride E.ldp2[l]).  Pre-activations are in
// the E.o_P1 buffers (critic forward with keepP).
template <typename T, int ROWS>
__device__ __forceinline__ void critic_unit_backward(const AS_C EngineDev& E, const AS_C NetDev& net, const lf* Gout, int ldo,
                                                     lf* lds, Pf<T>& pf) {
  const int Lh = net.L - 1;
  layer_bwd<T, ROWS>(Gout, ldo, net.l[Lh], lds + E.o_P1[Lh - 1], E.ldp1[Lh - 1], net.hid_act, lds + E.o_P2[Lh - 1],
                     E.ldp2[Lh - 1], pf, Lh - 1 >= 1 ? gw_bwd(net.l[Lh - 1]) : gw_none());
  __syncthreads();
  for (int l = Lh - 1; l >= 1; --l) {
    layer_bwd<T, ROWS>(lds + E.o_P2[l], E.ldp2[l], net.l[l], lds + E.o_P1[l - 1], E.ldp1[l - 1], net.hid_act,
                       lds + E.o_P2[l - 1], E.ldp2[l - 1], pf, l - 1 >= 1 ? gw_bwd(net.l[l - 1]) : gw_none());
    __syncthreads();
  }
}

// ============================================================================ phases B / D
__device__ __forceinline__ float adam_elem(float& p, float& m, float& v, float g, float w1, float b2, float w2,
                                           float bc2s, float eps, float neg_step) {
  const float mm = m + w1 * (g - m);  // exp_avg.lerp_(grad, 1-beta1)
  float vv = v * b2;                  // exp_avg_sq.mul_(beta2)
  vv = vv + (w2 * g) * g;             //   .addcmul_(grad, grad, 1-beta2)
  const float denom = sqrtf(vv) / bc2s + eps;
  const float pn = p + (neg_step * mm) / denom;  // param.addcdiv_(exp_avg, denom, -step_size)
  m = mm;
  v = vv;
  p = pn;
  return pn;
}

// One 32x32 weight tile of an update phase, UT threads:
//   1. all threads stage the tile's 32 dY^T rows and 32 X^T rows (the dW GEMM's
//      operands, K = batch) into LDS and fetch their elements' master weight,
//      Adam moments, target weight and bias state, all in one round trip;
//   2. the dW MFMAs run as 16 (sub-tile, K-quarter) pairs spread over the
//      waves (one pair per wave at 16 waves): pair p owns 16x16 sub-tile p & 3
//      and the MFMA K-steps ch = p >> 2 (mod 4) of every staged chunk; the four
//      K-quarter partials are summed in LDS in quarter order (the same bits for
//      any block size);
//   3. every thread updates 1024 / UT elements: Adam (torch single-tensor op
//      order), Polyak, master weights; the packed compute copies are written
//      from LDS as whole 16-B fragment pieces (plain stores: the reader is the
//      next launch).
// 16 waves (measured on C2: 256-thread tiles took B 8.7 / D 7.8 us vs 6.4 / 5.9)
#ifndef SAC_UPD_THREADS
#define SAC_UPD_THREADS 1024
#endif
#define SAC_UPD_BCH (512 / (int)sizeof(T))  // batch columns staged per chunk (512 B per row)
// dynamic LDS of an update tile: upd_slots x stage 64 x 528 B | 2 x [32][33] f32 | [32][17] f32 |
// upd_slots x [256] f32 seeds (>= the alpha block's 5 x 1024 floats)
#define SAC_UPD_SLOT_BYTES (64 * 528)
#define SAC_UPD_LDS_FOR(slots) ((slots) * SAC_UPD_SLOT_BYTES + 2 * 32 * 33 * 4 + 32 * 17 * 4 + (slots) * 256 * 4)
template <typename T, int UT, int GS = 1, int MS = 2>
__device__ __forceinline__ void dw_adam_tile(const AS_C EngineDev& E, const TileDesc* tdp_, bool polyak, int par,
                                             int par_x, lf* lds) {
  constexpr int KC = MM<T>::KC, KL = MM<T>::KL;
  constexpr int EPR = 16 / sizeof(T);  // elements per 16-B piece (= KL)
  constexpr int EPT = 1024 / UT;       // elements per thread
  static_assert(EPR == KL, "a piece is one lane's fragment slice");
  const AS_C TileDesc& td = *(const AS_C TileDesc*)tdp_;  // scalar loads
  STAMP(polyak ? 48 : 52);
  const int tid = threadIdx.x;
  const int Bp = td.bp;
  // LDS: stage [64][SAC_UPD_BCH + pad] of T | acc / new params [32][33] f32 | targets [32][33] | bias reduce [32][17]
  const int lds_row = SAC_UPD_BCH + 16 / (int)sizeof(T);  // +16 B per row: rows start on different banks
  AS_L T* stage = (AS_L T*)lds;
  const int nslot = E.upd_slots;
  // slots (MS: the kernel's cap -- 2, or 1 for the 512-thread phase B: a
  // second slot in flight bought nothing there, one slot is C3 bf16 +1%,
  // profiles/r05_ab_update_slots.txt), pieces per thread per operand (32 rows)
  // per full chunk
  constexpr int MAXS = MS, PPO = 32 * (SAC_UPD_BCH / EPR) / UT;
  const int ns = nslot < MAXS ? nslot : MAXS;  // slots per round
  const int slot_el = 64 * lds_row;  // T elements per stage slot
  lf* accs = lds + (ns * slot_el * (int)sizeof(T) + 15) / 16 * 4;
  lf* tgts = accs + 32 * 33;
  lf* red = tgts + 32 * 33;
  // this step's Adam scalars (written by phase A)
  const float neg_step = GPC(float, E.adam_sc)[par * 6 + td.opt * 2];
  const float bc2s = GPC(float, E.adam_sc)[par * 6 + td.opt * 2 + 1];
  // ---- 1. loads: the first round of staged operands, then element state + bias
  // state + bias partials, all before the first wait (one round trip; the bias
  // sums below wait for everything issued before them, in issue order)
  static_assert(PPO >= 1 && (32 * (SAC_UPD_BCH / EPR)) % UT == 0, "whole pieces per thread");
  const int rstep = ns * SAC_UPD_BCH;          // batch columns per round
  u32x4 rg[MAXS][GS + 1][PPO];                 // [slot][dY part 0..GS-1, then X][piece]
  // the batch columns' seeds (TileDesc::seed).  Per dY piece (sdr) they are 16x
  // redundant loads, as many bytes as the dY pieces themselves through each CU's
  // load path; with several rounds (fp32 at C3) each chunk's seeds are instead
  // loaded ONCE (by the first bch / 4 threads) and handed over through LDS, a
  // round's written at the end of the round before: C3 fp32 +3%, while at C2
  // (one round) the extra barrier cost phase B 0.5 us (profiles/r05_ab_seeds_lds.txt)
  const AS_G float* const seedp = GPC(float, td.seed);  // uniform
  const bool lseeds = seedp && sizeof(T) == 4 && Bp > rstep;  // uniform
  AS_L float* seedL = (AS_L float*)(red + 32 * 17);      // [MAXS][SAC_UPD_BCH]
  f32x4 sreg[MAXS];                                       // lseeds: the next round's seeds of slot sl (tid < bch / 4)
  constexpr int SQ = EPR / 4;                             // seed f32x4 per 16-B piece (fp32 1, bf16 2)
  f32x4 sdr[MAXS][PPO][SQ];                               // !lseeds: the seeds of this thread's dY pieces
  // the operands' bases as separate values: a per-lane choice between two
  // descriptor fields was compiled into a per-lane LOAD of the chosen field and a
  // wait before every piece (the pieces' loads ran one round trip after another)
  const AS_G T* const gsrc = GPC(T, td.GT);
  const AS_G T* const xsrc = GPC(T, td.XT) + par_x * td.xt_par;
  const long goff = GS > 1 ? td.goff : 0;
  const int ldg = td.ld, ldx = td.ldx;
  // round r0's slot sl -> rg[sl] (16-B pieces of the 32 dY^T rows of every part, then of the 32 X^T rows)
  // what: 1 operands, 2 seeds, 3 both
  auto issue_seeds = [&](int r0, auto slc) __attribute__((always_inline)) {
    constexpr int sl = decltype(slc)::value;
    const int b0 = r0 + sl * SAC_UPD_BCH;
    if (lseeds && sl < ns && b0 < Bp) {  // uniform
      const int bch = Bp - b0 < SAC_UPD_BCH ? Bp - b0 : SAC_UPD_BCH;
      if (threadIdx.x * 4 < bch) sreg[sl] = *(const AS_G f32x4*)(seedp + b0 + threadIdx.x * 4);
    }
  };
  // pieces: seeds = false for round 0 (its seeds were issued before any piece)
  auto issue = [&](int r0, auto slc, bool seeds = true) {
    constexpr int sl = decltype(slc)::value;
    const int b0 = r0 + sl * SAC_UPD_BCH;
    if (sl < ns && b0 < Bp) {  // uniform
      const int bch = Bp - b0 < SAC_UPD_BCH ? Bp - b0 : SAC_UPD_BCH;
      const int per_row = bch / EPR;  // 16-B pieces per operand row of this chunk
      // the slot's seeds before its pieces: their wait (end of round) then does
      // not include this slot's pieces
      if (seeds) issue_seeds(r0, slc);
#pragma unroll
      for (int op = 0; op <= GS; ++op)
#pragma unroll
        for (int pi = 0; pi < PPO; ++pi) {
          const int i = threadIdx.x + pi * UT;
          const int row = i / per_row, pc = i % per_row;
          const AS_G T* src = op < GS ? gsrc + op * goff + (size_t)row * ldg : xsrc + (size_t)row * ldx;
          if (i < 32 * per_row) rg[sl][op][pi] = *(const AS_G u32x4*)(src + b0 + pc * EPR);
          if (op == 0 && seedp && !lseeds && i < 32 * per_row)
#pragma unroll
            for (int q = 0; q < SQ; ++q) sdr[sl][pi][q] = *(const AS_G f32x4*)(seedp + b0 + pc * EPR + 4 * q);
        }
    }
  };
  // round 0: every slot's seeds, then the pieces (the seeds' wait below includes no piece)
  static_for<MAXS>([&](auto sl) { issue_seeds(0, sl); });
  static_for<MAXS>([&](auto sl) { issue(0, sl, false); });
  // the seeds of round r0 + rstep's slots -> LDS (after round r0's last reads of seedL)
  auto seeds_to_lds = [&](int r0) __attribute__((always_inline)) {
    if (lseeds)  // uniform
      static_for<MAXS>([&](auto slc) {
        constexpr int sl = decltype(slc)::value;
        const int b0 = r0 + sl * SAC_UPD_BCH;
        if (sl < ns && b0 < Bp) {
          const int bch = Bp - b0 < SAC_UPD_BCH ? Bp - b0 : SAC_UPD_BCH;
          if (tid * 4 < bch) *(AS_L f32x4*)(seedL + sl * SAC_UPD_BCH + tid * 4) = sreg[sl];
        }
      });
  };
  AS_G float* W = GP(float, td.W);
  AS_G float* Wm = GP(float, td.Wm);
  AS_G float* Wv = GP(float, td.Wv);
  AS_G float* tW = GP(float, td.tW);
  float p[EPT], m[EPT], v[EPT], tp[EPT];
  size_t idx[EPT];
  bool ok[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int el = tid + e * UT, en = el >> 5, ek = el & 31;  // element (n0 + en, k0 + ek)
    const int n = td.n0 + en, k = td.k0 + ek;
    ok[e] = n < td.N && k < td.K;
    idx[e] = ok[e] ? (size_t)n * td.K + k : 0;
    if (td.kpart < 2) {  // uniform: a producer part only computes its partial dW
      p[e] = W[idx[e]];
      m[e] = Wm[idx[e]];
      v[e] = Wv[idx[e]];
      tp[e] = polyak ? tW[idx[e]] : 0.f;
    } else {
      p[e] = m[e] = v[e] = tp[e] = 0.f;
    }
  }
  const bool do_bias = td.k0 == 0 && td.kpart <= 1;
  // the bias gradient is summed from the staged (seed-scaled) dY rows, every
  // batch part its own columns (handed over with the partial dW)
  const bool bias_acc = td.k0 == 0;
  float pb = 0.f, mb = 0.f, vb = 0.f, tbv = 0.f;
  if (do_bias && tid < 32 && td.n0 + tid < td.N) {
    pb = GPC(float, td.b)[td.n0 + tid];
    mb = GPC(float, td.bm)[td.n0 + tid];
    vb = GPC(float, td.bv)[td.n0 + tid];
    if (polyak) tbv = GPC(float, td.tb)[td.n0 + tid];
  }
  // bias partial lanes: 16 per column (512 lanes, BPT per thread: the same sums
  // for 8- and 16-wave blocks), summed in LDS in lane order below
  constexpr int BPT = (512 + UT - 1) / UT;
  float bsum[BPT];
#pragma unroll
  for (int j = 0; j < BPT; ++j) bsum[j] = 0.f;
  // ---- 2. dW = dY^T X over the batch, staged through LDS in 512-B row chunks,
  // nslot chunks per round; waves run (16x16 sub-tile, K-quarter) pairs, chunks
  // in batch order.  A slot's registers are re-issued for the next round as
  // soon as they are in LDS, so round r + 1's loads land under round r's MFMAs.
  const int lane = tid & 63, wave = wave_id();
  const int c = lane & 15, g = lane >> 4;
  constexpr int KQ = 4, NWV = UT / 64, PPW = 16 / NWV;  // K-quarters, waves, pairs per wave
  static_assert(UT % 64 == 0 && 16 % NWV == 0, "16 (sub-tile, K-quarter) pairs over whole waves");
  f32x4 acc[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // round 0's seeds -> LDS: issued first, so this waits for them alone, after
  // every load of the tile (operands, element state, bias) is in flight
  seeds_to_lds(0);
  if (lseeds) __syncthreads();  // uniform
  for (int r0 = 0; r0 < Bp; r0 += rstep) {
    // slot by slot: its pieces -> LDS (waits only for this slot's loads: they
    // complete in issue order), the next round's loads into its registers,
    // barrier, its MFMAs -- while the later slots' loads are still landing
    static_for<MAXS>([&](auto slc) {
      constexpr int sl = decltype(slc)::value;
      const int b0 = r0 + sl * SAC_UPD_BCH;
      if (sl < ns && b0 < Bp) {  // uniform
        const int bch = Bp - b0 < SAC_UPD_BCH ? Bp - b0 : SAC_UPD_BCH;
        const int per_row = bch / EPR;
#pragma unroll
        for (int op = 0; op < 2; ++op)
#pragma unroll
          for (int pi = 0; pi < PPO; ++pi) {
            const int i = tid + pi * UT;
            const int row = i / per_row + 32 * op, pc = i % per_row;
            u32x4 v = rg[sl][op ? GS : 0][pi];
            if constexpr (sizeof(T) == 4) {
              if constexpr (GS > 1)
                if (op == 0) {  // dY: the parts' partials added in part order
                  f32x4 a = __builtin_bit_cast(f32x4, v);
#pragma unroll
                  for (int q = 1; q < GS; ++q) a += __builtin_bit_cast(f32x4, rg[sl][q][pi]);
                  v = __builtin_bit_cast(u32x4, a);
                }
              if (op == 0 && seedp)
                v = __builtin_bit_cast(u32x4, __builtin_bit_cast(f32x4, v) *
                                                  (lseeds ? *(const AS_L f32x4*)(seedL + sl * SAC_UPD_BCH + pc * EPR)
                                                          : sdr[sl][pi][0]));
            } else if (op == 0 && (GS > 1 || seedp)) {
              // bf16 dY: the parts added in fp32 (part order), scaled by the
              // rows' seeds in fp32, rounded to bf16 once
              bf16x8 h = __builtin_bit_cast(bf16x8, v);
              float a[8];
#pragma unroll
              for (int e = 0; e < 8; ++e) a[e] = (float)h[e];
#pragma unroll
              for (int q = 1; q < GS; ++q) {
                const bf16x8 hq = __builtin_bit_cast(bf16x8, rg[sl][q][pi]);
#pragma unroll
                for (int e = 0; e < 8; ++e) a[e] += (float)hq[e];
              }
              if (seedp)  // bf16: per-piece seeds (lseeds is fp32 only)
#pragma unroll
                for (int e = 0; e < 8; ++e) a[e] *= sdr[sl][pi][e >> 2][e & 3];
#pragma unroll
              for (int e = 0; e < 8; ++e) h[e] = (bf16)a[e];
              v = __builtin_bit_cast(u32x4, h);
            }
            if (i < 32 * per_row) *(AS_L u32x4*)(stage + sl * slot_el + row * lds_row + pc * EPR) = v;
          }
        issue(r0 + rstep, slc);
        __syncthreads();
        if (r0 == 0 && sl == 0) STAMP(polyak ? 51 : 55);
        if (bias_acc) {  // bias gradient: this lane's columns of the slot's (scaled) dY rows
#pragma unroll
          for (int j = 0; j < BPT; ++j) {
            const int t = tid + j * UT, bn = t >> 4, bs = t & 15;
            if (t < 512)  // 16-B LDS reads: lane bs takes the row's 16-B pieces bs, bs + 16, ...
              for (int c = bs * EPR; c < bch; c += 16 * EPR) {
                const AS_L T* q = stage + sl * slot_el + bn * lds_row + c;
                if constexpr (sizeof(T) == 4) {
                  const f32x4 x = *(const AS_L f32x4*)q;
                  bsum[j] += (x[0] + x[1]) + (x[2] + x[3]);
                } else {
                  const bf16x8 x = *(const AS_L bf16x8*)q;
                  float s = 0.f;
#pragma unroll
                  for (int e = 0; e < 8; ++e) s += (float)x[e];
                  bsum[j] += s;
                }
              }
          }
        }
#pragma unroll
        for (int j = 0; j < PPW; ++j) {
          const int pr = wave + j * NWV, kq = pr >> 2;
          const int ns = ((pr & 3) >> 1) * 16, ks = (pr & 1) * 16;
          const AS_L T* arow = stage + sl * slot_el + (ns + c) * lds_row + g * KL;
          const AS_L T* brow = stage + sl * slot_el + (32 + ks + c) * lds_row + g * KL;
          for (int ch = kq; ch < bch / KC; ch += KQ) {
            typename MM<T>::Frag a, b;
            if constexpr (sizeof(T) == 2) {
              a = *(const AS_L bf16x8*)(arow + ch * KC);
              b = *(const AS_L bf16x8*)(brow + ch * KC);
            } else {
              a = *(const AS_L f32x4*)(arow + ch * KC);
              b = *(const AS_L f32x4*)(brow + ch * KC);
            }
            MM<T>::mma(acc[j], a, b);
          }
        }
      }
    });
    seeds_to_lds(r0 + rstep);  // every thread's reads of this round's seeds are behind a slot barrier
    __syncthreads();  // the stage is refilled by the next round
  }
  STAMP(polyak ? 49 : 53);
  {  // K-quarter partials -> the (free) stage area, summed in quarter order below
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int pr = wave + j * NWV;
      const int ns = ((pr & 3) >> 1) * 16, ks = (pr & 1) * 16;
      lf* part = (lf*)stage + (pr >> 2) * (32 * 33);
#pragma unroll
      for (int i = 0; i < 4; ++i) part[(ns + g * 4 + i) * 33 + ks + c] = acc[j][i];
    }
  }
  __syncthreads();
  for (int el = tid; el < 1024; el += UT) {
    const int o = (el >> 5) * 33 + (el & 31);
    const lf* part = (const lf*)stage;
    float sum = part[o];
#pragma unroll
    for (int q = 1; q < KQ; ++q) sum += part[q * (32 * 33) + o];
    accs[o] = sum;
  }
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    const int t = tid + j * UT;
    if (bias_acc && t < 512) red[(t >> 4) * 17 + (t & 15)] = bsum[j];
  }
  __syncthreads();
  // producer parts a consumer takes (the 512-thread tiles: up to 7, else 3)
  constexpr int MAXP = UT == 512 ? 7 : 3;
  float gbx[MAXP];  // staged-row bias: the producer parts' column sums (consumer, tid < 32)
#pragma unroll
  for (int q = 0; q < MAXP; ++q) gbx[q] = 0.f;
  if (td.kpart) {  // hidden-split layer 0: the batch parts of this tile meet here
    const uint32_t ep = *GPC(uint32_t, E.sync) + 1u;  // per launch (B and D have their own granules)
    if (td.kpart >= 2) {
      AS_G uint64_t* mine = GP(uint64_t, td.part) + (size_t)(td.kpart - 2) * SAC_PART_STRIDE;
      for (int el = tid; el < 1024; el += UT) {
        const uint64_t x = (uint64_t)__float_as_uint(accs[(el >> 5) * 33 + (el & 31)]) | ((uint64_t)ep << 32);
        __hip_atomic_store((uint64_t*)(mine + el), x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (bias_acc && tid < 32) {
        float gb = 0.f;
        for (int q = 0; q < 16; ++q) gb += red[tid * 17 + q];
        const uint64_t x = (uint64_t)__float_as_uint(gb) | ((uint64_t)ep << 32);
        __hip_atomic_store((uint64_t*)(mine + 1024 + tid), x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;  // uniform: part 1 runs Adam on the sum
    }
    // each thread polls all of its 1024 / UT elements' granules of every
    // producer part in one batch of loads per attempt (one round trip, not one
    // per element); parts are added in order
    constexpr int EL = 1024 / UT;
    static_assert(EL * UT == 1024 && EL <= 4, "granules per thread");
    const int np = td.nparts - 1;  // producer parts (1..MAXP)
    const bool pb_here = do_bias && tid < 32;
    float v[MAXP][EL];
    for (int it = 0;; ++it) {
      bool all = true;
#pragma unroll
      for (int q = 0; q < MAXP; ++q)
        if (q < np) {
#pragma unroll
          for (int j = 0; j < EL; ++j) {
            const uint64_t x = __hip_atomic_load(td.part + (size_t)q * SAC_PART_STRIDE + tid + j * UT,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            all = all && (uint32_t)(x >> 32) == ep;
            v[q][j] = __uint_as_float((uint32_t)x);
          }
          if (pb_here) {
            const uint64_t x = __hip_atomic_load(td.part + (size_t)q * SAC_PART_STRIDE + 1024 + tid,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            all = all && (uint32_t)(x >> 32) == ep;
            gbx[q] = __uint_as_float((uint32_t)x);
          }
        }
      if (all) break;
      if (it > E.spin_limit) {  // a producer part never ran: flag the error, do not hang
        __hip_atomic_store((uint32_t*)GP(uint32_t, E.sync) + 1 /* SYNC_TIMEOUT */, 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int j = 0; j < EL; ++j) {
      const int el = tid + j * UT, o = (el >> 5) * 33 + (el & 31);
      float sum = accs[o];
#pragma unroll
      for (int q = 0; q < MAXP; ++q)
        if (q < np) sum += v[q][j];
      accs[o] = sum;
    }
    __syncthreads();
  }
  STAMP(polyak ? 50 : 54);
  // ---- 3. elements: Adam + Polyak on the masters; new values -> LDS
  const float w1 = (float)(1.0 - (double)E.beta1), b2 = E.beta2, w2 = (float)(1.0 - (double)E.beta2);
  const float eps = E.adam_eps, tau = E.tau, omt = (float)(1.0 - (double)E.tau);
  float pn[EPT], tn[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int el = tid + e * UT;
    pn[e] = 0.f;
    tn[e] = 0.f;
    if (ok[e]) {
      pn[e] = adam_elem(p[e], m[e], v[e], accs[(el >> 5) * 33 + (el & 31)], w1, b2, w2, bc2s, eps, neg_step);
      W[idx[e]] = p[e];
      Wm[idx[e]] = m[e];
      Wv[idx[e]] = v[e];
      if (polyak) {
        tn[e] = tau * pn[e] + omt * tp[e];
        tW[idx[e]] = tn[e];
      }
    }
  }
  __syncthreads();  // every read of accs done
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int el = tid + e * UT;
    accs[(el >> 5) * 33 + (el & 31)] = pn[e];  // padding elements: 0, as packed
    if (polyak) tgts[(el >> 5) * 33 + (el & 31)] = tn[e];
  }
  if (do_bias && tid < 32 && td.n0 + tid < td.N) {
    float gb = 0.f;
    for (int q = 0; q < 16; ++q) gb += red[tid * 17 + q];
    if (td.kpart) {  // the other batch parts' sums, in part order
#pragma unroll
      for (int q = 0; q < MAXP; ++q)
        if (q < td.nparts - 1) gb += gbx[q];
    }
    const float pbn = adam_elem(pb, mb, vb, gb, w1, b2, w2, bc2s, eps, neg_step);
    GP(float, td.b)[td.n0 + tid] = pb;
    GP(float, td.bm)[td.n0 + tid] = mb;
    GP(float, td.bv)[td.n0 + tid] = vb;
    if (polyak) GP(float, td.tb)[td.n0 + tid] = tau * pbn + omt * tbv;  // read by the next step's launch only
  }
  __syncthreads();
  // ---- packed copies as 16-B pieces: Wc / tWc rows n (EPR consecutive k), WTc rows k
  constexpr int PPR = 32 / EPR;  // pieces per 32-element tile row
  for (int mat = 0; mat < (polyak ? 3 : 2); ++mat) {  // uniform: one buffer descriptor per matrix
    const void* base = mat == 0 ? td.Wc : mat == 1 ? td.WTc : td.tWc;
    for (int i = tid; i < 32 * PPR; i += UT) {
      const int row = i / PPR, pc = i % PPR;
      T vv[EPR];
      size_t off;
      if (mat == 1) {  // W^T: row k = k0 + row, columns n = n0 + pc * EPR + j
#pragma unroll
        for (int j = 0; j < EPR; ++j) vv[j] = MM<T>::cvt(accs[(pc * EPR + j) * 33 + row]);
        off = packed_off<T>(td.k0 + row, td.n0 + pc * EPR, td.Np);
      } else {  // W or target W: row n = n0 + row, columns k = k0 + pc * EPR + j
        const lf* srcm = mat == 0 ? accs : tgts;
#pragma unroll
        for (int j = 0; j < EPR; ++j) vv[j] = MM<T>::cvt(srcm[row * 33 + pc * EPR + j]);
        off = packed_off<T>(td.n0 + row, td.k0 + pc * EPR, td.Kp);
      }
      coh_store16<false>(base, (uint32_t)(off * sizeof(T)), *(const u32x4*)vv);
    }
  }
}

// a tile with summed dY parts (hidden-split layer 0) runs its own instance
template <typename T, int UT, int MS = 2>
__device__ __forceinline__ void dw_adam_tile_any(const AS_C EngineDev& E, const TileDesc* tdp_, bool polyak, int par,
                                                 int par_x, lf* lds) {
  if constexpr (UT != 512) {  // (the 512-thread phase B never runs the hidden split's summed tiles)
    const int gs = ((const AS_C TileDesc*)tdp_)->gsum;  // uniform
    if constexpr (sizeof(T) == 4)
      if (gs == 4) return dw_adam_tile<T, UT, 4, MS>(E, tdp_, polyak, par, par_x, lds);
    if (gs == 2) return dw_adam_tile<T, UT, 2, MS>(E, tdp_, polyak, par, par_x, lds);
  }
  dw_adam_tile<T, UT, 1, MS>(E, tdp_, polyak, par, par_x, lds);
}

// One block: reduces the step's loss partials into stats[0..3] and runs the
// float64 alpha Adam step (agent.py:263-280).  All blockDim.x threads take part
// (no early exit: the caller's completion barrier follows).  alpha_state is
// stored sc1 (from the fused step, where phase A's critics read alpha after the
// completion counter; phase A is the next launch since round 5).
__device__ __forceinline__ void alpha_and_losses(const AS_C EngineDev& E, int par, lf* red) {
  const int tid = threadIdx.x, NT = blockDim.x, B = E.B;
  const float H = E.target_entropy;
  AS_G double* st = GP(double, E.alpha_state);
  const double st0 = st[0];
  const float la32 = (float)st0;
  const float mB = -1.0f / (float)B;
  const AS_G float* lp = GPC(float, E.lp_st) + par * E.Br;
  const AS_G float* lossp = GPC(float, E.lossp) + par * E.nrt * 4;
  float sg = 0.f, sl = 0.f, l0 = 0.f, l1 = 0.f, l2 = 0.f;
  for (int b = tid; b < B; b += NT) {
    const float term = lp[b] + H;
    sg += mB * term;
    sl += la32 * term;
  }
  for (int rt = tid; rt < E.nrt; rt += NT) {
    l0 += lossp[rt * 4 + 0];
    l1 += lossp[rt * 4 + 1];
    l2 += lossp[rt * 4 + 2];
  }
  red[0 * NT + tid] = sg;
  red[1 * NT + tid] = sl;
  red[2 * NT + tid] = l0;
  red[3 * NT + tid] = l1;
  red[4 * NT + tid] = l2;
  __syncthreads();
  for (int s = NT / 2; s > 0; s >>= 1) {
    if (tid < s)
      for (int j = 0; j < 5; ++j) red[j * NT + tid] += red[j * NT + tid + s];
    __syncthreads();
  }
  if (tid == 0) {
    AS_G float* stats = GP(float, E.stats);
    stats[0] = red[2 * NT] / (float)B;
    stats[1] = red[3 * NT] / (float)B;
    stats[2] = red[4 * NT] / (float)B;
    stats[3] = E.auto_entropy ? -(red[1 * NT] / (float)B) : __builtin_nanf("");
    if (E.auto_entropy && E.alpha_update) {
      const double gr = (double)red[0];
      const double b1 = (double)E.beta1, b2 = (double)E.beta2;
      const double st2 = st[2], st3 = st[3];
      const double m = st2 + (1.0 - b1) * (gr - st2);
      const double v = st3 * b2 + (1.0 - b2) * gr * gr;
      const double bc1 = GPC(double, E.alpha_sc)[par * 2];
      const double bc2 = GPC(double, E.alpha_sc)[par * 2 + 1];
      const double denom = sqrt(v) / sqrt(bc2) + (double)E.adam_eps;
      const double la = st0 + (-(E.alpha_lr / bc1)) * m / denom;
      double* sd = (double*)E.alpha_state;
      __hip_atomic_store(sd + 0, la, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sd + 1, exp(la), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sd + 2, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sd + 3, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ============================================================================ role hand-offs
// With E.roles, phases A and C run as several workgroups per row tile, one per
// network ("role"), that hand small per-row results to each other inside the
// launch (MI355X_MICROARCH.md §visibility, write-through form): every payload
// store and load is an agent-scope (sc1) access, the storing waves drain their
// stores (s_waitcnt vmcnt(0)) before a workgroup barrier, then one lane stores
// the flag (sc1); the consumer polls the flag with sc1 loads from one lane and
// joins the others at a barrier.  Flags carry a per-launch epoch (E.sync[0] + 1,
// advanced by phase C), so they are never reset.  Producers have lower block
// indices than their consumers in every layout (phase A: pi(s') -> target
// critics -> critics; phase C: critics -> pi), so
// in-order dispatch gives every spinning consumer resident producers; spins are
// still bounded (E.spin_limit) and set E.sync[1] on a timeout, which the host
// API turns into an error (sac_engine_read_status, SacEngine._poll_status).
enum HandKind { HK_PI = 0, HK_T1 = 1, HK_T2 = 2, HK_C1 = 3, HK_C2 = 4, HK_COUNT = 5 };
// SYNC_STAGED (u64 at words 4-5): step whose phase A last used a staged batch record
enum SyncWord { SYNC_EPOCH = 0, SYNC_TIMEOUT = 1, SYNC_STAGED = 4, SYNC_CDONE = 64, SYNC_FLAGS = 128 };
#define SAC_HAND_STRIDE 576  // floats per (kind, row tile) payload: >= SAC_ROWS * (act_dim + 1)

__device__ __forceinline__ AS_G uint32_t* hand_flag(const AS_C EngineDev& E, int kind, int rbi) {
  return GP(uint32_t, E.sync) + SYNC_FLAGS + (kind * E.nrt + rbi) * 16;  // one 64-B line per flag
}
__device__ __forceinline__ AS_G float* hand_data(const AS_C EngineDev& E, int kind, int rbi) {
  return GP(float, E.hand) + (size_t)(kind * E.nrt + rbi) * SAC_HAND_STRIDE;
}
__device__ __forceinline__ void st_sc1(AS_G float* p, float v) {
  __hip_atomic_store((float*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const AS_G float* p) {
  return __hip_atomic_load((float*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// all threads: after this workgroup's sc1 payload stores
__device__ __forceinline__ void hand_publish(const AS_C EngineDev& E, int kind, int rbi, uint32_t ep) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store((uint32_t*)hand_flag(E, kind, rbi), ep, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
}
// all threads: returns once flag(kind, rbi) == ep (or the spin gave up)
__device__ __forceinline__ void hand_wait(const AS_C EngineDev& E, int kind, int rbi, uint32_t ep) {
  if (threadIdx.x == 0) {
    uint32_t* f = (uint32_t*)hand_flag(E, kind, rbi);
    for (int it = 0; __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ep; ++it) {
      if (it > E.spin_limit) {  // ~0.3 s: a producer never ran; flag the error, do not hang the GPU
        __hip_atomic_store((uint32_t*)GP(uint32_t, E.sync) + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
}

// all threads: returns once both flags == ep (one polling lane, one barrier)
__device__ __forceinline__ void hand_wait2(const AS_C EngineDev& E, int k1, int k2, int rbi, uint32_t ep) {
  if (threadIdx.x == 0) {
    uint32_t* f1 = (uint32_t*)hand_flag(E, k1, rbi);
    uint32_t* f2 = (uint32_t*)hand_flag(E, k2, rbi);
    for (int it = 0;; ++it) {
      const uint32_t a = __hip_atomic_load(f1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t b = __hip_atomic_load(f2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (a == ep && b == ep) break;
      if (it > E.spin_limit) {
        __hip_atomic_store((uint32_t*)GP(uint32_t, E.sync) + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
}

// Data-tagged granules (MI355X_MICROARCH.md, handoff-1to1) for the hand-offs
// whose consumer needs a few values per row: one 8-B sc1 store carries {value,
// epoch}, and the consumer's lanes poll the values themselves.  There is no
// drain, no separate flag, and one round trip.  Epochs advance once per step and
// are never reset, so a granule left from an earlier step never matches.
//   G_Q1T / G_Q2T: Q1t(s', a~') / Q2t per row (target critics -> critics),
//   G_LP:          log pi(a~'|s') per row (target critic 1 -> critics),
//   G_C1 / G_C2:   dQ_i/da~ [R][A] then q_i [R] (phase C critics -> pi),
//   G_PI:          a~' [R][A] then log pi' [R] (pi(s') -> target critics).
enum GranKind { G_Q1T = 0, G_Q2T = 1, G_LP = 2, G_C1 = 3, G_C2 = 4, G_PI = 5, G_COUNT = 6 };
__device__ __forceinline__ AS_G uint64_t* gran_at(const AS_C EngineDev& E, int kind, int rbi) {
  return GP(uint64_t, E.gran) + (size_t)(kind * E.nrt + rbi) * E.gstride;
}
__device__ __forceinline__ void gran_put(AS_G uint64_t* g, float v, uint32_t ep) {
  const uint64_t x = (uint64_t)__float_as_uint(v) | ((uint64_t)ep << 32);
  __hip_atomic_store((uint64_t*)g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one lane: the granule's value once it carries epoch ep (bounded spin; a
// timeout sets the engine's error flag, see sac_engine_check)
__device__ __forceinline__ float gran_get(const AS_C EngineDev& E, const AS_G uint64_t* g, uint32_t ep) {
  uint64_t x = 0;
  for (int it = 0;; ++it) {
    x = __hip_atomic_load((uint64_t*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)(x >> 32) == ep) break;
    if (it > E.spin_limit) {
      __hip_atomic_store((uint32_t*)GP(uint32_t, E.sync) + SYNC_TIMEOUT, 1u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return __uint_as_float((uint32_t)x);
}

// one lane: N granules polled together (every load of a poll in flight at once:
// one round trip once the producers have stored, not N in sequence)
// Pipelined hand-off polls (gran_getn): the s_sleep between a consumer's two
// polls in flight; 0 = one poll per round trip.  Same-box A/Bs, C2 fp32: 8 ->
// +0.6% steps/s over 0 (both interleaved reps), 20 -> -1%; then 4 -> +0.5%
// over 8, 12 mixed (profiles/r02_ab_poll2.txt, r02_ab_poll_spacing.txt).
#ifndef SAC_POLL2
#define SAC_POLL2 4
#endif
template <int N>
__device__ __forceinline__ bool gran_ok(const uint64_t (&x)[N], uint32_t ep) {
  bool all = true;
#pragma unroll
  for (int i = 0; i < N; ++i) all = all && (uint32_t)(x[i] >> 32) == ep;
  return all;
}
template <int N>
__device__ __forceinline__ void gran_issue(const AS_G uint64_t* const (&g)[N], uint64_t (&x)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) x[i] = __hip_atomic_load((uint64_t*)g[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one poll in flight (register-lean: N granules need 2N VGPRs, not 4N)
template <int N>
__device__ __forceinline__ void gran_getn1(const AS_C EngineDev& E, const AS_G uint64_t* const (&g)[N], uint32_t ep,
                                           float (&out)[N]) {
  uint64_t x[N];
  for (int it = 0;; ++it) {
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = __hip_atomic_load((uint64_t*)g[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool all = true;
#pragma unroll
    for (int i = 0; i < N; ++i) all = all && (uint32_t)(x[i] >> 32) == ep;
    if (all) break;
    if (it > E.spin_limit) {
      __hip_atomic_store((uint32_t*)GP(uint32_t, E.sync) + SYNC_TIMEOUT, 1u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = __uint_as_float((uint32_t)x[i]);
}
template <int N>
__device__ __forceinline__ void gran_getn(const AS_C EngineDev& E, const AS_G uint64_t* const (&g)[N], uint32_t ep,
                                          float (&out)[N]) {
#if SAC_POLL2
  // Two polls in flight, half a round trip apart: a failed check re-issues its
  // poll at once while the other one is still on its way, so a granule that
  // lands is seen ~RTT/4 after (on average) instead of ~RTT/2.  The check of
  // one poll waits only for its own loads (the other's were issued later).
  uint64_t x[N], y[N];
  gran_issue<N>(g, x);
  __builtin_amdgcn_s_sleep(SAC_POLL2);
  gran_issue<N>(g, y);
  for (int it = 0;; it += 2) {
    if (gran_ok<N>(x, ep)) {
#pragma unroll
      for (int i = 0; i < N; ++i) out[i] = __uint_as_float((uint32_t)x[i]);
      return;
    }
    gran_issue<N>(g, x);
    if (gran_ok<N>(y, ep)) {
#pragma unroll
      for (int i = 0; i < N; ++i) out[i] = __uint_as_float((uint32_t)y[i]);
      return;
    }
    if (it > E.spin_limit) {
      __hip_atomic_store((uint32_t*)GP(uint32_t, E.sync) + SYNC_TIMEOUT, 1u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int i = 0; i < N; ++i) out[i] = __uint_as_float((uint32_t)y[i]);
      return;
    }
    gran_issue<N>(g, y);
  }
#else
  gran_getn1<N>(E, g, ep, out);
#endif
}

// ============================================================================ sample + gather
// Row tile r0's replay slots for `step` (replay_buffer.py:32-39: distinct
// uniform logical rows, 0 = oldest; -1 for padding rows): threads tid < R.
__device__ __forceinline__ void tile_slots(const AS_C EngineDev& E, const sac_replay& rb, uint64_t step,
                                           int64_t rb_size, int64_t rb_pos, int r0, const AS_G int32_t* inj_idx,
                                           AS_L int64_t* slotB) {
  const int tid = threadIdx.x;
  if (tid < SAC_ROWS) {
    int64_t slot = -1;
    const int b = r0 + tid;
    if (b < E.B) {
      int64_t li;
      if (inj_idx) {
        li = inj_idx[b];
      } else {
        const Feistel f = feistel_make(E.seed, step, rb_size);
        li = feistel_sample(f, b, rb_size);
      }
      slot = rb_size < rb.capacity ? li : (rb_pos + li) % rb.capacity;
    }
    slotB[tid] = slot;
  }
}

// Gather the tile's rows (agent.py:166-193) into s, s2 [R][O], a [R][A], r, d [R]
// (LDS or global): one pass, every load unconditional (row 0 for padding rows).
template <typename Dst>
__device__ __forceinline__ void gather_rows(const sac_replay& rb, const AS_L int64_t* slotB, int O, int A, Dst s,
                                            Dst s2, Dst a, Dst r, Dst d) {
  constexpr int R = SAC_ROWS;
  const AS_G float* obs = GPC(float, rb.obs);
  const AS_G float* nobs = GPC(float, rb.next_obs);
  const AS_G float* ract = GPC(float, rb.act);
  const AS_G float* rrew = GPC(float, rb.rew);
  const AS_G float* rdone = GPC(float, rb.done);
  const RowStrides rs = row_strides(rb.row_stride, O, A);
  const int nI = R * (O > A ? O : A);
  for (int i = threadIdx.x; i < nI; i += SAC_THREADS) {
    const int io = i < R * O ? i : R * O - 1, ia = i < R * A ? i : R * A - 1, ir = i < R ? i : R - 1;
    const int64_t so = slotB[io / O], sa = slotB[ia / A], sr = slotB[ir];
    const int64_t po = (so < 0 ? 0 : so) * rs.obs + io % O, pa = (sa < 0 ? 0 : sa) * rs.act + ia % A,
                  pr = (sr < 0 ? 0 : sr) * rs.one;
    const float vo = obs[po], vn = nobs[po], va = ract[pa], vr = rrew[pr], vd = rdone[pr];
    if (i < R * O) {
      s[i] = so >= 0 ? vo : 0.f;
      s2[i] = so >= 0 ? vn : 0.f;
    }
    if (i < R * A) a[i] = sa >= 0 ? va : 0.f;
    if (i < R) {
      r[i] = sr >= 0 ? vr : 0.f;
      d[i] = sr >= 0 ? vd : 0.f;
    }
  }
}

// Stager block (phase C): step t+1's rows of row tile rbi into E.stg.  Phase C
// is the step's last reader of the previous record (phase A of step t consumed
// it before this launch began); the next launch sees the stores.
// The record of step s is slot s & 1 (stage_rec): the stager of step t + 1
// never overwrites the record step t's phase A reads (the fused step stages
// inside the same launch as that phase A).
__device__ __forceinline__ size_t stage_rec(const AS_C EngineDev& E, uint64_t step, int rbi) {
  return ((size_t)(step & 1) * E.nrt + rbi) * E.stg_stride;
}
__device__ __forceinline__ void stage_next_batch(const AS_C EngineDev& E, const sac_replay& rb, int rbi, lf* lds,
                                                 uint64_t cur_step) {
  constexpr int R = SAC_ROWS;
  const uint64_t step = cur_step + 1;  // the batch is step t + 1's
  const int64_t rb_size = GPC(int64_t, rb.state)[0], rb_pos = GPC(int64_t, rb.state)[1];
  AS_G float* rec = GP(float, E.stg) + stage_rec(E, step, rbi);
  AS_G uint64_t* hdr = (AS_G uint64_t*)rec;
  if (rb_size < E.B) {  // nothing to sample: leave no matching record
    if (threadIdx.x == 0) hdr[0] = ~0ull;
    return;
  }
  AS_L int64_t* slotB = (AS_L int64_t*)lds;
  tile_slots(E, rb, step, rb_size, rb_pos, rbi * R, nullptr, slotB);
  __syncthreads();
  const int O = E.O, A = E.A;
  AS_G float* p = rec + 16;
  gather_rows<AS_G float*>(rb, slotB, O, A, p, p + R * O, p + 2 * R * O, p + 2 * R * O + R * A,
                           p + 2 * R * O + R * A + R);
  if (threadIdx.x == 0) {
    hdr[0] = step;
    hdr[1] = (uint64_t)rb_size;
    hdr[2] = (uint64_t)rb_pos;
    hdr[3] = (uint64_t)(uintptr_t)rb.obs;
    hdr[4] = (uint64_t)GPC(int64_t, rb.state)[2];  // push generation: any push / clear() invalidates
  }
}

// ============================================================================ phase A
// sample + gather, pi on [s'; s], target twin-Q -> y, critics forward + backward.
// ROLES: block = role * nrt + row tile; role 0 pi on s' (target sample), 1/2
// target critics, 3/4 critics, 5 pi on s (actor sample, stashed for phase C).
template <typename T, bool ROLES>
__device__ __forceinline__ void target_critic_body(const EngineDev* __restrict__ Ep, const sac_replay& rb,
                                                   const int32_t* __restrict__ inj_idx_,
                                                   const float* __restrict__ inj_eps_) {
  PREFETCH_ARG(Ep);
  const AS_C EngineDev& E = *(const AS_C EngineDev*)Ep;
  extern __shared__ float lds_raw[];
  lf* lds = (lf*)lds_raw;
  constexpr int R = SAC_ROWS;
  const int tid = threadIdx.x;
  const int bid = blockIdx.x;
  int rbi, role;
  if (ROLES) {
    rbi = bid % E.nrt;
    role = bid / E.nrt;
  } else {
    if (blockIdx.x % E.xs) return;  // XCD placement: see EngineDev::xs
    rbi = blockIdx.x / E.xs;
    role = -1;
  }
  const bool do_pi = !ROLES || role == 0 || role == 5;
  STAMP(0);
  CLK_STAMP(40);
  const int B = E.B, Bp = E.Bp, O = E.O, A = E.A, ld = E.ld, ldo = E.ldo;
  const int r0 = rbi * R;
  const int nvalid = min(R, B - r0);
  const uint32_t ep = ROLES ? *GPC(uint32_t, E.sync) + 1u : 0u;
  const AS_G int32_t* inj_idx = GPC(int32_t, inj_idx_);
  const AS_G float* inj_eps = GPC(float, inj_eps_);
  lf* Xb = lds + E.o_X;
  lf* Yb = lds + E.o_Y;
  lf* sB = lds + E.o_s;
  lf* s2B = lds + E.o_s2;
  lf* aB = lds + E.o_a;
  lf* a2B = lds + E.o_a2;
  lf* rB = lds + E.o_r;
  lf* dB = lds + E.o_d;
  lf* etB = lds + E.o_et;
  lf* eaB = lds + E.o_ea;
  lf* outB = lds + E.o_out;
  lf* outP = lds + E.o_outp;
  lf* lp2B = lds + E.o_lp;
  lf* qtB = lds + E.o_qt;
  lf* yB = lds + E.o_y;
  lf* gqB = lds + E.o_gout;
  AS_L int64_t* slotB = (AS_L int64_t*)(lds + E.o_slot);
  const AS_C NetDev& pi = E.net[NET_PI];
  Pf<T> pf;  // this role's first GEMM streams in under the sample / gather
  pf_issue<T>(pf, !ROLES || do_pi ? gw_fwd(pi.l[0])
                  : gw_fwd(E.net[role <= 2 ? NET_Q1T + role - 1 : NET_Q1 + role - 3].l[0]));
  // pi(s') (the critical path): layers 0 and 1 held under the sample / gather
  Held<T, 1> ph0;
  Held<T, 8> ph1;
  ph0.tag = ph1.tag = nullptr;
  // late_ph1: layers 0 and 1's fragments are issued after the step counter's
  // and the staged record's loads, so waiting for those (vmcnt retires in issue
  // order) does not also wait for ~72 KB of cold weights (they land under the
  // eps draw and the X build)
  constexpr int MXS = 4;  // staged floats of s / s' per thread, at most
  const bool late_ph1 = ROLES && role == 0 && E.stage && !inj_idx_ &&
                        SAC_ROWS * E.O <= MXS * SAC_THREADS && SAC_ROWS * E.A <= SAC_THREADS;
  if (ROLES && role == 0 && !late_ph1) {
    held_issue<T, 1>(ph0, gw_fwd(pi.l[0]));
    held_issue<T, 8>(ph1, gw_fwd(pi.l[1]));
  }
  AS_G float* stats = GP(float, E.stats);

  // optimizer step counters and this step's Adam bias-correction scalars
  // (torch adam.py: step_size = lr / (1 - beta1^t), bias_correction2_sqrt), once per step
  // ---- sample (replay_buffer.py:32-39) + gather (agent.py:166-193); every role
  // draws the same indices from (seed, step), so no role waits for another's gather
  const uint64_t step = *GPC(uint64_t, E.rng_step);
  const int par = (int)(step & 1);  // step parity: selects the double-buffered per-step state
  if ((!ROLES || role == 0) && rbi == 0 && tid < 4 && (tid < 3 || (E.auto_entropy && E.alpha_update))) {
    const double t = GP(double, E.opt_steps)[tid] + 1.0;
    GP(double, E.opt_steps)[tid] = t;
    if (tid < 3) {
      const double lr = tid == 0 ? E.actor_lr : E.critic_lr;
      GP(float, E.adam_sc)[par * 6 + tid * 2] = (float)(-(lr / (1.0 - pow((double)E.beta1, t))));
      GP(float, E.adam_sc)[par * 6 + tid * 2 + 1] = (float)sqrt(1.0 - pow((double)E.beta2, t));
    } else {
      GP(double, E.alpha_sc)[par * 2] = 1.0 - pow((double)E.beta1, t);
      GP(double, E.alpha_sc)[par * 2 + 1] = 1.0 - pow((double)E.beta2, t);
    }
  }

  const int64_t rb_size = GPC(int64_t, rb.state)[0], rb_pos = GPC(int64_t, rb.state)[1];
  bool staged = false;
  if (E.stage && !inj_idx) {  // the record phase C staged for this step: copied speculatively,
    // its loads in flight together with the step / replay-state loads above
    const AS_G float* rec = GPC(float, E.stg) + stage_rec(E, step, rbi);
    const AS_C uint64_t* hdr = (const AS_C uint64_t*)rec;
    const AS_G float* p = rec + 16;
    if (late_ph1) {  // uniform: the record's loads, then layer 1's fragments, then the record's stores
      float vs[MXS], vs2[MXS], va = 0.f, vr = 0.f, vd = 0.f;
#pragma unroll
      for (int u = 0; u < MXS; ++u) {
        const int i = tid + u * SAC_THREADS;
        vs[u] = vs2[u] = 0.f;
        if (i < R * O) {
          vs[u] = p[i];
          vs2[u] = p[R * O + i];
        }
      }
      if (tid < R * A) va = p[2 * R * O + tid];
      if (tid < R) {
        vr = p[2 * R * O + R * A + tid];
        vd = p[2 * R * O + R * A + R + tid];
      }
      __builtin_amdgcn_sched_barrier(0);
      held_issue<T, 1>(ph0, gw_fwd(pi.l[0]));
      held_issue<T, 8>(ph1, gw_fwd(pi.l[1]));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < MXS; ++u) {
        const int i = tid + u * SAC_THREADS;
        if (i < R * O) {
          sB[i] = vs[u];
          s2B[i] = vs2[u];
        }
      }
      if (tid < R * A) aB[tid] = va;
      if (tid < R) {
        rB[tid] = vr;
        dB[tid] = vd;
      }
    } else {
      for (int i = tid; i < R * O; i += SAC_THREADS) {
        sB[i] = p[i];
        s2B[i] = p[R * O + i];
      }
      for (int i = tid; i < R * A; i += SAC_THREADS) aB[i] = p[2 * R * O + i];
      if (tid < R) {
        rB[tid] = p[2 * R * O + R * A + tid];
        dB[tid] = p[2 * R * O + R * A + R + tid];
      }
    }
    staged = hdr[0] == step && hdr[1] == (uint64_t)rb_size && hdr[2] == (uint64_t)rb_pos &&
             hdr[3] == (uint64_t)(uintptr_t)rb.obs && hdr[4] == (uint64_t)GPC(int64_t, rb.state)[2];
  }
  if (staged && rbi == 0 && (!ROLES || role == 0) && tid == 0)
    *(AS_G uint64_t*)(GP(uint32_t, E.sync) + 4) = step;  // SYNC_STAGED: the staged path ran (tests)
  if (!staged) {  // uniform
    tile_slots(E, rb, step, rb_size, rb_pos, r0, inj_idx, slotB);
    __syncthreads();
    gather_rows<lf*>(rb, slotB, O, A, sB, s2B, aB, rB, dB);
  }
  if (do_pi) {  // which = 0: target draw (role 0), 1: actor draw (role 5)
    const int NP = (A + 1) / 2;
    const int w_lo = ROLES ? (role == 5) : 0, w_n = ROLES ? 1 : 2;
    for (int i = tid; i < w_n * R * NP; i += SAC_THREADS) {
      const int which = w_lo + i / (R * NP), rem = i % (R * NP), r = rem / NP, p = rem % NP;
      const int b = r0 + r;
      float n0 = 0.f, n1 = 0.f;
      if (b < B) {
        if (inj_eps) {
          n0 = inj_eps[((size_t)which * B + b) * A + 2 * p];
          if (2 * p + 1 < A) n1 = inj_eps[((size_t)which * B + b) * A + 2 * p + 1];
        } else {
          philox_normal2(E.seed, step, (uint32_t)b, (uint32_t)which, (uint32_t)p, n0, n1);
        }
      }
      lf* dst = which ? eaB : etB;
      dst[r * A + 2 * p] = n0;
      if (2 * p + 1 < A) dst[r * A + 2 * p + 1] = n1;
    }
  }
  __syncthreads();
  STAMP(1);

  // ---- pi forward: fused, one pass over [s' ; s] (2R rows: target sample, then
  // actor sample); role split, role 0 runs the s' rows (on the critical path) and
  // role 5 the s rows (stashed for phase C).
  auto pi_forward_head = [&](auto rows_c, bool tgt, bool act) {
    constexpr int ROWS = decltype(rows_c)::value;
    const int a0 = tgt ? (act ? R : ROWS) : 0;  // first actor row
    if (act)
      for (int i = tid; i < R * O; i += SAC_THREADS) GP(float, E.s_st)[(size_t)r0 * O + i] = sB[i];
    const int Kp0 = pi.l[0].Kp;
    for (int i = tid; i < ROWS * Kp0; i += SAC_THREADS) {
      const int r = i / Kp0, k = i % Kp0;
      Xb[r * ld + k] = k < O ? (r < a0 ? s2B[r * O + k] : sB[(r - a0) * O + k]) : 0.f;
    }
    __syncthreads();
    STAMP(56);
    lf* X = Xb;
    lf* Y = Yb;
    for (int l = 0; l < pi.L; ++l) {
      const AS_C LayerDev& Ly = pi.l[l];
      if (act)  // actor rows' input, into this step's parity copy
        store_T<T, R>(X + a0 * ld, ld, Ly.Kp, Ly.K, (T*)Ly.XT + par * Ly.xt_par, Bp, r0, nvalid, nullptr);
      if (l == 0) STAMP(57);
      float* stash = act ? Ly.pstash + (size_t)r0 * Ly.Np : nullptr;
      const bool out = l == pi.L - 1;
      const int act_l = out ? pi.out_act : pi.hid_act;
      lf* Pl = out ? outP : nullptr;
      lf* Yl = out ? outB : Y;
      const int ldl = out ? ldo : ld;
      const GemmW nx = out ? gw_fwd(E.net[NET_Q1T].l[0]) : gw_fwd(pi.l[l + 1]);
      // held fragments exist only under the role split (ROWS = R); the fused
      // [s'; s] pass (ROWS = 2R) streams every layer.  (With the held variants
      // instantiated here -- their tags null, the held branch never taken -- the
      // bf16 build returned wrong accumulator elements 0-1 of the second row
      // tile, the actor rows, whenever a layer took the streamed path: hidden
      // widths other than 256.  Found by tests/test_gpu_parity.py::
      // test_bf16_one_step_from_the_engine_state; profiles/r06_bf16_rows_fault.txt.)
      if constexpr (ROLES) {
        if (l == 0)
          layer_fwd<T, ROWS, 1>(X, ld, Ly, pi.P + Ly.b_off, act_l, Pl, ldl, Yl, ldl, stash, a0, pf, nx, &ph0);
        else if (l == 1)
          layer_fwd<T, ROWS, 8>(X, ld, Ly, pi.P + Ly.b_off, act_l, Pl, ldl, Yl, ldl, stash, a0, pf, nx, &ph1);
        else
          layer_fwd<T, ROWS>(X, ld, Ly, pi.P + Ly.b_off, act_l, Pl, ldl, Yl, ldl, stash, a0, pf, nx);
      } else {
        layer_fwd<T, ROWS>(X, ld, Ly, pi.P + Ly.b_off, act_l, Pl, ldl, Yl, ldl, stash, a0, pf, nx);
      }
      __syncthreads();
      STAMP(2 + l);
      lf* t = X;
      X = Y;
      Y = t;
    }
    // squashed-Gaussian head (models.py:79-87): one lane per (row, action dim),
    // each row's A lanes contiguous inside one wave (AP = pow2 >= A), summed by shuffles
    const int AP = A <= 1 ? 1 : 1 << (32 - __builtin_clz(A - 1));
    const int rows_per_pass = SAC_THREADS / AP;
    for (int base = 0; base < ROWS; base += rows_per_pass) {
      const int r = base + tid / AP, j = tid % AP;
      const bool live = r < ROWS && j < A;
      const bool actor = r >= a0;
      const int rr = actor ? r - a0 : r;
      const int b = r0 + rr;
      float lp = 0.f, corr = 0.f;
      if (live) {
        const lf* o = outB + r * ldo;
        const float mu = o[j], lsr = o[A + j], e = (actor ? eaB : etB)[rr * A + j];
        const float lo = E.ls_min, hi = E.ls_max;
        const float ls = lsr < lo ? lo : (lsr > hi ? hi : lsr);
        const float sd = expf(ls);
        const float z = mu + e * sd;
        const float act_v = tanhf(z) * E.scale;
        const float diff = z - mu;
        const float var = sd * sd;
        lp = -(diff * diff) / (2.f * var) - logf(sd) - HALF_LOG_2PI;
        corr = 2.f * ((LOG2F - z) - softplus20(-2.f * z));
        if (actor) {
          AS_G float* h = GP(float, E.head_st) + (size_t)b * 4 * A;
          h[j] = mu;
          h[A + j] = lsr;
          h[2 * A + j] = z;
          h[3 * A + j] = e;
          GP(float, E.a_st)[(size_t)b * A + j] = act_v;
        } else {
          a2B[rr * A + j] = act_v;
          if (ROLES) gran_put(gran_at(E, G_PI, rbi) + rr * A + j, act_v, ep);
        }
      }
      for (int o = 1; o < AP; o <<= 1) {
        lp += __shfl_xor(lp, o, 64);
        corr += __shfl_xor(corr, o, 64);
      }
      if (live && j == 0) {
        const float v = lp - corr;
        if (actor) {
          GP(float, E.lp_st)[par * E.Br + b] = v;
          if (b < B) stats[4 + B + b] = v;
        } else {
          lp2B[rr] = v;
          if (ROLES) gran_put(gran_at(E, G_PI, rbi) + R * A + rr, v, ep);
        }
      }
    }
    __syncthreads();
    STAMP(6);
  };
  if (!ROLES) {
    pi_forward_head(std::integral_constant<int, 2 * R>(), true, true);
  } else if (role == 0 || role == 5) {
    STAMP(59);
    pi_forward_head(std::integral_constant<int, R>(), role == 0, role == 5);
  }

  // ---- target twin-Q (agent.py:195-211)
  const float alpha32 = (float)*GPC(double, E.alpha_state + 1);
  if (!ROLES || role == 1 || role == 2) {
    // role split: the target critic's layers 0 and 1 held while a~' is computed
    Held<T, 1> qh0;
    Held<T, 8> qh1;
    if (ROLES) {
      held_issue<T, 1>(qh0, gw_fwd(E.net[NET_Q1T + role - 1].l[0]));
      held_issue<T, 8>(qh1, gw_fwd(E.net[NET_Q1T + role - 1].l[1]));
      const AS_G uint64_t* h = gran_at(E, G_PI, rbi);  // a~' and log pi' from pi(s')
      for (int i = tid; i < R * A; i += SAC_THREADS) a2B[i] = gran_get(E, h + i, ep);
      if (role == 1 && tid < R) gran_put(gran_at(E, G_LP, rbi) + tid, gran_get(E, h + R * A + tid, ep), ep);
      __syncthreads();
    }
    for (int t = ROLES ? role - 1 : 0; t < (ROLES ? role : 2); ++t) {
      const AS_C NetDev& q = E.net[NET_Q1T + t];
      const int Kp0 = q.l[0].Kp;
      for (int i = tid; i < R * Kp0; i += SAC_THREADS) {
        const int r = i / Kp0, k = i % Kp0;
        Xb[r * ld + k] = k < O ? s2B[r * O + k] : (k < O + A ? a2B[r * A + (k - O)] : 0.f);
      }
      __syncthreads();
      mlp_forward<T, R, ROLES>(q, Xb, Yb, ld, outP, outB, ldo, E.o_P1, E.ldp1, lds, false, false, Bp, r0,
                                      nvalid, pf, gw_fwd(E.net[t ? NET_Q1 : NET_Q2T].l[0]), &qh0, &qh1);
      if (tid < R) {
        qtB[t * R + tid] = outB[tid * ldo];
        if (ROLES) gran_put(gran_at(E, t ? G_Q2T : G_Q1T, rbi) + tid, outB[tid * ldo], ep);
      }
      __syncthreads();
      STAMP(7 + t);
    }
    STAMP(9);
  }
  if (!ROLES) {
    if (tid < R) {
      const int b = r0 + tid;
      const float mq = fmin_nan(qtB[tid], qtB[R + tid]);
      const float y = rB[tid] + (E.gamma * (1.f - dB[tid])) * (mq - alpha32 * lp2B[tid]);
      yB[tid] = y;
      if (b < B) stats[4 + b] = y;
    }
    __syncthreads();
  }

  // ---- critics: forward, MSE, backward (agent.py:213-236)
  if (!ROLES || role == 3 || role == 4) {
    for (int qi = ROLES ? role - 3 : 0; qi < (ROLES ? role - 2 : 2); ++qi) {
      const AS_C NetDev& q = E.net[NET_Q1 + qi];
      const int Kp0 = q.l[0].Kp;
      for (int i = tid; i < R * Kp0; i += SAC_THREADS) {
        const int r = i / Kp0, k = i % Kp0;
        Xb[r * ld + k] = k < O ? sB[r * O + k] : (k < O + A ? aB[r * A + (k - O)] : 0.f);
      }
      __syncthreads();
      // the layer-0 input (s, a) is shared by Q1 and Q2: its X^T is stored once
      if (qi == 0) store_T<T, R>(Xb, ld, Kp0, q.l[0].K, q.l[0].XT, Bp, r0, nvalid, nullptr);
      lf* X = Xb;
      lf* Y = Yb;
      for (int l = 0; l < q.L; ++l) {
        const AS_C LayerDev& Ly = q.l[l];
        if (l > 0) store_T<T, R>(X, ld, Ly.Kp, Ly.K, Ly.XT, Bp, r0, nvalid, nullptr);
        if (l == q.L - 1)
          layer_fwd<T, R>(X, ld, Ly, q.P + Ly.b_off, q.out_act, outP, ldo, outB, ldo, nullptr, 0, pf, gw_bwd(Ly));
        else
          layer_fwd<T, R>(X, ld, Ly, q.P + Ly.b_off, q.hid_act, lds + E.o_P1[l], E.ldp1[l], Y, ld, nullptr, 0, pf,
                          gw_fwd(q.l[l + 1]));
        __syncthreads();
        lf* t = X;
        X = Y;
        Y = t;
      }
      STAMP(10 + 2 * qi);
      // Backward with a UNIT seed per row first: every layer's dY is linear in
      // the row's seed 2(q - y)/B, so U_l = dY_l / seed does not need y and runs
      // while the target critics finish (role split); U_l stays in LDS (the Q2
      // pre-activation buffers, unused here) and is scaled once y is known.
      if (tid < R) {
        float u = tid < nvalid ? 1.f : 0.f;
        if (q.out_act != ACT_ID) u = act_bwd(q.out_act, outP[tid * ldo], u);
        for (int n = 0; n < 32; ++n) gqB[tid * ldo + n] = n == 0 ? u : 0.f;
      }
      __syncthreads();
      critic_unit_backward<T, R>(E, q, gqB, ldo, lds, pf);
      STAMP(16);
      // y needs both target critics and log pi' (granules: each lane polls its row's three)
      STAMP(14);
      if (tid < 64) {  // wave 0: y, loss partial, seed dL/dq (mse_loss backward: 2(q-y)/B)
        float sq = 0.f;
        if (tid < R) {
          const int b = r0 + tid;
          const bool v = tid < nvalid;
          float y;
          if (ROLES) {
            const float q1t = gran_get(E, gran_at(E, G_Q1T, rbi) + tid, ep);
            const float q2t = gran_get(E, gran_at(E, G_Q2T, rbi) + tid, ep);
            const float lp2 = gran_get(E, gran_at(E, G_LP, rbi) + tid, ep);
            // alpha, written by the previous launch's phase D (an atomic load: kept from the
            // fused step, where D shared this launch)
            const float al = (float)__hip_atomic_load((double*)E.alpha_state + 1, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
            y = rB[tid] + (E.gamma * (1.f - dB[tid])) * (fmin_nan(q1t, q2t) - al * lp2);
            if (qi == 0 && b < B) stats[4 + b] = y;
          } else {
            y = yB[tid];
          }
          const float d = outB[tid * ldo] - y;
          sq = v ? d * d : 0.f;
          qtB[tid] = v ? (2.0f / (float)B) * d : 0.f;  // the row's seed
        }
        sq = wave_sum(sq);
        if (tid == 0) GP(float, E.lossp)[(par * E.nrt + rbi) * 4 + qi] = sq;
      }
      __syncthreads();
      STAMP(15);
      {  // dY of every layer = seed * U, stored as dY^T + bias partials for phase B
        const AS_C LayerDev& Lo = q.l[q.L - 1];
        store_T<T, R>(gqB, ldo, Lo.Np, Lo.N, Lo.GT, Bp, r0, nvalid, Lo.dbp, qtB);
        for (int l = q.L - 2; l >= 0; --l) {
          const AS_C LayerDev& Ly = q.l[l];
          store_T<T, R>(lds + E.o_P2[l], E.ldp2[l], Ly.Np, Ly.N, Ly.GT, Bp, r0, nvalid, Ly.dbp, qtB);
        }
        __syncthreads();
      }
      STAMP(11 + 2 * qi);
    }
  }
}

template <typename T, bool ROLES>
__global__ void __launch_bounds__(SAC_THREADS) sac_target_critic(const EngineDev* __restrict__ Ep, sac_replay rb,
                                                                  const int32_t* __restrict__ inj_idx_,
                                                                  const float* __restrict__ inj_eps_) {
  target_critic_body<T, ROLES>(Ep, rb, inj_idx_, inj_eps_);
  const AS_C EngineDev& E = *(const AS_C EngineDev*)Ep;
  (void)E;
  END_STAMP(60);
  CLK_STAMP(41);
}

// ============================================================================ phase C
// critics on (s, a~) with the updated weights, d a~, head backward, pi backward.
// ROLES: block = role * nrt + row tile; role 0 pi (head + pi backward), 1/2 critics.
// A critic role back-propagates a UNIT seed (d Q_i / d a~) and hands (q_i,
// dQ_i/da~) to the pi role, which applies the min-Q weights -1/B, -1/2B or 0
// (powers of two for power-of-two batches: bit-identical to seeding them).
template <typename T, bool ROLES>
__device__ __forceinline__ void actor_body(const EngineDev* __restrict__ Ep, int bid) {
  const AS_C EngineDev& E = *(const AS_C EngineDev*)Ep;
  extern __shared__ float lds_raw[];
  lf* lds = (lf*)lds_raw;
  constexpr int R = SAC_ROWS;
  const int tid = threadIdx.x;
  int rbi, role;
  if (ROLES) {
    // producers first: block groups 0 / 1 are the critic roles (1 / 2), group
    // 2 the pi role (0) that consumes their granules.  In-order dispatch then
    // guarantees that a spinning consumer's producers already hold a CU.
    rbi = bid % E.nrt;
    const int grp = bid / E.nrt;
    role = grp == 2 ? 0 : grp + 1;
  } else {
    if (bid % E.xs) return;  // XCD placement: see EngineDev::xs
    rbi = bid / E.xs;
    role = -1;
  }
  const bool do_pi = !ROLES || role == 0;
  STAMP(32);
  const int B = E.B, Bp = E.Bp, O = E.O, A = E.A, ld = E.ld, ldo = E.ldo;
  const int r0 = rbi * R;
  const int nvalid = min(R, B - r0);
  const uint32_t ep = ROLES ? *GPC(uint32_t, E.sync) + 1u : 0u;
  const int par = (int)(*GPC(uint64_t, E.rng_step) & 1);  // advanced by the last block of this phase
  lf* Xb = lds + E.o_X;
  lf* Yb = lds + E.o_Y;
  lf* sB = lds + E.o_s;
  lf* aB = lds + E.o_a;
  lf* lpB = lds + E.o_lp;
  lf* g1B = lds + E.o_g;
  lf* g2B = lds + E.o_g2;
  lf* gaB = lds + E.o_ga;
  lf* goutB = lds + E.o_gout;
  lf* out1 = lds + E.o_out;
  lf* outP1 = lds + E.o_outp;
  lf* out2 = lds + E.o_out2;
  lf* outP2 = lds + E.o_outp2;
  const AS_C NetDev& pi = E.net[NET_PI];
  const float alpha32 = (float)*GPC(double, E.alpha_state + 1);
  Pf<T> pf;  // this role's first GEMM streams in under the loads / the wait
  pf_issue<T>(pf, !ROLES ? gw_fwd(E.net[NET_Q1].l[0])
                  : role == 0 ? gw_bwd(pi.l[pi.L - 1]) : gw_fwd(E.net[NET_Q1 + role - 1].l[0]));

  if (!ROLES || role >= 1) {
    for (int i = tid; i < R * O; i += SAC_THREADS) sB[i] = GPC(float, E.s_st)[(size_t)r0 * O + i];
    for (int i = tid; i < R * A; i += SAC_THREADS) aB[i] = GPC(float, E.a_st)[(size_t)r0 * A + i];
  }
  if (do_pi) {
    for (int i = tid; i < R * A; i += SAC_THREADS) gaB[i] = 0.f;
    if (tid < R) lpB[tid] = GPC(float, E.lp_st)[par * E.Br + r0 + tid];
  }
  __syncthreads();

  if (!ROLES || role >= 1) {
    const int q_lo = ROLES ? role - 1 : 0, q_hi = ROLES ? role : 2;
    Held<T, 1> ch0;
    Held<T, 8> ch1;
    if (ROLES) {  // one critic per role: its layers 0 and 1 held under the input loads
      held_issue<T, 1, false>(ch0, gw_fwd(E.net[NET_Q1 + q_lo].l[0]));
      held_issue<T, 8, false>(ch1, gw_fwd(E.net[NET_Q1 + q_lo].l[1]));
    }
    STAMP(33);
    // ---- Q1, Q2 on (s, a~) with the updated critics (agent.py:244-248)
    for (int qi = q_lo; qi < q_hi; ++qi) {
      const AS_C NetDev& q = E.net[NET_Q1 + qi];
      const int Kp0 = q.l[0].Kp;
      for (int i = tid; i < R * Kp0; i += SAC_THREADS) {
        const int r = i / Kp0, k = i % Kp0;
        Xb[r * ld + k] = k < O ? sB[r * O + k] : (k < O + A ? aB[r * A + (k - O)] : 0.f);
      }
      __syncthreads();
      mlp_forward<T, R, ROLES>(q, Xb, Yb, ld, qi ? outP2 : outP1, qi ? out2 : out1, ldo,
                                       qi ? E.o_P2 : E.o_P1, qi ? E.ldp2 : E.ldp1, lds, true, false, Bp, r0, nvalid, pf,
                                       ROLES ? gw_bwd(q.l[q.L - 1])
                                       : qi ? gw_bwd(E.net[NET_Q1].l[E.net[NET_Q1].L - 1]) : gw_fwd(E.net[NET_Q2].l[0]),
                                       &ch0, &ch1);
      STAMP(36 + qi);
    }
    // ---- backward seeds.  L_pi = mean(alpha logpi - min Q) (agent.py:251-252); min
    // backward splits ties.  ROLES: unit seeds, the pi role applies the weights.
    if (tid < 64) {
      float term = 0.f;
      if (tid < R) {
        const bool v = tid < nvalid;
        float g1, g2;
        if (ROLES) {
          g1 = g2 = v ? 1.0f : 0.f;
        } else {
          const float q1 = out1[tid * ldo], q2 = out2[tid * ldo];
          const float m = fmin_nan(q1, q2);
          term = v ? alpha32 * lpB[tid] - m : 0.f;
          const float gm = v ? -1.0f / (float)B : 0.f;
          g1 = (q1 == q2) ? gm * 0.5f : (q1 > q2 ? 0.f : gm);
          g2 = (q1 == q2) ? gm * 0.5f : (q1 < q2 ? 0.f : gm);
        }
        if (E.net[NET_Q1].out_act != ACT_ID) {
          if (q_lo == 0) g1 = act_bwd(E.net[NET_Q1].out_act, outP1[tid * ldo], g1);
          if (q_hi == 2) g2 = act_bwd(E.net[NET_Q2].out_act, outP2[tid * ldo], g2);
        }
        for (int n = 0; n < 32; ++n) {
          g1B[tid * ldo + n] = n == 0 ? g1 : 0.f;
          g2B[tid * ldo + n] = n == 0 ? g2 : 0.f;
        }
      }
      if (!ROLES) {
        term = wave_sum(term);
        if (tid == 0) GP(float, E.lossp)[(par * E.nrt + rbi) * 4 + 2] = term;
      }
    }
    __syncthreads();

    // ---- d a~ through the critics: dX of layer 0, action columns
    for (int qi = q_lo; qi < q_hi; ++qi) {
      const AS_C NetDev& q = E.net[NET_Q1 + qi];
      lf* G0 = mlp_backward<T, R>(q, qi ? g2B : g1B, ldo, Xb, Yb, ld, qi ? E.o_P2 : E.o_P1, qi ? E.ldp2 : E.ldp1,
                                  lds, false, Bp, r0, nvalid, pf, gw_bwd(q.l[0]));
      lf* Gx = (G0 == Xb) ? Yb : Xb;
      layer_bwd<T, R>(G0, ld, q.l[0], nullptr, 0, -1, Gx, ld, pf,
                      qi ? gw_bwd(pi.l[pi.L - 1]) : gw_bwd(E.net[NET_Q2].l[E.net[NET_Q2].L - 1]));
      __syncthreads();
      if (ROLES) {
        AS_G uint64_t* g = gran_at(E, G_C1 + qi, rbi);
        for (int i = tid; i < R * A; i += SAC_THREADS) gran_put(g + i, Gx[(i / A) * ld + O + i % A], ep);
        if (tid < R) gran_put(g + R * A + tid, (qi ? out2 : out1)[tid * ldo], ep);
        __syncthreads();  // Gx is reused by the next critic's backward
      } else {
        for (int i = tid; i < R * A; i += SAC_THREADS) gaB[i] += Gx[(i / A) * ld + O + i % A];
        __syncthreads();
      }
      STAMP(38 + qi);
    }
  }
  if (!do_pi) return;

  // ---- squashed-Gaussian head backward + pi backward (agent.py:255-257)
  for (int l = 0; l < pi.L - 1; ++l) {
    const AS_C LayerDev& Ly = pi.l[l];
    const int ldp = E.ldp1[l];
    lf* P = lds + E.o_P1[l];
    const AS_G float* ps = GPC(float, Ly.pstash) + (size_t)r0 * Ly.Np;
    for (int i = tid; i < R * Ly.Np; i += SAC_THREADS) P[(i / Ly.Np) * ldp + i % Ly.Np] = ps[i];
  }
  // pi's last two dX steps held while the critics run (pi is not written in this launch)
  Held<T, 1> bh0;
  Held<T, 8> bh1;
  bh0.tag = bh1.tag = nullptr;
  if (ROLES) {
    held_issue<T, 1>(bh0, gw_bwd(pi.l[pi.L - 1]));
    held_issue<T, 8>(bh1, gw_bwd(pi.l[pi.L - 2]));
  }
  if (ROLES) {  // combine the critics' unit-seed gradients with the min-Q weights
    const AS_G uint64_t* h1 = gran_at(E, G_C1, rbi);
    const AS_G uint64_t* h2 = gran_at(E, G_C2, rbi);
    if (tid < 64) {
      float term = 0.f;
      if (tid < R) {
        const bool v = tid < nvalid;
        const float q1 = gran_get(E, h1 + R * A + tid, ep), q2 = gran_get(E, h2 + R * A + tid, ep);
        const float m = fmin_nan(q1, q2);
        term = v ? alpha32 * lpB[tid] - m : 0.f;
        const float gm = v ? -1.0f / (float)B : 0.f;
        g1B[tid] = (q1 == q2) ? gm * 0.5f : (q1 > q2 ? 0.f : gm);
        g2B[tid] = (q1 == q2) ? gm * 0.5f : (q1 < q2 ? 0.f : gm);
      }
      term = wave_sum(term);
      if (tid == 0) GP(float, E.lossp)[(par * E.nrt + rbi) * 4 + 2] = term;
    }
    __syncthreads();
    for (int i = tid; i < R * A; i += SAC_THREADS) {
      const int r = i / A;
      gaB[i] = (gaB[i] + g1B[r] * gran_get(E, h1 + i, ep)) + g2B[r] * gran_get(E, h2 + i, ep);
    }
    __syncthreads();
    STAMP(39);
  }
  for (int i = tid; i < R * A; i += SAC_THREADS) {  // one lane per (row, action dim)
    const int r = i / A, j = i % A, b = r0 + r;
    const bool v = r < nvalid;
    const float gl = v ? alpha32 * (1.0f / (float)B) : 0.f;
    const AS_G float* h = GPC(float, E.head_st) + (size_t)b * 4 * A;
    const float lo = E.ls_min, hi = E.ls_max, scale = E.scale;
    const float mu = h[j], lsr = h[A + j], z = h[2 * A + j], e = h[3 * A + j];
    const float ls = lsr < lo ? lo : (lsr > hi ? hi : lsr);
    const float sd = expf(ls);
    const float t = tanhf(z);
    const float diff = z - mu, var = sd * sd;
    float g_z = (gaB[r * A + j] * scale) * (1.f - t * t);
    g_z = g_z + (-gl) * 2.f * (-1.f + 2.f * softplus20_grad(-2.f * z));
    const float two_var = 2.f * var;
    const float g_sq = -gl / two_var;
    const float g_twovar = gl * (diff * diff) / (two_var * two_var);
    const float g_var = 2.f * g_twovar;
    float g_std = 2.f * sd * g_var - gl / sd;
    const float g_diff = 2.f * diff * g_sq;
    g_z = g_z + g_diff;
    const float g_mu = -g_diff + g_z;
    g_std = g_std + g_z * e;
    const float g_ls = g_std * sd;
    const bool in_range = (lsr >= lo) && (lsr <= hi);
    float gm = v ? g_mu : 0.f, gs = (v && in_range) ? g_ls : 0.f;
    if (pi.out_act != ACT_ID) {
      const AS_C LayerDev& Lo = pi.l[pi.L - 1];
      const AS_G float* ps = GPC(float, Lo.pstash) + (size_t)b * Lo.Np;
      gm = act_bwd(pi.out_act, ps[j], gm);
      gs = act_bwd(pi.out_act, ps[A + j], gs);
    }
    goutB[r * ldo + j] = gm;
    goutB[r * ldo + A + j] = gs;
  }
  {
    const int NOp = 32 * ((2 * A + 31) / 32), pad = NOp - 2 * A;
    for (int i = tid; i < R * pad; i += SAC_THREADS) goutB[(i / pad) * ldo + 2 * A + i % pad] = 0.f;
  }
  __syncthreads();
  // held fragments only under the role split (bh0 / bh1 are issued only there)
  mlp_backward<T, R, ROLES>(pi, goutB, ldo, Xb, Yb, ld, E.o_P1, E.ldp1, lds, true, Bp, r0, nvalid, pf, gw_none(),
                                   &bh0, &bh1);
  STAMP(35);
}

// The last block of phase C to finish advances the step: RNG step, hand-off
// epoch, and resets the completion counters (every reader of those words ran
// earlier in this launch or runs in a later one).
__device__ __forceinline__ void phase_c_done(const AS_C EngineDev& E) {
  if (threadIdx.x != 0) return;
  uint32_t* sync = (uint32_t*)E.sync;
  const uint32_t old = __hip_atomic_fetch_add(sync + SYNC_CDONE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old == gridDim.x - 1) {
    *GP(uint64_t, E.rng_step) += 1;
    sync[SYNC_EPOCH] += 1u;
    sync[SYNC_CDONE] = 0u;
  }
}

// After the role blocks: E.stage ? nrt stager blocks (next step's batch).
template <typename T, bool ROLES>
__global__ void __launch_bounds__(SAC_THREADS) sac_actor(const EngineDev* __restrict__ Ep, sac_replay rb) {
  PREFETCH_ARG(Ep);
  const AS_C EngineDev& E = *(const AS_C EngineDev*)Ep;
  extern __shared__ float lds_raw[];
  const int bid = (int)blockIdx.x;
  const int nrole = ROLES ? 3 * E.nrt : E.nrt * E.xs;
  if (bid >= nrole) {
    stage_next_batch(E, rb, bid - nrole, (lf*)lds_raw, *GPC(uint64_t, E.rng_step));
  } else {
    actor_body<T, ROLES>(Ep, bid);
  }
  phase_c_done(E);
  END_STAMP(61);
}

// ============================================================================ phases B / D kernels
// UT = 512 (SAC_UPD_UT=512): one slot per round and at most 128 VGPRs, so two
// workgroups share a CU (SAC_UPD_LDS_FOR(1) = 45 KB each)
template <typename T, int UT = SAC_UPD_THREADS>
__global__ void __launch_bounds__(UT, UT == 512 ? 4 : 1) sac_critic_update(const EngineDev* __restrict__ Ep,
                                                         const TileDesc* __restrict__ tiles) {
  const AS_C EngineDev& E = *(const AS_C EngineDev*)Ep;
  extern __shared__ float upd_lds[];
  // critic tiles: one X^T copy (xt_par = 0), so their operand loads need not wait for the step's parity
  dw_adam_tile_any<T, UT, UT == 512 ? 1 : 2>(E, tiles + blockIdx.x, true,
                                                          (int)(*GPC(uint64_t, E.rng_step) & 1), 0, (lf*)upd_lds);
  END_STAMP(62);  // standalone: the launch boundary publishes (no counter)
}

template <typename T>
__global__ void __launch_bounds__(SAC_UPD_THREADS) sac_actor_update(const EngineDev* __restrict__ Ep,
                                                                   const TileDesc* __restrict__ tiles, int ntiles) {
  const AS_C EngineDev& E = *(const AS_C EngineDev*)Ep;
  const int par = (int)((*GPC(uint64_t, E.rng_step) - 1) & 1);  // phase C already advanced the step
  extern __shared__ float upd_lds[];
  if ((int)blockIdx.x < ntiles)
    dw_adam_tile_any<T, SAC_UPD_THREADS>(E, tiles + blockIdx.x, false, par, par, (lf*)upd_lds);
  else
    alpha_and_losses(E, par, (lf*)upd_lds);
  END_STAMP(63);  // standalone: the launch boundary publishes (no counter)
}

// ============================================================================ policy
template <typename T>
__global__ void __launch_bounds__(SAC_THREADS) sac_policy_act_kernel(const EngineDev* __restrict__ Ep, const float* __restrict__ obs_, int n,
                                                             const float* __restrict__ eps_, float* __restrict__ action_,
                                                             float* __restrict__ log_pi_) {
  PREFETCH_ARG(Ep);
  const AS_C EngineDev& E = *(const AS_C EngineDev*)Ep;
  extern __shared__ float lds_raw[];
  lf* lds = (lf*)lds_raw;
  constexpr int R = SAC_ROWS;
  const int tid = threadIdx.x, O = E.O, A = E.A, ld = E.ld, ldo = E.ldo;
  const int r0 = blockIdx.x * R;
  const int nvalid = min(R, n - r0);
  const AS_G float* obs = GPC(float, obs_);
  const AS_G float* eps = GPC(float, eps_);
  AS_G float* action = GP(float, action_);
  AS_G float* log_pi = GP(float, log_pi_);
  lf* Xb = lds + E.o_X;
  lf* Yb = lds + E.o_Y;
  lf* outB = lds + E.o_out;
  lf* outP = lds + E.o_outp;
  const AS_C NetDev& pi = E.net[NET_PI];
  const int Kp0 = pi.l[0].Kp;
  for (int i = tid; i < R * Kp0; i += SAC_THREADS) {
    const int r = i / Kp0, k = i % Kp0;
    Xb[r * ld + k] = (k < O && r < nvalid) ? obs[(size_t)(r0 + r) * O + k] : 0.f;
  }
  __syncthreads();
  Pf<T> pf;
  pf.tag = nullptr;
  mlp_forward<T, R>(pi, Xb, Yb, ld, outP, outB, ldo, E.o_P1, E.ldp1, lds, false, false, 0, 0, 0, pf, gw_none());
  if (tid < nvalid) {
    const int b = r0 + tid;
    const lf* o = outB + tid * ldo;
    const float lo = E.ls_min, hi = E.ls_max, scale = E.scale;
    float lp_sum = 0.f, corr_sum = 0.f;
    for (int j = 0; j < A; ++j) {
      if (!eps) {
        action[(size_t)b * A + j] = tanhf(o[j]) * scale;
        continue;
      }
      const float mu = o[j], lsr = o[A + j], e = eps[(size_t)b * A + j];
      const float ls = lsr < lo ? lo : (lsr > hi ? hi : lsr);
      const float sd = expf(ls);
      const float z = mu + e * sd;
      action[(size_t)b * A + j] = tanhf(z) * scale;
      const float diff = z - mu;
      const float var = sd * sd;
      lp_sum += -(diff * diff) / (2.f * var) - logf(sd) - HALF_LOG_2PI;
      corr_sum += 2.f * ((LOG2F - z) - softplus20(-2.f * z));
    }
    if (eps && log_pi) log_pi[b] = lp_sum - corr_sum;
  }
}
