// sac_split.h — hidden-split role kernels of phases A and C.
//
// For nets with two hidden layers of width H = 256 (the reference's
// BipedalWalker / Donkey configs, C2/C4), every role of the role split
// (sac_phases.h "role hand-offs") runs as TWO workgroups per row tile, one per
// half h of layer 1's H outputs:
//
//   layer 0  (K0 -> H)   computed in full by both halves (K0 is small);
//   layer 1  (H -> H)    half h computes outputs [h H/2, (h+1) H/2): its half of
//                        W1 (128 KB fp32) is register-held, issued at launch
//                        start, so the layer runs at the MFMA rate;
//   layer 2  (H -> out)  half h sums over ITS inputs only: a partial output;
//                        consumers add the two partials (+ bias) themselves.
//
// Backward mirrors it: dY1 of a half is exact (elementwise in the seed for the
// critics), dY0 = dY1_h W1[h] is a PARTIAL over the half's n; the partial is
// masked (relu' is elementwise) and stored as its own batch columns of layer
// 0's dY^T, so phase B/D's dW = sum over 2 Bp columns adds the halves, and
// da (phase C) = the sum of the halves' partial dX0.
//
// No half waits for its peer on the critical path: a consumer reads both
// halves' partial granules.  Bit-identical to the reference up to fp32
// summation order (two partial sums instead of one), checked against the
// oracle in tests/test_gpu_parity.py.
//
// Reference cross-walk: target agent.py:195-211, critic agent.py:213-236,
// actor agent.py:238-260, policy head models.py:73-87.
#pragma once
#include "sac_phases.h"

#define SPLIT_H 256
#define SPLIT_HH 128
// Phase C splits layer 1 into split_wc parts: four in fp32 (3 roles x 4 parts x
// nrt = 192 workgroups at C2: its critical path is three layer-1 GEMMs -- critic
// forward, critic dX, pi dX -- each then a quarter of the MFMA-bound fp32 work
// per workgroup), two in bf16.  Quarters in bf16 ran faster on the round-5 build
// (C2 26.0K -> 26.8K steps/s) but failed the bf16 parity bar: pi's layer-0 dY
// arrives as four bf16-rounded partials instead of two, and the policy's
// per-step parameter drift against the oracle rose from under to above
// 0.05 lr (profiles/r05_ab_bf16_quarters_c.txt).
// Phase A keeps halves (6 roles x 2 x nrt = 192).
__host__ __device__ constexpr int split_wc(int elem_bytes) { return elem_bytes == 4 ? 4 : 2; }
// Phase C's critic roles: quarters in both precisions.  Their parts hand fp32
// granules to pi (no bf16-rounded partial is stored), so bf16 quarters change
// only fp32 summation order: C2 bf16 (profiles/r05_ab_bf16_critic_quarters.txt).
__host__ __device__ constexpr int split_wcq(int elem_bytes) { return (void)elem_bytes, 4; }
// Phase A's pi(s') role -- the head of the y chain -- gets the same parts as
// phase C (fp32: 4; the other five roles keep halves: (4 + 10) x nrt = 224
// workgroups at C2; quarters in bf16 measured 1.5% slower, profiles/r05_ab_misc.txt).
__host__ __device__ constexpr int split_wpi(int elem_bytes) { return split_wc(elem_bytes); }
#define SPLIT_GP 4  // granule part slots per (kind, row tile): max over precisions of split_wc

// Split granule kinds: [GS_COUNT][nrt][SPLIT_GP parts][E.gs2] 8-B granules
enum SplitGran {
  GS_PI = 0,   // pi(s') layer-2 partial [R][2A]              -> target critics
  GS_PS = 1,   // pi(s) layer-2 partial [R][2A]               -> the peer pi(s) half
  GS_QT1 = 2,  // target critic 1 partial q [R]               -> critics
  GS_QT2 = 3,  // target critic 2 partial q [R]               -> critics
  GS_LP = 4,   // log pi(a~'|s') [R] (half 0 only)           -> critics
  GS_QA1 = 5,  // critic 1 partial q [R]                      -> its peer half
  GS_QA2 = 6,  // critic 2 partial q [R]
  GS_C1 = 7,   // phase C critic 1: partial da [R][A], partial q [R] -> pi halves
  GS_C2 = 8,
  GS_COUNT = 9
};
__device__ __forceinline__ AS_G uint64_t* gs_at(const AS_C EngineDev& E, int kind, int rbi, int h) {
  return GP(uint64_t, E.gran2) + ((size_t)(kind * E.nrt + rbi) * SPLIT_GP + h) * E.gs2;
}

// ---------------------------------------------------------------------------- held GEMM
// The fragments of a wave's NTW output tiles (t = wave + j * SAC_NW) over the
// first HC reduction chunks of a packed B view, plus the bias of the lane's
// column in each tile.  Issued early (before waits); consumed by gemm_hs.
template <typename T, int NTW, int HC>
struct HTiles {
  typename MM<T>::Frag f[NTW][HC];
  float b[NTW];
};

template <typename T, int NTW, int HC, bool COH = false>
__device__ __forceinline__ void ht_issue(HTiles<T, NTW, HC>& ht, const GemmW& w) {
  constexpr uint32_t FSB = 64 * MM<T>::KL * sizeof(T);
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int nch = w.cols / MM<T>::KC;
  const __amdgpu_buffer_rsrc_t rs = coh_rsrc(w.p, 0xFFFFFFF0u);
  static_for<NTW>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    int t = wave + j * SAC_NW;
    const bool has = t < w.NT;  // wave-uniform: a wave without this tile loads nothing
    t = has ? t : w.NT - 1;
    const uint32_t o = (uint32_t)(((size_t)t * 16 * w.tcols + lane * MM<T>::KL) * sizeof(T));
    static_for<HC>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      const uint32_t cu = u < nch ? u : nch - 1;
      if (has)
        ht.f[j][u] = coh_frag<T, COH>(rs, o + cu * FSB);
      else
        ht.f[j][u] = typename MM<T>::Frag{};
    });
    if (w.bias) {
      const int n = t * 16 + (lane & 15);
      ht.b[j] = ldf<COH>(w.bias + (n < w.N ? n : w.N - 1));
    }
  });
}

// out tiles of A[16][cols] x B^T over the view's reduction: chunks [0, HC) from
// the held fragments (when ht != null), the rest streamed in batches of 8.
// Two accumulators per tile (even / odd chunk) cover the dependent-MFMA latency.
// epi(j, col, acc, bias) for every valid tile j of the wave.
template <typename T, int NTW, int HC, bool COH = false, typename Epi>
__device__ __forceinline__ void gemm_hs(const lf* __restrict__ A, int lda, const GemmW& w,
                                        const HTiles<T, NTW, HC>* ht, Epi&& epi) {
  typedef typename MM<T>::Frag F;
  constexpr int KC = MM<T>::KC, KL = MM<T>::KL;
  constexpr uint32_t FSB = 64 * KL * sizeof(T);
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int c = lane & 15, g = lane >> 4;
  const int nch = w.cols / KC;
  const lf* arow = A + c * lda + g * KL;
  f32x4 acc[NTW][2];
  static_for<NTW>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    acc[j][0] = acc[j][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  });
  int ch0 = 0;
  if (ht) {  // uniform
    F a[HC];
    static_for<HC>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      a[u] = MM<T>::from_lds(arow + (u < nch ? u : 0) * KC);
    });
    static_for<HC>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      if (u < nch)
        static_for<NTW>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          if (wave + j * SAC_NW < w.NT)  // wave-uniform: no MFMA issue for a wave without this tile
            MM<T>::mma(acc[j][u & 1], a[u], ht->f[j][u]);
        });
    });
    ch0 = HC;
  }
  if (ch0 < nch) {
    const __amdgpu_buffer_rsrc_t rs = coh_rsrc(w.p, 0xFFFFFFF0u);
    uint32_t o[NTW];
    static_for<NTW>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      int t = wave + j * SAC_NW;
      t = t < w.NT ? t : w.NT - 1;
      o[j] = (uint32_t)(((size_t)t * 16 * w.tcols + lane * KL) * sizeof(T));
    });
    for (int cb = ch0; cb < nch; cb += 8) {
      const int rem = nch - cb < 8 ? nch - cb : 8;
      F f[NTW][8], a[8];
      static_for<8>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        const uint32_t cu = cb + (u < rem ? u : rem - 1);
        static_for<NTW>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          f[j][u] = coh_frag<T, COH>(rs, o[j] + cu * FSB);
        });
      });
      static_for<8>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        a[u] = MM<T>::from_lds(arow + (cb + (u < rem ? u : rem - 1)) * KC);
      });
      static_for<8>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        if (u < rem)
          static_for<NTW>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            if (wave + j * SAC_NW < w.NT) MM<T>::mma(acc[j][u & 1], a[u], f[j][u]);
          });
      });
    }
  }
  static_for<NTW>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const int t = wave + j * SAC_NW;
    if (t < w.NT) epi(j, t * 16 + c, acc[j][0] + acc[j][1]);
  });
}

// ---------------------------------------------------------------------------- k-split GEMM
// Small-N steps (NT <= 2 output tiles, long reduction): the reduction is
// split over the waves (SAC_NW / NT waves per tile, consecutive chunk slices),
// partial tiles summed through LDS in slice order.  out[r][col] for col < 16 NT.
// A wave's slice of a k-split step held in registers: a step that follows a
// hand-off (the target critics' and pi(s')'s layer 2) issues its fragment
// before the poll instead of one more memory round trip after it.  Held when
// the slice is at most SAC_KS_MAXC32 chunks in fp32 / one chunk in bf16 (a
// 128-deep reduction over 8 waves).  Same-box A/Bs at C2
// (profiles/r02_ab_*.txt): bf16 +2.7% steps/s; fp32 phase A with 2- or 4-chunk
// slices held (issued under layer 1 / before the poll): no change, so fp32
// streams (MAXC32 = 1).  Phase C critics' two k-split steps held (SAC_KS_C):
// with both issued at launch start the fp32 kernel spilled 28 VGPRs (C 18.4 ->
// 19.8 us); with W0^T's 8 fp32 chunks issued once layer 1's held part is dead,
// no spill and C 18.6 -> 18.1 us, +0.8% steps/s fp32, +1.3% bf16.
#ifndef SAC_KS_HELD
#define SAC_KS_HELD 1
#endif
#ifndef SAC_KS_MAXC32
#define SAC_KS_MAXC32 1
#endif
#ifndef SAC_KS_C
#define SAC_KS_C 1
#endif
template <typename T, int MC = (sizeof(T) == 4 ? SAC_KS_MAXC32 : 1)>
struct KsHeld {
  static constexpr int MAXC = MC;
  typename MM<T>::Frag f[MAXC];
  bool ok;
};
template <typename T>
__device__ __forceinline__ void ks_slice(const GemmW& w, int& t, int& c0, int& c1, int& wpt) {
  const int wave = wave_id();
  const int NT = w.NT;  // 1 or 2
  wpt = SAC_NW / NT;
  t = wave % NT;
  const int sl = wave / NT;
  const int nch = w.cols / MM<T>::KC;
  const int per = (nch + wpt - 1) / wpt;
  c0 = sl * per;
  c1 = c0 + per < nch ? c0 + per : nch;
}
template <typename T, int MC, bool COH = false>
__device__ __forceinline__ void ks_issue(KsHeld<T, MC>& kh, const GemmW& w) {
  constexpr uint32_t FSB = 64 * MM<T>::KL * sizeof(T);
  int t, c0, c1, wpt;
  ks_slice<T>(w, t, c0, c1, wpt);
  const int nch = w.cols / MM<T>::KC, per = (nch + wpt - 1) / wpt;
  kh.ok = SAC_KS_HELD && per <= MC;  // uniform
  if (!kh.ok) return;
  const __amdgpu_buffer_rsrc_t rs = coh_rsrc(w.p, 0xFFFFFFF0u);
  const uint32_t o = (uint32_t)(((size_t)t * 16 * w.tcols + (threadIdx.x & 63) * MM<T>::KL) * sizeof(T));
  static_for<MC>([&](auto uc) {
    constexpr int u = decltype(uc)::value;
    if (c0 + u < c1) kh.f[u] = coh_frag<T, COH>(rs, o + (c0 + u) * FSB);
  });
}

template <typename T, bool COH = false, int MC = 1>
__device__ __forceinline__ void gemm_ksplit(const lf* __restrict__ A, int lda, const GemmW& w, lf* red, lf* out,
                                            int ldo, const KsHeld<T, MC>* kh = nullptr) {
  typedef typename MM<T>::Frag F;
  constexpr int KC = MM<T>::KC, KL = MM<T>::KL;
  constexpr uint32_t FSB = 64 * KL * sizeof(T);
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int c = lane & 15, g = lane >> 4;
  const int NT = w.NT;  // 1 or 2
  int t, c0, c1, wpt;
  ks_slice<T>(w, t, c0, c1, wpt);
  const __amdgpu_buffer_rsrc_t rs = coh_rsrc(w.p, 0xFFFFFFF0u);
  const uint32_t o = (uint32_t)(((size_t)t * 16 * w.tcols + lane * KL) * sizeof(T));
  const lf* arow = A + c * lda + g * KL;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (kh && kh->ok) {  // uniform: the slice's fragments are already in registers
    static_for<MC>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      if (c0 + u < c1) MM<T>::mma(acc, MM<T>::from_lds(arow + (c0 + u) * KC), kh->f[u]);
    });
    c1 = c0;  // nothing left to stream
  }
  for (int cb = c0; cb < c1; cb += 4) {
    const int rem = c1 - cb < 4 ? c1 - cb : 4;
    F f[4], a[4];
    static_for<4>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      const int cu = cb + (u < rem ? u : rem - 1);
      f[u] = coh_frag<T, COH>(rs, o + cu * FSB);
      a[u] = MM<T>::from_lds(arow + cu * KC);
    });
    static_for<4>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      if (u < rem) MM<T>::mma(acc, a[u], f[u]);
    });
  }
  // partial tile of (t, sl) -> red[wave][16][16]
#pragma unroll
  for (int i = 0; i < 4; ++i) red[wave * 256 + (g * 4 + i) * 16 + c] = acc[i];
  __syncthreads();
  for (int i = threadIdx.x; i < 256 * NT; i += SAC_THREADS) {
    const int tt = i / 256, e = i % 256, r = e / 16, cc = e % 16;
    float s = 0.f;
    for (int q = 0; q < wpt; ++q) s += red[(q * NT + tt) * 256 + e];
    out[r * ldo + tt * 16 + cc] = s;
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------- phase A
template <typename T>
__device__ __forceinline__ void target_critic_split_body(const EngineDev* __restrict__ Ep, const sac_replay& rb,
                                                         const int32_t* __restrict__ inj_idx_,
                                                         const float* __restrict__ inj_eps_, int bidA,
                                                         const StepCtx& sc) {
  const AS_C EngineDev& E = *(const AS_C EngineDev*)Ep;
  extern __shared__ float lds_raw[];
  lf* lds = (lf*)lds_raw;
  constexpr int R = SAC_ROWS, HH = SPLIT_HH;
  constexpr int KC = MM<T>::KC;
  constexpr int HC0 = 64 / KC;         // layer 0: chunks held (the rest streams)
  constexpr int NCH_H = SPLIT_H / KC;  // layer 1 reduction
  constexpr int NCH_HH = HH / KC;      // layer 1 dX reduction of a half
  const int tid = threadIdx.x;
  // blocks: pi(s') as WP parts x nrt, then roles 1..5 as 2 halves x nrt each
  constexpr int WP = split_wpi(sizeof(T));
  const int n2 = 2 * E.nrt, n0 = WP * E.nrt;
  const int grp = bidA < n0 ? 0 : 1 + (bidA - n0) / n2;
  const int idx = bidA < n0 ? bidA : (bidA - n0) % n2;
  const int h = bidA < n0 ? idx % WP : idx & 1, rbi = bidA < n0 ? idx / WP : idx >> 1;
  const int HHr = grp == 0 ? SPLIT_H / WP : SPLIT_HH;  // layer-1 outputs of this workgroup's part
  // roles in producer-first order: 0 pi(s'), 1/2 target critics, 3/4 critics, 5 pi(s)
  const int role = grp;
  const bool is_pi = role == 0 || role == 5;
  const int ni = is_pi ? NET_PI : role <= 2 ? NET_Q1T + role - 1 : NET_Q1 + role - 3;
  const AS_C NetDev& net = E.net[ni];
  const AS_C LayerDev& L0 = net.l[0];
  const AS_C LayerDev& L1 = net.l[1];
  const AS_C LayerDev& L2 = net.l[2];
  STAMP(0);
  // this role's weights: layer 0 (first HC0 chunks) first; the half of layer 1
  // (the bulk of the bytes) after the batch record's loads, so the waits for
  // the record do not include it (loads complete in issue order)
  const GemmW w0 = gw_fwd(L0);
  const GemmW w1 = gw_sub<T>(L1.Wc, L1.Kp, h * HHr, HHr, 0, L1.Kp, L1.bias + h * HHr, HHr);
  HTiles<T, 2, HC0> h0;
  HTiles<T, 1, NCH_H> h1;
  ht_issue<T, 2, HC0>(h0, w0);

  const int B = E.B, Bp = E.Bp, O = E.O, A = E.A, ld = E.ld, ldo = E.ldo;
  const int r0 = rbi * R;
  const int nvalid = min(R, B - r0);
  const uint32_t ep = sc.ep;
  const AS_G int32_t* inj_idx = GPC(int32_t, inj_idx_);
  const AS_G float* inj_eps = GPC(float, inj_eps_);
  lf* Xb = lds + E.o_X;           // layer-0 input [R][ld]; later dY0 partial
  lf* H0 = lds + E.o_Y;           // h0 [R][ld]
  lf* P0 = lds + E.o_P1[0];       // layer-0 pre-activation [R][ldp1[0]]
  lf* P1 = lds + E.o_P1[1];       // layer-1 half pre-activation
  lf* H1 = lds + E.o_P2[0];       // h1 half [R][ldp2[0]]
  lf* U1 = lds + E.o_P2[1];       // critics: unit-seed dY1 half
  const int ldp0 = E.ldp1[0], ldp1 = E.ldp1[1], ldh1 = E.ldp2[0], ldu1 = E.ldp2[1];
  lf* outB = lds + E.o_out;       // layer-2 partial [R][ldo]
  lf* red = lds + E.o_red;        // k-split partials
  lf* sB = lds + E.o_s;
  lf* s2B = lds + E.o_s2;
  lf* aB = lds + E.o_a;
  lf* a2B = lds + E.o_a2;
  lf* rB = lds + E.o_r;
  lf* dB = lds + E.o_d;
  lf* epsB = lds + E.o_et;
  lf* lpB = lds + E.o_lp;
  AS_L int64_t* slotB = (AS_L int64_t*)(lds + E.o_slot);
  AS_G float* stats = GP(float, E.stats);

  const uint64_t step = sc.step;
  const int par = sc.par;
#ifndef SAC_ADAM_LAST
#define SAC_ADAM_LAST 1
#endif
  const bool adam_blk = (SAC_ADAM_LAST ? (role == 5 && rbi == E.nrt - 1 && h == 1) : (role == 0 && rbi == 0 && h == 0));
  if (adam_blk && tid < 4 && (tid < 3 || (E.auto_entropy && E.alpha_update))) {
    // optimizer step counters and this step's Adam bias corrections (torch adam.py), read
    // by phases B and D only: done by the last pi(s) workgroup, off the y chain (a load
    // round trip + double pow() here delayed pi(s') of row tile 0, hence the whole launch)
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
  // ---- sample (replay_buffer.py:32-39) + gather (agent.py:166-193): the staged record or a gather
  const int64_t rb_size = GPC(int64_t, rb.state)[0], rb_pos = GPC(int64_t, rb.state)[1];
  bool staged = false;
  bool h1_issued = false;
  if (E.stage && !inj_idx) {
    const AS_G float* rec = GPC(float, E.stg) + stage_rec(E, step, rbi);
    const AS_C uint64_t* hdr = (const AS_C uint64_t*)rec;
    const AS_G float* p = rec + 16;
    constexpr int NS = (R * 32 + SAC_THREADS - 1) / SAC_THREADS;
    if (O <= 32) {  // uniform: record -> registers, layer-1 weights issued behind it, -> LDS
      float rs[2][NS], ra[NS], rr = 0.f, rd = 0.f;
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        const int i = tid + u * SAC_THREADS;
        rs[0][u] = i < R * O ? p[i] : 0.f;
        rs[1][u] = i < R * O ? p[R * O + i] : 0.f;
        ra[u] = i < R * A ? p[2 * R * O + i] : 0.f;
      }
      if (tid < R) {
        rr = p[2 * R * O + R * A + tid];
        rd = p[2 * R * O + R * A + R + tid];
      }
      ht_issue<T, 1, NCH_H>(h1, w1);
      h1_issued = true;
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        const int i = tid + u * SAC_THREADS;
        if (i < R * O) {
          sB[i] = rs[0][u];
          s2B[i] = rs[1][u];
        }
        if (i < R * A) aB[i] = ra[u];
      }
      if (tid < R) {
        rB[tid] = rr;
        dB[tid] = rd;
      }
      STAMP(22);  // probe: thread 0's record loads landed
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
  if (!h1_issued) ht_issue<T, 1, NCH_H>(h1, w1);
  // layer 2's k-split slice (layer 2 runs after the hand-off for the target
  // critics, and at the end of pi(s')'s chain): held from here
  GemmW w2n = gw_sub<T>(L2.Wc, L2.Kp, 0, L2.Np, h * HHr, HHr, nullptr, 0);
  w2n.NT = (L2.N + 15) >> 4;  // output tiles that hold data
  KsHeld<T> kh2;
  kh2.ok = false;
  if (sizeof(T) == 2) ks_issue<T>(kh2, w2n);  // bf16: one fragment, from the start
  if (staged && rbi == 0 && role == 0 && h == 0 && tid == 0)
    *(AS_G uint64_t*)(GP(uint32_t, E.sync) + 4) = step;  // SYNC_STAGED (tests)
  if (!staged) {  // uniform
    tile_slots(E, rb, step, rb_size, rb_pos, r0, inj_idx, slotB);
    __syncthreads();
    gather_rows<lf*>(rb, slotB, O, A, sB, s2B, aB, rB, dB);
  }
  // eps: the target draw (which = 0) for the roles that evaluate pi's head on s'
  // (target critics), the actor draw (which = 1) for pi(s)
  if (role == 1 || role == 2 || role == 5) {
    const int which = role == 5 ? 1 : 0;
    const int NP = (A + 1) / 2;
    for (int i = tid; i < R * NP; i += SAC_THREADS) {
      const int r = i / NP, pp = i % NP, b = r0 + r;
      float e0 = 0.f, e1 = 0.f;
      if (b < B) {
        if (inj_eps) {
          e0 = inj_eps[((size_t)which * B + b) * A + 2 * pp];
          if (2 * pp + 1 < A) e1 = inj_eps[((size_t)which * B + b) * A + 2 * pp + 1];
        } else {
          philox_normal2(E.seed, step, (uint32_t)b, (uint32_t)which, (uint32_t)pp, e0, e1);
        }
      }
      epsB[r * A + 2 * pp] = e0;
      if (2 * pp + 1 < A) epsB[r * A + 2 * pp + 1] = e1;
    }
  }
  __syncthreads();
  STAMP(1);

  // pi's squashed-Gaussian head (models.py:79-87) from two layer-2 partials:
  // o = p0 + p1 + b2 (same order in every consumer), one lane per (row, dim)
  // tgt: the WP parts of pi(s')'s layer-2 partial (g0 = part 0's granules; parts
  // are gs2 granules apart), summed in part order; else this half's own partial
  // (outB) and the peer half's granules g1, in half order
  auto head = [&](const AS_G uint64_t* g0, const AS_G uint64_t* g1, bool tgt, lf* actB, lf* lpOut, bool stash) {
    const AS_C NetDev& pn = E.net[NET_PI];
    const float* b2 = pn.l[2].bias;
    const int AP = A <= 1 ? 1 : 1 << (32 - __builtin_clz(A - 1));
    const int rpp = SAC_THREADS / AP;
    const int jj = tid % AP;
    // this lane's head biases, loaded before the polls (not one more round trip after them)
    const float b2mu = jj < A ? ldf<false>(b2 + jj) : 0.f, b2ls = jj < A ? ldf<false>(b2 + A + jj) : 0.f;
    for (int base = 0; base < R; base += rpp) {
      const int r = base + tid / AP, j = jj;
      const bool live = r < R && j < A;
      float lp = 0.f, corr = 0.f;
      if (live) {
        float mu, lsr;
        if (tgt) {
          const AS_G uint64_t* gg[2 * WP];
#pragma unroll
          for (int p = 0; p < WP; ++p) {
            gg[p] = g0 + (size_t)p * E.gs2 + r * 2 * A + j;
            gg[WP + p] = g0 + (size_t)p * E.gs2 + r * 2 * A + A + j;
          }
          float v[2 * WP];
          gran_getn<2 * WP>(E, gg, ep, v);
          float smu = v[0], sls = v[WP];
#pragma unroll
          for (int p = 1; p < WP; ++p) {
            smu += v[p];
            sls += v[WP + p];
          }
          mu = smu + b2mu;
          lsr = sls + b2ls;
        } else {  // g0 / g1 = this half's own partial (in outB) and the peer's granules, in half order
          const float pown0 = outB[r * ldo + j], pown1 = outB[r * ldo + A + j];
          const AS_G uint64_t* gg[2] = {g1 + r * 2 * A + j, g1 + r * 2 * A + A + j};
          float v[2];
          gran_getn<2>(E, gg, ep, v);
          const float ppe0 = v[0], ppe1 = v[1];
          mu = (h == 0 ? pown0 + ppe0 : ppe0 + pown0) + b2mu;
          lsr = (h == 0 ? pown1 + ppe1 : ppe1 + pown1) + b2ls;
        }
        const float e = epsB[r * A + j];
        const float lo = E.ls_min, hi = E.ls_max;
        const float ls = lsr < lo ? lo : (lsr > hi ? hi : lsr);
        const float sd = expf(ls);
        const float z = mu + e * sd;
        const float act_v = tanhf(z) * E.scale;
        const float diff = z - mu;
        const float var = sd * sd;
        lp = -(diff * diff) / (2.f * var) - logf(sd) - HALF_LOG_2PI;
        corr = 2.f * ((LOG2F - z) - softplus20(-2.f * z));
        actB[r * A + j] = act_v;
        if (stash) {
          const int b = r0 + r;
          float* hs = E.head_st + (size_t)b * 4 * A;
          st_f<false>(hs + j, mu);
          st_f<false>(hs + A + j, lsr);
          st_f<false>(hs + 2 * A + j, z);
          st_f<false>(hs + 3 * A + j, e);
          st_f<false>(E.a_st + (size_t)b * A + j, act_v);
        }
      }
      for (int o = 1; o < AP; o <<= 1) {
        lp += __shfl_xor(lp, o, 64);
        corr += __shfl_xor(corr, o, 64);
      }
      if (live && j == 0) lpOut[r] = lp - corr;
    }
    __syncthreads();
  };

  // ---- layer 0 (full) and layer 1 (this half) forward: H0, H1 in LDS; P0 / P1 kept
  auto no_hook = [] {};
  auto forward01 = [&](bool keepP, bool stXT, bool pi_actor, auto&& after_l1, bool l0_done = false) {
    // layer 0: X [R][Kp0] -> P0 / H0 [R][H] (l0_done: the caller computed H0)
    const int act = net.hid_act;
    if (!l0_done) gemm_hs<T, 2, HC0, false>(Xb, ld, w0, &h0, [&](int j, int col, const f32x4& acc) {
      const bool nv = col < L0.N;
      const float bn = h0.b[j];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = (((threadIdx.x & 63) >> 4) << 2) + i;
        const float p = nv ? acc[i] + bn : 0.f;
        if (keepP) P0[r * ldp0 + col] = p;
        H0[r * ld + col] = act == ACT_RELU ? (p > 0.f ? p : 0.f) : p;
      }
    });
    if (!l0_done) {
      if (act != ACT_RELU && act != ACT_ID) act_pass_fwd<R>(H0, ld, L0.Np >> 4, act);
      __syncthreads();
    }
    // pi's pre-activations for phase C's backward: only for a non-ReLU hidden
    // activation (a ReLU mask is read back from the next layer's stashed X^T)
    if (pi_actor && h == 0 && act != ACT_RELU) {
      float* ps = L0.pstash + (size_t)r0 * L0.Np;
      for (int i = tid; i < R * L0.Np; i += SAC_THREADS) st_f<false>(ps + i, P0[(i / L0.Np) * ldp0 + i % L0.Np]);
    }
    if (stXT && h == 0)
      store_T<T, R>(H0, ld, L1.Kp, L1.K, (T*)L1.XT + (pi_actor ? par * L1.xt_par : 0), Bp, r0, nvalid, nullptr);
    STAMP(2);
    if (sizeof(T) == 4 && !kh2.ok) ks_issue<T, KsHeld<T>::MAXC, false>(kh2, w2n);  // fp32: under layer 1 (target critics: before the poll)
    // layer 1, this half: H0 -> P1 / H1 [R][HH]
    gemm_hs<T, 1, NCH_H, false>(H0, ld, w1, &h1, [&](int j, int col, const f32x4& acc) {
      const float bn = h1.b[j];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = (((threadIdx.x & 63) >> 4) << 2) + i;
        const float p = acc[i] + bn;
        if (keepP) P1[r * ldp1 + col] = p;
        H1[r * ldh1 + col] = act == ACT_RELU ? (p > 0.f ? p : 0.f) : p;
      }
    });
    after_l1();  // layer 1's held weights are dead from here
    if (act != ACT_RELU && act != ACT_ID) act_pass_fwd<R>(H1, ldh1, HHr >> 4, act);
    __syncthreads();
    if (pi_actor && act != ACT_RELU) {  // this half's layer-1 pre-activations
      float* ps = L1.pstash + (size_t)r0 * L1.Np + h * HH;
      for (int i = tid; i < R * HH; i += SAC_THREADS) st_f<false>(ps + (i / HH) * L1.Np + i % HH, P1[(i / HH) * ldp1 + i % HH]);
    }
    if (stXT)  // layer 2's input, this half's rows of X^T
      store_T<T, R>(H1, ldh1, HH, HH, (T*)L2.XT + (pi_actor ? par * L2.xt_par : 0) + (size_t)h * HH * Bp, Bp, r0,
                       nvalid, nullptr);
    STAMP(3);
    // layer 2, this half's partial sum: outB [R][Np2]
    gemm_ksplit<T, false, decltype(kh2)::MAXC>(H1, ldh1, w2n, red, outB, ldo, &kh2);
    STAMP(4);
  };

  // X = [s or s', a or a'] (zero padded to Kp0)
  auto build_x = [&](const lf* st, const lf* ac, int na) {
    const int Kp0 = L0.Kp;
    for (int i = tid; i < R * Kp0; i += SAC_THREADS) {
      const int r = i / Kp0, k = i % Kp0;
      Xb[r * ld + k] = k < O ? st[r * O + k] : (k < O + na ? ac[r * A + (k - O)] : 0.f);
    }
    __syncthreads();
  };

  // alpha (agent.py:203): the previous step's phase D wrote it (the previous launch)
  const float alpha32 = (float)*GPC(double, E.alpha_state + 1);
  if (role == 0) {
    // ---- pi(s'): the critical path's head
    build_x(s2B, aB, 0);
    forward01(false, false, false, no_hook);
    AS_G uint64_t* g = gs_at(E, GS_PI, rbi, h);
    for (int i = tid; i < R * 2 * A; i += SAC_THREADS) gran_put(g + i, outB[(i / (2 * A)) * ldo + i % (2 * A)], ep);
    STAMP(6);
  } else if (role == 5) {
    // ---- pi(s): the actor sample for phase C (stashes), X^T of pi's layers
    if (h == 0)
      for (int i = tid; i < R * O; i += SAC_THREADS) st_f<false>(E.s_st + (size_t)r0 * O + i, sB[i]);
    build_x(sB, aB, 0);
    // layer-0 input X^T: both halves store it (columns h Bp + r0: the partial dW layout)
    store_T<T, R>(Xb, ld, L0.Kp, L0.K, (T*)L0.XT + par * L0.xt_par, 2 * Bp, h * Bp + r0, nvalid, nullptr);
    forward01(true, true, true, no_hook);
    AS_G uint64_t* g = gs_at(E, GS_PS, rbi, h);
    for (int i = tid; i < R * 2 * A; i += SAC_THREADS) gran_put(g + i, outB[(i / (2 * A)) * ldo + i % (2 * A)], ep);
    head(nullptr, gs_at(E, GS_PS, rbi, 1 - h), false, a2B, lpB, h == 0);
    if (h == 0 && tid < nvalid) {
      const int b = r0 + tid;
      st_f<false>(E.lp_st + par * E.Br + b, lpB[tid]);
      stats[4 + B + b] = lpB[tid];
    }
    STAMP(6);
  } else if (role == 1 || role == 2) {
    // ---- target critic t (agent.py:195-211): a~', log pi' from pi(s')'s two partials
    const int t = role - 1;
    if (sizeof(T) == 4) ks_issue<T, KsHeld<T>::MAXC, false>(kh2, w2n);
    // Layer 0 over the s' columns runs BEFORE the pi(s') hand-off (round 5,
    // VERDICT r04 item 2c): only the chunks holding a~' columns are left for
    // after the head.  Chunks [0, O / KC) are s' only; a chunk that holds both
    // (O % KC != 0: bf16 at C2, one 32-deep chunk) is multiplied once with its
    // a~' columns still 0 and once, after the head, with its s' columns
    // zeroed.  Chunk c goes to accumulator c & 1 as in gemm_hs, so with no
    // shared chunk (fp32 C2 / C4, bf16 C4) the result is the same bits.
    const int Kp0 = L0.Kp, nch0 = Kp0 / KC;
    const bool early0 = nch0 <= HC0;  // every layer-0 chunk held (C2, C4): else the plain path
    if (early0) {
      build_x(s2B, a2B, 0);  // [s', 0]
      const int cs = O / KC, cb = (O + KC - 1) / KC;  // s'-only chunks; chunks with any s' column
      const int lane = tid & 63, wave = wave_id(), c = lane & 15, g = lane >> 4;
      const lf* arow = Xb + c * ld + g * MM<T>::KL;
      f32x4 acc[2][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[j][0] = acc[j][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
      auto chunks = [&](int c0, int c1) __attribute__((always_inline)) {
        static_for<HC0>([&](auto uc) {
          constexpr int u = decltype(uc)::value;
          if (u >= c0 && u < c1) {  // uniform
            const typename MM<T>::Frag a = MM<T>::from_lds(arow + u * KC);
            static_for<2>([&](auto jc) {
              constexpr int j = decltype(jc)::value;
              if (wave + j * SAC_NW < w0.NT) MM<T>::mma(acc[j][u & 1], a, h0.f[j][u]);
            });
          }
        });
      };
      chunks(0, cb);
      __syncthreads();  // every wave has read the shared chunk's s' columns
      if (cb > cs)  // the shared chunk keeps only its a~' columns for the second pass
        for (int i = tid; i < R * KC; i += SAC_THREADS) {
          const int r = i / KC, k = cs * KC + i % KC;
          if (k < O) Xb[r * ld + k] = 0.f;
        }
      head(gs_at(E, GS_PI, rbi, 0), nullptr, true, a2B, lpB, false);
      if (t == 0 && h == 0 && tid < R) gran_put(gs_at(E, GS_LP, rbi, 0) + tid, lpB[tid], ep);
      STAMP(7);
      for (int i = tid; i < R * A; i += SAC_THREADS) Xb[(i / A) * ld + O + i % A] = a2B[i];
      __syncthreads();
      chunks(cs, nch0);
      const int act = net.hid_act;
      static_for<2>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        const int tt = wave + j * SAC_NW;
        if (tt < w0.NT) {
          const int col = tt * 16 + c;
          const bool nv = col < L0.N;
          const f32x4 sum = acc[j][0] + acc[j][1];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p = nv ? sum[i] + h0.b[j] : 0.f;
            H0[(g * 4 + i) * ld + col] = act == ACT_RELU ? (p > 0.f ? p : 0.f) : p;
          }
        }
      });
      if (act != ACT_RELU && act != ACT_ID) act_pass_fwd<R>(H0, ld, L0.Np >> 4, act);
      __syncthreads();
      forward01(false, false, false, no_hook, true);
    } else {
      head(gs_at(E, GS_PI, rbi, 0), nullptr, true, a2B, lpB, false);
      if (t == 0 && h == 0 && tid < R) gran_put(gs_at(E, GS_LP, rbi, 0) + tid, lpB[tid], ep);
      STAMP(7);
      build_x(s2B, a2B, A);
      forward01(false, false, false, no_hook);
    }
    if (tid < R) gran_put(gs_at(E, t ? GS_QT2 : GS_QT1, rbi, h) + tid, outB[tid * ldo], ep);
    STAMP(9);
    if (t == 0 && h == 0 && tid < 64) {
      // this half (Qt1, half 0) computes the row tile's targets y and both
      // critics' seeds dL/dq = 2 (q - y) / B and loss partials (agent.py:
      // 195-236; the critic roles store unit-seed operands and finish without
      // waiting for y: phase B applies the seeds).
      float sq[2] = {0.f, 0.f};
      if (tid < R) {
        const int b = r0 + tid;
        const bool v = tid < nvalid;
        const AS_C NetDev& t1 = E.net[NET_Q1T];
        const AS_C NetDev& t2 = E.net[NET_Q2T];
        const float bt1 = ldf<false>(t1.l[2].bias), bt2 = ldf<false>(t2.l[2].bias);
        const float bq[2] = {ldf<false>(E.net[NET_Q1].l[2].bias), ldf<false>(E.net[NET_Q2].l[2].bias)};
        const AS_G uint64_t* gg[7] = {gs_at(E, GS_QT1, rbi, 1) + tid, gs_at(E, GS_QT2, rbi, 0) + tid,
                                      gs_at(E, GS_QT2, rbi, 1) + tid, gs_at(E, GS_QA1, rbi, 0) + tid,
                                      gs_at(E, GS_QA1, rbi, 1) + tid, gs_at(E, GS_QA2, rbi, 0) + tid,
                                      gs_at(E, GS_QA2, rbi, 1) + tid};
        float gv[7];
        gran_getn<7>(E, gg, ep, gv);
        const float q1tp = outB[tid * ldo] + gv[0] + bt1;
        const float q2tp = gv[1] + gv[2] + bt2;
        const float q1t = t1.out_act == ACT_ID ? q1tp : act_fwd(t1.out_act, q1tp);
        const float q2t = t2.out_act == ACT_ID ? q2tp : act_fwd(t2.out_act, q2tp);
        const float y = rB[tid] + (E.gamma * (1.f - dB[tid])) * (fmin_nan(q1t, q2t) - alpha32 * lpB[tid]);
        if (b < B) stats[4 + b] = y;
#pragma unroll
        for (int qi = 0; qi < 2; ++qi) {
          const AS_C NetDev& qn = E.net[NET_Q1 + qi];
          const float qpre = (gv[3 + 2 * qi] + gv[4 + 2 * qi]) + bq[qi];
          const float q = qn.out_act == ACT_ID ? qpre : act_fwd(qn.out_act, qpre);
          const float d = q - y;
          sq[qi] = v ? d * d : 0.f;
          float seed = v ? (2.0f / (float)B) * d : 0.f;
          if (qn.out_act != ACT_ID) seed = act_bwd(qn.out_act, qpre, seed);
          st_f<false>(E.seedq + qi * Bp + b, seed);
        }
      }
#pragma unroll
      for (int qi = 0; qi < 2; ++qi) {
        const float s2 = wave_sum(sq[qi]);
        if (tid == 0) st_f<false>(E.lossp + (par * E.nrt + rbi) * 4 + qi, s2);
      }
    }
  } else {
    // ---- critic qi (agent.py:213-236): forward, unit-seed backward, seed once y is known
    const int qi = role - 3;
    // layer 1's dX operand for this half (rows k all, reduction over this half's n), held
    const GemmW wt1 = gw_sub<T>(L1.WTc, L1.Np, 0, L1.Kp, h * HH, HH, nullptr, 0);
    HTiles<T, 2, NCH_HH> ht1;
    // bf16: held from the start too; fp32 (no register room: 51 VGPRs would
    // spill) issued as soon as layer 1's forward GEMM has freed h1's registers.
    // W2's element for this thread's column n = tid % HH
    if constexpr (sizeof(T) == 2) ht_issue<T, 2, NCH_HH, false>(ht1, wt1);
    static_assert(SAC_THREADS % SPLIT_HH == 0, "one W2 column per thread in the unit-seed loop");
    const float w2n = ldf<false>(net.P + L2.w_off + h * HH + tid % HH);  // W2 [1][H] fp32 master
    build_x(sB, aB, A);
    // layer-0 input X^T is shared by Q1 and Q2: Q1's halves store it (columns h Bp + r0)
    if (qi == 0) store_T<T, R>(Xb, ld, L0.Kp, L0.K, L0.XT, 2 * Bp, h * Bp + r0, nvalid, nullptr);
    forward01(true, true, false, [&] {
      if constexpr (sizeof(T) == 4) ht_issue<T, 2, NCH_HH, false>(ht1, wt1);
    });
    if (tid < R) gran_put(gs_at(E, qi ? GS_QA2 : GS_QA1, rbi, h) + tid, outB[tid * ldo], ep);
    // unit-seed backward (every layer's dY is linear in the row's seed 2(q - y)/B):
    // U1[r][n] = act'(P1[r][n]) * W2[0][h HH + n];  U0p = act'(P0) * (U1 W1[half])
    {
      for (int i = tid; i < R * HH; i += SAC_THREADS) {
        const int r = i / HH, n = i % HH;  // n == tid % HH
        U1[r * ldu1 + n] = act_bwd(net.hid_act, P1[r * ldp1 + n], w2n);
      }
      __syncthreads();
      gemm_hs<T, 2, NCH_HH, false>(U1, ldu1, wt1, &ht1, [&](int j, int col, const f32x4& acc) {
        const bool kv = col < L1.K;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = (((threadIdx.x & 63) >> 4) << 2) + i;
          float v = kv ? acc[i] : 0.f;
          if (net.hid_act == ACT_RELU && !(P0[r * ldp0 + col] > 0.f)) v = 0.f;
          Xb[r * ld + col] = v;  // U0 partial
        }
      });
      if (net.hid_act != ACT_RELU && net.hid_act != ACT_ID)
        act_pass_bwd<R>(Xb, ld, P0, ldp0, L1.Kp >> 4, L1.K, net.hid_act);
      __syncthreads();
    }
    STAMP(16);
    // the role does not wait for y.  It stores every layer's UNIT-seed dY^T
    // (layer 2's: the indicator row); phase B scales each batch column by the
    // seed the first target-critic half computed (E.seedq) and sums the bias
    // gradients from the scaled rows.  (bf16: the unit dY is rounded to bf16
    // here and the scaled value once more in phase B, within the bf16 mode's
    // tolerances; round 5, VERDICT r04 item 2a -- before, the bf16 critics
    // waited for y and stored seed-scaled rows.)
    store_T<T, R>(U1, ldu1, HH, HH, (T*)L1.GT + (size_t)h * HH * Bp, Bp, r0, nvalid, nullptr);
    store_T<T, R>(Xb, ld, L0.Np, L0.N, L0.GT, 2 * Bp, h * Bp + r0, nvalid, nullptr);
    if (h == 0) {
      lf* g2 = outB;  // this half's q partial went out as a granule above
      for (int i = tid; i < R * 32; i += SAC_THREADS) g2[(i / 32) * ldo + i % 32] = (i % 32) == 0 ? 1.f : 0.f;
      __syncthreads();
      store_T<T, R>(g2, ldo, L2.Np, L2.N, L2.GT, Bp, r0, nvalid, nullptr);
    }
    STAMP(15);
    STAMP(11 + 2 * qi);
  }
}

template <typename T>
__global__ void __launch_bounds__(SAC_THREADS) sac_target_critic_split(const EngineDev* __restrict__ Ep, sac_replay rb,
                                                                        const int32_t* __restrict__ inj_idx_,
                                                                        const float* __restrict__ inj_eps_) {
#ifdef SAC_STAMPS
  const long long t_entry = __builtin_amdgcn_s_memrealtime();  // probe 20: before the descriptor prefetch
#endif
  PREFETCH_ARG(Ep);
  const AS_C EngineDev& E0 = *(const AS_C EngineDev*)Ep;
  const uint64_t step = *GPC(uint64_t, E0.rng_step);
  const StepCtx sc{step, *GPC(uint32_t, E0.sync) + 1u, (int)(step & 1)};
#ifdef SAC_STAMPS
  if (threadIdx.x == 0 && E0.stamps) {  // probe 21: the step counter loaded (the index depends on it)
    GP(long long, E0.stamps)[blockIdx.x * 64 + 20] = t_entry;
    GP(long long, E0.stamps)[blockIdx.x * 64 + 21 + (step == ~0ull ? 1 : 0)] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  int bidA = (int)blockIdx.x;
  if (E0.role_xcd) {  // uniform
    // blocks are dealt round-robin to the 8 XCDs (block b on XCD b % 8): XCD x
    // takes units [x G/8, (x+1) G/8) of the part-major order (every row tile of
    // pi(s') quarter 0, of quarter 1, ..., of each role half), so the 16
    // workgroups that stream one weight part share at most two XCDs' L2s
    constexpr int WP = split_wpi(sizeof(T));
    const int nrt = E0.nrt, n0 = WP * nrt, n2 = 2 * nrt;
    const int u = (bidA % 8) * ((int)gridDim.x / 8) + bidA / 8;
    if (u < n0) {
      bidA = (u % nrt) * WP + u / nrt;
    } else {
      const int v = u - n0, w = v % n2;
      bidA = n0 + (v / n2) * n2 + (w % nrt) * 2 + w / nrt;
    }
  }
  target_critic_split_body<T>(Ep, rb, inj_idx_, inj_eps_, bidA, sc);
  const AS_C EngineDev& E = *(const AS_C EngineDev*)Ep;
  (void)E;
  END_STAMP(60);
}

// ---------------------------------------------------------------------------- phase C
// pi's weights are read with plain loads (the previous launch's phase D wrote them).
template <typename T>
__device__ __forceinline__ void actor_split_body(const EngineDev* __restrict__ Ep, int bid, const StepCtx& sc) {
  const AS_C EngineDev& E = *(const AS_C EngineDev*)Ep;
  extern __shared__ float lds_raw[];
  lf* lds = (lf*)lds_raw;
  // WQ: the critic roles' parts of layer 1, WP: pi's (HQ / HH: layer-1 outputs of a part)
  constexpr int R = SAC_ROWS, WQ = split_wcq(sizeof(T)), WP = split_wc(sizeof(T));
  constexpr int HQ = SPLIT_H / WQ, HH = SPLIT_H / WP;
  constexpr int KC = MM<T>::KC;
  constexpr int HC0 = 64 / KC;
  constexpr int NCH_H = SPLIT_H / KC;
  constexpr int NCH_HH = HH / KC, NCH_HQ = HQ / KC;
  constexpr int NCH_32 = 32 / KC;
  const int tid = threadIdx.x;
  // producers first: groups 0 / 1 the critics (WQ parts per row tile), group 2 pi (WP parts)
  const int nq = WQ * E.nrt;
  const bool is_pi = bid >= 2 * nq;
  const int qi = is_pi ? 0 : bid / nq;  // critics
  const int idx = is_pi ? bid - 2 * nq : bid % nq;
  const int h = is_pi ? idx % WP : idx % WQ, rbi = is_pi ? idx / WP : idx / WQ;  // h: this workgroup's part of layer 1
  STAMP(32);
  const int B = E.B, Bp = E.Bp, O = E.O, A = E.A, ld = E.ld, ldo = E.ldo;
  const int r0 = rbi * R;
  const int nvalid = min(R, B - r0);
  const uint32_t ep = sc.ep;
  const int par = sc.par;
  lf* Xb = lds + E.o_X;
  lf* H0 = lds + E.o_Y;
  lf* P0 = lds + E.o_P1[0];
  lf* P1 = lds + E.o_P1[1];
  lf* H1 = lds + E.o_P2[0];
  lf* U1 = lds + E.o_P2[1];
  const int ldp0 = E.ldp1[0], ldp1 = E.ldp1[1], ldh1 = E.ldp2[0], ldu1 = E.ldp2[1];
  lf* outB = lds + E.o_out;
  lf* red = lds + E.o_red;
  lf* sB = lds + E.o_s;
  lf* aB = lds + E.o_a;
  lf* lpB = lds + E.o_lp;
  lf* gaB = lds + E.o_ga;
  lf* goutB = lds + E.o_gout;
  lf* g1B = lds + E.o_g;
  lf* g2B = lds + E.o_g2;
  const float alpha32 = (float)*GPC(double, E.alpha_state + 1);  // the previous launch's phase D

  if (!is_pi) {
    // ---- critic qi on (s, a~) with the UPDATED weights (agent.py:244-248), then d Q / d a~
    const AS_C NetDev& net = E.net[NET_Q1 + qi];
    const AS_C LayerDev& L0 = net.l[0];
    const AS_C LayerDev& L1 = net.l[1];
    const AS_C LayerDev& L2 = net.l[2];
    const GemmW w0 = gw_fwd(L0);
    const GemmW w1 = gw_sub<T>(L1.Wc, L1.Kp, h * HQ, HQ, 0, L1.Kp, L1.bias + h * HQ, HQ);
    HTiles<T, 2, HC0> h0;
    HTiles<T, 1, NCH_H> h1;
    // layer-1 dX operand of this half, held from the start as well (its fetch
    // would otherwise sit between the forward pass and the backward GEMM)
    const GemmW wt1 = gw_sub<T>(L1.WTc, L1.Np, 0, L1.Kp, h * HQ, HQ, nullptr, 0);
    HTiles<T, 2, NCH_HQ> ht1;
    ht_issue<T, 2, HC0>(h0, w0);
    ht_issue<T, 1, NCH_H>(h1, w1);
    ht_issue<T, 2, NCH_HQ>(ht1, wt1);
    // the two k-split steps of the critic's chain (layer 2's partial q, then
    // layer 0's dX for the action columns) read weights phase B has just
    // written: held (issued behind the inputs), not a cold round trip each
    // after layer 1 / after dY0 (SAC_KS_C=0: streamed)
    GemmW w2 = gw_sub<T>(L2.Wc, L2.Kp, 0, L2.Np, h * HQ, HQ, nullptr, 0);
    w2.NT = (L2.N + 15) >> 4;
    const int k0 = (O >> 4) << 4, k1 = (O + A + 15) >> 4 << 4;
    GemmW wt0 = gw_sub<T>(L0.WTc, L0.Np, k0, k1 - k0, 0, L0.Np, nullptr, 0);
    KsHeld<T, sizeof(T) == 4 ? 2 : 1> kc2;
    KsHeld<T, sizeof(T) == 4 ? 8 : 1> kc0;
    kc2.ok = kc0.ok = false;
    // the W2 (fp32 master) element of this thread's column n = tid % HQ of the unit-seed backward
    static_assert(SAC_THREADS % HQ == 0, "one W2 column per thread in the unit-seed loop");
    const float w2n = GPC(float, net.P + L2.w_off)[h * HQ + tid % HQ];
    for (int i = tid; i < R * O; i += SAC_THREADS) sB[i] = GPC(float, E.s_st)[(size_t)r0 * O + i];
    for (int i = tid; i < R * A; i += SAC_THREADS) aB[i] = GPC(float, E.a_st)[(size_t)r0 * A + i];
    if (SAC_KS_C) {  // behind the inputs: waiting for s / a~ must not wait for these (loads retire in order)
      ks_issue<T, decltype(kc2)::MAXC>(kc2, w2);
      if (sizeof(T) == 2) ks_issue<T, decltype(kc0)::MAXC>(kc0, wt0);  // fp32: after layer 1 (its held W1 part is dead then; from here it spilled)
    }
    __syncthreads();
    const int Kp0 = L0.Kp;
    for (int i = tid; i < R * Kp0; i += SAC_THREADS) {
      const int r = i / Kp0, k = i % Kp0;
      Xb[r * ld + k] = k < O ? sB[r * O + k] : (k < O + A ? aB[r * A + (k - O)] : 0.f);
    }
    __syncthreads();
    STAMP(33);
    const int act = net.hid_act;
    gemm_hs<T, 2, HC0, false>(Xb, ld, w0, &h0, [&](int j, int col, const f32x4& acc) {
      const bool nv = col < L0.N;
      const float bn = h0.b[j];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = (((threadIdx.x & 63) >> 4) << 2) + i;
        const float p = nv ? acc[i] + bn : 0.f;
        P0[r * ldp0 + col] = p;
        H0[r * ld + col] = act == ACT_RELU ? (p > 0.f ? p : 0.f) : p;
      }
    });
    if (act != ACT_RELU && act != ACT_ID) act_pass_fwd<R>(H0, ld, L0.Np >> 4, act);
    __syncthreads();
    gemm_hs<T, 1, NCH_H, false>(H0, ld, w1, &h1, [&](int j, int col, const f32x4& acc) {
      const float bn = h1.b[j];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = (((threadIdx.x & 63) >> 4) << 2) + i;
        const float p = acc[i] + bn;
        P1[r * ldp1 + col] = p;
        H1[r * ldh1 + col] = act == ACT_RELU ? (p > 0.f ? p : 0.f) : p;
      }
    });
    if (SAC_KS_C && sizeof(T) == 4) ks_issue<T, decltype(kc0)::MAXC>(kc0, wt0);
    if (act != ACT_RELU && act != ACT_ID) act_pass_fwd<R>(H1, ldh1, HQ >> 4, act);
    __syncthreads();
    gemm_ksplit<T, false, decltype(kc2)::MAXC>(H1, ldh1, w2, red, outB, ldo, &kc2);  // partial q
    STAMP(36 + qi);
    // unit-seed backward down to a~ (the pi role applies the min-Q weights and act'(q))
    {
      for (int i = tid; i < R * HQ; i += SAC_THREADS) {
        const int r = i / HQ, n = i % HQ;  // n == tid % HQ
        U1[r * ldu1 + n] = act_bwd(act, P1[r * ldp1 + n], w2n);
      }
      __syncthreads();
      gemm_hs<T, 2, NCH_HQ, false>(U1, ldu1, wt1, &ht1, [&](int j, int col, const f32x4& acc) {
        const bool kv = col < L1.K;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = (((threadIdx.x & 63) >> 4) << 2) + i;
          float v = kv ? acc[i] : 0.f;
          if (act == ACT_RELU && !(P0[r * ldp0 + col] > 0.f)) v = 0.f;
          Xb[r * ld + col] = v;
        }
      });
      if (act != ACT_RELU && act != ACT_ID) act_pass_bwd<R>(Xb, ld, P0, ldp0, L1.Kp >> 4, L1.K, act);
      __syncthreads();
      // dX of layer 0 for the action columns: the 16-row tiles of W0^T holding [O, O + A)
      gemm_ksplit<T, false, decltype(kc0)::MAXC>(Xb, ld, wt0, red, H0, ld, &kc0);  // H0 [R][k1 - k0]: partial dX0
      AS_G uint64_t* g = gs_at(E, GS_C1 + qi, rbi, h);
      for (int i = tid; i < R * A; i += SAC_THREADS) gran_put(g + i, H0[(i / A) * ld + (O - k0) + i % A], ep);
      if (tid < R) gran_put(g + R * A + tid, outB[tid * ldo], ep);
    }
    STAMP(38 + qi);
    return;
  }

  // ---- pi half h: head backward + pi backward (agent.py:251-257)
  const AS_C NetDev& pi = E.net[NET_PI];
  const AS_C LayerDev& L0 = pi.l[0];
  const AS_C LayerDev& L1 = pi.l[1];
  const AS_C LayerDev& L2 = pi.l[2];
  // operands: layer 2's dX (rows = this half's n, reduction over 2A -> 32),
  // layer 1's dX (rows k all, reduction over this half's n), both held
  const GemmW wt2 = gw_sub<T>(L2.WTc, L2.Np, h * HH, HH, 0, L2.Np, nullptr, 0);
  const GemmW wt1 = gw_sub<T>(L1.WTc, L1.Np, 0, L1.Kp, h * HH, HH, nullptr, 0);
  HTiles<T, 1, NCH_32> ht2;
  HTiles<T, 2, NCH_HH> ht1;
  ht_issue<T, 1, NCH_32, false>(ht2, wt2);
  ht_issue<T, 2, NCH_HH, false>(ht1, wt1);
  {  // the hidden layers' activation derivatives: for ReLU the masks, read from
     // the next layer's X^T that phase A's pi(s) role stashed for phase D
     // (relu(p) > 0 <=> p > 0); otherwise the stashed pre-activations
    if (pi.hid_act == ACT_RELU) {
      const AS_G T* x1 = GPC(T, L1.XT) + par * L1.xt_par + r0;  // relu(P0)^T [K1][Bp]
      for (int i = tid; i < R * L0.Np; i += SAC_THREADS) {
        const int k = i / R, r = i % R;
        P0[r * ldp0 + k] = k < L1.K ? (float)x1[(size_t)k * Bp + r] : 0.f;
      }
      const AS_G T* x2 = GPC(T, L2.XT) + par * L2.xt_par + (size_t)h * HH * Bp + r0;  // this half's relu(P1)^T
      for (int i = tid; i < R * HH; i += SAC_THREADS) {
        const int k = i / R, r = i % R;
        P1[r * ldp1 + k] = (float)x2[(size_t)k * Bp + r];
      }
    } else {
      const float* p0 = L0.pstash + (size_t)r0 * L0.Np;
      for (int i = tid; i < R * L0.Np; i += SAC_THREADS) P0[(i / L0.Np) * ldp0 + i % L0.Np] = ldf<false>(p0 + i);
      const float* p1 = L1.pstash + (size_t)r0 * L1.Np + h * HH;
      for (int i = tid; i < R * HH; i += SAC_THREADS)
        P1[(i / HH) * ldp1 + i % HH] = ldf<false>(p1 + (i / HH) * L1.Np + i % HH);
    }
    if (tid < R) lpB[tid] = ldf<false>(E.lp_st + par * E.Br + r0 + tid);
  }
  // the head stash of this thread's (row, dim) and the critics' output biases,
  // loaded now: after the critics' hand-off they would be one more round trip
  float hsv[4] = {0.f, 0.f, 0.f, 0.f};
  if (tid < R * A && r0 + tid / A < E.Br) {
    const float* hs = E.head_st + (size_t)(r0 + tid / A) * 4 * A;
#pragma unroll
    for (int q = 0; q < 4; ++q) hsv[q] = ldf<false>(hs + q * A + tid % A);
  }
  const float bq1 = ldf<false>(E.net[NET_Q1].l[2].bias), bq2 = ldf<false>(E.net[NET_Q2].l[2].bias);
  __syncthreads();
  STAMP(34);
  // combine the critics' unit-seed partials with the min-Q weights (L_pi = mean(alpha logpi - min Q))
  // the critics' parts, summed in part order by every consumer
  const AS_G uint64_t* c1p[WQ];
  const AS_G uint64_t* c2p[WQ];
#pragma unroll
  for (int p = 0; p < WQ; ++p) {
    c1p[p] = gs_at(E, GS_C1, rbi, p);
    c2p[p] = gs_at(E, GS_C2, rbi, p);
  }
  if (R * A <= 64) {  // uniform: wave 0 holds every (row, action dim) lane
    // ONE poll for everything this block takes from the critics: lane i = (r, j)
    // polls the da partials of (r, j) and lanes < R also the q partials of row
    // tid (lanes >= R re-poll row 0's: harmless), so the da values arrive with
    // the q values instead of one more round trip after them.  Row r's min-Q
    // weights then come from lane r by a cross-lane read.
    if (tid < 64) {
      const bool live = tid < R * A;
      const int i = live ? tid : 0, r = i / A, rq = tid < R ? tid : 0;
      const AS_G uint64_t* gg[4 * WQ];
#pragma unroll
      for (int p = 0; p < WQ; ++p) {
        gg[p] = c1p[p] + i;
        gg[WQ + p] = c2p[p] + i;
        gg[2 * WQ + p] = c1p[p] + R * A + rq;
        gg[3 * WQ + p] = c2p[p] + R * A + rq;
      }
      float gv[4 * WQ];
      gran_getn1<4 * WQ>(E, gg, ep, gv);
      float term = 0.f, w1 = 0.f, w2 = 0.f;
      if (tid < R) {
        const bool v = tid < nvalid;
        const AS_C NetDev& q1n = E.net[NET_Q1];
        const AS_C NetDev& q2n = E.net[NET_Q2];
        float q1p = gv[2 * WQ], q2p = gv[3 * WQ];
#pragma unroll
        for (int p = 1; p < WQ; ++p) {
          q1p += gv[2 * WQ + p];
          q2p += gv[3 * WQ + p];
        }
        q1p += bq1;
        q2p += bq2;
        const float q1 = q1n.out_act == ACT_ID ? q1p : act_fwd(q1n.out_act, q1p);
        const float q2 = q2n.out_act == ACT_ID ? q2p : act_fwd(q2n.out_act, q2p);
        const float m = fmin_nan(q1, q2);
        term = v ? alpha32 * lpB[tid] - m : 0.f;
        const float gm = v ? -1.0f / (float)B : 0.f;
        w1 = (q1 == q2) ? gm * 0.5f : (q1 > q2 ? 0.f : gm);
        w2 = (q1 == q2) ? gm * 0.5f : (q1 < q2 ? 0.f : gm);
        if (q1n.out_act != ACT_ID) w1 = act_bwd(q1n.out_act, q1p, w1);
        if (q2n.out_act != ACT_ID) w2 = act_bwd(q2n.out_act, q2p, w2);
      }
      term = wave_sum(term);
      if (tid == 0 && h == 0) st_f<false>(E.lossp + (par * E.nrt + rbi) * 4 + 2, term);
      const float w1r = __shfl(w1, r, 64), w2r = __shfl(w2, r, 64);
      if (live) {
        float da1 = gv[0], da2 = gv[WQ];
#pragma unroll
        for (int p = 1; p < WQ; ++p) {
          da1 += gv[p];
          da2 += gv[WQ + p];
        }
        gaB[i] = w1r * da1 + w2r * da2;
      }
    }
    __syncthreads();
  } else {
  if (tid < 64) {
    float term = 0.f;
    if (tid < R) {
      const bool v = tid < nvalid;
      const AS_C NetDev& q1n = E.net[NET_Q1];
      const AS_C NetDev& q2n = E.net[NET_Q2];
      const AS_G uint64_t* gg[2 * WQ];
#pragma unroll
      for (int p = 0; p < WQ; ++p) {
        gg[p] = c1p[p] + R * A + tid;
        gg[WQ + p] = c2p[p] + R * A + tid;
      }
      float gv[2 * WQ];
      gran_getn<2 * WQ>(E, gg, ep, gv);
      float q1p = gv[0], q2p = gv[WQ];
#pragma unroll
      for (int p = 1; p < WQ; ++p) {
        q1p += gv[p];
        q2p += gv[WQ + p];
      }
      q1p += bq1;
      q2p += bq2;
      const float q1 = q1n.out_act == ACT_ID ? q1p : act_fwd(q1n.out_act, q1p);
      const float q2 = q2n.out_act == ACT_ID ? q2p : act_fwd(q2n.out_act, q2p);
      const float m = fmin_nan(q1, q2);
      term = v ? alpha32 * lpB[tid] - m : 0.f;
      const float gm = v ? -1.0f / (float)B : 0.f;
      float w1 = (q1 == q2) ? gm * 0.5f : (q1 > q2 ? 0.f : gm);
      float w2 = (q1 == q2) ? gm * 0.5f : (q1 < q2 ? 0.f : gm);
      if (q1n.out_act != ACT_ID) w1 = act_bwd(q1n.out_act, q1p, w1);
      if (q2n.out_act != ACT_ID) w2 = act_bwd(q2n.out_act, q2p, w2);
      g1B[tid] = w1;
      g2B[tid] = w2;
    }
    term = wave_sum(term);
    if (tid == 0 && h == 0) st_f<false>(E.lossp + (par * E.nrt + rbi) * 4 + 2, term);
  }
  __syncthreads();
  for (int i = tid; i < R * A; i += SAC_THREADS) {
    const int r = i / A;
    const AS_G uint64_t* gg[2 * WQ];
#pragma unroll
    for (int p = 0; p < WQ; ++p) {
      gg[p] = c1p[p] + i;
      gg[WQ + p] = c2p[p] + i;
    }
    float gv[2 * WQ];
    gran_getn<2 * WQ>(E, gg, ep, gv);  // all in by now (the q granules above came after them)
    float da1 = gv[0], da2 = gv[WQ];
#pragma unroll
    for (int p = 1; p < WQ; ++p) {
      da1 += gv[p];
      da2 += gv[WQ + p];
    }
    gaB[i] = g1B[r] * da1 + g2B[r] * da2;
  }
  __syncthreads();
  }
  STAMP(39);
  // squashed-Gaussian head backward (models.py:79-87), one lane per (row, action dim)
  static_assert(SAC_ROWS * 32 <= SAC_THREADS, "one (row, action dim) per thread");
  if (tid < R * A) {
    const int i = tid;
    const int r = i / A, j = i % A;
    const bool v = r < nvalid;
    const float gl = v ? alpha32 * (1.0f / (float)B) : 0.f;
    const float lo = E.ls_min, hi = E.ls_max, scale = E.scale;
    const float mu = hsv[0], lsr = hsv[1], z = hsv[2], e = hsv[3];
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
    goutB[r * ldo + j] = v ? g_mu : 0.f;
    goutB[r * ldo + A + j] = (v && in_range) ? g_ls : 0.f;
  }
  {
    const int NOp = L2.Np, pad = NOp - 2 * A;
    for (int i = tid; i < R * pad; i += SAC_THREADS) goutB[(i / pad) * ldo + 2 * A + i % pad] = 0.f;
  }
  __syncthreads();
  // layer 2 dY^T (= dOut) + bias partials: half 0
  if (h == 0) store_T<T, R>(goutB, ldo, L2.Np, L2.N, L2.GT, Bp, r0, nvalid, L2.dbp);
  // dY1 (this half) = act'(P1) * (dOut W2[:, half])
  const int act = pi.hid_act;
  gemm_hs<T, 1, NCH_32, false>(goutB, ldo, wt2, &ht2, [&](int j, int col, const f32x4& acc) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (((threadIdx.x & 63) >> 4) << 2) + i;
      float v = acc[i];
      if (act == ACT_RELU && !(P1[r * ldp1 + col] > 0.f)) v = 0.f;
      U1[r * ldu1 + col] = v;
    }
  });
  if (act != ACT_RELU && act != ACT_ID) act_pass_bwd<R>(U1, ldu1, P1, ldp1, HH >> 4, HH, act);
  __syncthreads();
  store_T<T, R>(U1, ldu1, HH, HH, (T*)L1.GT + (size_t)h * HH * Bp, Bp, r0, nvalid, L1.dbp ? L1.dbp + h * HH : nullptr, nullptr, L1.N);
  // dY0 partial = act'(P0) * (dY1 W1[half])
  gemm_hs<T, 2, NCH_HH, false>(U1, ldu1, wt1, &ht1, [&](int j, int col, const f32x4& acc) {
    const bool kv = col < L1.K;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (((threadIdx.x & 63) >> 4) << 2) + i;
      float v = kv ? acc[i] : 0.f;
      if (act == ACT_RELU && !(P0[r * ldp0 + col] > 0.f)) v = 0.f;
      Xb[r * ld + col] = v;
    }
  });
  if (act != ACT_RELU && act != ACT_ID) act_pass_bwd<R>(Xb, ld, P0, ldp0, L1.Kp >> 4, L1.K, act);
  __syncthreads();
  store_T<T, R>(Xb, ld, L0.Np, L0.N, L0.GT, WP * Bp, h * Bp + r0, nvalid, L0.dbp);
  STAMP(35);
}

template <typename T>
__global__ void __launch_bounds__(SAC_THREADS) sac_actor_split(const EngineDev* __restrict__ Ep, sac_replay rb) {
  PREFETCH_ARG(Ep);
  const AS_C EngineDev& E = *(const AS_C EngineDev*)Ep;
  extern __shared__ float lds_raw[];
  const int bid = (int)blockIdx.x;
  const int nrole = (2 * split_wcq(sizeof(T)) + split_wc(sizeof(T))) * E.nrt;  // critics' + pi's parts x nrt
  if (bid >= nrole) {
    stage_next_batch(E, rb, bid - nrole, (lf*)lds_raw, *GPC(uint64_t, E.rng_step));
  } else {
    const uint64_t step = *GPC(uint64_t, E.rng_step);
    actor_split_body<T>(Ep, bid, StepCtx{step, *GPC(uint32_t, E.sync) + 1u, (int)(step & 1)});
  }
  phase_c_done(E);
  END_STAMP(61);
}
