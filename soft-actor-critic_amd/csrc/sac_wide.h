// sac_wide.h — large-batch phases A and C as layer-synchronous GEMM stages.
// Included by sac_engine.hip only (after sac_phases.h).  Design: DESIGN.md §3.6.
//
// At large batches (C3: B = 4096, reference notebooks/configs/bipedal_walker.yaml
// with train.batch_size 4096) the step is MFMA work, not a hand-off chain, and
// the per-row-tile kernels are per-CU weight-stream bound (every workgroup
// streams all five networks' weights for 16 rows).  Here each dense layer of
// the step (reference sac/agent.py:195-260, models.py:30-92) is one GEMM stage:
// 64-row x 64-column output tiles over the whole chip, K staged through LDS in
// 32-deep blocks (double-buffered, one barrier per block), and every
// elementwise step fused into a stage's prologue or epilogue:
//   forward      P = X W^T + b  -> pre-activation P (row-major fp32), act(P)^T
//                into the X^T stash of the update tiles, and for the last
//                hidden layer the output layer as per-column-block partials
//                (OUTP[cb][row][j] = sum_{n in cb} Wout[j][n] act(P[row][n]));
//   backward     dX = dY W -> dY_prev = act'(P_prev) * dX, stored as the dY^T
//                stash + per-16-row bias partials of the update tiles, and for
//                the critics' layer 0 the action-column product (d a~ partials);
//   output layer the first backward stage generates its own A operand from the
//                last hidden pre-activation: dY[r][n] = act'(P[r][n]) *
//                sum_j D[r][j] Wout[j][n], with D the row's output-layer seed
//                (target y + MSE seed, min-Q weights, or the squashed-Gaussian
//                head backward) computed by the item's row prologue.
// Stages of one step (two hidden layers; deeper nets add stages):
//   A: gather | fwd L0 (pi on [s'; s], Q1, Q2) | fwd L1 (+ output partials) |
//      pi heads | Qt fwd L0 | Qt fwd L1 | critic backward (y, seeds, losses)
//   B: sac_critic_update (unchanged)
//   C: critic fwd L0 | fwd L1 | critic dX (min-Q weights, d a~ partials) |
//      pi backward (head backward) -- the last block advances the step
//   D: sac_actor_update + alpha (unchanged)
// The stashes the update tiles read (X^T, dY^T, bias partials per 16-row tile,
// loss partials, log pi) have exactly the row-tile kernels' layout, so phases B
// and D are shared.
#pragma once

#define WG_T 256   // threads per stage workgroup (4 waves)
#define WBM 64     // rows per output tile
#define WBN 64     // columns per output tile
#define WLDE 68    // LDS row stride of the epilogue tile
#define WLDD 17    // LDS row stride of the per-row seeds (J <= 16)
#define WJMAX 16
#define WWS 1088   // floats of the epilogue weight slices (OUTP: Nout x 64; DA: A x 64)

enum WAMode { WA_PLAIN = 0, WA_ACT = 1, WA_OUTBWD = 2 };
enum WEMode { WE_FWD = 0, WE_BWD = 1 };
enum WRowPro { WR_NONE = 0, WR_YSEED = 1, WR_MINQ = 2, WR_PIHEAD = 3 };

// Buffers of the wide path that the row prologues, the gather and the head
// kernel need (the GEMM stages get everything else from their job).
struct WideDev {
  int B, Bp, Brw, nrt, O, A;
  int ldpi0, ldq0;   // row strides of the layer-0 inputs (Kp of pi / Q layer 0)
  float* Xpi0;       // [2 Brw][ldpi0]: s' rows [0, B), s rows [Brw, Brw + B)
  float* Xq0;        // [Brw][ldq0]: (s, a) of the critics
  float* Xqt0;       // [Brw][ldq0]: (s', a~') of the target critics (a~' from the head kernel)
  float* Xc0;        // [Brw][ldq0]: (s, a~) of phase C's critics
  float* R;          // [Brw] rewards
  float* Dn;         // [Brw] dones
  float* LP2;        // [Brw] log pi(a~'|s')
  float* PIOP;       // [Brw][2A] pi output pre-activation of the actor rows (pi out_act != identity)
  int ncb_pi, ncb_q;   // column blocks of pi's / Q's last hidden layer
  long cbs_pi, cbs_q;  // floats between column blocks of the partial outputs
  float* OUTPpi;       // [ncb_pi][2 Brw][2A]
  float* OUTPq[2];     // [ncb_q][Brw][1]: critics, phase A
  float* OUTPqt[2];    // target critics
  float* OUTPc[2];     // critics on (s, a~), phase C
  int ncb_da;          // column blocks of the critics' layer 0 outputs
  long cbs_da;
  float* DA[2];        // [ncb_da][Brw][A]: phase C critics' seeded d a~ partials
  // output layers' dY^T / bias partials written by the row prologues
  void* GTq_out[2];
  float* dbpq_out[2];
  void* GTpi_out;
  float* dbppi_out;
  int stamp_stage;  // stamps builds: the stage index that writes stamps (SAC_WIDE_STAMP_STAGE)
  const uint64_t* rng_step;  // = EngineDev::rng_step (read through the prefetched WideDev lines)
};

// One GEMM of a stage: output tiles (row block rb, column block cb), items
// [item0, item0 + nrb * ncb) of the stage's grid.
struct WJob {
  int M, K, Kp, N, Np;  // rows (multiple of 64); reduction (valid, padded to 32); outputs (valid, padded)
  int nrb, ncb, item0;
  // A operand: X [M][ldx] fp32 (WA_ACT: act(X); WA_OUTBWD: X = P of the layer, see header)
  int amode, aact;
  const float* X;
  int ldx;
  const float* Wo;  // WA_OUTBWD: output layer weights [J][ldwo] (fp32 master)
  int ldwo, J;
  int rowpro, qi;   // row prologue (WA_OUTBWD seeds) and its critic index
  // B operand: fragment-packed matrix (forward: Wc [Np][Kp]; backward: WTc [Kp][Np])
  const void* Wp;
  int tcols;
  const float* bias;  // forward
  int emode;
  // forward epilogue
  float* P;  // [M][ldp] pre-activation (null: not kept)
  int ldp;
  int oact;  // activation of the layer (X^T stash, output partials)
  void* XT;  // act(P)^T (T) of rows >= xt_row0 at column r - xt_row0; row stride xt_ld
  int xt_row0;
  long xt_ld;
  long xt_par;  // elements between the two step-parity copies (pi: phase D of step k reads one)
  const float* Wout;  // output layer [Nout][ldwout] (fp32 master) for OUTP
  int ldwout, Nout;
  float* OUTP;
  long outp_cb;
  // backward epilogue
  const float* Pprev;  // pre-activation of the layer below (act' of the dX); pact < 0: none
  int ldpp, pact;
  float* DY;  // [M][lddy] dY of the layer below (for a following backward stage)
  int lddy;
  void* GT;   // dY^T (T), row stride gt_ld = Bp
  long gt_ld;
  float* dbp;  // [nrt][dbp_ld] per-16-row bias partials
  int dbp_ld;
  const float* W0a;  // critics' layer 0 [N0][ldw0]: d a~ partials through the action columns
  int ldw0, a_off;
  float* DA;
  long da_cb;
  void* AGT;   // WA_OUTBWD: the generated operand's dY^T and bias partials (cb == 0 items)
  float* Adbp;
  int adbp_ld;
  int p_row0;  // forward: P is stored for rows >= p_row0 only
  int nbuf;    // K-block buffers in LDS (2..4): nbuf - 1 blocks in flight ahead of the MFMAs
};

static_assert(sizeof(WJob) <= 448, "extend wide_prefetch");
static_assert(sizeof(WideDev) <= 384, "extend wide_prefetch");

// Every 64-B line of the stage's job descriptor and of WideDev touched once at
// entry with back-to-back scalar loads (one latency instead of one per line
// at first use; see prefetch_engine).
__device__ __forceinline__ void wide_prefetch(const void* job, const void* wd) {
  const uint64_t a = (uint64_t)(uintptr_t)job, b = (uint64_t)(uintptr_t)wd;
  asm volatile("s_load_dword s95, %0, 0\n\t" "s_load_dword s95, %0, 64\n\t" "s_load_dword s95, %0, 128\n\t"
               "s_load_dword s95, %0, 192\n\t" "s_load_dword s95, %0, 256\n\t" "s_load_dword s95, %0, 320\n\t"
               "s_load_dword s95, %0, 384\n\t" "s_load_dword s95, %1, 0\n\t" "s_load_dword s95, %1, 64\n\t"
               "s_load_dword s95, %1, 128\n\t" "s_load_dword s95, %1, 192\n\t" "s_load_dword s95, %1, 256\n\t"
               "s_load_dword s95, %1, 320\n\t" "s_waitcnt lgkmcnt(0)" :: "s"(a), "s"(b) : "s95", "memory");
}

// In-kernel stamps of one stage (stamps builds: the stage whose index is
// WideDev::stamp_stage writes s_memrealtime at slot i of its block's row)
#ifdef SAC_STAMPS
#define WSTAMP(i)                                                                                          \
  do {                                                                                                     \
    if (wst && threadIdx.x == 0) GP(long long, E.stamps)[blockIdx.x * 64 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define WSTAMP(i) \
  do {            \
  } while (0)
#endif

__device__ __forceinline__ bool wrow_ok(const AS_C WideDev& W, int r) { return r % W.Brw < W.B; }

// T-typed 4-element store of 4 consecutive batch columns (16 B fp32 / 8 B bf16)
template <typename T>
__device__ __forceinline__ void st4(void* base, size_t off, const f32x4& v) {
  if constexpr (sizeof(T) == 4) {
    *(AS_G f32x4*)((AS_G float*)base + off) = v;
  } else {
    typedef bf16 bf16x4 __attribute__((ext_vector_type(4)));
    bf16x4 h;
    h[0] = (bf16)v[0]; h[1] = (bf16)v[1]; h[2] = (bf16)v[2]; h[3] = (bf16)v[3];
    *(AS_G bf16x4*)((AS_G bf16*)base + off) = h;
  }
}

// plain loads / stores of the buffers the stages hand to each other (every
// hand-off crosses a launch boundary)
__device__ __forceinline__ float ldh(const float* p) { return *GPC(float, p); }
__device__ __forceinline__ void sth(float* p, float v) { *GP(float, p) = v; }
__device__ __forceinline__ void st16h(float* base, size_t off, f32x4 v) { *(AS_G f32x4*)(GP(float, base) + off) = v; }
__device__ __forceinline__ f32x4 ld16h(const float* base, size_t off) { return *(const AS_G f32x4*)(GPC(float, base) + off); }

// ---------------------------------------------------------------------------- row prologues
// D[r][0..J) of the item's rows into Dl (LDS), plus the side outputs of the
// output layer (cb == 0 items only: losses, y, the output layer's dY^T / bias).
template <typename T>
__device__ __forceinline__ void wide_rowpro(const AS_C EngineDev& E, const AS_C WideDev& W, const AS_C WJob& jb,
                                            int row0, int cb, int par, lf* Dl) {
  const int tid = threadIdx.x, B = W.B, A = W.A;
  const float alpha32 = (float)*GPC(double, E.alpha_state + 1);
  if (jb.rowpro == WR_YSEED) {
    // target y (agent.py:195-211) and critic qi's MSE seed 2 (q - y) / B (agent.py:221-234)
    if (tid < 64) {
      const int lr = row0 + tid;
      const bool v = lr < B;
      const int qi = jb.qi;
      const AS_C NetDev& qt1 = E.net[NET_Q1T];
      const AS_C NetDev& qt2 = E.net[NET_Q2T];
      const AS_C NetDev& q = E.net[NET_Q1 + qi];
      float seed = 0.f, sq = 0.f, y = 0.f;
      if (v) {
        float a1 = 0.f, a2 = 0.f, aq = 0.f;
        for (int c0 = 0; c0 < W.ncb_q; c0 += 4) {  // every load of a batch of 4 blocks in flight together
          float x1[4], x2[4], xq[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int c = c0 + u < W.ncb_q ? c0 + u : W.ncb_q - 1;
            x1[u] = ldh(W.OUTPqt[0] + c * W.cbs_q + lr);
            x2[u] = ldh(W.OUTPqt[1] + c * W.cbs_q + lr);
            xq[u] = ldh(W.OUTPq[qi] + c * W.cbs_q + lr);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (c0 + u < W.ncb_q) {
              a1 += x1[u];
              a2 += x2[u];
              aq += xq[u];
            }
        }
        const float t1 = act_fwd(qt1.out_act, a1 + GPC(float, qt1.l[qt1.L - 1].bias)[0]);
        const float t2 = act_fwd(qt2.out_act, a2 + GPC(float, qt2.l[qt2.L - 1].bias)[0]);
        const float qp = aq + GPC(float, q.l[q.L - 1].bias)[0];
        y = ldh(W.R + lr) + (E.gamma * (1.f - ldh(W.Dn + lr))) * (fmin_nan(t1, t2) - alpha32 * ldh(W.LP2 + lr));
        const float d = act_fwd(q.out_act, qp) - y;
        sq = d * d;
        seed = (2.0f / (float)B) * d;
        if (q.out_act != ACT_ID) seed = act_bwd(q.out_act, qp, seed);
      }
      Dl[tid * WLDD] = seed;
      if (cb == 0) {
        if (qi == 0 && v) GP(float, E.stats)[4 + lr] = y;
        if (lr < W.Bp) {
          if constexpr (sizeof(T) == 4) GP(float, W.GTq_out[qi])[lr] = seed;
          else GP(bf16, W.GTq_out[qi])[lr] = (bf16)seed;
        }
        float s = seed;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          s += __shfl_xor(s, o, 64);
          sq += __shfl_xor(sq, o, 64);
        }
        const int rt = lr >> 4;
        if ((tid & 15) == 0 && rt < W.nrt) {
          if (W.dbpq_out[qi]) GP(float, W.dbpq_out[qi])[rt] = s;
          GP(float, E.lossp)[(par * E.nrt + rt) * 4 + qi] = sq;
        }
      }
    }
  } else if (jb.rowpro == WR_MINQ) {
    // min-Q weights of L_pi = mean(alpha log pi - min Q) (agent.py:244-252), ties split
    if (tid < 64) {
      const int lr = row0 + tid;
      const bool v = lr < B;
      const AS_C NetDev& q1 = E.net[NET_Q1];
      const AS_C NetDev& q2 = E.net[NET_Q2];
      float a1 = 0.f, a2 = 0.f;
      if (v)
        for (int c0 = 0; c0 < W.ncb_q; c0 += 4) {  // every load of a batch of 4 blocks in flight together
          float x1[4], x2[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int c = c0 + u < W.ncb_q ? c0 + u : W.ncb_q - 1;
            x1[u] = ldh(W.OUTPc[0] + c * W.cbs_q + lr);
            x2[u] = ldh(W.OUTPc[1] + c * W.cbs_q + lr);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (c0 + u < W.ncb_q) {
              a1 += x1[u];
              a2 += x2[u];
            }
        }
      const float p1 = a1 + GPC(float, q1.l[q1.L - 1].bias)[0], p2 = a2 + GPC(float, q2.l[q2.L - 1].bias)[0];
      const float o1 = act_fwd(q1.out_act, p1), o2 = act_fwd(q2.out_act, p2);
      const float m = fmin_nan(o1, o2);
      const float gm = v ? -1.0f / (float)B : 0.f;
      float g1 = (o1 == o2) ? gm * 0.5f : (o1 > o2 ? 0.f : gm);
      float g2 = (o1 == o2) ? gm * 0.5f : (o1 < o2 ? 0.f : gm);
      if (q1.out_act != ACT_ID) g1 = act_bwd(q1.out_act, p1, g1);
      if (q2.out_act != ACT_ID) g2 = act_bwd(q2.out_act, p2, g2);
      Dl[tid * WLDD] = jb.qi ? g2 : g1;
      if (cb == 0 && jb.qi == 0) {
        float term = v ? alpha32 * GPC(float, E.lp_st)[par * E.Br + lr] - m : 0.f;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) term += __shfl_xor(term, o, 64);
        const int rt = lr >> 4;
        if ((tid & 15) == 0 && rt < W.nrt) GP(float, E.lossp)[(par * E.nrt + rt) * 4 + 2] = term;
      }
    }
  } else if (jb.rowpro == WR_PIHEAD) {
    // squashed-Gaussian head backward (models.py:79-87 under agent.py:255-257):
    // d(mu), d(log_std) of each actor row from d a~ (the critics' seeded partials)
    const AS_C NetDev& pi = E.net[NET_PI];
    for (int i = tid; i < 64 * A; i += WG_T) {
      const int r = i / A, j = i % A, lr = row0 + r;
      const bool v = lr < B;
      float gm = 0.f, gs = 0.f;
      if (v) {
        float d1 = 0.f, d2 = 0.f;
        for (int c0 = 0; c0 < W.ncb_da; c0 += 4) {  // every load of a batch of 4 blocks in flight together
          float x1[4], x2[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int c = c0 + u < W.ncb_da ? c0 + u : W.ncb_da - 1;
            x1[u] = ldh(W.DA[0] + c * W.cbs_da + (size_t)lr * A + j);
            x2[u] = ldh(W.DA[1] + c * W.cbs_da + (size_t)lr * A + j);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (c0 + u < W.ncb_da) {
              d1 += x1[u];
              d2 += x2[u];
            }
        }
        const float ga = d1 + d2;
        const float gl = alpha32 * (1.0f / (float)B);
        const AS_G float* h = GPC(float, E.head_st) + (size_t)lr * 4 * A;
        const float lo = E.ls_min, hi = E.ls_max, scale = E.scale;
        const float mu = h[j], lsr = h[A + j], z = h[2 * A + j], e = h[3 * A + j];
        const float ls = lsr < lo ? lo : (lsr > hi ? hi : lsr);
        const float sd = expf(ls);
        const float t = tanhf(z);
        const float diff = z - mu, var = sd * sd;
        float g_z = (ga * scale) * (1.f - t * t);
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
        gm = g_mu;
        gs = in_range ? g_ls : 0.f;
        if (pi.out_act != ACT_ID) {
          gm = act_bwd(pi.out_act, GPC(float, W.PIOP)[(size_t)lr * 2 * A + j], gm);
          gs = act_bwd(pi.out_act, GPC(float, W.PIOP)[(size_t)lr * 2 * A + A + j], gs);
        }
      }
      Dl[r * WLDD + j] = gm;
      Dl[r * WLDD + A + j] = gs;
      if (cb == 0 && lr < W.Bp) {
        if constexpr (sizeof(T) == 4) {
          GP(float, W.GTpi_out)[(size_t)j * W.Bp + lr] = gm;
          GP(float, W.GTpi_out)[(size_t)(A + j) * W.Bp + lr] = gs;
        } else {
          GP(bf16, W.GTpi_out)[(size_t)j * W.Bp + lr] = (bf16)gm;
          GP(bf16, W.GTpi_out)[(size_t)(A + j) * W.Bp + lr] = (bf16)gs;
        }
      }
    }
    if (cb == 0 && W.dbppi_out) {  // bias partials of the output layer: per 16-row tile, column j < 2A
      __syncthreads();
      for (int i = tid; i < 4 * 2 * A; i += WG_T) {
        const int rt = i / (2 * A), j = i % (2 * A);
        const int grt = row0 / 16 + rt;
        float s = 0.f;
        for (int r = 0; r < 16; ++r) s += Dl[(rt * 16 + r) * WLDD + j];
        if (grt < W.nrt) GP(float, W.dbppi_out)[(size_t)grt * 2 * A + j] = s;
      }
    }
  }
}

// ---------------------------------------------------------------------------- one GEMM item
// K is staged through LDS in blocks of WK<T>::KB by LDS-DMA (global_load_lds,
// 16 B per lane, no register staging): the A block as fragment pieces (16 rows
// x 4 k per lane group, lane-linear in exactly the order a wave reads one MFMA
// operand), the B block as the packed weight fragments themselves.  Two
// buffers, one barrier per block; block kb + 1 lands while block kb is
// multiplied.  Every wave issues the same number of DMAs per block (a piece
// past Kp or a column tile past Np re-loads a valid address and is never
// multiplied), so blocks in flight are counted with vmcnt.
template <typename T>
struct WK {
  static constexpr int KC = MM<T>::KC, KL = MM<T>::KL;
  static constexpr int KB = sizeof(T) == 4 ? 32 : 64;  // K per block
  static constexpr int NCH = KB / KC;                   // MFMA chunks per block
  static constexpr int PR = KB / 16;                    // A pieces per 16-row tile
  static constexpr int APC = 4 * PR, BPC = 4 * NCH;     // A / B pieces per block
  static constexpr int ABUF = APC * 256, BUF = ABUF + BPC * 256;  // floats
  // in-block k of lane group gg's 4 elements in A piece h (fp32: piece = chunk;
  // bf16: chunk h / 2, elements 4 (h & 1).. of the lane's 8)
  static __device__ __forceinline__ int koff(int h, int gg) {
    if constexpr (sizeof(T) == 4) return h * 16 + gg * 4;
    else return (h >> 1) * 32 + gg * 8 + (h & 1) * 4;
  }
  static __device__ __forceinline__ int chunk(int h) { return sizeof(T) == 4 ? h : h >> 1; }
  // LDS float index of A element (row r, in-block k) in a block image
  static __device__ __forceinline__ int aloc(int r, int k) {
    int h, gg;
    if constexpr (sizeof(T) == 4) {
      h = k >> 4;
      gg = (k & 15) >> 2;
    } else {
      h = (k >> 5) * 2 + ((k >> 2) & 1);
      gg = (k & 31) >> 3;
    }
    return ((r >> 4) * PR + h) * 256 + (gg * 16 + (r & 15)) * 4 + (k & 3);
  }
};
static_assert(64 * WLDE <= 2 * WK<float>::BUF && 64 * WLDE <= 2 * WK<bf16>::BUF, "epilogue tile aliases the K buffers");

template <int AUX = 0>
__device__ __forceinline__ void glds16(const AS_G void* g, lf* l) {
  __builtin_amdgcn_global_load_lds(g, (AS_L void*)l, 16, 0, AUX);
}
// hidden activation and its derivative; HR: every hidden layer of the stage is ReLU
template <bool HR>
__device__ __forceinline__ float hact(int a, float p) {
  if constexpr (HR) return p > 0.f ? p : 0.f;
  else return act_fwd(a, p);
}
template <bool HR>
__device__ __forceinline__ float hactb(int a, float p, float g) {
  if constexpr (HR) return p > 0.f ? g : 0.f;
  else return act_bwd(a, p, g);
}

// 64 rows x 64 columns of Et dotted with No weight rows Ws[j][0..64): four
// threads per row, 16 columns each, reduced by two shuffles; act: apply the
// hidden activation to Et first (output-layer partials of a forward stage)
template <bool HR, bool ACTX>
__device__ __forceinline__ void wide_rowdot(const lf* Et, const lf* Ws, int No, int aact, float* dst) {
  const int tid = threadIdx.x, r = tid >> 2, kq = tid & 3;
  float x[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x4 v = *(const AS_L f32x4*)(Et + r * WLDE + kq * 16 + q * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) x[q * 4 + e] = ACTX ? hact<HR>(aact, v[e]) : v[e];
  }
  for (int j = 0; j < No; ++j) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 w = *(const AS_L f32x4*)(Ws + j * WBN + kq * 16 + q * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) s += x[q * 4 + e] * w[e];
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (kq == (j & 3)) sth(dst + (size_t)r * No + j, s);
  }
}

// item -> (row block, column block): the column blocks of one row block 8
// items apart, i.e. on one XCD under round-robin placement (speed only), so
// the row block's A operand is fetched into one L2 and re-read from there
__device__ __forceinline__ void wide_rbcb(const AS_C WJob& jb, int it, int& rb, int& cb) {
  if ((jb.nrb & 7) == 0 && (jb.item0 & 7) == 0) {
    const int grp = it / (8 * jb.ncb), rem = it % (8 * jb.ncb);
    cb = rem >> 3;
    rb = grp * 8 + (rem & 7);
  } else {
    rb = it / jb.ncb;
    cb = it % jb.ncb;
  }
}

template <typename T, int AM, bool HR>
__device__ __forceinline__ void wide_item(const AS_C EngineDev& E, const AS_C WideDev& W, const AS_C WJob& jb, int it,
                                          lf* lds, int par, bool wst) {
  typedef WK<T> K_;
  constexpr int KC = K_::KC, KL = K_::KL, KB = K_::KB, NCH = K_::NCH, PR = K_::PR;
  static_assert(3 * (PR + NCH) < 64, "vmcnt counts blocks in flight");
  constexpr bool XF = AM == WA_OUTBWD || (AM == WA_ACT && !HR);  // A transformed in place after landing
  typedef typename MM<T>::Frag F;
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
  const int c = lane & 15, g = lane >> 4;
  const int wr = wave >> 1, wc = wave & 1;
  int rb, cb;
  wide_rbcb(jb, it, rb, cb);
  const int row0 = rb * WBM, col0 = cb * WBN;
  const int rbase = row0 % W.Brw;  // row r of the block is a batch row iff rbase + r < B
  const int NT = jb.Np >> 4, t0 = col0 >> 4, nchT = jb.tcols / KC;
  const int Kp = jb.Kp, nkb = (Kp + KB - 1) / KB;
  const int NB = jb.nbuf;
  lf* Ws = lds + NB * K_::BUF;  // the epilogue's weight slices (WWS floats)
  lf* Dl = Ws + WWS;           // [64][WLDD] row seeds (WA_OUTBWD)
  lf* Wol = Dl + 64 * WLDD;    // [J][Kp] output layer weights (WA_OUTBWD)

  // ---- LDS-DMA sources: this wave's A pieces wave + 4 i, B pieces wave + 4 i
  const AS_G float* xa[PR];
#pragma unroll
  for (int i = 0; i < PR; ++i) {
    const int pa = wave + 4 * i, rt = pa / PR, h = pa % PR;
    xa[i] = GPC(float, jb.X) + (size_t)(row0 + rt * 16 + c) * jb.ldx + K_::koff(h, g);
  }
  const AS_G T* wb[NCH];
  bool bv[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int pb = wave + 4 * i, ct = pb / NCH, ch = pb % NCH, t = t0 + ct;
    bv[i] = t < NT;
    wb[i] = GPC(T, jb.Wp) + ((size_t)((bv[i] ? t : 0) * nchT + ch) * 64 + lane) * KL;
  }
  auto issue = [&](int kb, int buf) __attribute__((always_inline)) {
    lf* Aq = lds + buf * K_::BUF;
    lf* Bq = Aq + K_::ABUF;
    const int k0 = kb * KB;
#pragma unroll
    for (int i = 0; i < PR; ++i) {
      const int pa = wave + 4 * i, h = pa % PR;
      const bool v = k0 + K_::chunk(h) * KC < Kp;
      glds16(xa[i] + (v ? k0 : -K_::koff(h, g)), Aq + pa * 256);  // past Kp: the row's first 4 k
    }
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int pb = wave + 4 * i;
      const bool v = k0 + (pb % NCH) * KC < Kp;
      glds16(wb[i] + (v ? (size_t)kb * NCH * 64 * KL : 0), Bq + pb * 256);
    }
  };
  constexpr int CNT = PR + NCH;  // DMAs per wave per block
  // wait until this wave's DMAs of the block `ahead` blocks older than the
  // newest issued one have landed (vmcnt retires in issue order)
  auto wait_ahead = [&](int ahead) __attribute__((always_inline)) {
    if (ahead <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CNT) : "memory");
    else if (ahead == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * CNT) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * CNT) : "memory");
  };
  // a workgroup barrier that does not drain the DMAs in flight (__syncthreads
  // would wait vmcnt(0)): LDS traffic retired, then s_barrier
  auto bar = [&]() __attribute__((always_inline)) { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  // the output layer's weight slice [Nout][64] by DMA when the block's 64
  // columns are all inside the rows (issued first: retired by the first wait)
  const bool ws_dma = jb.OUTP && col0 + WBN <= jb.N && (jb.ldwout & 3) == 0 && ((uintptr_t)jb.Wout & 15) == 0;
  if (ws_dma) {
    const int j = 4 * wave + (lane >> 4);  // wave w: rows q0 + 4w..4w+3, 16 lanes x 16 B per row
    for (int q0 = 0; q0 < jb.Nout; q0 += 16)
      if (q0 + j < jb.Nout)
        glds16(GPC(float, jb.Wout) + (size_t)(q0 + j) * jb.ldwout + col0 + (lane & 15) * 4, Ws + (q0 + 4 * wave) * WBN);
  }
  for (int b = 0; b < NB && b < nkb; ++b) issue(b, b);

  // ---- prologue (under the first two blocks' DMA)
  const bool fwd = jb.emode == WE_FWD;
  float bias_r[2];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    const int n = col0 + wc * 32 + ct * 16 + c;
    bias_r[ct] = (fwd && n < jb.N) ? GPC(float, jb.bias)[n] : 0.f;
  }
  // the epilogue's weight slices, row-major [j][64 columns of this block]:
  // output layer columns (OUTP) or the critics' layer-0 action columns (DA)
  if (jb.OUTP && !ws_dma) {
    for (int i = tid; i < jb.Nout * WBN; i += WG_T) {
      const int j = i / WBN, k = i % WBN;
      Ws[i] = col0 + k < jb.N ? GPC(float, jb.Wout)[(size_t)j * jb.ldwout + col0 + k] : 0.f;
    }
  } else if (jb.DA) {
    for (int i = tid; i < W.A * WBN; i += WG_T) {
      const int j = i / WBN, k = i % WBN;
      Ws[i] = col0 + k < jb.N ? GPC(float, jb.W0a)[(size_t)(col0 + k) * jb.ldw0 + jb.a_off + j] : 0.f;
    }
  }
  // XF pass mapping: a thread transforms lanes pL, pL + 1 of the pieces of
  // row tile prt with h = (tid >> 7) + 2 i (its two rows are fixed)
  const int prt = (tid >> 5) & 3, pL = (tid & 31) * 2, pg = pL >> 4;
  const int J = jb.J;
  const int rA = prt * 16 + (pL & 15);  // the pass's two rows rA, rA + 1
  if constexpr (AM == WA_OUTBWD) {
    wide_rowpro<T>(E, W, jb, row0, cb, par, Dl);
    for (int i = tid; i < J * Kp; i += WG_T) {
      const int j = i / Kp, k = i % Kp;
      Wol[i] = k < jb.ldwo ? GPC(float, jb.Wo)[(size_t)j * jb.ldwo + k] : 0.f;
    }
    // (the loop's first barrier orders Dl / Wol before the first pass)
  }
  auto xform = [&](int kb, int buf) __attribute__((always_inline)) {
    lf* Aq = lds + buf * K_::BUF;
    const int k0 = kb * KB;
#pragma unroll
    for (int i = 0; i < PR / 2; ++i) {
      const int h = (tid >> 7) + 2 * i;
      if (k0 + K_::chunk(h) * KC >= Kp) continue;
      AS_L f32x4* q = (AS_L f32x4*)(Aq + (prt * PR + h) * 256 + pL * 4);
      f32x4 a = q[0], b = q[1];
      if constexpr (AM == WA_OUTBWD) {
        // dY[r][k] = act'(P[r][k]) * sum_j D[r][j] Wout[j][k]
        const int k = k0 + K_::koff(h, pg);
        f32x4 sa = {0.f, 0.f, 0.f, 0.f}, sb = {0.f, 0.f, 0.f, 0.f};
        for (int j = 0; j < J; ++j) {
          const f32x4 w = *(const AS_L f32x4*)(Wol + j * Kp + k);
          sa += Dl[rA * WLDD + j] * w;
          sb += Dl[(rA + 1) * WLDD + j] * w;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] = hactb<HR>(jb.aact, a[e], sa[e]);
          b[e] = hactb<HR>(jb.aact, b[e], sb[e]);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] = act_fwd(jb.aact, a[e]);
          b[e] = act_fwd(jb.aact, b[e]);
        }
      }
      q[0] = a;
      q[1] = b;
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto afrag = [&](const lf* Aq, int rt, int ch) __attribute__((always_inline)) -> F {
    constexpr bool RL = AM == WA_ACT && HR;  // ReLU applied as the fragment is read
    if constexpr (sizeof(T) == 4) {
      f32x4 v = *(const AS_L f32x4*)(Aq + (rt * PR + ch) * 256 + lane * 4);
      if constexpr (RL)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
      return v;
    } else {
      f32x4 u = *(const AS_L f32x4*)(Aq + (rt * PR + ch * 2) * 256 + lane * 4);
      f32x4 v = *(const AS_L f32x4*)(Aq + (rt * PR + ch * 2 + 1) * 256 + lane * 4);
      if constexpr (RL)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          u[e] = u[e] > 0.f ? u[e] : 0.f;
          v[e] = v[e] > 0.f ? v[e] : 0.f;
        }
      F f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        f[e] = (bf16)u[e];
        f[4 + e] = (bf16)v[e];
      }
      return f;
    }
  };
  auto comp = [&](int buf, int nc) __attribute__((always_inline)) {
    const lf* Aq = lds + buf * K_::BUF;
    const lf* Bq = Aq + K_::ABUF;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      if (ch >= nc) break;
      const F a0 = afrag(Aq, wr * 2, ch);
      const F a1 = afrag(Aq, wr * 2 + 1, ch);
      const F b0 = *(const AS_L F*)(Bq + ((wc * 2 + 0) * NCH + ch) * 256 + lane * 4);
      const F b1 = *(const AS_L F*)(Bq + ((wc * 2 + 1) * NCH + ch) * 256 + lane * 4);
      MM<T>::mma(acc[0][0], a0, b0);
      MM<T>::mma(acc[0][1], a0, b1);
      MM<T>::mma(acc[1][0], a1, b0);
      MM<T>::mma(acc[1][1], a1, b1);
    }
  };
  // the generated operand's dY^T + bias partials (WA_OUTBWD, cb == 0 items): from the transformed block
  // (spread over the row block's items: item cb stores the K blocks kb = cb mod ncb)
  const bool agt = AM == WA_OUTBWD && jb.AGT;
  auto agt_store = [&](int kb, int buf, int nk) __attribute__((always_inline)) {
    const int k0 = kb * KB;
    const lf* Aq = lds + buf * K_::BUF;
#pragma unroll
    for (int u = 0; u < KB / 16; ++u) {
      const int p = tid + WG_T * u, k = p >> 4, q = p & 15;  // column k0 + k, rows 4q..4q+3
      const int b0 = row0 + 4 * q;
      if (b0 < W.Bp && k < nk) {
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = Aq[K_::aloc(4 * q + e, k)];
        st4<T>(jb.AGT, (size_t)(k0 + k) * W.Bp + b0, v);
      }
    }
    if (jb.Adbp && tid < 4 * KB) {
      const int rt = tid / KB, k = tid % KB, grt = row0 / 16 + rt;
      float s = 0.f;
      for (int r = 0; r < 16; ++r) s += Aq[K_::aloc(rt * 16 + r, k)];
      if (grt < W.nrt && k < nk && k0 + k < jb.adbp_ld) GP(float, jb.Adbp)[(size_t)grt * jb.adbp_ld + k0 + k] = s;
    }
  };

  WSTAMP(1);
  int cur = 0;
  for (int kb = 0; kb < nkb; ++kb) {
    const int nc = min(NCH, (Kp - kb * KB) / KC);
    // newest block issued so far: NB - 1 at kb = 0, then kb + NB - 2
    const int last = min(nkb - 1, kb == 0 ? NB - 1 : kb + NB - 2);
    wait_ahead(last - kb);  // this wave's pieces of block kb have landed
    bar();                  // ... and every wave's; block kb - 1 is consumed
    if constexpr (XF) {
      xform(kb, cur);
      bar();
    }
    if (kb >= 1 && kb + NB - 1 < nkb) issue(kb + NB - 1, cur == 0 ? NB - 1 : cur - 1);  // block kb - 1's buffer
    if (kb < 8) WSTAMP(2 + kb);
    if (agt && kb % jb.ncb == cb) agt_store(kb, cur, nc * KC);
    comp(cur, nc);
    cur = cur + 1 == NB ? 0 : cur + 1;
  }
  WSTAMP(11);
  __syncthreads();  // the epilogue tile aliases the K buffers (no DMA in flight)

  // ---- epilogue through an LDS tile [64][WLDE]
  lf* Et = lds;
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      const int cl = wc * 32 + ct * 16 + c, n = col0 + cl;
      const float bn = bias_r[ct];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wr * 32 + rt * 16 + 4 * g + i;
        const bool ok = n < jb.N && rbase + r < W.B;
        Et[r * WLDE + cl] = ok ? acc[rt][ct][i] + bn : 0.f;
      }
    }
  __syncthreads();
  WSTAMP(12);
  if (!fwd) {  // dY of the layer below = act'(P_prev) * dX, in place (row pieces)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = tid + WG_T * u, r = p >> 4, q = p & 15, k = col0 + 4 * q;
      if (k < jb.Np) {
        f32x4 v = *(AS_L f32x4*)(Et + r * WLDE + 4 * q);
        if (jb.pact >= 0) {
          const f32x4 pp = ld16h(jb.Pprev, (size_t)(row0 + r) * jb.ldpp + k);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = hactb<HR>(jb.pact, pp[e], v[e]);
          *(AS_L f32x4*)(Et + r * WLDE + 4 * q) = v;
        }
        if (jb.DY) st16h(jb.DY, (size_t)(row0 + r) * jb.lddy + k, v);
      }
    }
    __syncthreads();
    // dY^T stash + per-16-row bias partials
    if (jb.GT) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int p = tid + WG_T * u, k = p >> 4, q = p & 15, b0 = row0 + 4 * q;
        if (col0 + k < jb.Np && b0 < W.Bp) {
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = Et[(4 * q + e) * WLDE + k];
          st4<T>(jb.GT, (size_t)(col0 + k) * jb.gt_ld + b0, v);
        }
      }
    }
    if (jb.dbp) {
      const int rt = tid >> 6, k = tid & 63, grt = row0 / 16 + rt;
      float s = 0.f;
      for (int r = 0; r < 16; ++r) s += Et[(rt * 16 + r) * WLDE + k];
      if (grt < W.nrt && col0 + k < jb.N) GP(float, jb.dbp)[(size_t)grt * jb.dbp_ld + col0 + k] = s;
    }
    // d a~ partials: sum over this block's hidden units of dY0[r][n] W0[n][O + j]
    if (jb.DA) wide_rowdot<HR, false>(Et, Ws, W.A, 0, jb.DA + cb * jb.da_cb + (size_t)row0 * W.A);
    return;
  }
  // forward: pre-activation rows (rows >= p_row0), act(P)^T stash, output-layer partials
  if (jb.P && row0 >= jb.p_row0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = tid + WG_T * u, r = p >> 4, q = p & 15;
      if (col0 + 4 * q < jb.Np)
        st16h(jb.P, (size_t)(row0 + r) * jb.ldp + col0 + 4 * q, *(AS_L f32x4*)(Et + r * WLDE + 4 * q));
    }
  }
  if (jb.XT && row0 >= jb.xt_row0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = tid + WG_T * u, n = p >> 4, q = p & 15, b0 = row0 - jb.xt_row0 + 4 * q;
      if (col0 + n < jb.Np && b0 < W.Bp) {
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = hact<HR>(jb.oact, Et[(4 * q + e) * WLDE + n]);
        st4<T>(jb.XT, (size_t)par * jb.xt_par + (size_t)(col0 + n) * jb.xt_ld + b0, v);
      }
    }
  }
  if (jb.OUTP)
    wide_rowdot<HR, true>(Et, Ws, jb.Nout, jb.oact, jb.OUTP + cb * jb.outp_cb + (size_t)row0 * jb.Nout);
}

// ---------------------------------------------------------------------------- gather
// One step's batch (replay_buffer.py:32-39, agent.py:166-193) into the row-major
// layer-0 inputs and the layer-0 X^T stashes, WGR rows per workgroup: each
// thread issues up to 8 independent replay loads before storing any (sampled
// rows are random lines: one memory latency per batch of loads, not per load),
// the (s, a) columns go through LDS to the k-major X^T stores.  Runs as its own
// launch for the first step of a call, and inside the last phase-C stage of
// step t for step t + 1 (every buffer it writes is past its last reader of
// step t: the layer-0 inputs and rewards are read in phase A and by phase C's
// first stage, the critics' X^T by phase B, and pi's X^T is the other step
// parity's copy from the one phase D of step t reads).
#define WGR 16
template <typename T>
__device__ __forceinline__ void wide_gather_rows(const AS_C EngineDev& E, const AS_C WideDev& W, const sac_replay& rb,
                                                 const int32_t* __restrict__ inj_idx_, uint64_t step, int blk,
                                                 lf* gl) {
  // LDS: [WGR][O + A] (s, a) of the block's rows, then the rows' replay slots
  // (all dynamic: a static array would push the stage kernel past the 160 KiB
  // dynamic-LDS attribute)
  const int tid = threadIdx.x, O = W.O, A = W.A, B = W.B, OA = O + A;
  AS_L int64_t* slot = (AS_L int64_t*)(gl + ((WGR * OA + 1) & ~1));
  const int row0 = blk * WGR;
  const int par = (int)(step & 1);
  if (tid < WGR) {
    const int64_t size = GPC(int64_t, rb.state)[0], pos = GPC(int64_t, rb.state)[1];
    const int b = row0 + tid;
    int64_t sl = -1;
    if (b < B) {
      int64_t li;
      if (inj_idx_) {
        li = GPC(int32_t, inj_idx_)[b];
      } else {
        const Feistel f = feistel_make(E.seed, step, size);
        li = feistel_sample(f, b, size);
      }
      sl = size < rb.capacity ? li : (pos + li) % rb.capacity;
    }
    slot[tid] = sl;
  }
  __syncthreads();
  const RowStrides rs = row_strides(rb.row_stride, O, A);
  const int Wf = 2 * O + A + 2, total = WGR * Wf;
  constexpr int U = 8;
  for (int base = 0; base < total; base += U * WG_T) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // every load of the batch first
      const int i = base + u * WG_T + tid;
      const int r = i / Wf, f = i % Wf;
      const int64_t sl = i < total ? slot[r] : -1;
      const int64_t src = sl < 0 ? 0 : sl;
      const AS_G float* p = f < O ? GPC(float, rb.obs) + src * rs.obs + f
                          : f < 2 * O ? GPC(float, rb.next_obs) + src * rs.obs + (f - O)
                          : f < 2 * O + A ? GPC(float, rb.act) + src * rs.act + (f - 2 * O)
                          : f == 2 * O + A ? GPC(float, rb.rew) + src * rs.one : GPC(float, rb.done) + src * rs.one;
      v[u] = *p;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * WG_T + tid;
      if (i >= total) continue;
      const int r = i / Wf, f = i % Wf, b = row0 + r;
      if (slot[r] < 0) continue;
      const float x = v[u];
      if (f < O) {
        sth(W.Xpi0 + (size_t)(W.Brw + b) * W.ldpi0 + f, x);
        sth(W.Xq0 + (size_t)b * W.ldq0 + f, x);
        GP(float, W.Xc0)[(size_t)b * W.ldq0 + f] = x;
        gl[r * OA + f] = x;
      } else if (f < 2 * O) {
        sth(W.Xpi0 + (size_t)b * W.ldpi0 + (f - O), x);
        sth(W.Xqt0 + (size_t)b * W.ldq0 + (f - O), x);
      } else if (f < 2 * O + A) {
        sth(W.Xq0 + (size_t)b * W.ldq0 + O + (f - 2 * O), x);
        gl[r * OA + O + (f - 2 * O)] = x;
      } else if (f == 2 * O + A) {
        sth(W.R + b, x);
      } else {
        sth(W.Dn + b, x);
      }
    }
  }
  __syncthreads();
  // X^T stashes of layer 0: the critics' (s, a) and the actor rows' s (the step's parity copy)
  const AS_C LayerDev& q0 = E.net[NET_Q1].l[0];
  const AS_C LayerDev& p0 = E.net[NET_PI].l[0];
  T* xq = (T*)q0.XT;
  T* xp = (T*)p0.XT + par * p0.xt_par;
  for (int i = tid; i < OA * WGR; i += WG_T) {  // k-major: WGR consecutive batch columns per k
    const int k = i / WGR, r = i % WGR, b = row0 + r;
    if (b >= B) continue;
    const float x = gl[r * OA + k];
    xq[(size_t)k * W.Bp + b] = MM<T>::cvt(x);
    if (k < O) xp[(size_t)k * W.Bp + b] = MM<T>::cvt(x);
  }
}

// The step's optimizer step counts and Adam bias corrections (torch adam.py:
// step_size = lr / (1 - beta1^t), sqrt(1 - beta2^t)), once per step by block 0
// of the step's first GEMM stage (the row-tile path does it in phase A).
__device__ __forceinline__ void wide_step_scalars(const AS_C EngineDev& E, int par) {
  const int tid = threadIdx.x;
  if (tid < 4 && (tid < 3 || (E.auto_entropy && E.alpha_update))) {
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
}

template <typename T>
__global__ void __launch_bounds__(WG_T) sac_wide_gather(const EngineDev* __restrict__ Ep, const WideDev* __restrict__ Wd,
                                                        sac_replay rb, const int32_t* __restrict__ inj_idx_) {
  const AS_C EngineDev& E = *(const AS_C EngineDev*)Ep;
  const AS_C WideDev& W = *(const AS_C WideDev*)Wd;
  extern __shared__ float lds_raw[];
  wide_gather_rows<T>(E, W, rb, inj_idx_, *GPC(uint64_t, E.rng_step), blockIdx.x, (lf*)lds_raw);
}

// ---------------------------------------------------------------------------- pi heads (phase A)
// Squashed-Gaussian sample (models.py:79-87) of every pi row: target rows
// (s', draw 0) -> a~' into the target critics' input and log pi' (LP2); actor
// rows (s, draw 1) -> a~ into phase C's critic input, the head stash, log pi.
// pi rows [rbase, rbase + nrows) (of the 2 Brw rows: s' then s), WG_T / AP
// rows per pass, one lane per (row, action dim)
template <typename T>
__device__ __forceinline__ void wide_head_rows(const AS_C EngineDev& E, const AS_C WideDev& W, int rbase, int nrows,
                                               const float* __restrict__ inj_eps_, uint64_t step) {
  const AS_C NetDev& pi = E.net[NET_PI];
  const int tid = threadIdx.x, A = W.A, B = W.B;
  const int par = (int)(step & 1);
  const int AP = A <= 1 ? 1 : 1 << (32 - __builtin_clz(A - 1));
  const int rpp = WG_T / AP;
  const int j = tid % AP;
  for (int p0 = 0; p0 < nrows; p0 += rpp) {
    const int r = rbase + p0 + tid / AP;  // r in [0, 2 Brw)
    const int which = r >= W.Brw ? 1 : 0, b = r - which * W.Brw;
    const bool live = p0 + tid / AP < nrows && r < 2 * W.Brw && b < B && j < A;
    float lp = 0.f, corr = 0.f;
    if (live) {
      float am = 0.f, as = 0.f;
      for (int c0 = 0; c0 < W.ncb_pi; c0 += 8) {  // every load of a batch of 8 blocks in flight together
        float xm[8], xs[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int c = c0 + u < W.ncb_pi ? c0 + u : W.ncb_pi - 1;
          xm[u] = ldh(W.OUTPpi + c * W.cbs_pi + (size_t)r * 2 * A + j);
          xs[u] = ldh(W.OUTPpi + c * W.cbs_pi + (size_t)r * 2 * A + A + j);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (c0 + u < W.ncb_pi) {
            am += xm[u];
            as += xs[u];
          }
      }
      const AS_G float* bo = GPC(float, pi.l[pi.L - 1].bias);
      const float pm = am + bo[j], ps = as + bo[A + j];
      const float mu = act_fwd(pi.out_act, pm), lsr = act_fwd(pi.out_act, ps);
      float e;
      if (inj_eps_) {
        e = GPC(float, inj_eps_)[((size_t)which * B + b) * A + j];
      } else {
        float n0, n1;
        philox_normal2(E.seed, step, (uint32_t)b, (uint32_t)which, (uint32_t)(j >> 1), n0, n1);
        e = (j & 1) ? n1 : n0;
      }
      const float lo = E.ls_min, hi = E.ls_max;
      const float ls = lsr < lo ? lo : (lsr > hi ? hi : lsr);
      const float sd = expf(ls);
      const float z = mu + e * sd;
      const float act_v = tanhf(z) * E.scale;
      const float diff = z - mu;
      const float var = sd * sd;
      lp = -(diff * diff) / (2.f * var) - logf(sd) - HALF_LOG_2PI;
      corr = 2.f * ((LOG2F - z) - softplus20(-2.f * z));
      if (which) {
        AS_G float* h = GP(float, E.head_st) + (size_t)b * 4 * A;
        h[j] = mu;
        h[A + j] = lsr;
        h[2 * A + j] = z;
        h[3 * A + j] = e;
        GP(float, E.a_st)[(size_t)b * A + j] = act_v;
        GP(float, W.Xc0)[(size_t)b * W.ldq0 + W.O + j] = act_v;
        if (pi.out_act != ACT_ID) {
          GP(float, W.PIOP)[(size_t)b * 2 * A + j] = pm;
          GP(float, W.PIOP)[(size_t)b * 2 * A + A + j] = ps;
        }
      } else {
        sth(W.Xqt0 + (size_t)b * W.ldq0 + W.O + j, act_v);
      }
    }
    for (int o = 1; o < AP; o <<= 1) {
      lp += __shfl_xor(lp, o, 64);
      corr += __shfl_xor(corr, o, 64);
    }
    if (live && j == 0) {
      const float v = lp - corr;
      if (which) {
        GP(float, E.lp_st)[par * E.Br + b] = v;
        GP(float, E.stats)[4 + B + b] = v;
      } else {
        sth(W.LP2 + b, v);
      }
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(WG_T) sac_wide_head(const EngineDev* __restrict__ Ep, const WideDev* __restrict__ Wd,
                                                      const float* __restrict__ inj_eps_) {
  const AS_C EngineDev& E = *(const AS_C EngineDev*)Ep;
  const AS_C WideDev& W = *(const AS_C WideDev*)Wd;
  const int A = W.A;
  const int AP = A <= 1 ? 1 : 1 << (32 - __builtin_clz(A - 1));
  const int rpb = WG_T / AP;
  wide_head_rows<T>(E, W, blockIdx.x * rpb, rpb, inj_eps_, *GPC(uint64_t, E.rng_step));
}

// ---------------------------------------------------------------------------- the stage kernel
// flags: bit 0 = the step's last launch before phase D (advances the step),
// bit 1 = the step's first GEMM stage (block 0 derives the step's Adam scalars),
// bit 2 = blocks [nitems, grid) gather the next step's batch; bits 8.. = the
// stage's index in the step (stamps builds).  AM: the A-operand mode of every
// job of the stage; HR: both networks' hidden activation is ReLU (applied and
// differentiated inline, no switch).
template <typename T, int AM, bool HR>
__global__ void __launch_bounds__(WG_T, 4) sac_wide_stage(const EngineDev* __restrict__ Ep, const WideDev* __restrict__ Wd,
                                                       const WJob* __restrict__ jobs, int njobs, int flags, int nitems,
                                                       sac_replay rb, const int32_t* __restrict__ next_idx) {
  const AS_C EngineDev& E = *(const AS_C EngineDev*)Ep;
  const AS_C WideDev& W = *(const AS_C WideDev*)Wd;
  extern __shared__ float lds_raw[];
  if ((int)blockIdx.x >= nitems) {  // flags & 4: the next step's batch (see wide_gather_rows)
    wide_gather_rows<T>(E, W, rb, next_idx, *GPC(uint64_t, E.rng_step) + 1, (int)blockIdx.x - nitems, (lf*)lds_raw);
    if (flags & 1) phase_c_done(E);
    return;
  }
  if ((flags & 2) && blockIdx.x == 0) wide_step_scalars(E, (int)(*GPC(uint64_t, E.rng_step) & 1));
#ifdef SAC_STAMPS
  const bool wst = E.stamps && (flags >> 8) == W.stamp_stage;
#else
  const bool wst = false;
#endif
  WSTAMP(0);
  int j = 0;
  while (j + 1 < njobs && (int)blockIdx.x >= ((const AS_C WJob*)jobs)[j + 1].item0) ++j;
  const AS_C WJob& jb = ((const AS_C WJob*)jobs)[j];
  wide_prefetch(jobs + j, Wd);
  const int par = (int)(*GPC(uint64_t, W.rng_step) & 1);
  const int it = (int)blockIdx.x - jb.item0;
  wide_item<T, AM, HR>(E, W, jb, it, (lf*)lds_raw, par, wst);
#ifdef SAC_STAMPS
  if (wst) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    WSTAMP(13);
  }
#endif
  if (flags & 1) phase_c_done(E);  // the step's last launch before phase D advances the step
}
