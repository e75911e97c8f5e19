// Pair-tile kernels of phases A and C for large batches (C3: B = 4096).
//
// The row-tile kernels (sac_phases.h, !ROLES) give one workgroup per 16-row
// tile and run every network through it: at C3 each of the 256 workgroups
// streams all five networks' weights for 16 rows, one pass after another
// (profiles/r05_stamps_c3_bf16.txt: phase A 49 us of ~7 weight passes).  Here a
// workgroup takes a PAIR of row tiles (32 rows: every weight fragment feeds two
// 16-row MFMA tiles) and one GROUP of networks, so that the same 256 workgroups
// each stream about half the weight passes:
//
//   phase A  critic group (blocks [0, npt)):  Q1 and Q2 forward on (s, a) and
//            their unit-seed backward; dY^T stored unscaled (phase B applies the
//            seeds, as the hidden-split kernels do), q published as granules.
//            target group (blocks [npt, 2 npt)):  pi(s') -> Q1t / Q2t -> y;
//            pi(s) (the actor sample and its stashes for phases C / D); then
//            polls the critics' q and writes the seeds dL/dq = 2 (q - y) / B and
//            the loss partials.
//   phase C  critic group (blocks [0, npt)):  Q2 on (s, a~) with the updated
//            weights, unit-seed backward to a~; publishes (dQ2/da~, q2).
//            actor group (blocks [npt, 2 npt)):  Q1 the same, then combines both
//            with the min-Q weights (polling Q2's granules), the head backward and
//            pi's backward (dY^T stored for phase D); then the stager blocks.
//
// The consumers are the higher block ids (in-order dispatch starts every
// producer first), and no producer waits.  Same arithmetic per row as the
// row-tile kernels, except that the critics' seeds are applied in phase B (fp32:
// one rounding of seed x dY instead of dY computed from a seeded output;
// checked against the oracle like every layout).
//
// Reference: agent.py:195-260 (target, critic and actor passes), models.py:73-92
// (policy head), replay_buffer.py:32-39 / agent.py:166-193 (sample + gather).
#pragma once
#include "sac_phases.h"

#define SAC_PR (2 * SAC_ROWS)  // rows per pair tile

// The pair's batch rows (s, s', a, r, d) into LDS: the two 16-row records phase
// C staged, or the tile's own sample + gather.  Both records' loads (and both
// headers') are issued before any LDS store: one round trip for the pair, not
// one per record.  Returns whether every live sub-tile came from a staged
// record (uniform).
__device__ __forceinline__ bool pair_batch(const AS_C EngineDev& E, const sac_replay& rb, uint64_t step, int pt,
                                           const AS_G int32_t* inj_idx, lf* sB, lf* s2B, lf* aB, lf* rB, lf* dB,
                                           AS_L int64_t* slotB) {
  constexpr int R = SAC_ROWS;
  const int tid = threadIdx.x, O = E.O, A = E.A;
  const int64_t rb_size = GPC(int64_t, rb.state)[0], rb_pos = GPC(int64_t, rb.state)[1];
  const int RO = R * O, RA = R * A, per = 2 * RO + RA + 2 * R;  // floats of one record
  bool staged[2] = {false, false};
  const bool live1 = 2 * pt + 1 < E.nrt;
  if (E.stage && !inj_idx) {  // uniform
    const AS_G float* rec[2] = {GPC(float, E.stg) + stage_rec(E, step, 2 * pt),
                                GPC(float, E.stg) + stage_rec(E, step, live1 ? 2 * pt + 1 : 2 * pt)};
    uint64_t h[2][5];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int k = 0; k < 5; ++k) h[sub][k] = ((const AS_C uint64_t*)rec[sub])[k];
    constexpr int MV = 4;  // record floats per thread and record, at most (R * (2 O + A + 2) <= 2048)
    float v[2][MV];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int u = 0; u < MV; ++u) {
        const int i = tid + u * SAC_THREADS;
        v[sub][u] = i < per ? rec[sub][16 + i] : 0.f;
      }
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      staged[sub] = h[sub][0] == step && h[sub][1] == (uint64_t)rb_size && h[sub][2] == (uint64_t)rb_pos &&
                    h[sub][3] == (uint64_t)(uintptr_t)rb.obs && h[sub][4] == (uint64_t)GPC(int64_t, rb.state)[2];
      // a sub-tile past the batch (odd nrt) is zero-filled below by other
      // threads of the same slots: no copy of the duplicate record into it
      if (sub == 1 && !live1) continue;  // uniform
#pragma unroll
      for (int u = 0; u < MV; ++u) {
        const int i = tid + u * SAC_THREADS;
        if (i < per) {
          if (i < RO) sB[sub * RO + i] = v[sub][u];
          else if (i < 2 * RO) s2B[sub * RO + i - RO] = v[sub][u];
          else if (i < 2 * RO + RA) aB[sub * RA + i - 2 * RO] = v[sub][u];
          else if (i < 2 * RO + RA + R) rB[sub * R + i - 2 * RO - RA] = v[sub][u];
          else dB[sub * R + i - 2 * RO - RA - R] = v[sub][u];
        }
      }
    }
  }
  bool all_staged = true;
#pragma unroll
  for (int sub = 0; sub < 2; ++sub) {
    const int rbi = 2 * pt + sub;
    lf* s = sB + sub * RO;
    lf* s2 = s2B + sub * RO;
    lf* a = aB + sub * RA;
    lf* r = rB + sub * R;
    lf* d = dB + sub * R;
    if (rbi >= E.nrt) {  // the pair's second tile past the batch: zero rows
      for (int i = tid; i < RO; i += SAC_THREADS) s[i] = s2[i] = 0.f;
      for (int i = tid; i < RA; i += SAC_THREADS) a[i] = 0.f;
      if (tid < R) r[tid] = d[tid] = 0.f;
      continue;
    }
    if (!staged[sub]) {  // uniform
      tile_slots(E, rb, step, rb_size, rb_pos, rbi * R, inj_idx, slotB + sub * R);
      __syncthreads();
      gather_rows<lf*>(rb, slotB + sub * R, O, A, s, s2, a, r, d);
    }
    all_staged = all_staged && staged[sub];
  }
  return all_staged;
}

// Unit-seed output gradient of a critic (1 per valid row, through the output
// activation): column 0 of G [PR][ldo], the other columns of the padded width 0.
__device__ __forceinline__ void unit_seed(const AS_C NetDev& q, const lf* outP, int ldo, lf* G, int nvalid) {
  const int tid = threadIdx.x;
  if (tid < SAC_PR) {
    float u = tid < nvalid ? 1.f : 0.f;
    if (q.out_act != ACT_ID) u = act_bwd(q.out_act, outP[tid * ldo], u);
    for (int n = 0; n < 32; ++n) G[tid * ldo + n] = n == 0 ? u : 0.f;
  }
}

// Critic forward over the pair's rows: pre-activations kept in the P1 buffers
// (keepP), every layer's input X^T stored for phase B (storeXT; the layer-0
// input (s, a) is shared by Q1 and Q2 and stored by Q1 only).  q in outB col 0.
template <typename T>
__device__ __forceinline__ void pair_critic_forward(const AS_C EngineDev& E, const AS_C NetDev& q, lf* lds, lf* Xb,
                                                    lf* Yb, lf* outP, lf* outB, bool storeXT, bool store_x0, int r0,
                                                    int nvalid, Pf<T>& pf) {
  const int ld = E.ld, ldo = E.ldo, Bp = E.Bp;
  lf* X = Xb;
  lf* Y = Yb;
  for (int l = 0; l < q.L; ++l) {
    const AS_C LayerDev& Ly = q.l[l];
    if (storeXT && (l > 0 || store_x0)) store_T<T, SAC_PR>(X, ld, Ly.Kp, Ly.K, Ly.XT, Bp, r0, nvalid, nullptr);
    if (l == q.L - 1)
      layer_fwd<T, SAC_PR>(X, ld, Ly, q.P + Ly.b_off, q.out_act, outP, ldo, outB, ldo, nullptr, 0, pf, gw_bwd(Ly));
    else
      layer_fwd<T, SAC_PR>(X, ld, Ly, q.P + Ly.b_off, q.hid_act, lds + E.o_P1[l], E.ldp1[l], Y, ld, nullptr, 0, pf,
                           gw_fwd(q.l[l + 1]));
    __syncthreads();
    lf* t = X;
    X = Y;
    Y = t;
  }
}

// ============================================================================ phase A
template <typename T>
__global__ void __launch_bounds__(SAC_THREADS) sac_target_critic_pairs(const EngineDev* __restrict__ Ep, sac_replay rb,
                                                                        const int32_t* __restrict__ inj_idx_,
                                                                        const float* __restrict__ inj_eps_) {
  PREFETCH_ARG(Ep);
  const AS_C EngineDev& E = *(const AS_C EngineDev*)Ep;
  extern __shared__ float lds_raw[];
  lf* lds = (lf*)lds_raw;
  constexpr int PR = SAC_PR;
  const int tid = threadIdx.x;
  const int npt = (E.nrt + 1) / 2;
  const bool critics = (int)blockIdx.x < npt;  // producers first
  const int pt = critics ? (int)blockIdx.x : (int)blockIdx.x - npt;
  STAMP(0);
  const int B = E.B, Bp = E.Bp, O = E.O, A = E.A, ld = E.ld, ldo = E.ldo;
  const int r0 = pt * PR;
  const int nvalid = min(PR, B - r0);
  const uint32_t ep = *GPC(uint32_t, E.sync) + 1u;
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
  AS_G float* stats = GP(float, E.stats);
  const AS_C NetDev& pi = E.net[NET_PI];
  Pf<T> pf;
  pf_issue<T>(pf, critics ? gw_fwd(E.net[NET_Q1].l[0]) : gw_fwd(pi.l[0]));

  const uint64_t step = *GPC(uint64_t, E.rng_step);
  const int par = (int)(step & 1);
  // optimizer step counters and this step's Adam bias-correction scalars, once per step
  if (!critics && pt == 0 && tid < 4 && (tid < 3 || (E.auto_entropy && E.alpha_update))) {
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
  const bool staged = pair_batch(E, rb, step, pt, inj_idx, sB, s2B, aB, rB, dB, slotB);
  if (staged && !critics && pt == 0 && tid == 0)
    *(AS_G uint64_t*)(GP(uint32_t, E.sync) + SYNC_STAGED) = step;  // the staged path ran (tests)
  if (!critics) {  // eps: target draw (which 0) and actor draw (which 1)
    const int NP = (A + 1) / 2;
    for (int i = tid; i < 2 * PR * NP; i += SAC_THREADS) {
      const int which = i / (PR * NP), rem = i % (PR * NP), r = rem / NP, p = rem % NP;
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

  if (critics) {
    // ---- Q1, Q2 on (s, a): forward, unit-seed backward (agent.py:213-236)
    for (int qi = 0; qi < 2; ++qi) {
      const AS_C NetDev& q = E.net[NET_Q1 + qi];
      const int Kp0 = q.l[0].Kp;
      for (int i = tid; i < PR * Kp0; i += SAC_THREADS) {
        const int r = i / Kp0, k = i % Kp0;
        Xb[r * ld + k] = k < O ? sB[r * O + k] : (k < O + A ? aB[r * A + (k - O)] : 0.f);
      }
      __syncthreads();
      pair_critic_forward<T>(E, q, lds, Xb, Yb, outP, outB, true, qi == 0, r0, nvalid, pf);
      // q to the target group (it computes y, the seeds and the loss partials)
      if (tid < PR && 2 * pt + (tid >> 4) < E.nrt)
        gran_put(gran_at(E, G_Q1T + qi, 2 * pt + (tid >> 4)) + (tid & 15), outB[tid * ldo], ep);
      STAMP(10 + 2 * qi);
      unit_seed(q, outP, ldo, gqB, nvalid);
      __syncthreads();
      // every layer's unit-seed dY^T, stored as it is made: phase B scales batch
      // column b by the seed (TileDesc::seed = E.seedq)
      mlp_backward<T, PR>(q, gqB, ldo, Xb, Yb, ld, E.o_P1, E.ldp1, lds, true, Bp, r0, nvalid, pf,
                          qi ? gw_none() : gw_fwd(E.net[NET_Q2].l[0]));
      STAMP(11 + 2 * qi);
    }
    END_STAMP(60);
    return;
  }

  // ---- target group: pi on s' (target sample) and on s (actor sample)
  auto pi_pass = [&](bool actor) {
    const lf* st = actor ? sB : s2B;
    if (actor)
      for (int i = tid; i < PR * O; i += SAC_THREADS) GP(float, E.s_st)[(size_t)r0 * O + i] = sB[i];
    const int Kp0 = pi.l[0].Kp;
    for (int i = tid; i < PR * Kp0; i += SAC_THREADS) {
      const int r = i / Kp0, k = i % Kp0;
      Xb[r * ld + k] = k < O ? st[r * O + k] : 0.f;
    }
    __syncthreads();
    lf* X = Xb;
    lf* Y = Yb;
    for (int l = 0; l < pi.L; ++l) {
      const AS_C LayerDev& Ly = pi.l[l];
      if (actor)  // the actor rows' layer input, into this step's parity copy (phase D)
        store_T<T, PR>(X, ld, Ly.Kp, Ly.K, (T*)Ly.XT + par * Ly.xt_par, Bp, r0, nvalid, nullptr);
      const bool out = l == pi.L - 1;
      // for phase C's pi backward: a ReLU hidden layer's mask as bits (written
      // below from the activations), every other layer's pre-activations
      const bool bits = !out && pi.hid_act == ACT_RELU;
      float* stash = actor && !bits ? Ly.pstash + (size_t)r0 * Ly.Np : nullptr;
      const GemmW nx = out ? gw_fwd(E.net[NET_Q1T].l[0]) : gw_fwd(pi.l[l + 1]);
      layer_fwd<T, PR>(X, ld, Ly, pi.P + Ly.b_off, out ? pi.out_act : pi.hid_act, out ? outP : nullptr,
                       out ? ldo : ld, out ? outB : Y, out ? ldo : ld, stash, 0, pf, nx);
      __syncthreads();
      if (actor && bits) {  // relu(p) > 0 <=> p > 0: one 32-unit word per (row, word) lane
        const int nw = Ly.Np >> 5;
        AS_G uint32_t* mk = GP(uint32_t, Ly.pmask) + (size_t)r0 * nw;
        for (int i = tid; i < PR * nw; i += SAC_THREADS) {
          const int r = i / nw, w = i % nw;
          const lf* y = Y + r * ld + 32 * w;
          uint32_t m = 0;
#pragma unroll
          for (int u = 0; u < 32; ++u) m |= (y[u] > 0.f ? 1u : 0u) << u;
          mk[i] = m;
        }
      }
      lf* t = X;
      X = Y;
      Y = t;
    }
    // squashed-Gaussian head (models.py:79-87): one lane per (row, action dim)
    const int AP = A <= 1 ? 1 : 1 << (32 - __builtin_clz(A - 1));
    const int rows_per_pass = SAC_THREADS / AP;
    for (int base = 0; base < PR; base += rows_per_pass) {
      const int r = base + tid / AP, j = tid % AP;
      const bool live = r < PR && j < A;
      const int b = r0 + r;
      float lp = 0.f, corr = 0.f;
      if (live) {
        const lf* o = outB + r * ldo;
        const float mu = o[j], lsr = o[A + j], e = (actor ? eaB : etB)[r * A + j];
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
          a2B[r * A + j] = act_v;
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
          lp2B[r] = v;
        }
      }
    }
    __syncthreads();
  };
  pi_pass(false);
  STAMP(6);

  // ---- target twin-Q and y (agent.py:195-211)
  const float alpha32 = (float)*GPC(double, E.alpha_state + 1);
  for (int t = 0; t < 2; ++t) {
    const AS_C NetDev& q = E.net[NET_Q1T + t];
    const int Kp0 = q.l[0].Kp;
    for (int i = tid; i < PR * Kp0; i += SAC_THREADS) {
      const int r = i / Kp0, k = i % Kp0;
      Xb[r * ld + k] = k < O ? s2B[r * O + k] : (k < O + A ? a2B[r * A + (k - O)] : 0.f);
    }
    __syncthreads();
    mlp_forward<T, PR>(q, Xb, Yb, ld, outP, outB, ldo, E.o_P1, E.ldp1, lds, false, false, Bp, r0, nvalid, pf,
                       t ? gw_fwd(pi.l[0]) : gw_fwd(E.net[NET_Q2T].l[0]));
    if (tid < PR) qtB[t * PR + tid] = outB[tid * ldo];
    __syncthreads();
    STAMP(7 + t);
  }
  if (tid < PR) {
    const int b = r0 + tid;
    const float mq = fmin_nan(qtB[tid], qtB[PR + tid]);
    const float y = rB[tid] + (E.gamma * (1.f - dB[tid])) * (mq - alpha32 * lp2B[tid]);
    yB[tid] = y;
    if (b < B) stats[4 + b] = y;
  }
  __syncthreads();

  // ---- pi(s): the actor sample, its stashes for phases C / D (the critics run meanwhile)
  pi_pass(true);
  STAMP(9);

  // ---- the critics' seeds dL/dq = 2 (q - y) / B (mse_loss backward) and loss partials
  if (tid < 64) {
    const int r = tid & (PR - 1), rbi = 2 * pt + (r >> 4);
    const bool live = tid < PR && rbi < E.nrt;
    float q[2] = {0.f, 0.f};
    if (live) {
      const AS_G uint64_t* const g[2] = {gran_at(E, G_Q1T, rbi) + (r & 15), gran_at(E, G_Q2T, rbi) + (r & 15)};
      gran_getn<2>(E, g, ep, q);
    }
    const bool v = live && r < nvalid;
#pragma unroll
    for (int qi = 0; qi < 2; ++qi) {
      const float d = q[qi] - yB[r];
      if (tid < PR) st_f<false>(E.seedq + qi * Bp + r0 + r, v ? (2.0f / (float)B) * d : 0.f);
      float sq = v ? d * d : 0.f;
      // per 16-row tile, as the row-tile kernels sum them
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) sq += __shfl_xor(sq, o, 64);
      if (live && (r & 15) == 0) GP(float, E.lossp)[(par * E.nrt + rbi) * 4 + qi] = sq;
    }
  }
  STAMP(14);
  END_STAMP(60);
}

// ============================================================================ phase C
template <typename T>
__device__ __forceinline__ void actor_pairs_body(const AS_C EngineDev& E, int bid) {
  extern __shared__ float lds_raw[];
  lf* lds = (lf*)lds_raw;
  constexpr int R = SAC_ROWS, PR = SAC_PR;
  const int tid = threadIdx.x;
  const int npt = (E.nrt + 1) / 2;
  const bool critic2 = bid < npt;  // producers first: the Q2 group
  const int pt = critic2 ? bid : bid - npt;
  STAMP(32);
  const int B = E.B, Bp = E.Bp, O = E.O, A = E.A, ld = E.ld, ldo = E.ldo;
  const int r0 = pt * PR;
  const int nvalid = min(PR, B - r0);
  const uint32_t ep = *GPC(uint32_t, E.sync) + 1u;
  const int par = (int)(*GPC(uint64_t, E.rng_step) & 1);  // advanced by the last block of this phase
  lf* Xb = lds + E.o_X;
  lf* Yb = lds + E.o_Y;
  lf* sB = lds + E.o_s;
  lf* aB = lds + E.o_a;
  lf* lpB = lds + E.o_lp;
  lf* gaB = lds + E.o_ga;
  lf* gwB = lds + E.o_g;  // min-Q weights: Q1's [PR], then Q2's [PR]
  lf* goutB = lds + E.o_gout;
  lf* outB = lds + E.o_out;
  lf* outP = lds + E.o_outp;
  lf* qtB = lds + E.o_qt;  // q1 [PR]
  const AS_C NetDev& pi = E.net[NET_PI];
  const float alpha32 = (float)*GPC(double, E.alpha_state + 1);
  const int qi = critic2 ? 1 : 0;
  const AS_C NetDev& q = E.net[NET_Q1 + qi];
  Pf<T> pf;
  pf_issue<T>(pf, gw_fwd(q.l[0]));
  for (int i = tid; i < PR * O; i += SAC_THREADS) sB[i] = r0 * O + i < E.Br * O ? GPC(float, E.s_st)[(size_t)r0 * O + i] : 0.f;
  for (int i = tid; i < PR * A; i += SAC_THREADS) aB[i] = r0 * A + i < E.Br * A ? GPC(float, E.a_st)[(size_t)r0 * A + i] : 0.f;
  if (!critic2) {
    for (int i = tid; i < PR * A; i += SAC_THREADS) gaB[i] = 0.f;
    if (tid < PR) lpB[tid] = r0 + tid < E.Br ? GPC(float, E.lp_st)[par * E.Br + r0 + tid] : 0.f;
  }
  __syncthreads();
  STAMP(33);

  // ---- this group's critic on (s, a~) with the updated weights (agent.py:244-248)
  {
    const int Kp0 = q.l[0].Kp;
    for (int i = tid; i < PR * Kp0; i += SAC_THREADS) {
      const int r = i / Kp0, k = i % Kp0;
      Xb[r * ld + k] = k < O ? sB[r * O + k] : (k < O + A ? aB[r * A + (k - O)] : 0.f);
    }
    __syncthreads();
    pair_critic_forward<T>(E, q, lds, Xb, Yb, outP, outB, false, false, r0, nvalid, pf);
    if (!critic2 && tid < PR) qtB[tid] = outB[tid * ldo];
    STAMP(36 + qi);
    unit_seed(q, outP, ldo, goutB, nvalid);
    __syncthreads();
    // d a~ through the critic: dX of layer 0, action columns (unit seed)
    lf* G0 = mlp_backward<T, PR>(q, goutB, ldo, Xb, Yb, ld, E.o_P1, E.ldp1, lds, false, Bp, r0, nvalid, pf,
                                 gw_bwd(q.l[0]));
    lf* Gx = (G0 == Xb) ? Yb : Xb;
    layer_bwd<T, PR>(G0, ld, q.l[0], nullptr, 0, -1, Gx, ld, pf, critic2 ? gw_none() : gw_bwd(pi.l[pi.L - 1]));
    __syncthreads();
    if (critic2) {  // (dQ2/da~, q2) to the actor group
      for (int i = tid; i < PR * A; i += SAC_THREADS) {
        const int r = i / A, j = i % A, rbi = 2 * pt + (r >> 4);
        if (rbi < E.nrt) gran_put(gran_at(E, G_C2, rbi) + (r & 15) * A + j, Gx[r * ld + O + j], ep);
      }
      if (tid < PR && 2 * pt + (tid >> 4) < E.nrt)
        gran_put(gran_at(E, G_C2, 2 * pt + (tid >> 4)) + R * A + (tid & 15), outB[tid * ldo], ep);
      STAMP(38 + qi);
      return;
    }
    // keep dQ1/da~ for the combination (Gx is reused by pi's backward)
    for (int i = tid; i < PR * A; i += SAC_THREADS) goutB[(i / A) * ldo + i % A] = Gx[(i / A) * ld + O + i % A];
    STAMP(38);
  }

  // ---- pi's pre-activations (relu masks etc.) from phase A's stash
  for (int l = 0; l < pi.L - 1; ++l) {
    const AS_C LayerDev& Ly = pi.l[l];
    const int ldp = E.ldp1[l];
    lf* P = lds + E.o_P1[l];
    if (pi.hid_act == ACT_RELU) {  // phase A's mask bits: 1 / 0 stand in for the pre-activation's sign
      const int nw = Ly.Np >> 5;
      const AS_G uint32_t* mk = GPC(uint32_t, Ly.pmask) + (size_t)r0 * nw;
      for (int i = tid; i < PR * nw; i += SAC_THREADS) {
        const int r = i / nw, w = i % nw;
        const uint32_t m = mk[i];
        lf* pr = P + r * ldp + 32 * w;
#pragma unroll
        for (int u = 0; u < 32; ++u) pr[u] = (m >> u) & 1u ? 1.f : 0.f;
      }
    } else {
      const AS_G float* ps = GPC(float, Ly.pstash) + (size_t)r0 * Ly.Np;
      for (int i = tid; i < PR * Ly.Np; i += SAC_THREADS) P[(i / Ly.Np) * ldp + i % Ly.Np] = ps[i];
    }
  }
  __syncthreads();
  // ---- combine the critics' unit-seed gradients with the min-Q weights
  // (L_pi = mean(alpha logpi - min Q), agent.py:251-252; min backward splits ties)
  if (tid < 64) {
    const int r = tid & (PR - 1), rbi = 2 * pt + (r >> 4);
    const bool live = tid < PR && rbi < E.nrt;
    float q2 = 0.f;
    if (live) q2 = gran_get(E, gran_at(E, G_C2, rbi) + R * A + (r & 15), ep);
    const bool v = live && r < nvalid;
    const float q1 = qtB[r];
    const float m = fmin_nan(q1, q2);
    float term = v ? alpha32 * lpB[r] - m : 0.f;
    const float gm = v ? -1.0f / (float)B : 0.f;
    if (tid < PR) {
      gwB[r] = (q1 == q2) ? gm * 0.5f : (q1 > q2 ? 0.f : gm);
      gwB[PR + r] = (q1 == q2) ? gm * 0.5f : (q1 < q2 ? 0.f : gm);
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) term += __shfl_xor(term, o, 64);
    if (live && (r & 15) == 0) GP(float, E.lossp)[(par * E.nrt + rbi) * 4 + 2] = term;
  }
  __syncthreads();
  for (int i = tid; i < PR * A; i += SAC_THREADS) {
    const int r = i / A, j = i % A, rbi = 2 * pt + (r >> 4);
    const float d2 = rbi < E.nrt ? gran_get(E, gran_at(E, G_C2, rbi) + (r & 15) * A + j, ep) : 0.f;
    gaB[i] = (gaB[i] + gwB[r] * goutB[r * ldo + j]) + gwB[PR + r] * d2;
  }
  __syncthreads();
  STAMP(39);
  // ---- squashed-Gaussian head backward (models.py:79-87), one lane per (row, action dim)
  for (int i = tid; i < PR * A; i += SAC_THREADS) {
    const int r = i / A, j = i % A, b = r0 + r;
    const bool v = r < nvalid;
    const float gl = v ? alpha32 * (1.0f / (float)B) : 0.f;
    const AS_G float* h = GPC(float, E.head_st) + (size_t)(v ? b : 0) * 4 * A;
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
      const AS_G float* ps = GPC(float, Lo.pstash) + (size_t)(v ? b : 0) * Lo.Np;
      gm = act_bwd(pi.out_act, ps[j], gm);
      gs = act_bwd(pi.out_act, ps[A + j], gs);
    }
    goutB[r * ldo + j] = gm;
    goutB[r * ldo + A + j] = gs;
  }
  {
    const int NOp = 32 * ((2 * A + 31) / 32), pad = NOp - 2 * A;
    for (int i = tid; i < PR * pad; i += SAC_THREADS) goutB[(i / pad) * ldo + 2 * A + i % pad] = 0.f;
  }
  __syncthreads();
  // ---- pi backward (agent.py:255-257): every layer's dY^T for phase D
  mlp_backward<T, PR>(pi, goutB, ldo, Xb, Yb, ld, E.o_P1, E.ldp1, lds, true, Bp, r0, nvalid, pf, gw_none());
  STAMP(35);
}

// After the 2 npt pair blocks: E.stage ? nrt stager blocks (next step's batch).
template <typename T>
__global__ void __launch_bounds__(SAC_THREADS) sac_actor_pairs(const EngineDev* __restrict__ Ep, sac_replay rb) {
  PREFETCH_ARG(Ep);
  const AS_C EngineDev& E = *(const AS_C EngineDev*)Ep;
  extern __shared__ float lds_raw[];
  const int bid = (int)blockIdx.x;
  const int nrole = 2 * ((E.nrt + 1) / 2);
  if (bid >= nrole)
    stage_next_batch(E, rb, bid - nrole, (lf*)lds_raw, *GPC(uint64_t, E.rng_step));
  else
    actor_pairs_body<T>(E, bid);
  phase_c_done(E);
  END_STAMP(61);
}
