// sac_engine.hip — MI355X (gfx950) SAC gradient-step engine, C ABI in
// include/sac_engine.h.  Design notes: DESIGN.md.
//
// One gradient step (reference sac/agent.py:302-327) = 4 launches:
//
//   A  sac_target_critic  row tiles of 16 batch rows, 8 waves.  Device sampler
//                         + replay gather (agent.py:166-193), pi forward on s' and s
//                         (models.py:79-87), target twin-Q and y (agent.py:195-211),
//                         Q1/Q2 forward + backward to every layer's pre-activation
//                         gradient (agent.py:221-234).  Writes X^T / dY^T tiles.
//   B  sac_critic_update  32x32 weight tiles: dW = dY^T X (MFMA over the batch),
//                         Adam (torch single-tensor math), Polyak (agent.py:282-300),
//                         packed compute copies of the new weights.
//   C  sac_actor          row tiles: Q1/Q2 forward on (s, a~) with the UPDATED
//                         critics, min-Q, backward to d a~, squashed-Gaussian head
//                         backward, pi backward (agent.py:238-260).
//   D  sac_actor_update   pi weight tiles + Adam; one extra block runs the float64
//                         alpha update (agent.py:263-280) and reduces the losses.
//
// Weights stay fp32 masters (the nn.Parameter storage); GEMM operands are packed
// compute copies in the MFMA dtype ([out][in] and [in][out], 32-padded) that the
// update kernels rewrite in place, so nothing is re-packed per step.
#include "../../include/sac_engine.h"

#include <algorithm>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>

#define SAC_VERSION "sac-mi355x 0.1.0"

#include "sac_phases.h"
#include "sac_split.h"
#include "sac_wide.h"
#include "sac_pairs.h"

// ============================================================================ params / replay
template <typename T>
__global__ void pack_weights(const float* __restrict__ W, int K, int N, int Kp, int Np, T* __restrict__ Wc,
                             T* __restrict__ WTc) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < Np * Kp; i += gridDim.x * blockDim.x) {
    const int n = i / Kp, k = i % Kp;
    const float v = (n < N && k < K) ? W[(size_t)n * K + k] : 0.f;
    Wc[packed_off<T>(n, k, Kp)] = MM<T>::cvt(v);
    if (WTc) WTc[packed_off<T>(k, n, Np)] = MM<T>::cvt(v);
  }
}

__global__ void replay_push_kernel(sac_replay rb, const float* __restrict__ rows, int64_t n, int64_t skip, int64_t pos,
                                   int64_t new_size, int64_t new_pos) {
  const int O = rb.obs_dim, A = rb.act_dim, W = 2 * O + A + 2;
  const RowStrides rs = row_strides(rb.row_stride, O, A);
  const int64_t total = (n - skip) * W;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t rr = i / W;
    const int c = (int)(i % W);
    const int64_t src = skip + rr;
    const int64_t slot = (pos + src) % rb.capacity;
    const float v = rows[src * W + c];
    if (c < O)
      rb.obs[slot * rs.obs + c] = v;
    else if (c < O + A)
      rb.act[slot * rs.act + (c - O)] = v;
    else if (c == O + A)
      rb.rew[slot * rs.one] = v;
    else if (c < 2 * O + A + 1)
      rb.next_obs[slot * rs.obs + (c - O - A - 1)] = v;
    else
      rb.done[slot * rs.one] = v;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    rb.state[0] = new_size;
    rb.state[1] = new_pos;
    rb.state[2] += 1;  // push generation (a staged batch record of an older generation is stale)
  }
}

// Replay gather by LOGICAL index (reference replay_buffer.py:32-39 +
// agent.py:166-193), one wave per 64 batch rows.  Lane l resolves row b0+l's
// ring slot ONCE (32-bit index load or the device sampler, one conditional
// subtract instead of a 64-bit modulo); then each field is copied
// row-vectorised: the wave's 64 output rows of a field are one contiguous span
// of the SoA output, swept 16 B per lane (4 B when the field width is not a
// multiple of 4 floats), each lane taking its source row's slot from the
// owner lane by a shuffle.  Loads are issued in batches of GATHER_GB before
// their stores (memory-level parallelism: a batch's rows are independent).
#ifndef GATHER_NT
#define GATHER_NT 1  // nontemporal output stores: 2.41 -> 3.01 TB/s at B = 1,048,576 (records)
#endif
#ifndef GATHER_GB
#define GATHER_GB 8
#endif
template <typename V>
__device__ __forceinline__ void gather_field(const float* __restrict__ src, int W, int64_t stride,
                                             float* __restrict__ dst, int nrow, int64_t slot, int lane) {
  constexpr int EV = sizeof(V) / 4;  // floats per access
  const int Q = W / EV;              // accesses per row
  const int64_t SV = stride / EV;    // accesses between consecutive source rows
  const int total = nrow * Q;
  const V* __restrict__ sv = (const V*)src;
  V* __restrict__ dv = (V*)dst;
  for (int i0 = 0; i0 < total; i0 += 64 * GATHER_GB) {
    V v[GATHER_GB];
    int64_t sl[GATHER_GB];
    int qq[GATHER_GB];
#pragma unroll
    for (int u = 0; u < GATHER_GB; ++u) {
      const int i = min(i0 + u * 64 + lane, total - 1);  // past the end: the last access again
      const int row = (unsigned)i / (unsigned)Q;
      qq[u] = i - row * Q;
      sl[u] = __shfl(slot, row < 64 ? row : 63, 64);  // every lane joins the shuffle
    }
    // loads unconditional: under a per-lane branch each one waited for the one before
#pragma unroll
    for (int u = 0; u < GATHER_GB; ++u)
      if (i0 + u * 64 < total) v[u] = sv[sl[u] * SV + qq[u]];  // wave-uniform test
#pragma unroll
    for (int u = 0; u < GATHER_GB; ++u) {
      const int i = i0 + u * 64 + lane;
      if (i < total) dv[i] = v[u];
    }
  }
}

// Transition-record layout with the standard field order (obs | next_obs |
// act | rew | done at offsets 0, O, 2O, 2O+A, 2O+A+1; O, A multiples of 4;
// row_stride = 4P floats with P | 64): ONE sweep reads each sampled record
// once, 16 B per lane (P lanes per record, 64 / P records per wave
// instruction, padding pieces skipped), and every 16-B piece lands whole in
// one output field.  The field of a lane's piece is the same in every
// iteration (piece = lane % P).
template <bool SAMPLE>
__global__ void __launch_bounds__(256) replay_gather_records_kernel(
    sac_replay rb, const int32_t* __restrict__ idx, int B, FeistelKeys fk, int32_t* __restrict__ idx_out,
    float* __restrict__ s, float* __restrict__ a, float* __restrict__ r, float* __restrict__ s2, float* __restrict__ d,
    int rpw) {
  // rpw rows per wave (64, or 16 for smaller batches: 4x the waves in flight)
  const int lane = threadIdx.x & 63;
  const int b0 = (int)(((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * rpw;
  if (b0 >= B) return;  // whole waves
  const int nrow = B - b0 < rpw ? B - b0 : rpw;
  const int O = rb.obs_dim, A = rb.act_dim;
  const int64_t size = rb.state[0], pos = rb.state[1], cap = rb.capacity;
  int64_t slot = 0;
  if (lane < nrow) {
    int64_t li;
    if (SAMPLE) {
      const Feistel f = feistel_from_keys(fk, size);
      li = feistel_sample(f, b0 + lane, size);
      if (idx_out) idx_out[b0 + lane] = (int32_t)li;
    } else {
      li = idx[b0 + lane];
    }
    const int64_t p = pos + li;
    slot = size < cap ? li : (p >= cap ? p - cap : p);
  }
  const int P = (int)(rb.row_stride >> 2);  // 16-B pieces per record
  const int RPI = 64 / P;                   // records per wave instruction
  const int piece = lane % P, sub = lane / P;
  const int f = 4 * piece;                  // first float of this lane's piece
  const int live = (2 * O + A + 2 + 3) >> 2;  // pieces holding data
  // this lane's destination: field base + column (fixed over the iterations)
  float* dst;
  int dw, col;
  if (f < O) { dst = s; dw = O; col = f; }
  else if (f < 2 * O) { dst = s2; dw = O; col = f - O; }
  else if (f < 2 * O + A) { dst = a; dw = A; col = f - 2 * O; }
  else { dst = nullptr; dw = 0; col = 0; }  // the rew | done piece
  const f32x4* __restrict__ rec = (const f32x4*)rb.obs;
  const int64_t SV = rb.row_stride >> 2;
  const int iters = (nrow + RPI - 1) / RPI;
  const int pcl = piece < live ? piece : live - 1;  // padding pieces re-read the row's last live one
  for (int i0 = 0; i0 < iters; i0 += GATHER_GB) {
    f32x4 v[GATHER_GB];
    int64_t sl[GATHER_GB];
#pragma unroll
    for (int u = 0; u < GATHER_GB; ++u) {
      const int row = (i0 + u) * RPI + sub;
      sl[u] = __shfl(slot, row < 64 ? row : 63, 64);  // rows past nrow: slot 0
    }
    // loads unconditional (no per-lane branch: under one each load waited for the
    // one before, so a wave's rows were fetched one round trip after another)
#pragma unroll
    for (int u = 0; u < GATHER_GB; ++u)
      if (i0 + u < iters) v[u] = rec[sl[u] * SV + pcl];  // wave-uniform test
#pragma unroll
    for (int u = 0; u < GATHER_GB; ++u) {
      const int row = (i0 + u) * RPI + sub;
      if (row < nrow && piece < live) {
        const int b = b0 + row;
        if (dst) {
#if GATHER_NT
          __builtin_nontemporal_store(v[u], (f32x4*)(dst + (size_t)b * dw + col));
#else
          *(f32x4*)(dst + (size_t)b * dw + col) = v[u];
#endif
        } else if (f == 2 * O + A) {
          r[b] = v[u][0];
          d[b] = v[u][1];
        }
      }
    }
  }
}

static bool standard_records(const sac_replay* rb) {
  const int64_t W = rb->row_stride;
  const int O = rb->obs_dim, A = rb->act_dim;
  return W > 0 && W <= 256 && (W & (W - 1)) == 0 && W >= 2 * O + A + 2 && (O & 3) == 0 && (A & 3) == 0 &&
         ((uintptr_t)rb->obs & 15) == 0 && rb->next_obs == rb->obs + O && rb->act == rb->obs + 2 * O &&
         rb->rew == rb->act + A && rb->done == rb->rew + 1;
}

template <bool SAMPLE>
__global__ void __launch_bounds__(256) replay_gather_kernel(sac_replay rb, const int32_t* __restrict__ idx, int B,
                                                            FeistelKeys fk, int32_t* __restrict__ idx_out,
                                                            float* __restrict__ s, float* __restrict__ a,
                                                            float* __restrict__ r, float* __restrict__ s2,
                                                            float* __restrict__ d) {
  const int lane = threadIdx.x & 63;
  const int b0 = (int)(((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 64;
  if (b0 >= B) return;  // whole waves
  const int nrow = B - b0 < 64 ? B - b0 : 64;
  const int O = rb.obs_dim, A = rb.act_dim;
  const int64_t size = rb.state[0], pos = rb.state[1], cap = rb.capacity;
  int64_t slot = 0;
  if (lane < nrow) {
    int64_t li;
    if (SAMPLE) {
      const Feistel f = feistel_from_keys(fk, size);
      li = feistel_sample(f, b0 + lane, size);
      if (idx_out) idx_out[b0 + lane] = (int32_t)li;
    } else {
      li = idx[b0 + lane];
    }
    const int64_t p = pos + li;  // li < size <= cap, pos < cap
    slot = size < cap ? li : (p >= cap ? p - cap : p);
  }
  // transition records: the five sweeps read the same 64 records, so after the
  // first sweep's misses the others hit the lines in L2
  const RowStrides rs = row_strides(rb.row_stride, O, A);
  auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if ((O & 3) == 0 && (rs.obs & 3) == 0 && a16(rb.obs) && a16(rb.next_obs)) {
    gather_field<f32x4>(rb.obs, O, rs.obs, s + (size_t)b0 * O, nrow, slot, lane);
    gather_field<f32x4>(rb.next_obs, O, rs.obs, s2 + (size_t)b0 * O, nrow, slot, lane);
  } else {
    gather_field<float>(rb.obs, O, rs.obs, s + (size_t)b0 * O, nrow, slot, lane);
    gather_field<float>(rb.next_obs, O, rs.obs, s2 + (size_t)b0 * O, nrow, slot, lane);
  }
  if ((A & 3) == 0 && (rs.act & 3) == 0 && a16(rb.act))
    gather_field<f32x4>(rb.act, A, rs.act, a + (size_t)b0 * A, nrow, slot, lane);
  else
    gather_field<float>(rb.act, A, rs.act, a + (size_t)b0 * A, nrow, slot, lane);
  if (lane < nrow) {
    r[b0 + lane] = rb.rew[slot * rs.one];
    d[b0 + lane] = rb.done[slot * rs.one];
  }
}

// The eps draws of one step exactly as the fused step makes them in its default
// (device RNG) mode: out[which][b][j] = philox_normal2(seed, step, b, which,
// j / 2), component j % 2 (sac_phases.h / sac_split.h eps loops).
__host__ __device__ inline void eps_pair(uint64_t seed, uint64_t step, int b, int which, int p, int B, int A,
                                         float* out) {
  float n0, n1;
  philox_normal2(seed, step, (uint32_t)b, (uint32_t)which, (uint32_t)p, n0, n1);
  float* o = out + ((size_t)which * B + b) * A;
  o[2 * p] = n0;
  if (2 * p + 1 < A) o[2 * p + 1] = n1;
}
__global__ void eps_draw_kernel(uint64_t seed, uint64_t step, int B, int A, float* __restrict__ out) {
  const int NP = (A + 1) / 2;
  const int64_t n = 2LL * B * NP;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int p = (int)(i % NP);
    const int64_t rw = i / NP;
    eps_pair(seed, step, (int)(rw % B), (int)(rw / B), p, B, A, out);
  }
}

__global__ void replay_sample_kernel(const int64_t* __restrict__ state, int B, FeistelKeys fk, int32_t* __restrict__ out) {
  const int64_t size = state[0];
  const Feistel f = feistel_from_keys(fk, size);
  for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < B; b += gridDim.x * blockDim.x)
    out[b] = (int32_t)feistel_sample(f, b, size);
}

// ============================================================================ host side
static thread_local std::string g_err;
static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x)                                                                                  \
  do {                                                                                             \
    hipError_t _e = (x);                                                                           \
    if (_e != hipSuccess) return fail(SAC_E_HIP, std::string(#x ": ") + hipGetErrorString(_e));    \
  } while (0)

// Workspace offsets of the large-batch stage path (sac_wide.h), from plan()
struct WideLay {
  int on = 0, Brw = 0, hp = 0, hq = 0;
  size_t o_dev = 0, o_jobs = 0;
  size_t o_xpi0 = 0, o_xq0 = 0, o_xqt0 = 0, o_xc0 = 0, o_r = 0, o_d = 0, o_lp2 = 0, o_piop = 0;
  size_t o_outpi = 0, o_outq[2] = {0, 0}, o_outqt[2] = {0, 0}, o_outc[2] = {0, 0}, o_da[2] = {0, 0};
  size_t o_P[5][SAC_DEV_LAYERS] = {};      // phase A pre-activations (pi on [s'; s], Q1, Q2, Q1t, Q2t)
  size_t o_Pc[2][SAC_DEV_LAYERS] = {};     // phase C critics
  size_t o_DYq[2][SAC_DEV_LAYERS] = {}, o_DYc[2][SAC_DEV_LAYERS] = {}, o_DYpi[SAC_DEV_LAYERS] = {};
};
#define WIDE_MAX_JOBS 64

struct sac_engine {
  sac_engine_config cfg;
  sac_engine_buffers buf;
  EngineDev h;            // host mirror of the device struct
  EngineDev* d = nullptr; // in workspace
  TileDesc* tilesB = nullptr;
  TileDesc* tilesD = nullptr;
  std::vector<TileDesc> hostB, hostD;
  int nB = 0, nD = 0;
  size_t lds_bytes = 0;
  size_t upd_lds = 0;  // dynamic LDS of an update tile (SAC_UPD_LDS_FOR(upd_slots))
  int upd_ut_b = SAC_UPD_THREADS;  // phase B's workgroup size (SAC_UPD_UT=512: two per CU, two slots)
  size_t upd_lds_b = 0;
  int nrt = 0;
  int ncu = 256;  // compute units of the device
  // large-batch stage path (sac_wide.h): layout offsets, stages, jobs
  WideLay wl;
  int wide = 0;
  WideDev wdh;
  WideDev* wdd = nullptr;
  WJob* wjobs = nullptr;
  std::vector<WJob> hostW;
  struct WStage {
    int kind;   // 0 gather, 1 GEMM jobs [j0, j1), 2 pi heads, 3 phase B, 4 phase D
    int j0, j1, grid, phase, last;  // grid: workgroups
    size_t lds;
  };
  std::vector<WStage> wst;
  // graph cache
  hipGraphExec_t gexec = nullptr;
  hipGraph_t graph = nullptr;
  int gchunk = 0;
  sac_replay gkey{};
  hipStream_t cap = nullptr;
};

static inline int rup(int x, int m) { return (x + m - 1) / m * m; }


struct Layout {
  size_t off = 0;
  size_t take(size_t bytes) {
    off = (off + 255) & ~(size_t)255;
    const size_t o = off;
    off += bytes;
    return o;
  }
};

static int validate(const sac_engine_config* c) {
  if (!c) return fail(SAC_E_INVALID, "null config");
  if (c->obs_dim < 1 || c->act_dim < 1 || c->act_dim > 32) return fail(SAC_E_INVALID, "obs_dim >= 1, 1 <= act_dim <= 32");
  if (c->batch < 1 || c->batch > (1 << 20)) return fail(SAC_E_INVALID, "batch out of range");
  if (c->q_layers < 2 || c->q_layers > SAC_DEV_LAYERS || c->pi_layers < 2 || c->pi_layers > SAC_DEV_LAYERS)
    return fail(SAC_E_INVALID, "networks need 1..5 hidden layers");
  if (c->q_dims[0] != c->obs_dim + c->act_dim || c->q_dims[c->q_layers] != 1)
    return fail(SAC_E_INVALID, "q_dims must run obs+act -> ... -> 1");
  if (c->pi_dims[0] != c->obs_dim || c->pi_dims[c->pi_layers] != 2 * c->act_dim)
    return fail(SAC_E_INVALID, "pi_dims must run obs -> ... -> 2*act");
  for (int i = 0; i <= c->q_layers; ++i)
    if (c->q_dims[i] < 1) return fail(SAC_E_INVALID, "bad q dim");
  for (int i = 0; i <= c->pi_layers; ++i)
    if (c->pi_dims[i] < 1) return fail(SAC_E_INVALID, "bad pi dim");
  const int acts[4] = {c->q_hidden_act, c->q_out_act, c->pi_hidden_act, c->pi_out_act};
  for (int a : acts)
    if (a < 0 || a > 6) return fail(SAC_E_INVALID, "bad activation code");
  if (c->precision != SAC_PREC_FP32 && c->precision != SAC_PREC_BF16) return fail(SAC_E_INVALID, "bad precision");
  if (c->layout < SAC_LAYOUT_AUTO || c->layout > SAC_LAYOUT_PAIRS || c->stage_path < -1 || c->stage_path > 1 ||
      c->stage_batch < -1 || c->stage_batch > 0 || c->upd_parts < 0 || c->upd_parts > 4 ||
      (c->upd_threads != 0 && c->upd_threads != 512 && c->upd_threads != 1024))
    return fail(SAC_E_INVALID, "bad layout override (layout 0..3, stage_path -1..1, stage_batch -1..0, "
                               "upd_parts 0..4, upd_threads 0 / 512 / 1024)");
  return SAC_OK;
}

// Lays out everything; when e != nullptr also fills e->h pointers (base = workspace).
static void xcd_order(std::vector<TileDesc>& tiles);


// The large-batch path's device descriptor, jobs and stage list (sac_wide.h):
// per step  gather | A forward stages | pi heads | Qt forward stages | critic
// backward stages | B | C critic forward | critic dX | pi backward | D.
static void build_wide(sac_engine* e, char* base) {
  const WideLay& wl = e->wl;
  const EngineDev& h = e->h;
  const int esz = e->cfg.precision == SAC_PREC_BF16 ? 2 : 4;
  auto F = [&](size_t o) { return (float*)(base + o); };
  WideDev& W = e->wdh;
  memset(&W, 0, sizeof(W));
  const int B = h.B, A = h.A, O = h.O, Brw = wl.Brw, hp = wl.hp, hq = wl.hq;
  const NetDev& np = h.net[NET_PI];
  const NetDev& nq1 = h.net[NET_Q1];
  W.B = B;
  W.Bp = h.Bp;
  W.Brw = Brw;
  W.nrt = h.nrt;
  W.O = O;
  W.A = A;
  W.ldpi0 = np.l[0].Kp;
  W.ldq0 = nq1.l[0].Kp;
  W.Xpi0 = F(wl.o_xpi0);
  W.Xq0 = F(wl.o_xq0);
  W.Xqt0 = F(wl.o_xqt0);
  W.Xc0 = F(wl.o_xc0);
  W.R = F(wl.o_r);
  W.Dn = F(wl.o_d);
  W.LP2 = F(wl.o_lp2);
  W.PIOP = F(wl.o_piop);
  W.ncb_pi = (np.l[hp - 1].Np + 63) / 64;
  W.ncb_q = (nq1.l[hq - 1].Np + 63) / 64;
  W.ncb_da = (nq1.l[0].Np + 63) / 64;
  W.cbs_pi = (long)2 * Brw * 2 * A;
  W.cbs_q = Brw;
  W.cbs_da = (long)Brw * A;
  W.OUTPpi = F(wl.o_outpi);
  for (int qi = 0; qi < 2; ++qi) {
    W.OUTPq[qi] = F(wl.o_outq[qi]);
    W.OUTPqt[qi] = F(wl.o_outqt[qi]);
    W.OUTPc[qi] = F(wl.o_outc[qi]);
    W.DA[qi] = F(wl.o_da[qi]);
    W.GTq_out[qi] = h.net[NET_Q1 + qi].l[hq].GT;
    W.dbpq_out[qi] = h.net[NET_Q1 + qi].l[hq].dbp;
  }
  W.GTpi_out = np.l[hp].GT;
  W.dbppi_out = np.l[hp].dbp;
  W.rng_step = e->buf.rng_step;
  W.stamp_stage = -1;
#ifdef SAC_STAMPS  // diagnostic build only: the stage that writes stamps (tools/wide_stamps.py)
  if (const char* v = getenv("SAC_WIDE_STAMP_STAGE")) W.stamp_stage = atoi(v);
#endif
  e->wdd = (WideDev*)(base + wl.o_dev);
  e->wjobs = (WJob*)(base + wl.o_jobs);
  std::vector<WJob>& JB = e->hostW;
  JB.clear();
  e->wst.clear();
  // the two K-block buffers + the epilogue's weight slices (WWS floats); WA_OUTBWD
  // adds the row seeds and the output layer's weights
  // K-block buffers: as many (2..4) as keep the stage's workgroups co-resident
  // in one round (items / CUs per CU) in 160 KiB of LDS per CU
  const size_t kbuf = esz == 4 ? WK<float>::BUF : WK<bf16>::BUF;  // floats
  const int ncu = e->ncu > 0 ? e->ncu : 256;
  auto stage_gemm = [&](std::vector<WJob> js, int phase, int last) {
    int item = 0;
    size_t extra = WWS;  // floats past the K buffers
    for (WJob& j : js) {
      if (j.amode != js[0].amode) fprintf(stderr, "sac_engine: internal: mixed A modes in one stage\n"), abort();
      j.item0 = item;
      item += j.nrb * j.ncb;
      if (j.amode == WA_OUTBWD) extra = std::max(extra, (size_t)WWS + 64 * WLDD + (size_t)j.J * j.Kp);
      if ((j.OUTP && (size_t)j.Nout * WBN > WWS) || (j.DA && (size_t)WBN * A > WWS)) extra = ~(size_t)0 / 64;  // refused
    }
    const int per_cu = std::max(1, (item + ncu - 1) / ncu);
    int nb = 2;
    for (int b = 4; b > 2; --b)
      if ((size_t)per_cu * (b * kbuf + extra) * 4 <= 160 * 1024) {
        nb = b;
        break;
      }
    for (WJob& j : js) j.nbuf = nb;
    const size_t lf = nb * kbuf + extra;
    sac_engine::WStage st{1, (int)JB.size(), (int)(JB.size() + js.size()), item, phase, last, lf * 4};
    e->wst.push_back(st);
    JB.insert(JB.end(), js.begin(), js.end());
  };
  auto fwd = [&](int ni, int l, int M, const float* X, float* Pd, void* XT, int xt_row0, long xt_par, float* OUTP,
                 int p_row0 = 0) {
    const NetDev& nd = h.net[ni];
    const LayerDev& ly = nd.l[l];
    WJob j;
    memset(&j, 0, sizeof(j));
    j.M = M;
    j.K = ly.K;
    j.Kp = ly.Kp;
    j.N = ly.N;
    j.Np = ly.Np;
    j.nrb = M / 64;
    j.ncb = (ly.Np + 63) / 64;
    j.amode = l == 0 ? WA_PLAIN : WA_ACT;
    j.aact = nd.hid_act;
    j.X = X;
    j.ldx = ly.Kp;
    j.Wp = ly.Wc;
    j.tcols = ly.Kp;
    j.bias = nd.P + ly.b_off;
    j.emode = WE_FWD;
    j.P = Pd;
    j.p_row0 = p_row0;
    j.ldp = ly.Np;
    j.oact = nd.hid_act;
    j.XT = XT;
    j.xt_row0 = xt_row0;
    j.xt_ld = h.Bp;
    j.xt_par = xt_par;
    if (OUTP) {
      const LayerDev& lo = nd.l[nd.L - 1];
      j.Wout = nd.P + lo.w_off;
      j.ldwout = lo.K;
      j.Nout = lo.N;
      j.OUTP = OUTP;
      j.outp_cb = (long)M * lo.N;
    }
    j.pact = -1;
    return j;
  };
  // backward GEMM through layer d: dX_d = dY_d W_d -> dY_{d-1} = act'(P_{d-1}) dX_d
  auto bwd = [&](int ni, int d, int M, const float* X, bool first, int rowpro, int qi, const float* Pprev, float* DY,
                 void* GT, float* dbp, float* DA) {
    const NetDev& nd = h.net[ni];
    const LayerDev& ly = nd.l[d];
    const LayerDev& lb = nd.l[d - 1];
    const LayerDev& lo = nd.l[nd.L - 1];
    WJob j;
    memset(&j, 0, sizeof(j));
    j.M = M;
    j.K = ly.N;
    j.Kp = ly.Np;
    j.N = ly.K;
    j.Np = ly.Kp;
    j.nrb = M / 64;
    j.ncb = (ly.Kp + 63) / 64;
    j.amode = first ? WA_OUTBWD : WA_PLAIN;
    j.aact = nd.hid_act;
    j.X = X;
    j.ldx = ly.Np;
    if (first) {
      j.Wo = nd.P + lo.w_off;
      j.ldwo = lo.K;
      j.J = lo.N;
      j.rowpro = rowpro;
      j.qi = qi;
      if (GT) {  // phase A / pi: the generated dY of layer d is a dW operand too
        j.AGT = ly.GT;
        j.Adbp = ly.dbp;
        j.adbp_ld = ly.N;
      }
    }
    j.Wp = ly.WTc;
    j.tcols = ly.Np;
    j.emode = WE_BWD;
    j.Pprev = Pprev;
    j.ldpp = lb.Np;
    j.pact = nd.hid_act;
    j.DY = DY;
    j.lddy = lb.Np;
    j.GT = GT;
    j.gt_ld = h.Bp;
    j.dbp = dbp;
    j.dbp_ld = lb.N;
    if (DA) {
      const LayerDev& l0 = nd.l[0];
      j.W0a = nd.P + l0.w_off;
      j.ldw0 = l0.K;
      j.a_off = O;
      j.DA = DA;
      j.da_cb = (long)Brw * A;
    }
    return j;
  };
  auto add = [&](int kind, int grid, int phase) {
    sac_engine::WStage st{kind, 0, 0, grid, phase, 0, 0};
    e->wst.push_back(st);
  };
  // ---- phase A
  add(0, (B + WGR - 1) / WGR, 0);  // gather
  for (int d = 0; d < std::max(hp, hq); ++d) {
    std::vector<WJob> js;
    if (d < hp)
      // the last hidden layer's P is read by pi's backward only: actor rows [Brw, 2 Brw)
      js.push_back(fwd(NET_PI, d, 2 * Brw, d ? F(wl.o_P[0][d - 1]) : W.Xpi0, F(wl.o_P[0][d]), np.l[d + 1].XT, Brw,
                       np.l[d + 1].xt_par, d == hp - 1 ? W.OUTPpi : nullptr, d == hp - 1 ? Brw : 0));
    for (int qi = 0; qi < 2; ++qi)
      if (d < hq)
        js.push_back(fwd(NET_Q1 + qi, d, Brw, d ? F(wl.o_P[1 + qi][d - 1]) : W.Xq0, F(wl.o_P[1 + qi][d]),
                         h.net[NET_Q1 + qi].l[d + 1].XT, 0, 0, d == hq - 1 ? W.OUTPq[qi] : nullptr));
    stage_gemm(js, 0, 0);
  }
  {
    const int AP = A <= 1 ? 1 : 1 << (32 - __builtin_clz(A - 1));
    const int rpb = WG_T / AP;
    add(2, (2 * Brw + rpb - 1) / rpb, 0);  // pi heads
  }
  for (int d = 0; d < hq; ++d) {
    std::vector<WJob> js;
    for (int qi = 0; qi < 2; ++qi)
      js.push_back(fwd(NET_Q1T + qi, d, Brw, d ? F(wl.o_P[3 + qi][d - 1]) : W.Xqt0,
                       d < hq - 1 ? F(wl.o_P[3 + qi][d]) : nullptr, nullptr, 0, 0,  // no backward: last P unread
                       d == hq - 1 ? W.OUTPqt[qi] : nullptr));
    stage_gemm(js, 0, 0);
  }
  for (int d = hq - 1; d >= 1; --d) {
    std::vector<WJob> js;
    for (int qi = 0; qi < 2; ++qi) {
      const NetDev& nq = h.net[NET_Q1 + qi];
      const bool first = d == hq - 1;
      js.push_back(bwd(NET_Q1 + qi, d, Brw, first ? F(wl.o_P[1 + qi][d]) : F(wl.o_DYq[qi][d]), first, WR_YSEED, qi,
                       F(wl.o_P[1 + qi][d - 1]), d - 1 >= 1 ? F(wl.o_DYq[qi][d - 1]) : nullptr, nq.l[d - 1].GT,
                       nq.l[d - 1].dbp, nullptr));
    }
    stage_gemm(js, 0, 0);
  }
  add(3, 0, 1);  // phase B
  // ---- phase C
  for (int d = 0; d < hq; ++d) {
    std::vector<WJob> js;
    for (int qi = 0; qi < 2; ++qi)
      js.push_back(fwd(NET_Q1 + qi, d, Brw, d ? F(wl.o_Pc[qi][d - 1]) : W.Xc0, F(wl.o_Pc[qi][d]), nullptr, 0, 0,
                       d == hq - 1 ? W.OUTPc[qi] : nullptr));
    stage_gemm(js, 2, 0);
  }
  for (int d = hq - 1; d >= 1; --d) {
    std::vector<WJob> js;
    for (int qi = 0; qi < 2; ++qi) {
      const bool first = d == hq - 1;
      js.push_back(bwd(NET_Q1 + qi, d, Brw, first ? F(wl.o_Pc[qi][d]) : F(wl.o_DYc[qi][d]), first, WR_MINQ, qi,
                       F(wl.o_Pc[qi][d - 1]), d - 1 >= 1 ? F(wl.o_DYc[qi][d - 1]) : nullptr, nullptr, nullptr,
                       d == 1 ? W.DA[qi] : nullptr));
    }
    stage_gemm(js, 2, 0);
  }
  for (int d = hp - 1; d >= 1; --d) {
    const bool first = d == hp - 1;
    std::vector<WJob> js;
    js.push_back(bwd(NET_PI, d, Brw, first ? F(wl.o_P[0][d]) + (size_t)Brw * np.l[d].Np : F(wl.o_DYpi[d]), first,
                     WR_PIHEAD, 0, F(wl.o_P[0][d - 1]) + (size_t)Brw * np.l[d - 1].Np,
                     d - 1 >= 1 ? F(wl.o_DYpi[d - 1]) : nullptr, np.l[d - 1].GT, np.l[d - 1].dbp, nullptr));
    stage_gemm(js, 2, d == 1);
  }
  add(4, 0, 3);  // phase D
}

static size_t plan(const sac_engine_config* c, sac_engine* e, char* base) {
  const int esz = c->precision == SAC_PREC_BF16 ? 2 : 4;
  // Br: rows of the per-row stashes, whole pairs of row tiles (the pair-tile kernels write 2R rows)
  const int B = c->batch, Bp = rup(B, 32), nrt = (B + SAC_ROWS - 1) / SAC_ROWS, Br = rup(nrt, 2) * SAC_ROWS;
  const int O = c->obs_dim, A = c->act_dim;
  Layout lay;
  const size_t o_E = lay.take(4096);  // EngineDev, padded for prefetch_engine()
  EngineDev h;
  memset(&h, 0, sizeof(h));
  auto P = [&](size_t o) -> void* { return base ? (void*)(base + o) : nullptr; };
  int maxKp = 32, maxNo = 32;
  size_t xt_q0 = 0;
  const int nrt0 = (B + SAC_ROWS - 1) / SAC_ROWS;
  // dims-only pre-pass: the padded widths the phase kernels' LDS layout needs
  EngineDev probe;
  memset(&probe, 0, sizeof(probe));
  for (int ni = 0; ni < 5; ++ni) {
    const bool is_pi = ni == NET_PI;
    const int L = is_pi ? c->pi_layers : c->q_layers;
    const int* dims = is_pi ? c->pi_dims : c->q_dims;
    for (int l = 0; l < L; ++l) {
      probe.net[ni].l[l].Kp = rup(dims[l], SAC_PAD);
      probe.net[ni].l[l].Np = rup(dims[l + 1], SAC_PAD);
      maxKp = std::max(maxKp, probe.net[ni].l[l].Kp);
      if (l < L - 1) maxKp = std::max(maxKp, probe.net[ni].l[l].Np);
      else maxNo = std::max(maxNo, probe.net[ni].l[l].Np);
    }
  }
  int split = 0;  // decided below; the layout lambda reads it
  // pairs: the pair-tile kernels (sac_pairs.h): every per-row buffer 2R rows,
  // pre-activations for one critic or pi at a time (no P2 / second outputs)
  auto lds_layout = [&](EngineDev& hh, int xrows, bool full, bool pairs = false) -> int {
    const int R = pairs ? 2 * SAC_ROWS : SAC_ROWS;
    hh.ld = maxKp + 4;
    hh.ldo = maxNo + 4;
    int lo = 0;
    auto lt = [&](int floats) {
      lo = (lo + 3) & ~3;  // 16-B alignment
      const int o = lo;
      lo += floats;
      return o;
    };
    hh.o_X = lt(xrows * hh.ld);
    hh.o_Y = lt(xrows * hh.ld);
    const int Lhq = c->q_layers - 1, Lhp = c->pi_layers - 1;
    for (int l = 0; full && l < std::max(Lhq, Lhp); ++l) {
      int np = 0;
      if (l < Lhq) np = std::max(np, hh.net[NET_Q1].l[l].Np);
      if (l < Lhp) np = std::max(np, hh.net[NET_PI].l[l].Np);
      hh.ldp1[l] = np + 4;
      hh.o_P1[l] = lt(R * hh.ldp1[l]);
    }
    for (int l = 0; full && !pairs && l < Lhq; ++l) {
      hh.ldp2[l] = hh.net[NET_Q2].l[l].Np + 4;
      hh.o_P2[l] = lt(R * hh.ldp2[l]);
    }
    hh.o_s = lt(R * O);
    hh.o_s2 = lt(R * O);
    hh.o_a = lt(R * A);
    hh.o_a2 = lt(R * A);
    hh.o_r = lt(R);
    hh.o_d = lt(R);
    hh.o_et = lt(R * A);
    hh.o_ea = lt(R * A);
    hh.o_out = lt(xrows * hh.ldo);
    hh.o_outp = lt(xrows * hh.ldo);
    hh.o_out2 = pairs ? 0 : lt(R * hh.ldo);
    hh.o_outp2 = pairs ? 0 : lt(R * hh.ldo);
    hh.o_lp = lt(R);
    hh.o_qt = lt(2 * R);
    hh.o_y = lt(R);
    hh.o_g = lt(pairs ? 2 * R : R * hh.ldo);
    hh.o_g2 = pairs ? 0 : lt(R * hh.ldo);
    hh.o_ga = lt(R * A);
    hh.o_gout = lt(R * hh.ldo);
    hh.o_slot = lt(2 * R);  // int64[R]
    hh.o_red = split ? lt(SAC_NW * 256) : 0;
    return lo;
  };
  // does the phase kernels' layout fit a CU?  (per-network roles: R rows; one
  // block per row tile: pi on [s'; s], 2R rows)
  const bool lds_fits_roles = (size_t)lds_layout(probe, SAC_ROWS, true) * 4 <= 160 * 1024;
  const bool lds_fits_rows = (size_t)lds_layout(probe, 2 * SAC_ROWS, true) * 4 <= 160 * 1024;
  const bool lds_fits_pairs = (size_t)lds_layout(probe, 2 * SAC_ROWS, true, true) * 4 <= 160 * 1024;
  // hidden-split role kernels (sac_split.h): two hidden layers of width 256 in
  // both nets, identity pi output, 2 act <= 32, and 12 * nrt co-resident blocks
  split = lds_fits_roles && c->q_layers == 3 && c->pi_layers == 3 && c->q_dims[1] == SPLIT_H && c->q_dims[2] == SPLIT_H &&
              c->pi_dims[1] == SPLIT_H && c->pi_dims[2] == SPLIT_H && c->pi_out_act == SAC_ACT_IDENTITY &&
              2 * A <= 32 && (10 + split_wpi(esz)) * nrt0 <= 256 && (2 * split_wcq(esz) + split_wc(esz) + 1) * nrt0 <= 256 &&
              SAC_ROWS * (A + 1) <= SAC_HAND_STRIDE;
  split = split && c->layout == SAC_LAYOUT_AUTO;
  // batch columns of layer 0's operands under the split: X^T 2 Bp (phase A's two
  // halves store it), dY^T 2 Bp for the critics (phase A halves), split_wc Bp for
  // pi (phase C parts)
  const int wc = split_wc(esz);
  const int bp0 = split ? 2 * Bp : Bp;
  const int bp0_pi = split ? wc * Bp : Bp;
  for (int ni = 0; ni < 5; ++ni) {
    const bool is_pi = ni == NET_PI;
    const bool trainable = ni <= NET_Q2;
    const int L = is_pi ? c->pi_layers : c->q_layers;
    const int* dims = is_pi ? c->pi_dims : c->q_dims;
    NetDev& nd = h.net[ni];
    nd.L = L;
    nd.hid_act = is_pi ? c->pi_hidden_act : c->q_hidden_act;
    nd.out_act = is_pi ? c->pi_out_act : c->q_out_act;
    int off = 0;
    for (int l = 0; l < L; ++l) {
      LayerDev& ly = nd.l[l];
      ly.K = dims[l];
      ly.N = dims[l + 1];
      ly.Kp = rup(ly.K, SAC_PAD);
      ly.Np = rup(ly.N, SAC_PAD);
      ly.w_off = off;
      off += ly.K * ly.N;
      ly.b_off = off;
      off += ly.N;
      maxKp = std::max(maxKp, ly.Kp);
      if (l < L - 1) maxKp = std::max(maxKp, ly.Np);
      else maxNo = std::max(maxNo, ly.Np);
      ly.Wc = P(lay.take((size_t)ly.Np * ly.Kp * esz));
      if (trainable) {
        const int bpl = l == 0 ? bp0 : Bp;
        ly.WTc = P(lay.take((size_t)ly.Kp * ly.Np * esz));
        if (ni == NET_Q2 && l == 0) {
          ly.XT = P(xt_q0);
        } else {
          // pi: two copies by step parity (from the fused step, where phase D of
          // step k read one while phase A of step k + 1 wrote the other in one
          // launch; with one phase per launch they only alternate)
          const size_t o = lay.take((size_t)ly.Kp * bpl * esz * (is_pi ? 2 : 1));
          if (ni == NET_Q1 && l == 0) xt_q0 = o;
          ly.XT = P(o);
          ly.xt_par = is_pi ? (long)ly.Kp * bpl : 0;
        }
        const int bpg = (l == 0 && is_pi) ? bp0_pi : bpl;
        ly.GT = P(lay.take((size_t)ly.Np * bpg * esz));
        // the update tiles sum the bias gradient from their staged dY^T rows:
        // no per-row-tile partials (TileDesc / store_T with dbp == null)
        ly.dbp = nullptr;
      }
      if (is_pi) ly.pstash = (float*)P(lay.take((size_t)Br * ly.Np * 4));
      if (is_pi) ly.pmask = (uint32_t*)P(lay.take((size_t)Br * ((ly.Np + 31) / 32) * 4));
    }
  }
  h.s_st = (float*)P(lay.take((size_t)Br * O * 4));
  h.a_st = (float*)P(lay.take((size_t)Br * A * 4));
  h.lp_st = (float*)P(lay.take((size_t)2 * Br * 4));
  h.head_st = (float*)P(lay.take((size_t)Br * 4 * A * 4));
  h.lossp = (float*)P(lay.take((size_t)2 * nrt * 4 * 4));
  h.seedq = (float*)P(lay.take((size_t)2 * Bp * 4));
  h.adam_sc = (float*)P(lay.take(2 * 6 * 4));
  h.alpha_sc = (double*)P(lay.take(2 * 2 * 8));
  h.sync = (uint32_t*)P(lay.take((size_t)(SYNC_FLAGS + HK_COUNT * nrt * 16) * 4));
  h.hand = (float*)P(lay.take((size_t)HK_COUNT * nrt * SAC_HAND_STRIDE * 4));
  h.gstride = SAC_ROWS * (A + 1);
  h.gran = (uint64_t*)P(lay.take((size_t)G_COUNT * nrt * h.gstride * 8));
  h.stg_stride = (16 + 2 * SAC_ROWS * O + SAC_ROWS * A + 2 * SAC_ROWS + 15) / 16 * 16;
  h.stg = (float*)P(lay.take((size_t)2 * nrt * h.stg_stride * 4));  // two records per row tile: by step parity
  h.split = split;
  h.gs2 = SAC_ROWS * std::max(2 * A, A + 1);
  h.gran2 = (uint64_t*)P(lay.take((size_t)GS_COUNT * nrt * SPLIT_GP * h.gs2 * 8));
  // Batch parts of an update tile (TileDesc.kpart): the hidden split's layer 0
  // reduces over its parts' columns (critics 2: phase A halves; pi wc: phase C
  // parts); a large batch (Bp > 1024) is split into P <= 4 parts per phase, P
  // chosen for the fewest block rounds x the longest block: a block takes about
  // 2 us + its operand bytes at ~25 GB/s (one workgroup per CU; measured on C3:
  // 1024 fp32 columns = 256 KB of dY^T / X^T in ~12 us), so at C3 (160 critic
  // tiles, 80 policy tiles) P = 3: 480 blocks (2 rounds) for B and 240 (one) for D.
  // fp32 hidden-split layer 0: the parts' partial dY summed while staging in one
  // block (TileDesc.gsum), which also sees every batch column of the tile -- the
  // seeded bias sums of TileDesc.seed rely on that; bf16: a block per dY part
  // with a granule hand-off to part 1
  // fp32 split layer 0 (wc / 2 summed dY parts: the longest tiles of phases D /
  // B, 5 / 3 operand row sets) is also split into 2 batch parts with a granule
  // hand-off (the critics' producer parts also hand over their seeded bias
  // sums): measured D 8.3 -> 7.6 us on C2.  bf16: the parts' bf16 dY added in
  // fp32 and rounded once while staging, one block per tile (23.1K -> 23.6K
  // steps/s on C2, B 7.0 -> 6.6, D 6.7 -> 6.2 us, profiles/r04_ab_gsum_bf16_c2.txt)
  const int pi0_parts = esz == 4 ? 2 : 1, q0_parts = esz == 4 ? 2 : 1;
  const int TS = 32;  // update tiles are 32 x 32 weight blocks (64 x 64 measured slower at C3: profiles/r04_ab_tile64_c3.txt)
  // the 32 x 32 tiles sum the bias gradient from their staged dY rows (16-B
  // LDS reads) instead of loading per-row-tile partials (at C3 256 strided
  // loads per column made the k0 == 0 tiles the tail of phases B and D): C3
  // 4.47K -> 4.57K fp32, 7.63K -> 8.0K bf16; C2 19.3K -> 19.5K fp32, 23.45K ->
  // 24.0K bf16 (profiles/r04_ab_bias_staged.txt)
  const size_t part_stride = SAC_PART_STRIDE;
  auto ntiles_of = [&](const LayerDev& ly) { return ((ly.Np + TS - 1) / TS) * ((ly.Kp + TS - 1) / TS); };
  int tilesBD[2] = {0, 0};  // [critics (B), policy (D)]
  for (int ni = NET_PI; ni <= NET_Q2; ++ni)
    for (int l = 0; l < h.net[ni].L; ++l) tilesBD[ni == NET_PI] += ntiles_of(h.net[ni].l[l]);
  auto batch_parts = [&](int ntiles, int extra) {
    if (Bp <= 1024) return 1;
    if (c->upd_parts > 0) return std::min(4, (int)c->upd_parts);
    int best = 4;
    double bc = 1e30;
    for (int P = 2; P <= 4; ++P) {
      const int rounds = (ntiles * P + extra + 255) / 256;
      const double c = rounds * (2.0 + 64.0 * rup((Bp + P - 1) / P, 32) * esz / 25e3);  // us
      if (c < bc - 1e-9) bc = c, best = P;
    }
    return best;
  };
  const int bpartsB = batch_parts(tilesBD[0], 0);
  const int bpartsD = batch_parts(tilesBD[1], 1);
  auto tile_parts = [&](int ni, int l) {
    if (l == 0 && split) return std::min(ni == NET_PI ? pi0_parts : q0_parts, Bp / 32);
    return ni == NET_PI ? bpartsD : bpartsB;
  };
  int nB = 0, nD = 0, nhalf = 0;
  for (int ni = NET_PI; ni <= NET_Q2; ++ni)
    for (int l = 0; l < h.net[ni].L; ++l) {
      const int t = ntiles_of(h.net[ni].l[l]);
      const int parts = tile_parts(ni, l);
      (ni == NET_PI ? nD : nB) += t * parts;
      nhalf += t * (parts - 1);  // producer parts: one granule slot each
    }
  // Layer-synchronous stage path (sac_wide.h): where the phase
  // kernels' LDS layout does not fit a CU (hidden layers wider than 256, wide
  // inputs: the stage path takes any width), for nets with at least two hidden
  // layers.  At C3 the row-tile kernels are faster (profiles/r04_ab_c3_paths.txt),
  // so they keep the batches they fit; config.stage_path = 1 forces the stage
  // path on any batch past the hidden split, -1 refuses it.
  WideLay wl;
  {
    const int roles_pre = 6 * nrt0 <= 256 && SAC_ROWS * (A + 1) <= SAC_HAND_STRIDE && c->layout != SAC_LAYOUT_ROWS &&
                          c->layout != SAC_LAYOUT_PAIRS;
    const bool too_big = !(roles_pre ? lds_fits_roles : lds_fits_rows);
    const bool able = !split && c->q_layers >= 3 && c->pi_layers >= 3 && 2 * A <= WJMAX;
    int on = able && too_big;
    if (c->stage_path > 0) on = able;
    if (c->stage_path < 0) on = 0;
    wl.on = on;
  }
  if (wl.on) {
    const int Brw = rup(B, 64);
    const NetDev& np = h.net[NET_PI];
    const NetDev& nq = h.net[NET_Q1];
    const int hp = c->pi_layers - 1, hq = c->q_layers - 1;
    wl.Brw = Brw;
    wl.hp = hp;
    wl.hq = hq;
    wl.o_dev = lay.take(sizeof(WideDev));
    wl.o_jobs = lay.take(WIDE_MAX_JOBS * sizeof(WJob));
    wl.o_xpi0 = lay.take((size_t)2 * Brw * np.l[0].Kp * 4);
    wl.o_xq0 = lay.take((size_t)Brw * nq.l[0].Kp * 4);
    wl.o_xqt0 = lay.take((size_t)Brw * nq.l[0].Kp * 4);
    wl.o_xc0 = lay.take((size_t)Brw * nq.l[0].Kp * 4);
    wl.o_r = lay.take((size_t)Brw * 4);
    wl.o_d = lay.take((size_t)Brw * 4);
    wl.o_lp2 = lay.take((size_t)Brw * 4);
    wl.o_piop = lay.take((size_t)Brw * 2 * A * 4);
    const int ncb_pi = (np.l[hp - 1].Np + 63) / 64, ncb_q = (nq.l[hq - 1].Np + 63) / 64, ncb_da = (nq.l[0].Np + 63) / 64;
    wl.o_outpi = lay.take((size_t)ncb_pi * 2 * Brw * 2 * A * 4);
    for (int qi = 0; qi < 2; ++qi) {
      wl.o_outq[qi] = lay.take((size_t)ncb_q * Brw * 4);
      wl.o_outqt[qi] = lay.take((size_t)ncb_q * Brw * 4);
      wl.o_outc[qi] = lay.take((size_t)ncb_q * Brw * 4);
      wl.o_da[qi] = lay.take((size_t)ncb_da * Brw * A * 4);
    }
    for (int l = 0; l < hp; ++l) wl.o_P[0][l] = lay.take((size_t)2 * Brw * np.l[l].Np * 4);
    for (int l = 1; l + 1 < hp; ++l) wl.o_DYpi[l] = lay.take((size_t)Brw * np.l[l].Np * 4);
    for (int qi = 0; qi < 2; ++qi) {
      for (int l = 0; l < hq; ++l) {
        const size_t bytes = (size_t)Brw * nq.l[l].Np * 4;
        wl.o_P[1 + qi][l] = lay.take(bytes);
        wl.o_P[3 + qi][l] = lay.take(bytes);
        wl.o_Pc[qi][l] = lay.take(bytes);
      }
      for (int l = 1; l + 1 < hq; ++l) {
        wl.o_DYq[qi][l] = lay.take((size_t)Brw * nq.l[l].Np * 4);
        wl.o_DYc[qi][l] = lay.take((size_t)Brw * nq.l[l].Np * 4);
      }
    }
  }
  const size_t o_tB = lay.take((size_t)nB * sizeof(TileDesc));
  const size_t o_tD = lay.take((size_t)nD * sizeof(TileDesc));
  const size_t o_part = lay.take((size_t)nhalf * part_stride * 8);  // batch-part partial dW granules
  const size_t total = lay.take(0);

  // LDS layout (floats) of the row-tile / role kernels (policy_act included).
  // role split of phases A/C (decided here: it sizes the LDS): 6 * nrt
  // workgroups must be co-resident (one per CU).  Only the one-block-per-row-
  // tile kernels run pi on [s'; s] (2R rows); with roles every MLP pass is R rows.
  // The stage path (wl.on) launches none of them but policy_act: R rows, no
  // pre-activation buffers.
  int roles = 6 * nrt <= 256 && SAC_ROWS * (A + 1) <= SAC_HAND_STRIDE && c->layout != SAC_LAYOUT_ROWS &&
              c->layout != SAC_LAYOUT_PAIRS;
  roles = roles && !wl.on;
  // pair-tile kernels (sac_pairs.h): two row tiles and one group of networks per
  // workgroup; the critics' seeds are applied by phase B (TileDesc::seed).  The
  // default past the role split wherever its LDS layout fits: C3 4.66K -> 4.90K
  // steps/s fp32, 8.26K -> 9.58K bf16 (profiles/r05_ab_pair_tiles_c3.txt)
  const int pairs = !split && !roles && !wl.on &&
                    (c->layout == SAC_LAYOUT_PAIRS || c->layout == SAC_LAYOUT_AUTO) && lds_fits_pairs &&
                    SAC_ROWS * (A + 1) <= SAC_HAND_STRIDE &&
                    SAC_ROWS * (2 * O + A + 2) <= 4 * SAC_THREADS;  // pair_batch: a record in 4 loads per thread
  const int lo = pairs ? lds_layout(h, 2 * SAC_ROWS, true, true)
                       : lds_layout(h, wl.on || roles ? SAC_ROWS : 2 * SAC_ROWS, !wl.on);

  if (e) {
    h.B = B;
    h.Bp = Bp;
    h.Br = Br;
    h.O = O;
    h.A = A;
    h.nrt = nrt;
    {
      int xs = 1;  // largest power of two <= 8 with nrt * xs <= 256 blocks
      while (xs < 8 && nrt * xs * 2 <= 256) xs *= 2;
      h.xs = xs;
      // phase A's weight parts on one or two XCDs each: A's fetched bytes 11.0 -> 5.1
      // MB per launch, phase B 8.6 -> 8.1 us, +1.2% steps/s (C2 fp32,
      // profiles/r03_ab_role_xcd.txt)
      h.role_xcd = split && (10 + split_wpi(esz)) * nrt % 8 == 0;
      // role split of phases A/C: 6 * nrt workgroups must be co-resident (one per CU)
      h.roles = roles;
      h.pairs = pairs;
      // phase C stages the next step's batch (config.stage_batch = -1 turns it off)
      h.stage = c->stage_batch >= 0;
    }
    h.auto_entropy = c->auto_entropy;
    h.alpha_update = 1;
    h.gamma = c->gamma;
    h.tau = c->tau;
    h.ls_min = c->log_std_min;
    h.ls_max = c->log_std_max;
    h.scale = c->action_scale;
    h.actor_lr = c->actor_lr;
    h.critic_lr = c->critic_lr;
    h.beta1 = c->beta1;
    h.beta2 = c->beta2;
    h.adam_eps = c->adam_eps;
    h.target_entropy = c->target_entropy;
    h.alpha_lr = c->alpha_lr;
    h.seed = c->seed;
    h.spin_limit = 1 << 22;
    float* parts[5] = {e->buf.pi, e->buf.q1, e->buf.q2, e->buf.q1t, e->buf.q2t};
    float* ms[3] = {e->buf.pi_m, e->buf.q1_m, e->buf.q2_m};
    float* vs[3] = {e->buf.pi_v, e->buf.q1_v, e->buf.q2_v};
    for (int ni = 0; ni < 5; ++ni) {
      h.net[ni].P = parts[ni];
      h.net[ni].M = ni < 3 ? ms[ni] : nullptr;
      h.net[ni].V = ni < 3 ? vs[ni] : nullptr;
      for (int l = 0; l < h.net[ni].L; ++l) h.net[ni].l[l].bias = parts[ni] + h.net[ni].l[l].b_off;
    }
    h.alpha_state = e->buf.alpha_state;
    h.opt_steps = e->buf.opt_steps;
    h.rng_step = e->buf.rng_step;
    h.stats = e->buf.stats;
    e->h = h;
    e->d = (EngineDev*)(base + o_E);
    e->tilesB = (TileDesc*)(base + o_tB);
    e->tilesD = (TileDesc*)(base + o_tD);
    e->nB = nB;
    e->nD = nD;
    e->h.tilesB = e->tilesB;
    e->h.tilesD = e->tilesD;
    e->h.nB = nB;
    e->h.nD = nD;
    e->lds_bytes = (size_t)lo * 4;
    {  // update tiles stage up to 2 batch chunks of 512 B per operand row per round
       // (every tile reduces over at most Bp columns: split layer 0 is two half tiles)
      const int bch = 512 / esz;
      e->h.upd_slots = std::min(2, (Bp + bch - 1) / bch);
      e->upd_lds = SAC_UPD_LDS_FOR(e->h.upd_slots);
      // phase B in 2 rounds of 1024-thread blocks (C3: 480 blocks) -> 512-thread
      // blocks with 2 slots, two per CU, one round: C3 B 37.0 -> 33.5 us fp32,
      // 20.0 -> 18.1 bf16 (profiles/r04_ab_upd_ut512_c3.txt); config.upd_threads =
      // 512 / 1024 forces it (no summed layer-0 tiles: GS 1 only, so never with the
      // hidden split)
      int ut512 = nB > 256 && nB <= 512;
      if (c->upd_threads) ut512 = c->upd_threads == 512;
      e->upd_ut_b = SAC_UPD_THREADS;
      e->upd_lds_b = e->upd_lds;
      if (ut512 && !split) {
        e->upd_ut_b = 512;
        e->upd_lds_b = SAC_UPD_LDS_FOR(1);  // one slot (sac_phases.h, dw_adam_tile)
      }
    }
    e->nrt = nrt;
    // self-contained update tiles (phase B: critics + Polyak, phase D: policy)
    const int esz2 = esz;
    e->hostB.clear();
    e->hostD.clear();
    std::vector<TileDesc> halvesB, halvesD;
    int ihalf = 0;
    for (int ni = NET_PI; ni <= NET_Q2; ++ni) {
      const NetDev& nd = h.net[ni];
      const NetDev& tn = h.net[ni == NET_PI ? NET_PI : ni + 2];
      for (int l = 0; l < nd.L; ++l) {
        const LayerDev& ly = nd.l[l];
        for (int nt = 0; nt < (ly.Np + TS - 1) / TS; ++nt)
          for (int kt = 0; kt < (ly.Kp + TS - 1) / TS; ++kt) {
            TileDesc t;
            memset(&t, 0, sizeof(t));
            const int bpl = (l == 0 && split) ? 2 * Bp : Bp;                     // X^T row stride
            const int bpg = (l == 0 && split) ? (ni == NET_PI ? wc : 2) * Bp : Bp;  // dY^T row stride
            t.GT = (const char*)ly.GT + (size_t)nt * TS * bpg * esz2;
            t.XT = (const char*)ly.XT + (size_t)kt * TS * bpl * esz2;
            t.W = nd.P + ly.w_off;
            t.Wm = nd.M + ly.w_off;
            t.Wv = nd.V + ly.w_off;
            t.b = nd.P + ly.b_off;
            t.bm = nd.M + ly.b_off;
            t.bv = nd.V + ly.b_off;
            t.Wc = ly.Wc;
            t.WTc = ly.WTc;
            if (ni != NET_PI) {
              t.tW = tn.P + ly.w_off;
              t.tb = tn.P + ly.b_off;
              t.tWc = tn.l[l].Wc;
            }
            t.xt_par = ly.xt_par;
            t.bp = (l == 0 && split) ? 2 * Bp : Bp;
            t.K = ly.K;
            t.N = ly.N;
            t.Kp = ly.Kp;
            t.Np = ly.Np;
            t.n0 = nt * TS;
            t.k0 = kt * TS;
            t.opt = ni;
            t.ld = t.bp;
            t.ldx = t.bp;
            t.kpart = 0;
            t.nparts = 1;
            t.gsum = 1;
            t.goff = 0;
            t.seed = nullptr;
            if ((split || pairs) && ni != NET_PI) t.seed = h.seedq + (size_t)(ni - NET_Q1) * Bp;
            if (l == 0 && split) {  // one block: dY parts [p Bp, (p+1) Bp) summed, X^T [0, Bp)
              t.gsum = ni == NET_PI ? wc : 2;
              t.goff = Bp;
              t.bp = Bp;
              t.ld = bpg;
              t.ldx = 2 * Bp;
            }
            const int parts = tile_parts(ni, l);
            if (parts > 1) {
              // consumer part 1 (batch columns [0, bpp)) + producer parts 2..P ([(p-1) bpp, p bpp));
              // split layer 0 (gsum): batch parts of the summed operands
              const int total = Bp;
              const int bpp = rup((Bp + parts - 1) / parts, 32);
              if (!(l == 0 && split)) {
                t.ld = Bp;
                t.ldx = Bp;
              }
              t.bp = bpp;
              t.kpart = 1;
              t.nparts = parts;
              t.part = (uint64_t*)(base + o_part) + (size_t)ihalf * part_stride;
              ihalf += parts - 1;
              for (int pp = 2; pp <= parts; ++pp) {
                TileDesc pt = t;
                const int off = (pp - 1) * bpp;
                pt.kpart = pp;
                pt.bp = std::min(bpp, total - off);
                pt.GT = (const char*)t.GT + (size_t)off * esz2;
                pt.XT = (const char*)t.XT + (size_t)off * esz2;
                if (t.seed) pt.seed = t.seed + off;
                (ni == NET_PI ? halvesD : halvesB).push_back(pt);
              }
            }
            (ni == NET_PI ? e->hostD : e->hostB).push_back(t);
          }
      }
    }
    auto order = [&](std::vector<TileDesc>& cons, std::vector<TileDesc>& prod) {
      xcd_order(cons);
      // producer parts first: in-order dispatch starts every producer before its consumer
      cons.insert(cons.begin(), prod.begin(), prod.end());
    };
    order(e->hostB, halvesB);
    order(e->hostD, halvesD);
    e->h.nBq[0] = e->h.nBq[1] = 0;
    for (const TileDesc& t : e->hostB) ++e->h.nBq[t.opt - 1];
    e->wl = wl;
    e->wide = wl.on;
    if (wl.on) build_wide(e, base);
  }
  return total + 256;
}

// Update-tile order for the XCDs (speed only; any order gives the same bits).
// Blocks are dealt round-robin to the 8 XCDs (block b on XCD b % 8), and the
// dW operands come from other XCDs' L2s (fetched through the Infinity Fabric
// at ~11 B/cycle per CU). A layer's tile (nt, kt) reads dY^T rows nt and X^T
// rows kt; tiles sharing them on one XCD fetch them once into that L2. So each
// net's tiles are bucketed by XCD -- a 256x256 layer's 8x8 tiles as 2 nt x 4 kt
// blocks per XCD (6 row groups fetched per XCD instead of 16), one-column /
// one-row layers dealt across the XCDs -- and emitted so that position p holds
// a tile of bucket p % 8.
static void xcd_order(std::vector<TileDesc>& tiles) {
  std::vector<TileDesc> out;
  out.reserve(tiles.size());
  size_t i = 0;
  while (i < tiles.size()) {
    size_t j = i;  // one net: consecutive tiles of the same optimizer
    while (j < tiles.size() && tiles[j].opt == tiles[i].opt) ++j;
    std::vector<TileDesc> bucket[8];
    for (size_t t = i; t < j; ++t) {
      const TileDesc& d = tiles[t];
      const int NT = d.Np / 32, KT = d.Kp / 32, nt = d.n0 / 32, kt = d.k0 / 32;
      int x;
      if (KT == 1) x = nt % 8;
      else if (NT == 1) x = kt % 8;
      else if (NT >= 4 && KT >= 2) x = (nt * 4 / NT) * 2 + (kt * 2 / KT);
      else x = (nt * KT + kt) % 8;
      bucket[x].push_back(d);
    }
    size_t taken[8] = {0};
    for (size_t left = j - i; left;) {
      for (int x = 0; x < 8; ++x)
        if (taken[x] < bucket[x].size()) {
          out.push_back(bucket[x][taken[x]++]);
          --left;
        }
    }
    i = j;
  }
  tiles.swap(out);
}

template <typename T>
static void set_lds_attrs(size_t bytes) {
  (void)bytes;
  const int b = 160 * 1024;  // the launch passes what it needs; the attribute is the cap
  (void)hipFuncSetAttribute((const void*)sac_target_critic<T, false>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_target_critic<T, true>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_actor<T, false>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_actor<T, true>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_policy_act_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_target_critic_split<T>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_target_critic_pairs<T>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_actor_pairs<T>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_actor_split<T>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_critic_update<T>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_critic_update<T, 512>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_actor_update<T>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_wide_stage<T, WA_PLAIN, false>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_wide_stage<T, WA_ACT, false>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_wide_stage<T, WA_OUTBWD, false>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_wide_stage<T, WA_PLAIN, true>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_wide_stage<T, WA_ACT, true>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_wide_stage<T, WA_OUTBWD, true>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_wide_gather<T>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
  (void)hipFuncSetAttribute((const void*)sac_wide_head<T>, hipFuncAttributeMaxDynamicSharedMemorySize, b);
}

// empty kernel: the dispatch + event gap of sac_engine_time_phases
__global__ void sac_noop_kernel() {}
// one wave spinning `ticks` of the 100 MHz realtime clock: holds the stream
// while the host enqueues a timed sequence, so its launches run back to back
// at device speed instead of host-submission speed
__global__ void sac_spin_kernel(long long ticks) {
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

// Launch kinds of a step: A B C D.
enum LaunchKind { L_A = 0, L_B = 1, L_C = 2, L_D = 3 };

template <typename T>
static void launch_kind(sac_engine* e, int kind, const sac_replay* rb, const int32_t* idx, const float* eps,
                        hipStream_t s) {
  const size_t lf = std::max(e->lds_bytes, e->upd_lds);
  const int stg = e->h.stage ? e->nrt : 0;  // stager blocks of phase C
  switch (kind) {
    case L_A:
      if (e->h.split)
        sac_target_critic_split<T><<<e->nrt * (10 + split_wpi((int)sizeof(T))), SAC_THREADS, lf, s>>>(e->d, *rb, idx,
                                                                                                  eps);
      else if (e->h.roles)
        sac_target_critic<T, true><<<e->nrt * 6, SAC_THREADS, lf, s>>>(e->d, *rb, idx, eps);
      else if (e->h.pairs)
        sac_target_critic_pairs<T><<<2 * ((e->nrt + 1) / 2), SAC_THREADS, lf, s>>>(e->d, *rb, idx, eps);
      else
        sac_target_critic<T, false><<<e->nrt * e->h.xs, SAC_THREADS, lf, s>>>(e->d, *rb, idx, eps);
      break;
    case L_B:
      if (e->upd_ut_b == 512)
        sac_critic_update<T, 512><<<e->nB, 512, e->upd_lds_b, s>>>(e->d, e->tilesB);
      else
        sac_critic_update<T><<<e->nB, SAC_UPD_THREADS, e->upd_lds, s>>>(e->d, e->tilesB);
      break;
    case L_C:
      if (e->h.split)
        sac_actor_split<T><<<e->nrt * (2 * split_wcq((int)sizeof(T)) + split_wc((int)sizeof(T))) + stg, SAC_THREADS,
                             lf, s>>>(e->d, *rb);
      else if (e->h.roles)
        sac_actor<T, true><<<e->nrt * 3 + stg, SAC_THREADS, lf, s>>>(e->d, *rb);
      else if (e->h.pairs)
        sac_actor_pairs<T><<<2 * ((e->nrt + 1) / 2) + stg, SAC_THREADS, lf, s>>>(e->d, *rb);
      else
        sac_actor<T, false><<<e->nrt * e->h.xs + stg, SAC_THREADS, lf, s>>>(e->d, *rb);
      break;
    case L_D:
      sac_actor_update<T><<<e->nD + 1, SAC_UPD_THREADS, e->upd_lds, s>>>(e->d, e->tilesD, e->nD);
      break;
  }
}

// One launch of the large-batch stage path (sac_wide.h).
template <typename T>
static void launch_wide_stage(sac_engine* e, const sac_engine::WStage& st, const sac_replay* rb, const int32_t* idx,
                              const float* eps, hipStream_t s, bool stage_next, const int32_t* next_idx) {
  const size_t glds = (size_t)((WGR * (e->cfg.obs_dim + e->cfg.act_dim) + 1) & ~1) * 4 + WGR * 8;
  switch (st.kind) {
    case 0:
      sac_wide_gather<T><<<st.grid, WG_T, glds, s>>>(e->d, e->wdd, *rb, idx);
      break;
    case 1: {
      // the last phase-C stage also gathers the next step's batch (when there is one in this call)
      const int ng = st.last && stage_next ? (e->cfg.batch + WGR - 1) / WGR : 0;
      const int flags = st.last | (&st == &e->wst[1] ? 2 : 0) | (ng ? 4 : 0) | (int)((&st - e->wst.data()) << 8);
      const bool relu = e->cfg.q_hidden_act == ACT_RELU && e->cfg.pi_hidden_act == ACT_RELU;
      const int am = e->hostW[st.j0].amode;  // one A-operand mode per stage (build_wide)
      auto k = relu ? (am == WA_PLAIN ? sac_wide_stage<T, WA_PLAIN, true>
                       : am == WA_ACT ? sac_wide_stage<T, WA_ACT, true> : sac_wide_stage<T, WA_OUTBWD, true>)
                    : (am == WA_PLAIN ? sac_wide_stage<T, WA_PLAIN, false>
                       : am == WA_ACT ? sac_wide_stage<T, WA_ACT, false> : sac_wide_stage<T, WA_OUTBWD, false>);
      k<<<st.grid + ng, WG_T, std::max(st.lds, ng ? glds : 0), s>>>(e->d, e->wdd, e->wjobs + st.j0, st.j1 - st.j0,
                                                                    flags, st.grid, *rb, next_idx);
      break;
    }
    case 2:
      sac_wide_head<T><<<st.grid, WG_T, 0, s>>>(e->d, e->wdd, eps);
      break;
    case 3:
      launch_kind<T>(e, L_B, rb, idx, eps, s);
      break;
    case 4:
      launch_kind<T>(e, L_D, rb, idx, eps, s);
      break;
  }
}
static void launch_wide(sac_engine* e, const sac_engine::WStage& st, const sac_replay* rb, const int32_t* idx,
                        const float* eps, hipStream_t s, bool stage_next = false, const int32_t* next_idx = nullptr) {
  if (e->cfg.precision == SAC_PREC_BF16)
    launch_wide_stage<bf16>(e, st, rb, idx, eps, s, stage_next, next_idx);
  else
    launch_wide_stage<float>(e, st, rb, idx, eps, s, stage_next, next_idx);
}

// The launches of n consecutive steps (and, per launch, its kind in *kinds).
static void launch_steps(sac_engine* e, const sac_replay* rb, int n, const int32_t* indices, const float* eps,
                         hipStream_t s, std::vector<int>* kinds = nullptr, std::vector<hipEvent_t>* ev = nullptr) {
  const size_t B = e->cfg.batch, A = e->cfg.act_dim;
  auto go = [&](int kind, int step) {
    const int32_t* ix = indices ? indices + (size_t)step * B : nullptr;
    const float* ep = eps ? eps + (size_t)step * 2 * B * A : nullptr;
    if (e->cfg.precision == SAC_PREC_BF16)
      launch_kind<bf16>(e, kind, rb, ix, ep, s);
    else
      launch_kind<float>(e, kind, rb, ix, ep, s);
    if (kinds) kinds->push_back(kind);
    if (ev) {
      hipEvent_t x;
      (void)hipEventCreate(&x);
      (void)hipEventRecord(x, s);
      ev->push_back(x);
    }
  };
  if (e->wide) {  // the stage sequence of sac_wide.h per step
    for (int i = 0; i < n; ++i) {
      const int32_t* ix = indices ? indices + (size_t)i * B : nullptr;
      const float* ep = eps ? eps + (size_t)i * 2 * B * A : nullptr;
      // step i > 0 of the call uses the batch step i - 1 gathered in its last phase-C stage
      const bool next = i + 1 < n;
      const int32_t* nix = indices && next ? indices + (size_t)(i + 1) * B : nullptr;
      for (const sac_engine::WStage& st : e->wst) {
        if (st.kind == 0 && i > 0) continue;
        launch_wide(e, st, rb, ix, ep, s, next, nix);
        if (kinds) kinds->push_back(st.phase);
        if (ev) {
          hipEvent_t x;
          (void)hipEventCreate(&x);
          (void)hipEventRecord(x, s);
          ev->push_back(x);
        }
      }
    }
    return;
  }
  for (int i = 0; i < n; ++i)
    for (int k = L_A; k <= L_D; ++k) go(k, i);
}

static int check_replay(sac_engine* e, const sac_replay* rb) {
  if (!rb || !rb->obs || !rb->act || !rb->rew || !rb->next_obs || !rb->done || !rb->state)
    return fail(SAC_E_INVALID, "null replay buffer");
  if (rb->obs_dim != e->cfg.obs_dim || rb->act_dim != e->cfg.act_dim)
    return fail(SAC_E_INVALID, "replay dims do not match the engine");
  if (rb->capacity < e->cfg.batch) return fail(SAC_E_NOT_ENOUGH, "replay capacity smaller than the batch");
  return SAC_OK;
}

extern "C" {

const char* sac_last_error(void) { return g_err.c_str(); }
const char* sac_version(void) { return SAC_VERSION; }

size_t sac_engine_workspace_bytes(const sac_engine_config* cfg) {
  if (validate(cfg) != SAC_OK) return 0;
  return plan(cfg, nullptr, nullptr);
}

const char* sac_phase_kernel_name(int32_t phase) {
  switch (phase) {
    case 0: return "sac_target_critic";
    case 1: return "sac_critic_update";
    case 2: return "sac_actor";
    case 3: return "sac_actor_update";
    default: return "";
  }
}

int sac_engine_sync_params(sac_engine* e, void* stream) {
  if (!e) return fail(SAC_E_INVALID, "null engine");
  hipStream_t s = (hipStream_t)stream;
  const bool bf = e->cfg.precision == SAC_PREC_BF16;
  for (int ni = 0; ni < 5; ++ni) {
    const NetDev& nd = e->h.net[ni];
    for (int l = 0; l < nd.L; ++l) {
      const LayerDev& ly = nd.l[l];
      const int blocks = std::min(1024, (ly.Np * ly.Kp + 255) / 256);
      if (bf)
        pack_weights<bf16><<<blocks, 256, 0, s>>>(nd.P + ly.w_off, ly.K, ly.N, ly.Kp, ly.Np, (bf16*)ly.Wc, (bf16*)ly.WTc);
      else
        pack_weights<float><<<blocks, 256, 0, s>>>(nd.P + ly.w_off, ly.K, ly.N, ly.Kp, ly.Np, (float*)ly.Wc,
                                                   (float*)ly.WTc);
    }
  }
  HIPCHK(hipGetLastError());
  return SAC_OK;
}

int sac_engine_create(const sac_engine_config* cfg, const sac_engine_buffers* buf, void* stream, sac_engine** out) {
  if (!out || !buf) return fail(SAC_E_INVALID, "null argument");
  *out = nullptr;
  int rc = validate(cfg);
  if (rc) return rc;
  const size_t need = plan(cfg, nullptr, nullptr);
  if (!buf->workspace || buf->workspace_bytes < need)
    return fail(SAC_E_INVALID, "workspace too small: need " + std::to_string(need) + " bytes");
  if (((uintptr_t)buf->workspace) & 255) return fail(SAC_E_INVALID, "workspace must be 256-byte aligned");
  if (!buf->pi || !buf->q1 || !buf->q2 || !buf->q1t || !buf->q2t || !buf->pi_m || !buf->pi_v || !buf->q1_m ||
      !buf->q1_v || !buf->q2_m || !buf->q2_v || !buf->alpha_state || !buf->opt_steps || !buf->rng_step || !buf->stats)
    return fail(SAC_E_INVALID, "null device buffer");
  sac_engine* e = new sac_engine();
  e->cfg = *cfg;
  e->buf = *buf;
  {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      e->ncu = n;
  }
  plan(cfg, e, (char*)buf->workspace);
  {  // an explicit layout override runs the kernels it names or fails (as stage_path = -1 does)
    const bool rows = !e->h.split && !e->h.roles && !e->h.pairs && !e->wide;
    const char* miss = nullptr;
    if (cfg->layout == SAC_LAYOUT_ROLES && !e->h.roles) miss = "roles (needs 6 * row tiles <= 256 co-resident workgroups)";
    if (cfg->layout == SAC_LAYOUT_PAIRS && !e->h.pairs) miss = "pairs (the pair-tile LDS layout or record does not fit)";
    if (cfg->layout == SAC_LAYOUT_ROWS && !rows) miss = "rows (the row-tile LDS layout does not fit: stage path)";
    if (miss) {
      delete e;
      return fail(SAC_E_INVALID, std::string("layout override cannot be honoured: ") + miss);
    }
  }
  if (std::max(e->lds_bytes, e->upd_lds) > 160 * 1024) {
    const size_t lb = e->lds_bytes;
    delete e;
    return fail(SAC_E_INVALID, "layer widths need " + std::to_string(lb) + " B of LDS per workgroup (max 163840)");
  }
  if (e->wide) {
    // the stage launches' LDS, and the batch gather's [WGR][obs + act] rows + slots
    size_t mx = (size_t)((WGR * (cfg->obs_dim + cfg->act_dim) + 1) & ~1) * 4 + WGR * 8;
    for (const sac_engine::WStage& st : e->wst) mx = std::max(mx, st.lds);
    if (e->hostW.size() > WIDE_MAX_JOBS || mx > 160 * 1024) {
      const std::string m = "internal: stage path plans " + std::to_string(e->hostW.size()) + " jobs, " +
                            std::to_string(mx) + " B of LDS";
      delete e;
      return fail(SAC_E_INVALID, m);
    }
  }
  if ((int)e->hostB.size() != e->nB || (int)e->hostD.size() != e->nD) {  // the grids launch nB / nD tiles
    const std::string m = "internal: update tiles planned " + std::to_string(e->nB) + " / " + std::to_string(e->nD) +
                          ", built " + std::to_string(e->hostB.size()) + " / " + std::to_string(e->hostD.size());
    delete e;
    return fail(SAC_E_INVALID, m);
  }
  if (cfg->precision == SAC_PREC_BF16)
    set_lds_attrs<bf16>(e->lds_bytes);
  else
    set_lds_attrs<float>(e->lds_bytes);
  hipStream_t s = (hipStream_t)stream;
  hipError_t err = hipMemsetAsync(buf->workspace, 0, buf->workspace_bytes, s);
  if (err == hipSuccess) err = hipMemcpyAsync(e->d, &e->h, sizeof(EngineDev), hipMemcpyHostToDevice, s);
  if (err == hipSuccess) err = hipMemcpyAsync(e->tilesB, e->hostB.data(), e->hostB.size() * sizeof(TileDesc), hipMemcpyHostToDevice, s);
  if (err == hipSuccess) err = hipMemcpyAsync(e->tilesD, e->hostD.data(), e->hostD.size() * sizeof(TileDesc), hipMemcpyHostToDevice, s);
  if (err == hipSuccess && e->wide) err = hipMemcpyAsync(e->wdd, &e->wdh, sizeof(WideDev), hipMemcpyHostToDevice, s);
  if (err == hipSuccess && e->wide)
    err = hipMemcpyAsync(e->wjobs, e->hostW.data(), e->hostW.size() * sizeof(WJob), hipMemcpyHostToDevice, s);
  if (err == hipSuccess) err = hipStreamSynchronize(s);
  if (err != hipSuccess) {
    delete e;
    return fail(SAC_E_HIP, std::string("engine upload: ") + hipGetErrorString(err));
  }
  rc = sac_engine_sync_params(e, stream);
  if (rc) {
    delete e;
    return rc;
  }
  *out = e;
  return SAC_OK;
}

int sac_engine_set_alpha_update(sac_engine* e, int32_t enabled, void* stream) {
  if (!e) return fail(SAC_E_INVALID, "null engine");
  e->h.alpha_update = enabled ? 1 : 0;
  HIPCHK(hipMemcpyAsync((char*)e->d + offsetof(EngineDev, alpha_update), &e->h.alpha_update, sizeof(int),
                        hipMemcpyHostToDevice, (hipStream_t)stream));
  return SAC_OK;
}

int sac_engine_check(sac_engine* e, void* stream) {
  if (!e) return fail(SAC_E_INVALID, "null engine");
  uint32_t w[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(w, e->h.sync, sizeof(w), hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  if (w[1]) return fail(SAC_E_HIP, "a workgroup hand-off timed out: results of the affected steps are invalid");
  return SAC_OK;
}

int sac_engine_debug_staged_step(sac_engine* e, uint64_t* step_out, void* stream) {
  if (!e || !step_out) return fail(SAC_E_INVALID, "bad debug_staged_step arguments");
  HIPCHK(hipMemcpyAsync(step_out, e->h.sync + SYNC_STAGED, sizeof(uint64_t), hipMemcpyDeviceToHost,
                        (hipStream_t)stream));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  return SAC_OK;
}

void sac_engine_destroy(sac_engine* e) {
  if (!e) return;
  if (e->gexec) (void)hipGraphExecDestroy(e->gexec);
  if (e->graph) (void)hipGraphDestroy(e->graph);
  if (e->cap) (void)hipStreamDestroy(e->cap);
  delete e;
}

int sac_engine_train(sac_engine* e, const sac_replay* rb, int32_t n_steps, const int32_t* indices, const float* eps,
                     void* stream) {
  if (!e) return fail(SAC_E_INVALID, "null engine");
  int rc = check_replay(e, rb);
  if (rc) return rc;
  launch_steps(e, rb, n_steps, indices, eps, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return SAC_OK;
}

int sac_engine_train_graph(sac_engine* e, const sac_replay* rb, int32_t n_steps, int32_t chunk, void* stream) {
  if (!e) return fail(SAC_E_INVALID, "null engine");
  int rc = check_replay(e, rb);
  if (rc) return rc;
  if (chunk < 1) return fail(SAC_E_INVALID, "chunk >= 1");
  hipStream_t s = (hipStream_t)stream;
  const bool same = e->gexec && e->gchunk == chunk && !memcmp(&e->gkey, rb, sizeof(sac_replay));
  if (!same && (n_steps >= chunk || n_steps == 0)) {  // n_steps == 0: capture only
    if (e->gexec) (void)hipGraphExecDestroy(e->gexec);
    if (e->graph) (void)hipGraphDestroy(e->graph);
    e->gexec = nullptr;
    e->graph = nullptr;
    if (!e->cap) HIPCHK(hipStreamCreateWithFlags(&e->cap, hipStreamNonBlocking));
    HIPCHK(hipStreamBeginCapture(e->cap, hipStreamCaptureModeThreadLocal));
    launch_steps(e, rb, chunk, nullptr, nullptr, e->cap);
    HIPCHK(hipStreamEndCapture(e->cap, &e->graph));
    HIPCHK(hipGraphInstantiate(&e->gexec, e->graph, nullptr, nullptr, 0));
    // device-side setup of the executable graph now, on the caller's stream,
    // not inside its first replay (the timed region of a short run)
    HIPCHK(hipGraphUpload(e->gexec, s));
    e->gchunk = chunk;
    e->gkey = *rb;
  }
  int done = 0;
  if (e->gexec)
    for (; done + chunk <= n_steps; done += chunk) HIPCHK(hipGraphLaunch(e->gexec, s));
  if (done < n_steps) launch_steps(e, rb, n_steps - done, nullptr, nullptr, s);
  HIPCHK(hipGetLastError());
  return SAC_OK;
}

int sac_policy_act(sac_engine* e, const float* obs, int32_t n, const float* eps, float* action, float* log_pi,
                   void* stream) {
  if (!e || !obs || !action || n < 1) return fail(SAC_E_INVALID, "bad policy_act arguments");
  hipStream_t s = (hipStream_t)stream;
  const int blocks = (n + SAC_ROWS - 1) / SAC_ROWS;
  if (e->cfg.precision == SAC_PREC_BF16)
    sac_policy_act_kernel<bf16><<<blocks, SAC_THREADS, e->lds_bytes, s>>>(e->d, obs, n, eps, action, log_pi);
  else
    sac_policy_act_kernel<float><<<blocks, SAC_THREADS, e->lds_bytes, s>>>(e->d, obs, n, eps, action, log_pi);
  HIPCHK(hipGetLastError());
  return SAC_OK;
}

int sac_replay_push(const sac_replay* rb, const float* rows, int64_t n, int64_t size_host, int64_t pos_host,
                    void* stream) {
  if (!rb || !rows || n < 0 || rb->capacity < 1) return fail(SAC_E_INVALID, "bad replay_push arguments");
  if (n == 0) return SAC_OK;
  const int64_t cap = rb->capacity;
  const int64_t skip = n > cap ? n - cap : 0;
  const int64_t new_size = std::min(cap, size_host + n);
  const int64_t new_pos = (pos_host + n) % cap;
  const int64_t total = (n - skip) * (2 * rb->obs_dim + rb->act_dim + 2);
  const int blocks = (int)std::min<int64_t>(4096, (total + 255) / 256);
  replay_push_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(*rb, rows, n, skip, pos_host, new_size, new_pos);
  HIPCHK(hipGetLastError());
  return SAC_OK;
}

// rows per wave of the records gather: 16 (4x the waves in flight of 64 rows per wave:
// 65,536 rows 1.51 -> 2.42 TB/s, 1,048,576 rows 3.00 -> 3.17 TB/s)
static int gather_rpw(int batch) {
  (void)batch;
  return 16;
}

int sac_replay_gather(const sac_replay* rb, const int32_t* logical_idx, int32_t batch, float* s, float* a, float* r,
                      float* s2, float* d, void* stream) {
  if (!rb || !logical_idx || batch < 1 || !s || !a || !r || !s2 || !d) return fail(SAC_E_INVALID, "bad gather arguments");
  const int blocks = (batch + 255) / 256;  // one wave per 64 rows
  const int rpw = gather_rpw(batch);
  if (standard_records(rb))
    replay_gather_records_kernel<false><<<(batch + 4 * rpw - 1) / (4 * rpw), 256, 0, (hipStream_t)stream>>>(
        *rb, logical_idx, batch, FeistelKeys{}, nullptr, s, a, r, s2, d, rpw);
  else
    replay_gather_kernel<false><<<blocks, 256, 0, (hipStream_t)stream>>>(*rb, logical_idx, batch, FeistelKeys{}, nullptr, s,
                                                                         a, r, s2, d);
  HIPCHK(hipGetLastError());
  return SAC_OK;
}

int sac_replay_sample_gather(const sac_replay* rb, int32_t batch, uint64_t seed, uint64_t step, int32_t* idx_out,
                             float* s, float* a, float* r, float* s2, float* d, void* stream) {
  if (!rb || batch < 1 || !s || !a || !r || !s2 || !d) return fail(SAC_E_INVALID, "bad sample_gather arguments");
  const int blocks = (batch + 255) / 256;
  const int rpw = gather_rpw(batch);
  if (standard_records(rb))
    replay_gather_records_kernel<true><<<(batch + 4 * rpw - 1) / (4 * rpw), 256, 0, (hipStream_t)stream>>>(
        *rb, nullptr, batch, feistel_keys(seed, step), idx_out, s, a, r, s2, d, rpw);
  else
    replay_gather_kernel<true><<<blocks, 256, 0, (hipStream_t)stream>>>(*rb, nullptr, batch, feistel_keys(seed, step), idx_out, s,
                                                                        a, r, s2, d);
  HIPCHK(hipGetLastError());
  return SAC_OK;
}

int sac_engine_read_status(sac_engine* e, uint32_t* host_dst, void* stream) {
  if (!e || !host_dst) return fail(SAC_E_INVALID, "bad read_status arguments");
  HIPCHK(hipMemcpyAsync(host_dst, e->h.sync, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, (hipStream_t)stream));
  return SAC_OK;
}

int sac_engine_clear_status(sac_engine* e, void* stream) {
  if (!e) return fail(SAC_E_INVALID, "null engine");
  HIPCHK(hipMemsetAsync(e->h.sync + SYNC_TIMEOUT, 0, sizeof(uint32_t), (hipStream_t)stream));
  return SAC_OK;
}

int sac_engine_debug_set_spin_limit(sac_engine* e, int32_t polls, void* stream) {
  if (!e || polls < 0) return fail(SAC_E_INVALID, "bad spin limit");
  e->h.spin_limit = polls;
  HIPCHK(hipMemcpyAsync(e->d, &e->h, sizeof(EngineDev), hipMemcpyHostToDevice, (hipStream_t)stream));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  return SAC_OK;
}

int sac_replay_sample_indices(const sac_replay* rb, int32_t batch, uint64_t seed, uint64_t step, int32_t* out,
                              void* stream) {
  if (!rb || !out || batch < 1) return fail(SAC_E_INVALID, "bad sample arguments");
  const int blocks = std::min(4096, (batch + 255) / 256);
  replay_sample_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(rb->state, batch, feistel_keys(seed, step), out);
  HIPCHK(hipGetLastError());
  return SAC_OK;
}

int sac_engine_debug_stamps(sac_engine* e, long long* dev_buf, void* stream) {
  if (!e) return fail(SAC_E_INVALID, "null engine");
  e->h.stamps = dev_buf;
  HIPCHK(hipMemcpyAsync(e->d, &e->h, sizeof(EngineDev), hipMemcpyHostToDevice, (hipStream_t)stream));
#ifdef SAC_STAMPS
  HIPCHK(hipMemcpyToSymbolAsync(HIP_SYMBOL(sac_dbg_stamps), &dev_buf, sizeof(dev_buf), 0, hipMemcpyHostToDevice,
                                (hipStream_t)stream));
#endif
  if (e->gexec) {  // graphs captured the old kernel arguments
    (void)hipGraphExecDestroy(e->gexec);
    (void)hipGraphDestroy(e->graph);
    e->gexec = nullptr;
    e->graph = nullptr;
  }
  return SAC_OK;
}

int sac_debug_sample_indices_host(int64_t size, int32_t batch, uint64_t seed, uint64_t step, int32_t* out) {
  if (!out || batch < 0 || size < batch) return fail(SAC_E_INVALID, "need 0 <= batch <= size and out != NULL");
  const Feistel f = feistel_make(seed, step, size);
  for (int32_t b = 0; b < batch; ++b) out[b] = (int32_t)feistel_sample(f, b, size);
  return SAC_OK;
}

int sac_debug_eps_host(uint64_t seed, uint64_t step, int32_t batch, int32_t act_dim, float* out) {
  if (!out || batch < 1 || act_dim < 1) return fail(SAC_E_INVALID, "need batch >= 1, act_dim >= 1, out != NULL");
  for (int which = 0; which < 2; ++which)
    for (int b = 0; b < batch; ++b)
      for (int p = 0; p < (act_dim + 1) / 2; ++p) eps_pair(seed, step, b, which, p, batch, act_dim, out);
  return SAC_OK;
}

int sac_debug_eps_device(uint64_t seed, uint64_t step, int32_t batch, int32_t act_dim, float* out, void* stream) {
  if (!out || batch < 1 || act_dim < 1) return fail(SAC_E_INVALID, "need batch >= 1, act_dim >= 1, out != NULL");
  const int64_t n = 2LL * batch * ((act_dim + 1) / 2);
  const int blocks = (int)std::min<int64_t>(4096, (n + 255) / 256);
  eps_draw_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(seed, step, batch, act_dim, out);
  HIPCHK(hipGetLastError());
  return SAC_OK;
}

int sac_engine_uses_roles(const sac_engine* e) { return e && e->h.roles ? 1 : 0; }

int sac_engine_uses_split(const sac_engine* e) { return e && e->h.split ? 1 : 0; }

int sac_engine_uses_pairs(const sac_engine* e) { return e && e->h.pairs ? 1 : 0; }

int sac_engine_uses_wide(const sac_engine* e) { return e && e->wide ? (int)e->wst.size() : 0; }

int sac_engine_phase_launches(const sac_engine* e, int32_t* out) {
  if (!e || !out) return fail(SAC_E_INVALID, "null argument");
  for (int k = 0; k < 4; ++k) out[k] = 1;
  if (e->wide) {
    for (int k = 0; k < 4; ++k) out[k] = 0;
    for (const sac_engine::WStage& st : e->wst)
      if (st.kind != 0 && st.phase >= 0 && st.phase < 4) ++out[st.phase];
  }
  return SAC_OK;
}

int sac_engine_debug_launch(sac_engine* e, const sac_replay* rb, int32_t kind, void* stream) {
  if (!e || !rb || kind < L_A || kind > L_D) return fail(SAC_E_INVALID, "bad debug_launch arguments");
  if (e->wide) {  // every launch of that phase
    for (const sac_engine::WStage& st : e->wst)
      if (st.phase == kind) launch_wide(e, st, rb, nullptr, nullptr, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return SAC_OK;
  }
  if (e->cfg.precision == SAC_PREC_BF16)
    launch_kind<bf16>(e, kind, rb, nullptr, nullptr, (hipStream_t)stream);
  else
    launch_kind<float>(e, kind, rb, nullptr, nullptr, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return SAC_OK;
}

int sac_engine_debug_stamped(void) {
#ifdef SAC_STAMPS
  return 1;
#else
  return 0;
#endif
}

int sac_engine_time_phases(sac_engine* e, const sac_replay* rb, int32_t n_steps, float* ms_host, void* stream) {
  if (!e || !ms_host || n_steps < 1) return fail(SAC_E_INVALID, "bad time_phases arguments");
  int rc = check_replay(e, rb);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  // events after every launch of the step sequence; a launch's time = its event
  // minus the previous one
  std::vector<int> kinds;
  std::vector<hipEvent_t> ev;
  hipEvent_t start;
  HIPCHK(hipEventCreate(&start));
  // hold the stream while the whole sequence is enqueued (~0.2 ms of host time
  // per step), so the intervals are device time, not host-submission time
  const long long hold = std::min(20000000LL, 20000LL * n_steps + 200000LL);
  sac_spin_kernel<<<1, 64, 0, s>>>(hold);
  HIPCHK(hipEventRecord(start, s));
  launch_steps(e, rb, n_steps, nullptr, nullptr, s, &kinds, &ev);
  HIPCHK(hipStreamSynchronize(s));
  double sum[4] = {0, 0, 0, 0};
  int cnt[4] = {0, 0, 0, 0};
  for (size_t i = 0; i < ev.size(); ++i) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, i ? ev[i - 1] : start, ev[i]));
    sum[kinds[i]] += ms;
    ++cnt[kinds[i]];
  }
  // per phase and step (the stage path has several launches per phase)
  auto avg = [&](int k) { return cnt[k] ? (float)(sum[k] / (e->wide ? n_steps : cnt[k])) : 0.f; };
  for (int p = 0; p < 4; ++p) ms_host[p] = avg(p);
  // the same event pattern around empty launches: the per-launch gap
  {
    const int n = 64;
    std::vector<hipEvent_t> ez(n + 1);
    for (auto& x : ez) HIPCHK(hipEventCreate(&x));
    sac_spin_kernel<<<1, 64, 0, s>>>(200000LL);  // 2 ms: every empty launch queued behind it
    HIPCHK(hipEventRecord(ez[0], s));
    for (int i = 1; i <= n; ++i) {
      sac_noop_kernel<<<1, 64, 0, s>>>();
      HIPCHK(hipEventRecord(ez[i], s));
    }
    HIPCHK(hipStreamSynchronize(s));
    double tot = 0.0;
    for (int i = 1; i <= n; ++i) {
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, ez[i - 1], ez[i]));
      tot += ms;
    }
    ms_host[4] = (float)(tot / n);
    for (auto& x : ez) (void)hipEventDestroy(x);
  }
  (void)hipEventDestroy(start);
  for (auto& x : ev) (void)hipEventDestroy(x);
  return SAC_OK;
}

}  // extern "C"
