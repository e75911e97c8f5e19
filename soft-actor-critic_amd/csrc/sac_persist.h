// sac_persist.h — the whole SAC gradient step as ONE persistent launch of K
// steps (the hidden-split configurations: C2, C4, C4').
//
// The four phase kernels of a step (A target + critic backward, B critic
// update + Polyak, C actor, D actor update + alpha; reference
// sac/agent.py:302-327) become phases of one launch of G workgroups, one per
// CU, all co-resident.  Every workgroup holds a fixed task per phase (a phase-A
// role, a phase-B tile, a phase-C role, a phase-D tile; any may be absent:
// PTask) and runs them in phase order for each of the K steps.  The kernel
// boundaries become readiness counters (sharded per XCD, monotonic inside the
// launch) that a task polls before it touches what its producers wrote:
//
//   PC_AQ   phase-A critic + target-critic roles done  -> phase B tiles
//           (dY^T, X^T, seeds; and the target weights the target critics have
//            read before Polyak overwrites them)
//   PC_PS   phase-A pi(s) roles done                   -> phase C (stashes)
//   PC_BQ1/2 phase-B tiles of critic 1 / 2 done        -> phase C critic 1 / 2,
//                                                         next step's critics and
//                                                         target critics
//   PC_CP   phase-C pi roles done                      -> phase D
//   PC_D    phase-D tiles + the alpha block done       -> next step's pi roles
//
// Every other dependency is ordered transitively through these and the
// data-tagged granule hand-offs inside phases A and C (DESIGN.md §3.5 lists the
// read-after-write and write-after-read pairs and the edge that orders each).
// Cross-workgroup data is stored sc1 (write-through) and loaded sc1
// (MI355X_MICROARCH.md, visibility: the write-through form), producers drain
// their stores (s_waitcnt vmcnt(0)) before they arrive on a counter.  What a
// phase waits for is what the kernel boundary used to provide, so no task
// waits on a later task of its own workgroup, and every spin is bounded: a
// timeout sets the engine's error flag and ends that workgroup's loop.
//
// What the launch saves against four launches per step: per step four
// dispatches, drains and cold starts (EngineDev and tile descriptor loads, the
// first weight round trip of every block), and the phase-B / phase-C inputs
// that do not depend on the previous phase are fetched while it is still
// running (a tile's masters and moments, phase C's stashes).  The numerics are
// the phase kernels' own device code: the results are the same bits.
#pragma once
#include "sac_split.h"

enum PCtr { PC_AQ = 0, PC_PS = 1, PC_BQ1 = 2, PC_BQ2 = 3, PC_CP = 4, PC_D = 5, PC_AQP = 6, PC_COUNT = 7 };
#define PC_SHARDS 8
#define PC_STRIDE 16  // uint32 per shard: one 64-B line each

struct PTask {
  int16_t a, b, c, d;  // phase-A role block, phase-B tile, phase-C role block, phase-D tile (nD: alpha); -1 none
};

__device__ __forceinline__ uint32_t* pc_word(const AS_C EngineDev& E, int ctr, int shard) {
  return E.pctr + (ctr * PC_SHARDS + shard) * PC_STRIDE;
}

// all threads: this workgroup's stores of the task are drained, then one lane
// adds 1 to the counter's shard of this workgroup
__device__ __forceinline__ void pc_arrive(const AS_C EngineDev& E, int ctr) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(pc_word(E, ctr, blockIdx.x & (PC_SHARDS - 1)), 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// all threads: returns true once counter c0 (and c1 if >= 0) reach their targets
// (sum over the shards).  Wave 0 polls: lanes 0..7 the shards of c0, 8..15
// those of c1, lane 16 the engine's timeout flag, all in one batch of sc1
// loads; false (for every thread) if the spin bound ran out or another
// workgroup has already timed out.
__device__ __forceinline__ bool pc_wait(const AS_C EngineDev& E, int c0, uint32_t t0, int c1, uint32_t t1,
                                        volatile AS_L int* flag) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const uint32_t* w = lane < 8 ? pc_word(E, c0, lane)
                                 : lane < 16 ? pc_word(E, c1 >= 0 ? c1 : c0, lane - 8)
                                             : (const uint32_t*)E.sync + SYNC_TIMEOUT;
    int ok = 1;
    for (int it = 0;; ++it) {
      const uint32_t v = lane <= 16 ? __hip_atomic_load((uint32_t*)w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      uint32_t s0 = lane < 8 ? v : 0u, s1 = (lane >= 8 && lane < 16) ? v : 0u;
      const uint32_t to = __shfl(v, 16, 64);
#pragma unroll
      for (int o = 4; o > 0; o >>= 1) {
        s0 += __shfl_xor(s0, o, 64);
        s1 += __shfl_xor(s1, o, 64);
      }
      s0 = __shfl(s0, 0, 64);
      s1 = __shfl(s1, 8, 64);
      if (to) {
        ok = 0;
        break;
      }
      if (s0 >= t0 && (c1 < 0 || s1 >= t1)) break;
      if (it > E.spin_limit) {
        if (lane == 0)
          __hip_atomic_store((uint32_t*)E.sync + SYNC_TIMEOUT, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0 && !ok) *flag = 0;
  }
  __syncthreads();
  return *flag != 0;
}

// Adam scalars of step t of an optimizer (torch adam.py, single tensor, as
// phase A's Adam block computes them for the phase kernels)
__device__ __forceinline__ UpdStep upd_step(const AS_C EngineDev& E, int opt, double t, uint32_t ep) {
  const double lr = opt == NET_PI ? E.actor_lr : E.critic_lr;
  UpdStep u;
  u.neg_step = (float)(-(lr / (1.0 - pow((double)E.beta1, t))));
  u.bc2s = (float)sqrt(1.0 - pow((double)E.beta2, t));
  u.ep = ep;
  return u;
}

// The step's context and this workgroup's task, re-read (scalar loads) by
// every phase instead of kept live across the phases: the launch's constants
// (step counter, epoch, optimizer steps) only change when the last workgroup
// leaves (below), and values kept live across the four bodies cost SGPR and
// then VGPR spills.
__device__ __forceinline__ StepCtx step_now(const AS_C EngineDev& E) {
  const uint64_t step = *GPC(uint64_t, E.rng_step);
  return StepCtx{step, *GPC(uint32_t, E.sync) + 1u, (int)(step & 1)};
}
__device__ __forceinline__ const EngineDev* fresh_ptr(const EngineDev* Ep) {
  uint64_t p = (uint64_t)(uintptr_t)Ep;
  asm volatile("" : "+s"(p));  // opaque: nothing derived from it is hoisted across phases
  return (const EngineDev*)(uintptr_t)p;
}
__device__ __forceinline__ const AS_C PTask& my_task(const AS_C EngineDev& E) {
  return ((const AS_C PTask*)E.ptasks)[blockIdx.x];
}

// One gradient step per launch: a step loop inside the launch (K > 1) was
// measured to push the merged kernel into 130+ VGPR spills (the compiler keeps
// the phases' thread-index address arithmetic live across iterations), while
// the straight-line four-phase step stays near the phase kernels' register
// counts.  So the previous step's phase D -> this step's phase A edge is the
// kernel boundary (phase A waits for nothing); B, C and D wait on counters.
template <typename T>
__global__ void __launch_bounds__(SAC_THREADS) sac_persist(const EngineDev* __restrict__ Ep, sac_replay rb,
                                                           const int32_t* __restrict__ inj_idx_,
                                                           const float* __restrict__ inj_eps_) {
  PREFETCH_ARG(Ep);
  extern __shared__ float lds_raw[];
  lf* lds = (lf*)lds_raw;
  const int o_flag = ((const AS_C EngineDev*)Ep)->o_pflag;
  volatile AS_L int* flag = (volatile AS_L int*)(lds + o_flag);
  if (threadIdx.x == 0) *flag = 1;
  __syncthreads();
  // ---- phase A: sample + gather, pi(s'), target critics, critics, pi(s)
  {
    const EngineDev* Ek = fresh_ptr(Ep);
    const AS_C EngineDev& E = *(const AS_C EngineDev*)Ek;
    const int a = my_task(E).a;
    if (a >= 0) {
      int role_done = -1;
      target_critic_split_body<T, true>(Ek, rb, inj_idx_, inj_eps_, a, step_now(E), [&](int role) {
        if (role < 0) {
          if (E.p_aqp) pc_arrive(E, PC_AQP);  // a critic's pre-seed operands are stored
        } else {
          role_done = role;
        }
      });
      if (role_done >= 1 && role_done <= 4) pc_arrive(E, PC_AQ);
      else if (role_done == 5) pc_arrive(E, PC_PS);
      STAMP(24);
    }
  }
  // ---- phase B: critic dW + Adam + Polyak tiles
  {
    const AS_C EngineDev& E = *(const AS_C EngineDev*)fresh_ptr(Ep);
    const int b = my_task(E).b;
    if (b >= 0 && *flag) {
      const StepCtx sc = step_now(E);
      const TileDesc* td = E.tilesB + b;
      const int opt = ((const AS_C TileDesc*)td)->opt;
      const UpdStep us = upd_step(E, opt, GPC(double, E.opt_steps)[opt] + 1.0, sc.ep);
      // fp32 layers 0 / 1: operands once every critic role has stored its pre-seed
      // operands (PC_AQP), the rest once the critics and targets are done (PC_AQ)
      const bool pre = sizeof(T) == 4 && E.p_aqp && ((const AS_C TileDesc*)td)->N > 1;
      dw_adam_tile_any<T, SAC_THREADS, true, true>(E, td, true, sc.par, 0, lds, &us, [&](int stage) {
        if (stage == 0 && pre) {
          pc_wait(E, PC_AQP, E.pc_n[PC_AQP], -1, 0, flag);
        } else if (stage == 1 || !pre) {
          if (stage == 1 && !pre) return;  // waited at stage 0
          pc_wait(E, PC_AQ, E.pc_n[PC_AQ], -1, 0, flag);
          STAMP(25);
        }
      });
      pc_arrive(E, opt == 1 ? PC_BQ1 : PC_BQ2);
      STAMP(26);
    }
  }
  // ---- phase C: critics on (s, a~) with the updated weights, pi backward
  {
    const EngineDev* Ek = fresh_ptr(Ep);
    const AS_C EngineDev& E = *(const AS_C EngineDev*)Ek;
    const int c = my_task(E).c;
    const int nrole = 3 * split_wc(sizeof(T)) * E.nrt;
    if (c >= nrole) {  // stager: the next step's batch of row tile c - nrole (read by the next launch)
      stage_next_batch(E, rb, c - nrole, lds, step_now(E).step);
      __syncthreads();
    } else if (c >= 0 && *flag) {
      actor_split_body<T, true>(Ek, c, step_now(E), [&](int w) {
        if (w == 0)
          pc_wait(E, PC_PS, E.pc_n[PC_PS], -1, 0, flag);
        else if (w == 1 || w == 2)
          pc_wait(E, w == 1 ? PC_BQ1 : PC_BQ2, E.pc_n[w == 1 ? PC_BQ1 : PC_BQ2], -1, 0, flag);
        else
          pc_wait(E, PC_BQ1, E.pc_n[PC_BQ1], PC_BQ2, E.pc_n[PC_BQ2], flag);
        STAMP(27 + (w > 0));
      });
      if (c >= 2 * split_wc(sizeof(T)) * E.nrt) pc_arrive(E, PC_CP);  // pi roles (after the critics' blocks)
      STAMP(29);
    }
  }
  // ---- phase D: pi dW + Adam tiles; the last task is the float64 alpha step + losses
  {
    const AS_C EngineDev& E = *(const AS_C EngineDev*)fresh_ptr(Ep);
    const int d = my_task(E).d;
    if (d >= 0 && *flag) {
      const StepCtx sc = step_now(E);
      auto waitD = [&](int stage = 0) {
        if (stage) return;
        pc_wait(E, PC_CP, E.pc_n[PC_CP], -1, 0, flag);
        STAMP(30);
      };
      if (d < E.nD) {
        const UpdStep us = upd_step(E, NET_PI, GPC(double, E.opt_steps)[NET_PI] + 1.0, sc.ep);
        // pi's new weights are read by the next launch only: plain stores (COH off)
        dw_adam_tile_any<T, SAC_THREADS, false, true>(E, E.tilesD + d, false, sc.par, sc.par, lds, &us, waitD);
      } else {
        const double t3 = GPC(double, E.opt_steps)[3] + 1.0;
        const double bc[2] = {1.0 - pow((double)E.beta1, t3), 1.0 - pow((double)E.beta2, t3)};
        waitD();
        alpha_and_losses<true>(E, sc.par, lds, bc);
      }
      pc_arrive(E, PC_D);
      STAMP(31);
    }
  }
  // ---- the last workgroup out advances the engine's step state and resets the
  // counters for the next launch (every wait of this launch is over: each
  // workgroup counts itself out after its last task)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < 64) {  // wave 0: lane 0 counts the workgroup out; the last one's lanes reset in parallel
    const AS_C EngineDev& E = *(const AS_C EngineDev*)fresh_ptr(Ep);
    uint32_t* done = E.pctr + PC_COUNT * PC_SHARDS * PC_STRIDE;
    uint32_t n = 0;
    if (threadIdx.x == 0) n = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    n = __shfl(n, 0, 64);
    if (n == gridDim.x - 1) {
      const int lane = threadIdx.x;
      if (lane < PC_COUNT * PC_SHARDS) E.pctr[lane * PC_STRIDE] = 0u;  // the word each shard uses
      if (lane == 63) {
        *done = 0u;
        *GP(uint64_t, E.rng_step) += 1;
        GP(uint32_t, E.sync)[SYNC_EPOCH] += 1u;
      }
      if (lane < 3 || (lane == 3 && E.auto_entropy && E.alpha_update)) GP(double, E.opt_steps)[lane] += 1.0;
    }
  }
  {
    const AS_C EngineDev& E = *(const AS_C EngineDev*)Ep;
    (void)E;
    END_STAMP(60);
  }
}
