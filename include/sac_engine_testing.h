/*
 * sac_engine_testing.h — diagnostic exports of libsac_engine.so (not part of
 * the drop-in boundary; used by tools/ and tests/ only).
 */
#ifndef SAC_ENGINE_TESTING_H
#define SAC_ENGINE_TESTING_H
#include "sac_engine.h"
#ifdef __cplusplus
extern "C" {
#endif
/* Point the phase kernels at a device buffer of int64 s_memtime stamps
 * ([grid][64]); only builds with -DSAC_STAMPS write them. */
int sac_engine_debug_stamps(sac_engine *e, long long *dev_buf, void *stream);
int sac_engine_debug_stamped(void);
/* Launch ONE phase kernel of the current step (kind: 0 A, 1 B, 2 C, 3 D) on
 * the stream.  Timing experiments only:
 * re-running a phase out of sequence advances or corrupts the training state. */
int sac_engine_debug_launch(sac_engine* e, const sac_replay* rb, int32_t kind, void* stream);
/* The last step whose phase A took its batch from the record phase C staged
 * (0: none yet); synchronises the stream. */
int sac_engine_debug_staged_step(sac_engine* e, uint64_t* step_out, void* stream);
/* 1 if phases A/C run role-split (per-network workgroups with in-launch
 * hand-offs), 0 if one workgroup per row tile runs all networks. */
int sac_engine_uses_roles(const sac_engine *e);
/* 1 if phases A/C run the hidden-split role kernels (sac_split.h: two
 * workgroups per role and row tile, each with half of the 256-wide layer 1). */
int sac_engine_uses_split(const sac_engine *e);
/* 1 if phases A/C run the pair-tile kernels (sac_pairs.h: one workgroup per
 * pair of row tiles and group of networks; config.layout = SAC_LAYOUT_PAIRS). */
int sac_engine_uses_pairs(const sac_engine *e);
/* Launches per gradient step of the large-batch stage path (sac_wide.h:
 * layer-synchronous GEMM stages for phases A and C, used where the per-network
 * role kernels do not fit), else 0. */
int sac_engine_uses_wide(const sac_engine *e);
/* Launches per step of each phase A, B, C, D into out[4] (the stage path runs
   several per phase; its first-step gather is not counted); returns 0. */
int sac_engine_phase_launches(const sac_engine *e, int32_t *out);
/* Host evaluation of the device sampler (the same inline code as the sampler
 * inside sac_engine_train and sac_replay_sample_indices): out[b] = b-th element
 * of the Philox-keyed Feistel permutation of [0, size) for RNG (seed, step). */
int sac_debug_sample_indices_host(int64_t size, int32_t batch, uint64_t seed, uint64_t step, int32_t *out);
/* Host evaluation of the device eps draws of one step (the same inline
 * philox_normal2 the phase kernels call in their default device-RNG mode, compiled
 * for the host): out[which][b][j], which = 0 the target rsample (agent.py:204),
 * 1 the actor rsample (agent.py:241), rows b < batch, action dims j < act_dim
 * (models.py:83: eps of rsample).  Counter (step, b, which << 16 | j / 2), key
 * seed; Box-Muller gives dims 2p and 2p + 1. */
int sac_debug_eps_host(uint64_t seed, uint64_t step, int32_t batch, int32_t act_dim, float *out);
/* The same draws computed on the device (out: device [2][batch][act_dim]). */
int sac_debug_eps_device(uint64_t seed, uint64_t step, int32_t batch, int32_t act_dim, float *out, void *stream);
/* Polls a hand-off wait makes before it gives up and sets the timeout flag
 * (default 1 << 22, about 0.3 s); synchronises the stream.  A bound of 0
 * forces the timeout path (tests/test_gpu_engine.py): the API must raise. */
int sac_engine_debug_set_spin_limit(sac_engine *e, int32_t polls, void *stream);
#ifdef __cplusplus
}
#endif
#endif
