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
#ifdef __cplusplus
}
#endif
#endif
