// Debug-build (-DNIMBLE_STAGE_TIMING) shader-clock instrumentation used by
// tools/stage_timing*.py; compiled out otherwise.
#pragma once
#include <hip/hip_runtime.h>
#ifdef NIMBLE_STAGE_TIMING
// debug builds: per-stage shader-clock stamps into the snapshot workspace
#define STAMP(k)                                                                   \
  do {                                                                             \
    if (lane == 0 && g_stamp) g_stamp[k] = (double)__builtin_amdgcn_s_memtime(); \
  } while (0)
// accumulating timers (slots >= 60): TACC_BEGIN(t) ... TACC_END(slot, t)
#define TACC_BEGIN(t) const long long t = (long long)__builtin_amdgcn_s_memtime()
#define TACC_END(k, t)                                                                            \
  do {                                                                                            \
    if (lane == 0 && g_stamp) g_stamp[k] += (double)((long long)__builtin_amdgcn_s_memtime() - t); \
  } while (0)
__device__ double* g_stamp_dummy;
#else
#define STAMP(k) do { } while (0)
#define TACC_BEGIN(t) do { } while (0)
#define TACC_END(k, t) do { } while (0)
#endif
