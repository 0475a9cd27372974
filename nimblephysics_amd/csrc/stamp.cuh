// Debug-build (-DNIMBLE_STAGE_TIMING) shader-clock instrumentation used by
// tools/stage_timing*.py; compiled out otherwise.
#pragma once
#include <hip/hip_runtime.h>
// slot map of the 128 stamp doubles (tools/stage_timing.py checks it against
// the sources): single stamps 0..51, 70..77, 86..88, 90..98, the board's
// 100..103 and the wide kernel's own start / reload / v1 / end 104..107 (a
// deferred world's 10..13 are the one-row kernel's); accumulators 60..66,
// 76..77, 80..85; multi-slot debug blocks:
#define SLOT_PGS 54        // pgsFallback: 5 doubles (sweeps, contact rows, 3 phase clocks) -> 54..58
#define SLOT_COD 67        // codFactor prof: 3 doubles -> 67..69
#define SLOT_DANTZIG 110   // Dantzig: pivots, row, 8 phase clocks -> 110..119
#define SLOT_COUNT 128
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
