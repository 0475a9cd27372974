// Wave-level primitives for the 64-lane CDNA4 wavefront: vectors of length
// <= 64 are held one element per lane in registers; reductions use DPP
// within 16-lane rows and v_readlane across rows, so their results are
// wave-uniform (SGPR) values usable directly in control flow.
#pragma once
#include <hip/hip_runtime.h>

__device__ __forceinline__ double rdl(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ int rdli(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

// Barrier of the one wave that owns a world.  The forward kernel runs a
// second (helper) wave per workgroup that never joins the world's barriers,
// so synchronisation is wave-scoped: workgroup-scope fences order the LDS
// traffic (a wave's LDS operations execute in order) and the wave barrier
// keeps the compiler from moving memory operations across it.
#define WSYNC()                                            \
  do {                                                     \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); \
    __builtin_amdgcn_wave_barrier();                       \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup"); \
  } while (0)

// Scalar (SGPR) copy of a value all lanes hold equally -- counts and flags
// read from LDS or global memory look lane-varying to the compiler, which
// then turns every loop and branch on them into exec-masked vector code.
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ double unid(double v) {
  const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
  const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
  return __hiloint2double(hi, lo);
}

// Hides a wave-uniform value from the optimiser (an empty asm that pins it
// in an SGPR pair), so an algebraic form chosen for the ISA is not folded
// back.  The host emulator of the kernels (tests/cpp/wave_emu) defines it
// away.
#ifndef NIMBLE_OPAQUE_SGPR
#define NIMBLE_OPAQUE_SGPR(x) asm("" : "+s"(x))
#endif

template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// LDS-typed pointers.  Device functions that are not inlined receive LDS
// data through generic pointers, and the compiler then emits FLAT accesses
// (slower, and each waits on both the vector-memory and the LDS counters).
// Buffers that may live in LDS or in HBM are passed as Space<kLds>::dptr:
// an address_space(3) pointer for LDS, so every access through it is a
// ds_read/ds_write, and a plain pointer for the HBM fallback.  Casting a
// generic pointer to the LDS type is only valid if it points into LDS.
typedef __attribute__((address_space(3))) double lds_double;
typedef __attribute__((address_space(3))) int lds_int;
template <bool kLds> struct Space;
template <> struct Space<true> { typedef lds_double* dptr; typedef const lds_double* cdptr; };
template <> struct Space<false> { typedef double* dptr; typedef const double* cdptr; };
template <bool kLds>
__device__ __forceinline__ typename Space<kLds>::dptr sp(double* p) { return (typename Space<kLds>::dptr)p; }
template <bool kLds>
__device__ __forceinline__ typename Space<kLds>::cdptr spc(const double* p) { return (typename Space<kLds>::cdptr)p; }
// generic view of a known-LDS pointer that keeps the LDS provenance visible
// inside the current function
template <bool kLds, class T>
__device__ __forceinline__ T* lds(T* p) {
  if constexpr (kLds) return (T*)((__attribute__((address_space(3))) T*)p);
  else return p;
}

// generic view of a known-global (HBM) pointer: global_load/store instead of
// FLAT (which also waits on the LDS counter)
template <class T>
__device__ __forceinline__ T* gbl(T* p) {
  return (T*)((__attribute__((address_space(1))) T*)p);
}

// sum over all 64 lanes (every lane must be active); wave-uniform result
__device__ __forceinline__ double waveSum(double v) {
  v += dppd<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dppd<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dppd<0x124>(v);  // row_ror:4
  v += dppd<0x128>(v);  // row_ror:8
  return (rdl(v, 0) + rdl(v, 16)) + (rdl(v, 32) + rdl(v, 48));
}

// min over all lanes; wave-uniform
__device__ __forceinline__ double waveMin(double v) {
  v = fmin(v, dppd<0xB1>(v));
  v = fmin(v, dppd<0x4E>(v));
  v = fmin(v, dppd<0x124>(v));
  v = fmin(v, dppd<0x128>(v));
  return fmin(fmin(rdl(v, 0), rdl(v, 16)), fmin(rdl(v, 32), rdl(v, 48)));
}

// lowest lane index whose predicate holds (-1 if none); wave-uniform
__device__ __forceinline__ int waveFirst(bool pred) {
  const unsigned long long m = __ballot(pred);
  return m ? __ffsll((long long)m) - 1 : -1;
}

// value held by lane (lane + 1) (the last lane gets its own value)
__device__ __forceinline__ double shiftDown1(double v, int lane) {
  return __shfl(v, lane + 1 < 64 ? lane + 1 : lane);
}
__device__ __forceinline__ int shiftDown1i(int v, int lane) { return __shfl(v, lane + 1 < 64 ? lane + 1 : lane); }

// ---------------------------------------------------------------------------
// Row-distributed vectors of up to 64 R elements: row i lives on lane
// (i & 63) in register slot (i >> 6) (R = 1 is the plain one-element-per-lane
// layout above; R = 2 carries the 65..128-row LCPs of worlds with more than
// 21 frictional contacts).  Row indices passed to these helpers are
// wave-uniform.
template <int R>
__device__ __forceinline__ double rdlR(const double (&v)[R], int i) {
  if constexpr (R == 1) return rdl(v[0], i);
  else return rdl((i >> 6) ? v[1] : v[0], i & 63);
}
template <int R>
__device__ __forceinline__ int rdliR(const int (&v)[R], int i) {
  if constexpr (R == 1) return rdli(v[0], i);
  else return rdli((i >> 6) ? v[1] : v[0], i & 63);
}
// row index of slot s on this lane
__device__ __forceinline__ int rowAt(int s, int lane) { return lane + 64 * s; }
// sum over all rows' partial values
template <int R>
__device__ __forceinline__ double waveSumR(const double (&v)[R]) {
  double t = v[0];
#pragma unroll
  for (int s = 1; s < R; s++) t += v[s];
  return waveSum(t);
}
// set row i of v (i wave-uniform) to val (this lane's value)
template <int R>
__device__ __forceinline__ void setR(double (&v)[R], int i, int lane, double val) {
#pragma unroll
  for (int s = 0; s < R; s++)
    if (rowAt(s, lane) == i) v[s] = val;
}
template <int R>
__device__ __forceinline__ void setRi(int (&v)[R], int i, int lane, int val) {
#pragma unroll
  for (int s = 0; s < R; s++)
    if (rowAt(s, lane) == i) v[s] = val;
}
// bit i of a row mask
template <int R>
__device__ __forceinline__ bool bitR(const unsigned long long (&mk)[R], int i) {
  if constexpr (R == 1) return (mk[0] >> i) & 1ull;
  else return (((i >> 6) ? mk[1] : mk[0]) >> (i & 63)) & 1ull;
}
template <int R>
__device__ __forceinline__ int popR(const unsigned long long (&mk)[R]) {
  int c = 0;
#pragma unroll
  for (int s = 0; s < R; s++) c += __popcll(mk[s]);
  return c;
}
// number of set rows below row i
template <int R>
__device__ __forceinline__ int rankR(const unsigned long long (&mk)[R], int i) {
  int c = 0;
#pragma unroll
  for (int s = 0; s < R; s++) {
    const int lo = 64 * s;
    if (i >= lo + 64) c += __popcll(mk[s]);
    else if (i > lo) c += __popcll(mk[s] & ((1ull << (i - lo)) - 1ull));
  }
  return c;
}
// lowest row whose predicate holds (-1 if none)
template <int R>
__device__ __forceinline__ int waveFirstR(const bool (&pred)[R]) {
#pragma unroll
  for (int s = 0; s < R; s++) {
    const unsigned long long m = __ballot(pred[s]);
    if (m) return 64 * s + __ffsll((long long)m) - 1;
  }
  return -1;
}
template <int R>
__device__ __forceinline__ double waveMinR(const double (&v)[R]) {
  double t = v[0];
#pragma unroll
  for (int s = 1; s < R; s++) t = fmin(t, v[s]);
  return waveMin(t);
}
// row i receives row i + 1 (the last row keeps its own value)
template <int R>
__device__ __forceinline__ void shiftDownR(double (&v)[R], int lane) {
  double nx[R];
#pragma unroll
  for (int s = 0; s < R; s++) {
    nx[s] = __shfl(v[s], lane + 1 < 64 ? lane + 1 : lane);
    const double next = s + 1 < R ? rdl(v[s + 1 < R ? s + 1 : s], 0) : v[s];
    if (lane == 63) nx[s] = next;
  }
#pragma unroll
  for (int s = 0; s < R; s++) v[s] = nx[s];
}
template <int R>
__device__ __forceinline__ void shiftDownRi(int (&v)[R], int lane) {
  int nx[R];
#pragma unroll
  for (int s = 0; s < R; s++) {
    nx[s] = __shfl(v[s], lane + 1 < 64 ? lane + 1 : lane);
    const int next = s + 1 < R ? rdli(v[s + 1 < R ? s + 1 : s], 0) : v[s];
    if (lane == 63) nx[s] = next;
  }
#pragma unroll
  for (int s = 0; s < R; s++) v[s] = nx[s];
}
// value of row `src` (lane-varying) of v, for every slot's row: a gather
// across rows (the R = 1 case is __shfl)
template <int R>
__device__ __forceinline__ double gatherR(const double (&v)[R], int src) {
  if constexpr (R == 1) return __shfl(v[0], src & 63);
  else {
    const double a = __shfl(v[0], src & 63), b = __shfl(v[1], src & 63);
    return (src >> 6) ? b : a;
  }
}
template <int R>
__device__ __forceinline__ int gatherRi(const int (&v)[R], int src) {
  if constexpr (R == 1) return __shfl(v[0], src & 63);
  else {
    const int a = __shfl(v[0], src & 63), b = __shfl(v[1], src & 63);
    return (src >> 6) ? b : a;
  }
}
