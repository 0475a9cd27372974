// Host emulation of the HIP kernels' execution model for the wave-level code
// in nimblephysics_amd/csrc (test infrastructure only, never part of the
// product): every GPU thread is a host thread; a workgroup's waves are 64
// threads each, and every cross-lane operation (readlane, ballot, bpermute,
// DPP, MFMA, wave barrier) is a rendezvous of the wave's 64 threads, so the
// emulation is exact for code that enters each cross-lane operation with the
// whole wave (the contract the kernels state).  Workgroups run one after
// another; LDS is one host array.  Host API (hipMalloc, hipMemcpy,
// hipLaunchKernelGGL, ...) maps onto host memory and the emulated launch, so
// the C-ABI (capi.cpp) runs unchanged on the CPU.  Built with
// AddressSanitizer by tests/test_wave_emu.py to catch out-of-bounds accesses.
#pragma once
#include <atomic>
#include <chrono>
#include <barrier>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

using std::fabs;
using std::fmin;
using std::isfinite;
using std::isnan;
using std::sqrt;

#define __device__
#define __host__
#define __global__
#define __shared__
#define __forceinline__ inline
#define __noinline__ __attribute__((noinline))
#define __launch_bounds__(...)
#define NIMBLE_OPAQUE_SGPR(x) ((void)(x))
#define amdgpu_waves_per_eu(...) unused

struct dim3 {
  unsigned x = 1, y = 1, z = 1;
  dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};

namespace wave_emu {
constexpr int kMaxWaves = 2;
inline std::barrier<>* waveBar[kMaxWaves] = {nullptr, nullptr};
inline std::barrier<>* blockBar = nullptr;
inline thread_local int tl_lane = 0;
inline thread_local int tl_wave = 0;
inline thread_local dim3 tl_tid, tl_bid, tl_bdim, tl_gdim;
inline uint64_t slots[kMaxWaves][64];
inline uint64_t slots2[kMaxWaves][64];
// per-lane count of the wave's rendezvous: every lane must have taken the
// same number when it arrives at one (a lane that skipped a cross-lane
// operation inside lane-divergent code would desynchronise the emulation --
// the check turns that into an abort with the lanes' stacks)
inline thread_local uint64_t tl_seq = 0;
inline uint64_t seqs[kMaxWaves][64];
}  // namespace wave_emu
extern "C" void __sanitizer_print_stack_trace();
namespace wave_emu {
inline uint64_t sites[kMaxWaves][64];
// hash of the calling frames' return addresses (frame-pointer walk; the
// driver is built with -O0 -fno-omit-frame-pointer so every call site of a
// cross-lane operation has its own frames): lanes that meet at one
// rendezvous from different call sites are out of step
__attribute__((noinline)) inline uint64_t callSite() {
  uint64_t h = 1469598103934665603ull;
  void** fp = (void**)__builtin_frame_address(0);
  for (int d = 0; d < 12 && fp; d++) {
    void** next = (void**)fp[0];
    h = (h ^ (uint64_t)fp[1]) * 1099511628211ull;
    if (next <= fp || (char*)next - (char*)fp > (1 << 20)) break;
    fp = next;
  }
  return h;
}
inline void waveSync() {
  seqs[tl_wave][tl_lane] = ++tl_seq;
  sites[tl_wave][tl_lane] = callSite();
  waveBar[tl_wave]->arrive_and_wait();
  const uint64_t s0 = seqs[tl_wave][0];
  const bool bad = seqs[tl_wave][tl_lane] != s0 || sites[tl_wave][tl_lane] != sites[tl_wave][0];
  waveBar[tl_wave]->arrive_and_wait();
  if (bad) {
    std::fprintf(stderr, "wave_emu: lane %d (rendezvous %llu) out of step with lane 0 (%llu) -- lane %d's stack:\n",
                 tl_lane, (unsigned long long)tl_seq, (unsigned long long)s0, tl_lane);
    __sanitizer_print_stack_trace();
    std::abort();
  }
}
inline uint64_t exchange(uint64_t v, int src) {
  slots[tl_wave][tl_lane] = v;
  waveSync();
  const uint64_t r = slots[tl_wave][src & 63];
  waveSync();
  return r;
}
inline int readlane(int v, int l) { return (int)(uint32_t)exchange((uint32_t)v, l); }
inline unsigned long long ballot(bool p) {
  slots[tl_wave][tl_lane] = p ? 1 : 0;
  waveSync();
  unsigned long long m = 0;
  for (int i = 0; i < 64; i++) m |= (slots[tl_wave][i] ? 1ull : 0ull) << i;
  waveSync();
  return m;
}
// DPP controls used by wave.cuh: quad_perm [1,0,3,2] (0xB1), [2,3,0,1]
// (0x4E), row_ror:4 (0x124), row_ror:8 (0x128)
inline int dpp(int old, int src, int ctrl) {
  (void)old;
  const int l = tl_lane, row = l & ~15, q = l & ~3;
  int s = l;
  if (ctrl == 0xB1) s = q + ((l & 3) ^ 1);
  else if (ctrl == 0x4E) s = q + ((l & 3) ^ 2);
  else if (ctrl == 0x124) s = row + (((l & 15) + 4) & 15);
  else if (ctrl == 0x128) s = row + (((l & 15) + 8) & 15);
  else std::abort();
  return (int)(uint32_t)exchange((uint32_t)src, s);
}
inline double asD(uint64_t u) { double d; std::memcpy(&d, &u, 8); return d; }
inline uint64_t asU(double d) { uint64_t u; std::memcpy(&u, &d, 8); return u; }
typedef double double4v __attribute__((ext_vector_type(4)));
// v_mfma_f64_16x16x4f64: A (16 x 4) lane l = row l % 16, k = l / 16; B (4 x
// 16) lane l = column l % 16, k = l / 16; D element e of lane l = row
// l / 16 + 4 e, column l % 16
inline double4v mfma16x16x4(double a, double b, double4v c) {
  slots[tl_wave][tl_lane] = asU(a);
  slots2[tl_wave][tl_lane] = asU(b);
  waveSync();
  double4v d = c;
  const int col = tl_lane & 15, r0 = tl_lane >> 4;
  for (int e = 0; e < 4; e++) {
    const int row = r0 + 4 * e;
    double acc = 0.0;
    for (int k = 0; k < 4; k++) acc += asD(slots[tl_wave][row + 16 * k]) * asD(slots2[tl_wave][col + 16 * k]);
    d[e] += acc;
  }
  waveSync();
  return d;
}

template <class T>
inline T atomicLoadUniform(T* p) {
  const T v = __atomic_load_n(p, __ATOMIC_SEQ_CST);
  return (T)exchange((uint64_t)(int64_t)v, 0);
}

// the emulated launch: workgroups in order, each with blockDim host threads
template <class K, class... A>
void launch(K kernel, dim3 grid, dim3 block, size_t lds, A... args) {
  (void)lds;
  const int threads = (int)block.x;
  const int waves = (threads + 63) / 64;
  if (waves > kMaxWaves || threads % 64) std::abort();
  std::barrier<> wb0(64), wb1(64), bb(threads);
  waveBar[0] = &wb0;
  waveBar[1] = &wb1;
  blockBar = &bb;
  for (unsigned b = 0; b < grid.x; b++) {
    std::vector<std::thread> ths;
    for (int t = 0; t < threads; t++)
      ths.emplace_back([&, t] {
        tl_seq = 0;
        tl_lane = t & 63;
        tl_wave = t >> 6;
        tl_tid = dim3(t);
        tl_bid = dim3(b);
        tl_bdim = block;
        tl_gdim = grid;
        kernel(args...);
      });
    for (auto& th : ths) th.join();
  }
}
}  // namespace wave_emu

#define threadIdx (wave_emu::tl_tid)
#define blockIdx (wave_emu::tl_bid)
#define blockDim (wave_emu::tl_bdim)
#define gridDim (wave_emu::tl_gdim)
#define __syncthreads() wave_emu::blockBar->arrive_and_wait()

#define __builtin_amdgcn_readlane(v, l) wave_emu::readlane((v), (l))
// readfirstlane (uni / unid) is applied only to values every lane holds
// equally (wave.cuh's contract): the identity, no rendezvous -- so it may
// sit in lane-divergent code, as on the GPU
#define __builtin_amdgcn_readfirstlane(v) (v)
#define __builtin_amdgcn_update_dpp(o, s, c, r, b, bc) wave_emu::dpp((o), (s), (c))
#define __builtin_amdgcn_fence(a, b) std::atomic_thread_fence(std::memory_order_seq_cst)
#define __builtin_amdgcn_wave_barrier() wave_emu::waveSync()
#define __builtin_amdgcn_s_memtime() 0ll
// (the two-wave deadlock guard never expires under emulation: an emulated
// wave can legitimately wait for seconds)
#define __builtin_amdgcn_s_memrealtime() 0ll
#define __builtin_amdgcn_s_getreg(r) 0u
#define __builtin_amdgcn_s_setprio(p) ((void)0)
#define __builtin_amdgcn_s_sleep(n) std::this_thread::sleep_for(std::chrono::microseconds(50))
#define __builtin_amdgcn_rsq(x) (1.0 / std::sqrt(x))
#define __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, x, y, z) wave_emu::mfma16x16x4((a), (b), (c))
// the kernels poll LDS flags with uni(atomic load) in whole-wave spin loops:
// lane 0's observation is broadcast (a rendezvous), so the wave leaves the
// loop together, as the readfirstlane makes it do on the GPU
#define __hip_atomic_load(p, o, s) wave_emu::atomicLoadUniform(p)
#define __hip_atomic_store(p, v, o, s) __atomic_store_n((p), (v), __ATOMIC_SEQ_CST)
// (lane 0 only, in the kernels; the winner is broadcast with a readlane)
#define __hip_atomic_compare_exchange_strong(p, e, d, o1, o2, s) \
  __atomic_compare_exchange_n((p), (e), (d), false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)
#define __HIP_MEMORY_SCOPE_WORKGROUP 0
#define __HIP_MEMORY_SCOPE_AGENT 1
// (lane 0 only: the deferred-world lists)
#define __hip_atomic_fetch_add(p, v, o, s) __atomic_fetch_add((p), (v), __ATOMIC_SEQ_CST)

inline int __double2loint(double d) { return (int)(uint32_t)wave_emu::asU(d); }
inline int __double2hiint(double d) { return (int)(uint32_t)(wave_emu::asU(d) >> 32); }
inline double __hiloint2double(int hi, int lo) {
  return wave_emu::asD(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
inline unsigned long long __ballot(bool p) { return wave_emu::ballot(p); }
inline int __ffsll(long long v) { return __builtin_ffsll(v); }
inline int __popcll(unsigned long long v) { return __builtin_popcountll(v); }
inline double __shfl(double v, int src) { return wave_emu::asD(wave_emu::exchange(wave_emu::asU(v), src & 63)); }
inline int __shfl(int v, int src) { return (int)(uint32_t)wave_emu::exchange((uint32_t)v, src & 63); }
inline unsigned __shfl_xor(unsigned v, int m) { return (unsigned)wave_emu::exchange(v, (wave_emu::tl_lane ^ m) & 63); }
inline int __shfl_xor(int v, int m) { return (int)(uint32_t)wave_emu::exchange((uint32_t)v, (wave_emu::tl_lane ^ m) & 63); }
inline double __shfl_xor(double v, int m) {
  return wave_emu::asD(wave_emu::exchange(wave_emu::asU(v), (wave_emu::tl_lane ^ m) & 63));
}
inline int __shfl_up(int v, unsigned d) {
  const int src = wave_emu::tl_lane - (int)d;
  const int r = (int)(uint32_t)wave_emu::exchange((uint32_t)v, src < 0 ? wave_emu::tl_lane : src);
  return r;
}

// host API over host memory
typedef int hipError_t;
typedef void* hipStream_t;
typedef void* hipFunction_t;
enum { hipSuccess = 0, hipMemcpyHostToDevice = 1, hipMemcpyDeviceToHost = 2, hipMemcpyDeviceToDevice = 3 };
inline hipError_t hipMalloc(void** p, size_t n) { *p = std::calloc(1, n ? n : 1); return *p ? 0 : 2; }
template <class T>
inline hipError_t hipMalloc(T** p, size_t n) { return hipMalloc((void**)p, n); }
inline hipError_t hipFree(void* p) { std::free(p); return 0; }
inline hipError_t hipMemcpy(void* d, const void* s, size_t n, int) { std::memcpy(d, s, n); return 0; }
inline hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t) { std::memset(p, v, n); return 0; }
inline hipError_t hipGetLastError() { return 0; }
inline const char* hipGetErrorString(hipError_t) { return "emulated"; }
#define hipLaunchKernelGGL(k, g, b, lds, st, ...) wave_emu::launch(k, dim3(g), dim3(b), (size_t)(lds), __VA_ARGS__)
