// COD micro-benchmark (tools/micro/cod_bench.py): one n x n problem per
// 64-lane workgroup, factorised and solved in LDS by codFactor /
// codSolveWave; per problem: shader clocks, rank and the min-norm solution.
// Built three times: register QR (default), -DNIMBLE_COD_LDS_ONLY, and the
// register QR with -DNIMBLE_COD_PROFILE (per-phase clocks in o[3..6]).
#include "../../nimblephysics_amd/csrc/lcp_wave.cuh"

extern "C" __global__ void __launch_bounds__(64)
cod_bench_kernel(int nmax, const int* nArr, const double* Ag, const double* bg, double* out, int rec) {
  extern __shared__ double ldsbuf[];
  const int lane = threadIdx.x;
  const int pb = blockIdx.x;
  const int n = nArr[pb];
  double* M = ldsbuf;                // n x n
  double* ws = M + nmax * nmax;    // carveCod workspace + v + z
  for (int t = lane; t < n * n; t += 64) M[t] = Ag[(size_t)pb * nmax * nmax + t];
  for (int t = lane; t < 12 * nmax + 64; t += 64) ws[t] = 0.0;
  __syncthreads();
  double* v = ws + 6 * nmax + 16;
  double* z = v + (nmax > 24 ? nmax : 24);
  const double b = lane < n ? bg[pb * nmax + lane] : 0.0;
  const long long t0 = __builtin_amdgcn_s_memtime();
  codFactor<true>(sp<true>(M), sp<true>(ws), n, n, n, sp<true>(v), lane);
  const long long t1 = __builtin_amdgcn_s_memtime();
  const double x = codSolveWave<true>(sp<true>(M), sp<true>(ws), n, n, n, b, sp<true>(z), lane);
  const long long t2 = __builtin_amdgcn_s_memtime();
  double* o = out + (size_t)pb * rec;
  Cod c;
  carveCod(ws, M, n, n, n, c);
  if (lane == 0) {
    o[0] = (double)(t1 - t0);
    o[1] = (double)(t2 - t1);
    o[2] = *c.rank;
  }
  if (lane < n) o[8 + lane] = x;
#ifdef NIMBLE_COD_PROFILE
  // per-phase clocks of the register QR (cod_wave.cuh codQrRegs)
  if (lane < 4) o[3 + lane] = g_codProf[blockIdx.x * 8 + lane];
#endif
}

extern "C" int cod_bench_launch(int P, int nmax, const int* nArr, const double* A, const double* b, double* out, int rec,
                                void* stream) {
  const size_t lds = (size_t)(nmax * nmax + 12 * nmax + 64) * sizeof(double);
#ifdef NIMBLE_COD_PROFILE
  static double* prof = nullptr;
  static int profN = 0;
  if (profN < P) {
    if (prof) (void)hipFree(prof);
    if (hipMalloc(&prof, (size_t)P * 8 * sizeof(double)) != hipSuccess) return 1;
    profN = P;
  }
  if (hipMemsetAsync(prof, 0, (size_t)P * 8 * sizeof(double), (hipStream_t)stream) != hipSuccess ||
      hipMemcpyToSymbolAsync(HIP_SYMBOL(g_codProf), &prof, sizeof(prof), 0, hipMemcpyHostToDevice,
                             (hipStream_t)stream) != hipSuccess)
    return 1;
#endif
  hipLaunchKernelGGL(cod_bench_kernel, dim3(P), dim3(64), lds, (hipStream_t)stream, nmax, nArr, A, b, out, rec);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// Wide variant (cod_bench.py wide): one n x n problem (n <= 128) per 64-lane
// workgroup with the two-slot factorisation codFactorR<true, 2> the wide
// forward kernel runs on its LDS stage; with -DNIMBLE_COD_PROFILE the per-step
// phase clocks of that path land in o[3..6].
extern "C" __global__ void __launch_bounds__(64)
cod_bench_wide_kernel(int nmax, const int* nArr, const double* Ag, const double* bg, double* out, int rec) {
  extern __shared__ double ldsbuf[];
  const int lane = threadIdx.x;
  const int pb = blockIdx.x;
  const int n = nArr[pb];
  double* M = ldsbuf;
  double* ws = M + nmax * nmax;
  for (int t = lane; t < n * n; t += 64) M[t] = Ag[(size_t)pb * nmax * nmax + t];
  for (int t = lane; t < 12 * nmax + 64; t += 64) ws[t] = 0.0;
  __syncthreads();
  double* v = ws + 6 * nmax + 16;
  double* z = v + nmax;
  double b[2], x[2];
  for (int s = 0; s < 2; s++) b[s] = lane + 64 * s < n ? bg[pb * nmax + lane + 64 * s] : 0.0;
  const long long t0 = __builtin_amdgcn_s_memtime();
  codFactorR<true, 2>(sp<true>(M), sp<true>(ws), n, n, n, sp<true>(v), lane);
  const long long t1 = __builtin_amdgcn_s_memtime();
  codSolveWaveR<true, 2>(sp<true>(M), sp<true>(ws), n, n, n, b, sp<true>(z), lane, x);
  const long long t2 = __builtin_amdgcn_s_memtime();
  double* o = out + (size_t)pb * rec;
  Cod c;
  carveCod(ws, M, n, n, n, c);
  if (lane == 0) {
    o[0] = (double)(t1 - t0);
    o[1] = (double)(t2 - t1);
    o[2] = *c.rank;
  }
  for (int s = 0; s < 2; s++)
    if (lane + 64 * s < n) o[8 + lane + 64 * s] = x[s];
#ifdef NIMBLE_COD_PROFILE
  if (lane < 5) o[3 + lane] = g_codProf[blockIdx.x * 8 + lane];
#endif
}

extern "C" int cod_bench_wide_launch(int P, int nmax, const int* nArr, const double* A, const double* b, double* out,
                                     int rec, void* stream) {
  const size_t lds = (size_t)(nmax * nmax + 12 * nmax + 64) * sizeof(double);
#ifdef NIMBLE_COD_PROFILE
  static double* prof = nullptr;
  static int profN = 0;
  if (profN < P) {
    if (prof) (void)hipFree(prof);
    if (hipMalloc(&prof, (size_t)P * 8 * sizeof(double)) != hipSuccess) return 1;
    profN = P;
  }
  if (hipMemsetAsync(prof, 0, (size_t)P * 8 * sizeof(double), (hipStream_t)stream) != hipSuccess ||
      hipMemcpyToSymbolAsync(HIP_SYMBOL(g_codProf), &prof, sizeof(prof), 0, hipMemcpyHostToDevice,
                             (hipStream_t)stream) != hipSuccess)
    return 1;
#endif
  if (nmax > 128 || lds > 160 * 1024) return 1;
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute((const void*)cod_bench_wide_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
          hipSuccess)
    return 1;
  hipLaunchKernelGGL(cod_bench_wide_kernel, dim3(P), dim3(64), lds, (hipStream_t)stream, nmax, nArr, A, b, out, rec);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
