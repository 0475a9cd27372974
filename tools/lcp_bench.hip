// Stand-alone harness for the wave LCP solvers (tools/lcp_bench.py): one
// problem per 64-lane workgroup, A staged in LDS as in the forward kernel,
// shader clocks of each solver written per problem.  Built with
// -DLCP_PROFILE for the Dantzig per-phase split.
#include "../nimblephysics_amd/csrc/lcp_wave.cuh"

struct Rec {  // per problem output (doubles)
  enum { OK_D = 0, CLK_D, OK_P, CLK_P, PIV, PIVROW, PGS_IT, PROF = 8, X_D = 16, X_P = 64, PGSPROF = 112, CODPROF = 120, SIZE = 128 };
};

extern "C" __global__ void __launch_bounds__(64)
lcp_bench_kernel(int nmax, int nl, const int* nArr, const double* Ag, const double* bg, const double* log_,
                 const double* hig, const int* fig, const double* x0g, double* out) {
  extern __shared__ double ldsbuf[];
  const int lane = threadIdx.x;
  const int pb = blockIdx.x;
  const int n = nArr[pb];
  const int ldA = nl * nl;
  double* A = ldsbuf;
  double* M1 = A + ldA;
  double* Lb = M1 + ldA;
  double* scr = Lb + nl * (nl | 1);
  double* o = out + (size_t)pb * Rec::SIZE;
  for (int t = lane; t < n * n; t += 64) A[t] = Ag[(size_t)pb * nmax * nmax + t];
  __syncthreads();
  const double b = lane < n ? bg[pb * nmax + lane] : 0.0;
  const double lo = lane < n ? log_[pb * nmax + lane] : 0.0;
  const double hi = lane < n ? hig[pb * nmax + lane] : 0.0;
  const int fi = lane < n ? fig[pb * nmax + lane] : -1;
  double dbg[16];
  for (int k = 0; k < 16; k++) dbg[k] = 0.0;
  __shared__ double dshared[24];
  if (lane < 24) dshared[lane] = 0.0;
  __syncthreads();

  for (int t = lane; t < n * n; t += 64) M1[t] = A[t];
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  double xd = 0.0;
  const bool okD = waveDantzig<true>(n, spc<true>(A), sp<true>(Lb), sp<true>(scr), xd, b, lo, hi, fi, lane, dshared);
  long long t1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  double xp = lane < n ? x0g[pb * nmax + lane] : 0.0;
  long long t2 = __builtin_amdgcn_s_memtime();
  const bool okP = wavePgs<true>(n, spc<true>(A), xp, b, lo, hi, fi, lane, dshared + 12);
  long long t3 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  (void)dbg;
  // COD of the full problem matrix (construct-sized Q) and a solve
  for (int t = lane; t < n * n; t += 64) M1[t] = A[t];
  for (int t = lane; t < 10 * nl + 16; t += 64) Lb[t] = 0.0;
  __syncthreads();
  long long t4 = __builtin_amdgcn_s_memtime();
  codFactor<true>(sp<true>(M1), sp<true>(Lb), n, n, n, sp<true>(Lb + 8 * nl + 16), lane);
  long long t5 = __builtin_amdgcn_s_memtime();
  const double zc = codSolveWave<true>(sp<true>(M1), sp<true>(Lb), n, n, n, b, sp<true>(Lb + 9 * nl + 16), lane);
  long long t6 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    o[Rec::PGSPROF + 3] = (double)(t5 - t4);
    o[Rec::PGSPROF + 4] = (double)(t6 - t5);
  }
  if (lane < n && !isfinite(zc)) o[Rec::PGSPROF + 7] = 1;
  if (lane == 0) {
    o[Rec::OK_D] = okD ? 1 : 0;
    o[Rec::CLK_D] = (double)(t1 - t0);
    o[Rec::OK_P] = okP ? 1 : 0;
    o[Rec::CLK_P] = (double)(t3 - t2);
    o[Rec::PIV] = dshared[0];
    o[Rec::PIVROW] = dshared[1];
    o[Rec::PGS_IT] = dshared[12];
    o[Rec::PGS_IT + 1] = dshared[13];
    for (int k = 0; k < 3; k++) o[Rec::PGSPROF + k] = dshared[14 + k];
    for (int k = 0; k < 8; k++) o[Rec::PROF + k] = dshared[2 + k];
  }
  if (lane < n) {
    o[Rec::X_D + lane] = xd;
    o[Rec::X_P + lane] = xp;
  }
}

extern "C" int lcp_bench_launch(int P, int nmax, int nl, const int* nArr, const double* A, const double* b, const double* lo,
                                const double* hi, const int* fi, const double* x0, double* out, void* stream) {
  const size_t ldsBytes = (size_t)(3 * nl * nl + 2 * nl * (nl | 1) + 64) * sizeof(double);
  hipLaunchKernelGGL(lcp_bench_kernel, dim3(P), dim3(64), ldsBytes, (hipStream_t)stream, nmax, nl, nArr, A, b, lo, hi, fi, x0,
                     out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// The wide kernels' Dantzig (R = 2, up to 128 rows) as the forward stages it:
// L, A's packed lower triangle and the scatter vector in LDS.  One problem
// per 64-lane workgroup; per problem: ok, clocks, pivots, the per-phase split
// (LCP_PROFILE: swap, solveL1, solveL1T, ldltRemove, w_i, pivot body), x.
// kPL: L in the packed panels the wide forward kernel's stage holds
template <bool kPL>
__global__ void __launch_bounds__(64)
lcp_bench_wide_kernel(int nmax, int nl, const int* nArr, const double* Ag, const double* bg, const double* log_,
                      const double* hig, const int* fig, double* out) {
  extern __shared__ double ldsbuf[];
  const int lane = threadIdx.x;
  const int pb = blockIdx.x;
  const int n = nArr[pb];
  lds_double* L = (lds_double*)ldsbuf;
  lds_double* Ap = L + nl * (nl | 1);
  lds_double* scr = Ap + nl * (nl + 1) / 2;
  double* o = out + (size_t)pb * Rec::SIZE;
  for (int i = 0; i < n; i++)
    for (int j = lane; j <= i; j += 64) Ap[i * (i + 1) / 2 + j] = Ag[(size_t)pb * nmax * nmax + i * n + j];
  __syncthreads();
  double b[2], lo[2], hi[2], x[2];
  int fi[2];
  for (int s = 0; s < 2; s++) {
    const int r = lane + 64 * s;
    b[s] = r < n ? bg[pb * nmax + r] : 0.0;
    lo[s] = r < n ? log_[pb * nmax + r] : 0.0;
    hi[s] = r < n ? hig[pb * nmax + r] : 0.0;
    fi[s] = r < n ? fig[pb * nmax + r] : -1;
  }
  __shared__ double dshared[24];
  if (lane < 24) dshared[lane] = 0.0;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  const bool ok = waveDantzigR<true, 2, true, true, kPL>(n, Ap, L, scr, x, b, lo, hi, fi, lane, dshared);
  const long long t1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  if (lane == 0) {
    o[Rec::OK_D] = ok ? 1 : 0;
    o[Rec::CLK_D] = (double)(t1 - t0);
    o[Rec::PIV] = dshared[0];
    o[Rec::PIVROW] = dshared[1];
    for (int k = 0; k < 8; k++) o[Rec::PROF + k] = dshared[2 + k];
  }
  for (int s = 0; s < 2; s++) {
    const int r = lane + 64 * s;
    if (r < n && 16 + r < Rec::SIZE) o[16 + r] = x[s];
  }
}

extern "C" int lcp_bench_wide_launch(int P, int nmax, int nl, const int* nArr, const double* A, const double* b,
                                     const double* lo, const double* hi, const int* fi, double* out, void* stream) {
  const size_t ldsBytes = (size_t)(nl * (nl | 1) + nl * (nl + 1) / 2 + nl + 8) * sizeof(double);
  if (getenv("LCP_WIDE_PACKED") && atoi(getenv("LCP_WIDE_PACKED")))
    hipLaunchKernelGGL(lcp_bench_wide_kernel<true>, dim3(P), dim3(64), ldsBytes, (hipStream_t)stream, nmax, nl, nArr, A,
                       b, lo, hi, fi, out);
  else
    hipLaunchKernelGGL(lcp_bench_wide_kernel<false>, dim3(P), dim3(64), ldsBytes, (hipStream_t)stream, nmax, nl, nArr,
                       A, b, lo, hi, fi, out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
