// fp64 MFMA vs the VALU lane tiles for the two dense products of the
// timestep that have matrix shape ("Bound"):
//   gram : A = Y^T Y, Y n x m (n = 33 dofs, m <= 24 LCP rows), the LCP matrix
//          A = J Minv J^T with Y = L^-1 J^T (contact.cuh, 8 x 8 lane tiles);
//   syrk : C -= L21 L21^T, the trailing update of a blocked 33 x 33 Cholesky
//          of M (L21: 17 x 16), the only MFMA-shaped part of that factor.
// One world per 64-lane wave, 1024 worlds (the bench batch), operands in LDS
// as in the kernel; each variant is timed with s_memtime over REPS calls and
// checked against the VALU result.  Prints JSON.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>

#define REPS 200
typedef double double4_t __attribute__((ext_vector_type(4)));

template <int N, int M>
__device__ void gramValu(const double* Y, double* A, int lane) {
  const int rl = lane >> 3, cl = lane & 7;
  for (int r0 = 0; r0 < M; r0 += 8)
    for (int c0 = r0; c0 < M; c0 += 8) {
      const int r = r0 + rl, c = c0 + cl;
      if (r < M && c < M && r <= c) {
        double acc = 0;
#pragma unroll 8
        for (int i = 0; i < N; i++) acc += Y[i * M + r] * Y[i * M + c];
        A[r * M + c] = acc;
        A[c * M + r] = acc;
      }
    }
}

// v_mfma_f64_16x16x4f64: A operand lane l = row l%16, k = l/16; B operand
// lane l = col l%16, k = l/16; D register e of lane l holds col l%16,
// row l/16 + 4e (the f64 form does not use the f32 C/D map)
template <int N, int M>
__device__ void gramMfma(const double* Y, double* A, int lane) {
  const int i16 = lane & 15, kq = lane >> 4;
  constexpr int T = (M + 15) / 16;
#pragma unroll
  for (int ti = 0; ti < T; ti++)
#pragma unroll
    for (int tj = ti; tj < T; tj++) {
      double4_t acc = {0, 0, 0, 0};
      const int ri = ti * 16 + i16, cj = tj * 16 + i16;
#pragma unroll
      for (int k0 = 0; k0 < N; k0 += 4) {
        const int k = k0 + kq;
        const double a = (k < N && ri < M) ? Y[k * M + ri] : 0.0;
        const double b = (k < N && cj < M) ? Y[k * M + cj] : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
      }
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int r = ti * 16 + kq + 4 * e, c = tj * 16 + i16;
        if (r < M && c < M) { A[r * M + c] = acc[e]; A[c * M + r] = acc[e]; }
      }
    }
}

// trailing update C (P x P) -= L (P x K) L^T, K = 16
template <int P, int K>
__device__ void syrkValu(const double* L, double* C, int lane) {
  for (int t = lane; t < P * P; t += 64) {
    const int r = t / P, c = t % P;
    double acc = C[t];
#pragma unroll 8
    for (int k = 0; k < K; k++) acc -= L[r * K + k] * L[c * K + k];
    C[t] = acc;
  }
}
template <int P, int K>
__device__ void syrkMfma(const double* L, double* C, int lane) {
  const int i16 = lane & 15, kq = lane >> 4;
  constexpr int T = (P + 15) / 16;
#pragma unroll
  for (int ti = 0; ti < T; ti++)
#pragma unroll
    for (int tj = 0; tj < T; tj++) {
      double4_t acc;
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int r = ti * 16 + kq + 4 * e, c = tj * 16 + i16;
        acc[e] = (r < P && c < P) ? C[r * P + c] : 0.0;
      }
      const int ri = ti * 16 + i16, cj = tj * 16 + i16;
#pragma unroll
      for (int k0 = 0; k0 < K; k0 += 4) {
        const int k = k0 + kq;
        const double a = ri < P ? -L[ri * K + k] : 0.0;
        const double b = cj < P ? L[cj * K + k] : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
      }
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int r = ti * 16 + kq + 4 * e, c = tj * 16 + i16;
        if (r < P && c < P) C[r * P + c] = acc[e];
      }
    }
}

constexpr int N = 33, M = 24, P = 17, K = 16;

__global__ void __launch_bounds__(64) bench(const double* __restrict__ Yg, const double* __restrict__ Lg,
                                            double* __restrict__ out, long long* __restrict__ clk) {
  __shared__ double Y[N * M], A1[M * M], A2[M * M], L[P * K], C1[P * P], C2[P * P];
  const int lane = threadIdx.x;
  const double* y = Yg + (size_t)blockIdx.x * N * M;
  for (int i = lane; i < N * M; i += 64) Y[i] = y[i];
  for (int i = lane; i < P * K; i += 64) L[i] = Lg[(size_t)blockIdx.x * P * K + i];
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REPS; r++) { gramValu<N, M>(Y, A1, lane); __builtin_amdgcn_wave_barrier(); }
  long long t1 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REPS; r++) { gramMfma<N, M>(Y, A2, lane); __builtin_amdgcn_wave_barrier(); }
  long long t2 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REPS; r++) {
    for (int i = lane; i < P * P; i += 64) C1[i] = 0.0;
    syrkValu<P, K>(L, C1, lane);
    __builtin_amdgcn_wave_barrier();
  }
  long long t3 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REPS; r++) {
    for (int i = lane; i < P * P; i += 64) C2[i] = 0.0;
    syrkMfma<P, K>(L, C2, lane);
    __builtin_amdgcn_wave_barrier();
  }
  long long t4 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  double e1 = 0, e2 = 0;
  for (int i = lane; i < M * M; i += 64) e1 = fmax(e1, fabs(A1[i] - A2[i]) / (fabs(A1[i]) + 1e-300));
  for (int i = lane; i < P * P; i += 64) e2 = fmax(e2, fabs(C1[i] - C2[i]) / (fabs(C1[i]) + 1e-300));
  out[blockIdx.x * 128 + lane] = e1;
  out[blockIdx.x * 128 + 64 + lane] = e2;
  if (lane == 0) {
    clk[blockIdx.x * 4 + 0] = (t1 - t0) / REPS;
    clk[blockIdx.x * 4 + 1] = (t2 - t1) / REPS;
    clk[blockIdx.x * 4 + 2] = (t3 - t2) / REPS;
    clk[blockIdx.x * 4 + 3] = (t4 - t3) / REPS;
  }
}

int main() {
  const int W = 1024;
  std::vector<double> Y((size_t)W * N * M), L((size_t)W * P * K);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1103515245u + 12345u; return ((s >> 8) & 0xFFFF) / 65536.0 - 0.5; };
  for (auto& v : Y) v = rnd();
  for (auto& v : L) v = rnd();
  double *dY, *dL, *dO;
  long long* dC;
  (void)hipMalloc(&dY, Y.size() * 8); (void)hipMalloc(&dL, L.size() * 8);
  (void)hipMalloc(&dO, (size_t)W * 128 * 8); (void)hipMalloc(&dC, (size_t)W * 4 * 8);
  (void)hipMemcpy(dY, Y.data(), Y.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dL, L.data(), L.size() * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(bench, dim3(W), dim3(64), 0, 0, dY, dL, dO, dC);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(bench, dim3(W), dim3(64), 0, 0, dY, dL, dO, dC);
  (void)hipEventRecord(e1);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<double> O((size_t)W * 128);
  std::vector<long long> C((size_t)W * 4);
  (void)hipMemcpy(O.data(), dO, O.size() * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(C.data(), dC, C.size() * 8, hipMemcpyDeviceToHost);
  double err1 = 0, err2 = 0, c[4] = {0, 0, 0, 0};
  for (int w = 0; w < W; w++) {
    for (int l = 0; l < 64; l++) { err1 = fmax(err1, O[w * 128 + l]); err2 = fmax(err2, O[w * 128 + 64 + l]); }
    for (int k = 0; k < 4; k++) c[k] += (double)C[w * 4 + k] / W;
  }
  printf("{\"worlds\": %d, \"reps\": %d, \"gram_33x24\": {\"valu_clk\": %.0f, \"mfma_clk\": %.0f, \"max_rel_diff\": %.3g}, "
         "\"syrk_17x16\": {\"valu_clk\": %.0f, \"mfma_clk\": %.0f, \"max_rel_diff\": %.3g}, \"kernel_ms\": %.3f}\n",
         W, REPS, c[0], c[1], err1, c[2], c[3], err2, ms);
  return 0;
}
