// Cholesky variants for the 33 x 33 packed joint-space mass matrix (one world
// per 64-lane wave, 1024 worlds, 40 KB LDS per workgroup as in the forward
// kernel so 4 worlds share a CU):
//   left  : the kernel's left-looking Crout (one lane per row, j-long dot
//           product per column, csrc/chol_wave.cuh)
//   right : right-looking, one lane per row; column j's multipliers stay in
//           the lanes' registers and the trailing update is (n-j) independent
//           LDS read-modify-writes per lane (same per-element subtraction
//           order, so bit-identical to `left`)
//   left4 : left-looking with four partial sums (shorter FMA chains, not
//           bit-identical)
// Prints JSON: mean clocks per factorisation and the max |diff| vs `left`.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>

#define REPS 40
#define NDOF 33
__device__ __forceinline__ int tri(int i, int k) { return ((i * (i + 1)) >> 1) + k; }
__device__ __forceinline__ double rdl(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}
#define WSYNC()                                            \
  do {                                                     \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); \
    __builtin_amdgcn_wave_barrier();                       \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup"); \
  } while (0)

__device__ void cholLeft(double* A, double* dinv, int n, int lane) {
  for (int j = 0; j < n; j++) {
    double sum = 0.0;
    if (lane >= j && lane < n) {
      const int ri = tri(lane, 0), rj = tri(j, 0);
      sum = A[ri + j];
#pragma unroll 8
      for (int k = 0; k < j; k++) sum -= A[ri + k] * A[rj + k];
    }
    const double djj = sqrt(rdl(sum, j));
    if (lane == j) { A[tri(j, j)] = djj; dinv[j] = 1.0 / djj; }
    else if (lane > j && lane < n) A[tri(lane, j)] = sum / djj;
    WSYNC();
  }
}

__device__ void cholRight(double* A, double* dinv, int n, int lane) {
  const int ri = tri(lane < n ? lane : 0, 0);
  for (int j = 0; j < n; j++) {
    const double ajj = A[tri(j, j)];
    const double aij = (lane > j && lane < n) ? A[ri + j] : 0.0;
    const double djj = sqrt(ajj);
    const double lij = aij / djj;
    if (lane == j) { A[tri(j, j)] = djj; dinv[j] = 1.0 / djj; }
    else if (lane > j && lane < n) A[ri + j] = lij;
    // trailing update of row `lane`: A_ik -= L_ij L_kj, k = j+1 .. lane
#pragma unroll 4
    for (int k = j + 1; k < n; k++) {
      const double lkj = rdl(lij, k);
      if (lane >= k && lane < n) A[ri + k] -= lij * lkj;
    }
    WSYNC();
  }
}

__device__ void cholLeft4(double* A, double* dinv, int n, int lane) {
  for (int j = 0; j < n; j++) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    if (lane >= j && lane < n) {
      const int ri = tri(lane, 0), rj = tri(j, 0);
      s0 = A[ri + j];
      int k = 0;
      for (; k + 4 <= j; k += 4) {
        s0 -= A[ri + k] * A[rj + k];
        s1 -= A[ri + k + 1] * A[rj + k + 1];
        s2 -= A[ri + k + 2] * A[rj + k + 2];
        s3 -= A[ri + k + 3] * A[rj + k + 3];
      }
      for (; k < j; k++) s0 -= A[ri + k] * A[rj + k];
    }
    const double sum = (s0 + s1) + (s2 + s3);
    const double djj = sqrt(rdl(sum, j));
    if (lane == j) { A[tri(j, j)] = djj; dinv[j] = 1.0 / djj; }
    else if (lane > j && lane < n) A[tri(lane, j)] = sum / djj;
    WSYNC();
  }
}

// left-looking, one reciprocal per column (multiply instead of divide)
__device__ void cholLeftR(double* A, double* dinv, int n, int lane) {
  for (int j = 0; j < n; j++) {
    double sum = 0.0;
    if (lane >= j && lane < n) {
      const int ri = tri(lane, 0), rj = tri(j, 0);
      sum = A[ri + j];
#pragma unroll 8
      for (int k = 0; k < j; k++) sum -= A[ri + k] * A[rj + k];
    }
    const double ajj = rdl(sum, j);
    const double djj = sqrt(ajj);
    const double rj = 1.0 / djj;
    if (lane == j) { A[tri(j, j)] = djj; dinv[j] = rj; }
    else if (lane > j && lane < n) A[tri(lane, j)] = sum * rj;
    WSYNC();
  }
}
// left-looking with the fast reciprocal square root (v_rsq_f64 + one Newton
// step): dinv = rsqrt(a) refined, L_jj = a * dinv
__device__ void cholLeftQ(double* A, double* dinv, int n, int lane) {
  for (int j = 0; j < n; j++) {
    double sum = 0.0;
    if (lane >= j && lane < n) {
      const int ri = tri(lane, 0), rj = tri(j, 0);
      sum = A[ri + j];
#pragma unroll 8
      for (int k = 0; k < j; k++) sum -= A[ri + k] * A[rj + k];
    }
    const double ajj = rdl(sum, j);
    double y = __builtin_amdgcn_rsq(ajj);
    y = y * (1.5 - 0.5 * ajj * y * y);
    y = y * (1.5 - 0.5 * ajj * y * y);
    const double djj = ajj * y;
    if (lane == j) { A[tri(j, j)] = djj; dinv[j] = y; }
    else if (lane > j && lane < n) A[tri(lane, j)] = sum * y;
    WSYNC();
  }
}
// left-looking, dot products in whole chunks of U (zero-selected past j: no
// remainder loop) and the rsqrt-based column scaling
template <int U>
__device__ void cholLeftPad(double* A, double* dinv, int n, int lane) {
  for (int j = 0; j < n; j++) {
    double sum = 0.0;
    if (lane >= j && lane < n) {
      const int ri = tri(lane, 0), rj = tri(j, 0);
      sum = A[ri + j];
      for (int k0 = 0; k0 < j; k0 += U) {
        double a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; u++) { a[u] = A[ri + k0 + u]; b[u] = A[rj + k0 + u]; }
#pragma unroll
        for (int u = 0; u < U; u++) sum -= (k0 + u < j ? a[u] : 0.0) * (k0 + u < j ? b[u] : 0.0);
      }
    }
    const double ajj = rdl(sum, j);
    double y = __builtin_amdgcn_rsq(ajj);
    y = y * (1.5 - 0.5 * ajj * y * y);
    y = y * (1.5 - 0.5 * ajj * y * y);
    const double djj = ajj * y;
    if (lane == j) { A[tri(j, j)] = djj; dinv[j] = y; }
    else if (lane > j && lane < n) A[tri(lane, j)] = sum * y;
    WSYNC();
  }
}
// the loop floor: no square root / division at all (wrong values)
__device__ void cholFloor(double* A, double* dinv, int n, int lane) {
  for (int j = 0; j < n; j++) {
    double sum = 0.0;
    if (lane >= j && lane < n) {
      const int ri = tri(lane, 0), rj = tri(j, 0);
      sum = A[ri + j];
#pragma unroll 8
      for (int k = 0; k < j; k++) sum -= A[ri + k] * A[rj + k];
    }
    const double djj = rdl(sum, j);
    if (lane == j) { A[tri(j, j)] = djj; dinv[j] = djj; }
    else if (lane > j && lane < n) A[tri(lane, j)] = sum * 1e-3;
    WSYNC();
  }
}

template <int V>
__global__ void __launch_bounds__(64) bench(const double* __restrict__ Mg, double* __restrict__ out,
                                            long long* __restrict__ clk) {
  extern __shared__ double lds[];
  double* A = lds;
  double* dinv = lds + 600;
  const int lane = threadIdx.x;
  const int n = NDOF, P = NDOF * (NDOF + 1) / 2;
  const double* M = Mg + (size_t)blockIdx.x * P;
  long long tot = 0;
  for (int r = 0; r < REPS; r++) {
    for (int t = lane; t < P; t += 64) A[t] = M[t];
    WSYNC();
    const long long t0 = __builtin_amdgcn_s_memtime();
    if (V == 0) cholLeft(A, dinv, n, lane);
    else if (V == 1) cholRight(A, dinv, n, lane);
    else if (V == 2) cholLeft4(A, dinv, n, lane);
    else if (V == 3) cholLeftR(A, dinv, n, lane);
    else if (V == 4) cholLeftQ(A, dinv, n, lane);
    else if (V == 5) cholFloor(A, dinv, n, lane);
    else if (V == 6) cholLeftPad<8>(A, dinv, n, lane);
    else cholLeftPad<4>(A, dinv, n, lane);
    const long long t1 = __builtin_amdgcn_s_memtime();
    tot += t1 - t0;
  }
  for (int t = lane; t < P; t += 64) out[(size_t)blockIdx.x * P + t] = A[t];
  if (lane == 0) clk[blockIdx.x] = tot / REPS;
}

int main() {
  const int W = 1024, n = NDOF, P = n * (n + 1) / 2;
  std::vector<double> M((size_t)W * P);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1103515245u + 12345u; return ((s >> 8) & 0xFFFFFF) / 16777216.0 - 0.5; };
  for (int w = 0; w < W; w++) {
    std::vector<double> B(n * n), F(n * n, 0.0);
    for (auto& v : B) v = rnd();
    for (int i = 0; i < n; i++)
      for (int j = 0; j < n; j++) {
        double acc = i == j ? n : 0.0;
        for (int k = 0; k < n; k++) acc += B[i * n + k] * B[j * n + k];
        F[i * n + j] = acc;
      }
    for (int i = 0; i < n; i++)
      for (int k = 0; k <= i; k++) M[(size_t)w * P + i * (i + 1) / 2 + k] = F[i * n + k];
  }
  double *dM, *dO[8];
  long long* dC[8];
  (void)hipMalloc(&dM, M.size() * 8);
  (void)hipMemcpy(dM, M.data(), M.size() * 8, hipMemcpyHostToDevice);
  for (int v = 0; v < 8; v++) { (void)hipMalloc(&dO[v], M.size() * 8); (void)hipMalloc(&dC[v], W * 8); }
  const size_t lds = 40 * 1024;
  hipLaunchKernelGGL(bench<0>, dim3(W), dim3(64), lds, 0, dM, dO[0], dC[0]);
  hipLaunchKernelGGL(bench<1>, dim3(W), dim3(64), lds, 0, dM, dO[1], dC[1]);
  hipLaunchKernelGGL(bench<2>, dim3(W), dim3(64), lds, 0, dM, dO[2], dC[2]);
  hipLaunchKernelGGL(bench<3>, dim3(W), dim3(64), lds, 0, dM, dO[3], dC[3]);
  hipLaunchKernelGGL(bench<4>, dim3(W), dim3(64), lds, 0, dM, dO[4], dC[4]);
  hipLaunchKernelGGL(bench<5>, dim3(W), dim3(64), lds, 0, dM, dO[5], dC[5]);
  hipLaunchKernelGGL(bench<6>, dim3(W), dim3(64), lds, 0, dM, dO[6], dC[6]);
  hipLaunchKernelGGL(bench<7>, dim3(W), dim3(64), lds, 0, dM, dO[7], dC[7]);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::vector<double> O[8];
  double clk[8];
  for (int v = 0; v < 8; v++) {
    O[v].resize(M.size());
    std::vector<long long> C(W);
    (void)hipMemcpy(O[v].data(), dO[v], M.size() * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(C.data(), dC[v], W * 8, hipMemcpyDeviceToHost);
    clk[v] = 0;
    for (auto c : C) clk[v] += (double)c / W;
  }
  double d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int v = 1; v < 8; v++)
    for (size_t i = 0; i < M.size(); i++) d[v] = fmax(d[v], fabs(O[v][i] - O[0][i]) / (fabs(O[0][i]) + 1e-300));
  const char* nm[8] = {"left", "right", "left4", "left_recip", "left_rsq", "floor_no_sqrt_div", "pad8_rsq", "pad4_rsq"};
  printf("{\"n\": %d, \"worlds\": %d", n, W);
  for (int v = 0; v < 8; v++) printf(", \"%s\": {\"clk\": %.0f, \"max_rel_diff\": %.3g}", nm[v], clk[v], d[v]);
  printf("}\n");
  return 0;
}
