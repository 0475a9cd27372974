// fp64 MFMA for the classification COD's trailing update (VERDICT r2, next
// 4): a blocked (WY / LAPACK dlaqps-style) column-pivoted QR of the m <= 24
// clamping matrix would replace nb = 4 of the register QR's rank-1 reflector
// updates by one rank-4 update C -= V F^T, which is one v_mfma_f64_16x16x4f64
// per 16 x 16 tile.  This times that update both ways, one problem per
// 64-lane wave, 1024 waves (the bench batch), REPS repetitions each:
//   valu_regs : the register QR's layout (lane = column, 24 rows in VGPRs),
//               V broadcast from LDS, 4 x 24 FMAs per lane;
//   valu_lds  : the same with C in LDS (column per lane, read-modify-write);
//   mfma_lds  : C in LDS as 2 x 2 tiles of 16 x 16 (24 x 24 padded), each
//               tile loaded into the f64 accumulator layout, one MFMA with
//               K = 4 (V: A operand, F: B operand), stored back.
// The per-step phase split of the register QR itself comes from
// cod_bench.hip built with -DNIMBLE_COD_PROFILE (tools/micro/cod_bench.py).
// Prints JSON (clocks per update, mean over waves) and checks the three
// results agree.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

#define REPS 64
#define M 24
typedef double double4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void wsync() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); }

extern "C" __global__ void __launch_bounds__(64) rank4_kernel(const double* Cg, const double* Vg, const double* Fg,
                                                               double* out, double* clk) {
  __shared__ double C[32 * 32], V[32 * 4], F[32 * 4];
  const int lane = threadIdx.x, w = blockIdx.x;
  const double* Cw = Cg + (size_t)w * M * M;
  for (int t = lane; t < 32 * 32; t += 64) {
    const int r = t / 32, c = t % 32;
    C[t] = (r < M && c < M) ? Cw[r * M + c] : 0.0;
  }
  for (int t = lane; t < 32 * 4; t += 64) {
    const int r = t / 4, k = t % 4;
    V[t] = r < M ? Vg[(size_t)w * M * 4 + r * 4 + k] : 0.0;
    F[t] = r < M ? Fg[(size_t)w * M * 4 + r * 4 + k] : 0.0;
  }
  __syncthreads();
  double* o = out + (size_t)w * 3 * M * M;
  // valu_regs: column `lane` in registers
  {
    double a[M];
    const int cl = lane < M ? lane : 0;
#pragma unroll
    for (int i = 0; i < M; i++) a[i] = C[i * 32 + cl];
    wsync();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int rep = 0; rep < REPS; rep++) {
      double f[4];
#pragma unroll
      for (int k = 0; k < 4; k++) f[k] = F[cl * 4 + k];
#pragma unroll
      for (int i = 0; i < M; i++) {
        const double* vi = V + i * 4;
        a[i] -= vi[0] * f[0] + vi[1] * f[1] + vi[2] * f[2] + vi[3] * f[3];
      }
      // keep the loop from being folded: a dependency through LDS per rep
      if (lane == 0) F[31 * 4] = a[0] * 0.0;
      wsync();
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (lane < M)
#pragma unroll
      for (int i = 0; i < M; i++) o[i * M + lane] = a[i];
    if (lane == 0) clk[w * 3 + 0] = (double)(t1 - t0) / REPS;
  }
  // valu_lds: column `lane` read-modify-write in LDS (private copy)
  __shared__ double C2[32 * 32];
  for (int t = lane; t < 32 * 32; t += 64) C2[t] = C[t];
  wsync();
  {
    const int cl = lane < M ? lane : 0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int rep = 0; rep < REPS; rep++) {
      double f[4];
#pragma unroll
      for (int k = 0; k < 4; k++) f[k] = F[cl * 4 + k];
      if (lane < M)
#pragma unroll
        for (int i = 0; i < M; i++) {
          const double* vi = V + i * 4;
          C2[i * 32 + cl] -= vi[0] * f[0] + vi[1] * f[1] + vi[2] * f[2] + vi[3] * f[3];
        }
      wsync();
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (lane < M)
      for (int i = 0; i < M; i++) o[M * M + i * M + lane] = C2[i * 32 + lane];
    if (lane == 0) clk[w * 3 + 1] = (double)(t1 - t0) / REPS;
  }
  // mfma_lds: 2 x 2 tiles; A operand lane l = row l % 16, k = l / 16 (V);
  // B operand lane l = column l % 16, k = l / 16 (F); D element e of lane l
  // = row l / 16 + 4 e, column l % 16
  {
    const int i16 = lane & 15, kq = lane >> 4;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int rep = 0; rep < REPS; rep++) {
#pragma unroll
      for (int ti = 0; ti < 2; ti++)
#pragma unroll
        for (int tj = 0; tj < 2; tj++) {
          double4_t acc;
#pragma unroll
          for (int e = 0; e < 4; e++) acc[e] = C[(ti * 16 + kq + 4 * e) * 32 + tj * 16 + i16];
          const double va = -V[(ti * 16 + i16) * 4 + kq];
          const double fb = F[(tj * 16 + i16) * 4 + kq];
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(va, fb, acc, 0, 0, 0);
#pragma unroll
          for (int e = 0; e < 4; e++) C[(ti * 16 + kq + 4 * e) * 32 + tj * 16 + i16] = acc[e];
        }
      wsync();
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    for (int t = lane; t < M * M; t += 64) o[2 * M * M + t] = C[(t / M) * 32 + t % M];
    if (lane == 0) clk[w * 3 + 2] = (double)(t1 - t0) / REPS;
  }
}

int main() {
  const int W = 1024;
  std::vector<double> C((size_t)W * M * M), V((size_t)W * M * 4), F((size_t)W * M * 4);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xffff) / 65536.0 - 0.5; };
  for (auto& x : C) x = rnd();
  for (auto& x : V) x = rnd() * 0.1;
  for (auto& x : F) x = rnd() * 0.1;
  double *dC, *dV, *dF, *dO, *dK;
  hipMalloc(&dC, C.size() * 8); hipMalloc(&dV, V.size() * 8); hipMalloc(&dF, F.size() * 8);
  hipMalloc(&dO, (size_t)W * 3 * M * M * 8); hipMalloc(&dK, (size_t)W * 3 * 8);
  hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dV, V.data(), V.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dF, F.data(), F.size() * 8, hipMemcpyHostToDevice);
  for (int it = 0; it < 2; it++) hipLaunchKernelGGL(rank4_kernel, dim3(W), dim3(64), 0, 0, dC, dV, dF, dO, dK);
  if (hipDeviceSynchronize() != hipSuccess) { std::printf("{\"error\": \"launch\"}\n"); return 1; }
  std::vector<double> O((size_t)W * 3 * M * M), K((size_t)W * 3);
  hipMemcpy(O.data(), dO, O.size() * 8, hipMemcpyDeviceToHost);
  hipMemcpy(K.data(), dK, K.size() * 8, hipMemcpyDeviceToHost);
  double d01 = 0, d02 = 0;
  for (int w = 0; w < W; w++)
    for (int t = 0; t < M * M; t++) {
      const double* o = O.data() + (size_t)w * 3 * M * M;
      d01 = std::fmax(d01, std::fabs(o[t] - o[M * M + t]));
      d02 = std::fmax(d02, std::fabs(o[t] - o[2 * M * M + t]));
    }
  double k[3] = {0, 0, 0};
  for (int w = 0; w < W; w++)
    for (int j = 0; j < 3; j++) k[j] += K[w * 3 + j] / W;
  // (REPS updates applied in place: the reference value is the VALU one)
  std::printf("{\"what\": \"rank-4 trailing update C -= V F^T of a 24 x 24 COD step block, clocks per update, mean of %d waves\", "
              "\"valu_regs_clk\": %.1f, \"valu_lds_clk\": %.1f, \"mfma_lds_clk\": %.1f, \"max_diff_valu_lds\": %.3g, "
              "\"max_diff_mfma\": %.3g}\n", W, k[0], k[1], k[2], d01, d02);
  return 0;
}
