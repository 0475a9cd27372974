// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the access widths the
// timestep kernels use (MI355X_MICROARCH.md: only 16 B/lane streaming is
// calibrated).  Each kernel moves a known byte count; run under
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./bytes_calib
//   rocprofv3 --pmc WRITE_SIZE --kernel-trace -- ./bytes_calib
// and divide the counter (KiB) by the printed byte counts.
//   rd8  : 8 B/lane, each wave reads 512 contiguous bytes (the per-world row
//          loads of state / snapshot / dynamics cache)
//   wr8  : 8 B/lane contiguous stores (snapshot / next-state / cache writes)
//   rd16 : 16 B/lane streaming reads (the guide's calibrated case)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void rd8(const double* __restrict__ a, double* __restrict__ out, size_t n) {
  double acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += a[i];
  if (acc == 12345.678) out[0] = acc;  // keep the loads
}
__global__ void wr8(double* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (double)i;
}
__global__ void rd16(const double2* __restrict__ a, double* __restrict__ out, size_t n2) {
  double acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
    const double2 v = a[i];
    acc += v.x + v.y;
  }
  if (acc == 12345.678) out[0] = acc;
}

int main() {
  const size_t n = 64ull << 20;  // 64 Mi doubles = 512 MiB (past the 256 MiB L3)
  double *a, *out;
  if (hipMalloc(&a, n * 8) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  hipLaunchKernelGGL(wr8, dim3(4096), dim3(256), 0, 0, a, n);
  hipLaunchKernelGGL(rd8, dim3(4096), dim3(256), 0, 0, a, out, n);
  hipLaunchKernelGGL(rd16, dim3(4096), dim3(256), 0, 0, (const double2*)a, out, n / 2);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("{\"bytes_per_kernel\": %zu, \"kernels\": [\"wr8\", \"rd8\", \"rd16\"]}\n", n * 8);
  (void)hipFree(a);
  (void)hipFree(out);
  return 0;
}
