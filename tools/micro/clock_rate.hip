// s_memrealtime vs s_memtime rates on the device (the kernels' deadlock guard
// counts s_memrealtime ticks): one wave spins s_sleep(1) for a fixed number
// of polls and reports both counters' deltas and the first raw values.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(long long* out, int polls) {
  const long long r0 = (long long)__builtin_amdgcn_s_memrealtime();
  const long long c0 = (long long)__builtin_amdgcn_s_memtime();
  for (int i = 0; i < polls; i++) __builtin_amdgcn_s_sleep(1);
  const long long r1 = (long long)__builtin_amdgcn_s_memrealtime();
  const long long c1 = (long long)__builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = r0; out[1] = r1; out[2] = c0; out[3] = c1; }
}
int main() {
  long long* d;
  long long h[4];
  hipMalloc(&d, 4 * sizeof(long long));
  for (int polls : {64, 4096, 262144}) {
    probe<<<1, 64>>>(d, polls);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("polls %7d realtime %lld -> %lld (d %lld)  memtime d %lld  ratio %.2f\n", polls, h[0], h[1], h[1] - h[0],
           h[3] - h[2], (double)(h[3] - h[2]) / (double)(h[1] - h[0]));
  }
  return 0;
}
