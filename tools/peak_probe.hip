// Calibration probe: sustained v_mfma_f64_16x16x4_f64 throughput (independent accumulators,
// operands in registers, every CU) and a float4 HBM copy.  Prints one JSON line.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void mfma_loop(double* out, int iters, double seed) {
  d4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = d4{0, 0, 0, 0};
  double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 2e-3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void copy4(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int ncu = p.multiProcessorCount;
  double* out;
  const int blocks = ncu * 8, iters = 4096;
  hipMalloc(&out, (size_t)blocks * 256 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  mfma_loop<<<blocks, 256>>>(out, 64, 1.0);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0);
    mfma_loop<<<blocks, 256>>>(out, iters, 1.0 + r);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  const double flops = (double)blocks * 4 /*waves*/ * iters * 8 * 2048.0;
  const double tf = flops / (best * 1e-3) / 1e12;
  const size_t n = (size_t)1 << 28;  // 4 GiB per buffer of float4? -> 2^28 * 16 B = 4 GiB
  float4 *a, *b;
  hipMalloc(&a, n * 16);
  hipMalloc(&b, n * 16);
  hipMemset(a, 0, n * 16);
  copy4<<<ncu * 8, 256>>>(a, b, n);
  hipDeviceSynchronize();
  float bms = 1e30f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0);
    copy4<<<ncu * 8, 256>>>(a, b, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < bms) bms = ms;
  }
  const double gbs = 2.0 * n * 16 / (bms * 1e-3) / 1e9;
  printf("{\"device\": \"%s\", \"cus\": %d, \"fp64_mfma_tflops\": %.2f, \"hbm_copy_gbs\": %.1f}\n", p.name, ncu, tf, gbs);
  return 0;
}
