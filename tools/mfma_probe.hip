// f64 MFMA issue / dependency probe on MI355X (v_mfma_f64_16x16x4_f64), for the chain's tile sizing.
// Every CU runs one workgroup of W waves (W / 4 per SIMD); each wave issues N MFMAs spread over A
// independent accumulators (A = 1: one fully dependent chain).  Per wave: shader cycles
// (s_memtime) and wall nanoseconds (s_memrealtime, 100 MHz) per MFMA, median over waves.
// Prints one JSON line per (W, A).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e = (x);                                                   \
    if (e != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
      return 1;                                                           \
    }                                                                     \
  } while (0)

template <int A>
__global__ void k_mfma(const double* in, double* out, unsigned long long* ts, int n) {
  const int lane = threadIdx.x & 63;
  double a = in[lane], b = in[64 + lane];
  d4 acc[A];
#pragma unroll
  for (int j = 0; j < A; ++j) acc[j] = d4{0.0, 0.0, 0.0, 0.0};
  __builtin_amdgcn_s_barrier();
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < n; i += A) {
#pragma unroll
    for (int j = 0; j < A; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < A; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (lane == 0) {
    const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    ts[2 * w] = c1 - c0;
    ts[2 * w + 1] = r1 - r0;
  }
}

template <int A>
int run(int W, int n, int ncu) {
  const int nw = ncu * W;
  double *in, *out;
  unsigned long long* ts;
  CK(hipMalloc(&in, 128 * 8));
  CK(hipMalloc(&out, (size_t)nw * 64 * 8));
  CK(hipMalloc(&ts, (size_t)nw * 16));
  std::vector<double> h(128);
  for (int i = 0; i < 128; ++i) h[i] = 0.5 + 1e-3 * ((i * 37) % 101);
  CK(hipMemcpy(in, h.data(), 128 * 8, hipMemcpyHostToDevice));
  for (int it = 0; it < 3; ++it) k_mfma<A><<<ncu, W * 64>>>(in, out, ts, n);
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> t(2 * (size_t)nw);
  CK(hipMemcpy(t.data(), ts, t.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> cyc(nw), ns(nw);
  for (int w = 0; w < nw; ++w) {
    cyc[w] = (double)t[2 * w] / n;
    ns[w] = (double)t[2 * w + 1] * 10.0 / n;
  }
  std::sort(cyc.begin(), cyc.end());
  std::sort(ns.begin(), ns.end());
  printf("{\"waves_per_wg\": %d, \"waves_per_simd\": %d, \"acc\": %d, \"n\": %d, \"cycles_per_mfma\": %.1f, "
         "\"ns_per_mfma\": %.2f, \"ns_max\": %.2f, \"simd_tflops\": %.1f}\n",
         W, W / 4, A, n, cyc[nw / 2], ns[nw / 2], ns[nw - 1], 2048.0 * (W / 4) / ns[nw / 2] * 1e-3 * ncu * 4);
  hipFree(in);
  hipFree(out);
  hipFree(ts);
  return 0;
}

int main() {
  int ncu = 256;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) == hipSuccess) ncu = p.multiProcessorCount;
  const int n = 4096;
  for (int W : {4, 8, 16}) {
    if (run<1>(W, n, ncu) || run<2>(W, n, ncu) || run<4>(W, n, ncu)) return 1;
  }
  return 0;
}
