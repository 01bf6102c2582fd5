// Does fp64 VALU FMA work run beside fp64 MFMA work on the same SIMD (separate pipes), and at what
// combined rate?  Every CU runs one 512-thread workgroup (two waves per SIMD):
//   mfma : all 8 waves issue v_mfma_f64_16x16x4_f64 (4 independent accumulators)
//   valu : all 8 waves issue v_fma_f64 (16 independent chains per lane)
//   mixed: waves 0-3 MFMA, waves 4-7 VALU (one of each per SIMD)
//   inter: every wave interleaves K v_fma_f64 after each MFMA (K = 4, 8, 12)
// Prints one JSON line per configuration: wall time, MFMA / VALU / total fp64 TFLOP/s.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e = (x);                                                   \
    if (e != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
      return 1;                                                           \
    }                                                                     \
  } while (0)

constexpr int NJ = 16;  // independent VALU chains per lane

__device__ __forceinline__ void mfma_loop(const double* in, double* out, int n) {
  const int lane = threadIdx.x & 63;
  double a = in[lane], b = in[64 + lane];
  d4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = d4{0.0, 0.0, 0.0, 0.0};
  for (int i = 0; i < n; i += 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__device__ __forceinline__ void valu_loop(const double* in, double* out, int n) {
  const int lane = threadIdx.x & 63;
  double x[NJ], acc[NJ];
  const double b = in[64 + lane];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    x[j] = in[(lane + j) & 63];
    acc[j] = 0.0;
  }
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = __builtin_fma(x[j], b, acc[j]);
    asm volatile("" : "+v"(acc[0]));  // keep the loop
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < NJ; ++j) s += acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
__global__ __launch_bounds__(512) void k_probe(const double* in, double* out, int nm, int nv) {
  const int wave = threadIdx.x >> 6;
  if (MODE == 0) mfma_loop(in, out, nm);
  else if (MODE == 1) valu_loop(in, out, nv);
  else if (wave < 4) mfma_loop(in, out, nm);
  else valu_loop(in, out, nv);
}

template <int K>
__global__ __launch_bounds__(512) void k_inter(const double* in, double* out, int nm) {
  const int lane = threadIdx.x & 63;
  double a = in[lane], b = in[64 + lane];
  d4 acc[4];
  double x[K > 0 ? K : 1], va[K > 0 ? K : 1];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int j = 0; j < K; ++j) {
    x[j] = in[(lane + j) & 63];
    va[j] = 0.0;
  }
  for (int i = 0; i < nm; i += 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < K; ++q) va[q] = __builtin_fma(x[q], b, va[q]);
    }
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
#pragma unroll
  for (int j = 0; j < K; ++j) s += va[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class F>
float timed(F launch) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 2; ++i) launch();
  hipEventRecord(e0);
  const int reps = 5;
  for (int i = 0; i < reps; ++i) launch();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return ms / reps;
}

int main() {
  int ncu = 256;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) == hipSuccess) ncu = p.multiProcessorCount;
  double *in, *out;
  CK(hipMalloc(&in, 128 * 8));
  CK(hipMalloc(&out, (size_t)ncu * 512 * 8));
  double h[128];
  for (int i = 0; i < 128; ++i) h[i] = 0.5 + 1e-3 * ((i * 37) % 101);
  CK(hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice));
  const int nm = 8192, nv = 16384;
  const double fm = (double)ncu * 8 * nm * 2048.0;      // all 8 waves MFMA
  const double fv = (double)ncu * 8 * nv * NJ * 64 * 2.0;  // all 8 waves VALU
  float t0 = timed([&] { k_probe<0><<<ncu, 512>>>(in, out, nm, nv); });
  float t1 = timed([&] { k_probe<1><<<ncu, 512>>>(in, out, nm, nv); });
  float t2 = timed([&] { k_probe<2><<<ncu, 512>>>(in, out, nm, nv); });
  CK(hipDeviceSynchronize());
  printf("{\"mode\": \"mfma\", \"ms\": %.4f, \"mfma_tflops\": %.1f}\n", t0, fm / t0 * 1e-9);
  printf("{\"mode\": \"valu\", \"ms\": %.4f, \"valu_tflops\": %.1f}\n", t1, fv / t1 * 1e-9);
  printf("{\"mode\": \"mixed\", \"ms\": %.4f, \"mfma_tflops\": %.1f, \"valu_tflops\": %.1f, \"total_tflops\": %.1f}\n", t2,
         0.5 * fm / t2 * 1e-9, 0.5 * fv / t2 * 1e-9, 0.5 * (fm + fv) / t2 * 1e-9);
  auto inter = [&](auto kfn, int K) {
    float t = timed([&] { kfn<<<ncu, 512>>>(in, out, nm); });
    const double fvk = (double)ncu * 8 * nm * K * 64 * 2.0;
    printf("{\"mode\": \"inter\", \"K\": %d, \"ms\": %.4f, \"mfma_tflops\": %.1f, \"valu_tflops\": %.1f, \"total_tflops\": %.1f}\n",
           K, t, fm / t * 1e-9, fvk / t * 1e-9, (fm + fvk) / t * 1e-9);
  };
  inter(k_inter<4>, 4);
  inter(k_inter<8>, 8);
  inter(k_inter<12>, 12);
  inter(k_inter<16>, 16);
  CK(hipDeviceSynchronize());
  return 0;
}
