// Latency probe for the per-step chain on MI355X: back-to-back dependent launches on one stream.
//   empty        kernel that does nothing (launch + drain cost)
//   chaseL2 N    one wave follows a pointer chain of N loads in a 1 MiB buffer (L2-resident)
//   chaseHBM N   same in a 512 MiB buffer (HBM)
//   exch G       G workgroups publish a 2 KiB partial each (sc1 stores), count on an atomic, and
//                the last one sums all partials (the tile_kernel's split reduction)
//   fence G      same with __threadfence() publication instead of sc1 stores
// Prints one JSON object: microseconds per launch for each.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void k_empty(int* p) {
  if (p && threadIdx.x == 1000000) p[0] = 1;
}

__global__ void k_chase(const unsigned* __restrict__ next, int n, unsigned* out) {
  unsigned i = threadIdx.x;
  for (int k = 0; k < n; ++k) i = next[i];
  if (threadIdx.x == 0) out[blockIdx.x] = i;
}

__global__ void k_exch(double* part, unsigned* cnt, double* out, int G, int fence) {
  __shared__ unsigned last;
  const double v = threadIdx.x + blockIdx.x;
  if (fence) {
    part[(size_t)blockIdx.x * 256 + threadIdx.x] = v;
    __threadfence();
  } else {
    __hip_atomic_store(part + (size_t)blockIdx.x * 256 + threadIdx.x, v, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == (unsigned)G - 1;
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (fence) __threadfence();
  }
  __syncthreads();
  if (!last) return;
  double s = 0;
  for (int g = 0; g < G; ++g)
    s += fence ? part[(size_t)g * 256 + threadIdx.x]
               : __hip_atomic_load(part + (size_t)g * 256 + threadIdx.x, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
  out[threadIdx.x] = s;
}

template <class F>
double time_us(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 20; ++i) f();
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3 / reps;
}

std::vector<unsigned> chain(size_t n, unsigned seed) {
  // random cyclic permutation, 64 independent lanes start at 0..63
  std::vector<unsigned> perm(n), next(n);
  for (size_t i = 0; i < n; ++i) perm[i] = (unsigned)i;
  srand(seed);
  for (size_t i = n - 1; i > 0; --i) {
    size_t j = ((size_t)rand() * 65536u + (size_t)rand()) % (i + 1);
    std::swap(perm[i], perm[j]);
  }
  for (size_t i = 0; i < n; ++i) next[perm[i]] = perm[(i + 1) % n];
  return next;
}

int main() {
  unsigned* out;
  CK(hipMalloc(&out, 1 << 20));
  printf("{");
  printf("\"empty_us\": %.2f", time_us([&] { k_empty<<<1, 64>>>(nullptr); }, 2000));
  printf(", \"empty_256wg_us\": %.2f", time_us([&] { k_empty<<<256, 256>>>(nullptr); }, 2000));
  printf(", \"empty_1024wg_us\": %.2f", time_us([&] { k_empty<<<1024, 256>>>(nullptr); }, 2000));
  const size_t nL2 = (1 << 20) / 4, nH = (size_t)1 << 27;
  std::vector<unsigned> c1 = chain(nL2, 1);
  unsigned *dL2, *dH;
  CK(hipMalloc(&dL2, nL2 * 4));
  CK(hipMemcpy(dL2, c1.data(), nL2 * 4, hipMemcpyHostToDevice));
  std::vector<unsigned> c2 = chain(nH, 2);
  CK(hipMalloc(&dH, nH * 4));
  CK(hipMemcpy(dH, c2.data(), nH * 4, hipMemcpyHostToDevice));
  c2.clear();
  for (int n : {0, 16, 64}) {
    printf(", \"chaseL2_%d_us\": %.2f", n, time_us([&] { k_chase<<<1, 64>>>(dL2, n, out); }, 500));
    printf(", \"chaseHBM_%d_us\": %.2f", n, time_us([&] { k_chase<<<1, 64>>>(dH, n, out); }, 200));
  }
  double *part, *res;
  unsigned* cnt;
  CK(hipMalloc(&part, 1024 * 256 * 8));
  CK(hipMalloc(&res, 256 * 8));
  CK(hipMalloc(&cnt, 4));
  CK(hipMemset(cnt, 0, 4));
  for (int G : {1, 4, 16, 114, 760}) {
    printf(", \"exch_sc1_%d_us\": %.2f", G, time_us([&] { k_exch<<<G, 256>>>(part, cnt, res, G, 0); }, 1000));
    printf(", \"exch_fence_%d_us\": %.2f", G, time_us([&] { k_exch<<<G, 256>>>(part, cnt, res, G, 1); }, 1000));
  }
  printf("}\n");
  CK(hipDeviceSynchronize());
  return 0;
}
