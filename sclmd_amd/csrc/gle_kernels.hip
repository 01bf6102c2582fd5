// HIP kernels of the GLE stepper for gfx950 (MI355X).
//
//  contract_kernel<RN>  memory-kernel friction contraction (and every other dense product of the
//                       step) on v_mfma_f64_16x16x4_f64: A = kernel slices streamed from HBM in
//                       fragment-native order straight into registers; X = a sliding window of
//                       the velocity-history ring staged once per k-chunk in LDS and shared by the
//                       4 waves (one 16-row tile each) across all slices of the work item.
//  reduce_kernel        fixed-order sum of split-K / split-slice partial tiles (+ far field).
//  finalize_kernel      heat current / kinetic energy per step from the chain's partial table.
//  (the per-step chain of md.vv is in gle_chain.hip)
//  philox / fft_noise   coloured-noise generator (noise.py:50-100, 149-206).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>
#include <cstdio>
#include <cstdlib>

#include "gle_internal.h"
#include "gle_cgemm.h"

namespace gle {

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int64_t pmod(int64_t a, int64_t m) {
  int64_t r = a % m;
  return r < 0 ? r + m : r;
}

// explicit global-address-space load (pointers read from work-item structs are otherwise flat)
__device__ __forceinline__ double gld(const double* p) {
  return *(const __attribute__((address_space(1))) double*)p;
}


// ------------------------------------------------------------------------------------------
// contraction
//
// Per work item: for each k-stage (KC = 2 k-steps = 8 rows of X), the window of X columns that all
// slices of the current slice-chunk need is staged in LDS; while the MFMAs of stage s run, the
// next stage's X columns (CU per thread per row) and the first A fragments are already in flight
// into registers (software pipelining without a second LDS buffer).
template <int RN, int CU>
__global__ __launch_bounds__(WG, 2) void contract_kernel(const CItem* __restrict__ items,
                                                         StepArgs ta) {
  __shared__ double lds[KROWS * LDS_COLS];
  // profiling (ta.ts, launch-uniform): [0] <- first workgroup start, [1] <- last workgroup end
  if (ta.ts && threadIdx.x == 0) atomicMin(ta.ts, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  constexpr int NT = 16 * RN;
  constexpr int WWCAP = (256 * CU < LDS_WW_MAX) ? 256 * CU : LDS_WW_MAX;
  // XCD-aware order (grids are padded to a multiple of 8): blocks b, b+8, b+16, ... share an XCD
  // and its L2, so they take consecutive work items -- the row groups of one slice range, which
  // stage the same history window.
  const int nblk = gridDim.x;
  const int bid = (nblk & 7) ? (int)blockIdx.x : (int)(blockIdx.x & 7) * (nblk >> 3) + (int)(blockIdx.x >> 3);
  const CItem it = items[bid];
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int64_t t = ta.t;

  d4 acc[RN];
#pragma unroll
  for (int n = 0; n < RN; ++n) acc[n] = d4{0.0, 0.0, 0.0, 0.0};

  const int ns_max = it.ring ? (WWCAP - NT) / it.cs + 1 : 1;
  const bool active = wave < it.nrt;
  const double* Aw = it.A + (int64_t)wave * it.a_rt + lane;
  const int brow = lane >> 4;
  const int bcol = lane & 15;
  const int nst = it.nks / KC;

  for (int s0 = 0; s0 < it.ni; s0 += ns_max) {
    const int ns = min(ns_max, it.ni - s0);
    const int ww = (ns - 1) * it.cs + NT;
    const int wwp = ((ww + 31) & ~31) + 16;  // row stride = 16 mod 32 doubles: rows r, r+1 on
                                             // complementary LDS bank halves for ds_read_b64
    int64_t wbase = it.col0;
    if (it.ring) {
      const int64_t tt = it.tdiv > 1 ? t / it.tdiv : t;
      const int64_t tau = tt + it.tshift - (int64_t)(it.ia + s0 + ns - 1);
      wbase += pmod(tau, it.ring) * it.cs;
    }
    const double* xs0 = it.X + wbase;
    const double* As0 = Aw + (int64_t)s0 * 64;
    double xr[KROWS * CU];
    double na0 = 0.0, na1 = 0.0;
    // prefetch stage 0
#pragma unroll
    for (int r = 0; r < KROWS; ++r)
#pragma unroll
      for (int u = 0; u < CU; ++u) {
        const int c = tid + WG * u;
        xr[r * CU + u] = (c < ww) ? BLD(&xs0[(int64_t)r * it.ldx + c]) : 0.0;
      }
    if (active) {
      na0 = BLD(&As0[0]);
      na1 = BLD(&As0[it.a_ks]);
    }
    for (int st = 0; st < nst; ++st) {
      __syncthreads();  // previous stage's LDS reads are done
#pragma unroll
      for (int r = 0; r < KROWS; ++r)
#pragma unroll
        for (int u = 0; u < CU; ++u) {
          const int c = tid + WG * u;
          if (c < ww) lds[r * wwp + c] = xr[r * CU + u];
        }
      __syncthreads();
      double a0 = na0, a1 = na1;
      const double* Ak = As0 + (int64_t)(st * KC) * it.a_ks;
      if (st + 1 < nst) {  // next stage in flight during this stage's MFMAs
        const double* xs = xs0 + (int64_t)(4 * KC * (st + 1)) * it.ldx;
#pragma unroll
        for (int r = 0; r < KROWS; ++r)
#pragma unroll
          for (int u = 0; u < CU; ++u) {
            const int c = tid + WG * u;
            xr[r * CU + u] = (c < ww) ? BLD(&xs[(int64_t)r * it.ldx + c]) : 0.0;
          }
        if (active) {
          na0 = BLD(&Ak[KC * it.a_ks]);
          na1 = BLD(&Ak[(KC + 1) * it.a_ks]);
        }
      }
      if (active) {
        // A fragments run two slices ahead of the MFMAs that consume them
        double m0 = 0.0, m1 = 0.0;
        if (ns > 1) {
          m0 = BLD(&Ak[64]);
          m1 = BLD(&Ak[it.a_ks + 64]);
        }
        for (int ss = 0; ss < ns; ++ss) {
          double n0 = 0.0, n1 = 0.0;
          if (ss + 2 < ns) {
            n0 = BLD(&Ak[(ss + 2) * 64]);
            n1 = BLD(&Ak[it.a_ks + (ss + 2) * 64]);
          }
          const int off = (ns - 1 - ss) * it.cs;
          const double* b0 = lds + brow * wwp + off + bcol;
          const double* b1 = b0 + 4 * wwp;
#pragma unroll
          for (int n = 0; n < RN; ++n)
            acc[n] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0[16 * n], acc[n], 0, 0, 0);
#pragma unroll
          for (int n = 0; n < RN; ++n)
            acc[n] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1[16 * n], acc[n], 0, 0, 0);
          a0 = m0;
          a1 = m1;
          m0 = n0;
          m1 = n1;
        }
      }
    }
  }
  if (active) {
    // f64 MFMA C/D map: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
    for (int n = 0; n < RN; ++n) {
      const int col = 16 * n + bcol;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wave * 16 + brow + 4 * r;
        if (row < it.nrows && col < it.ncols) {
          GLE_BCHK(&it.out[(int64_t)row * it.ldo + col]);
          it.out[(int64_t)row * it.ldo + col] = acc[n][r];
        }
      }
    }
  }
  if (ta.ts) {
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(ta.ts + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
}

void bounds_publish_kernels(const BoundsTab& t) {
#ifdef GLE_BOUNDS
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_btab), &t, sizeof(t));
#else
  (void)t;
#endif
}

template <int RN>
static void launch_rn(int cu, const CItem* items, int nitems, StepArgs ta, hipStream_t s) {
  dim3 g(nitems), b(WG);
  switch (cu) {
    case 1: contract_kernel<RN, 1><<<g, b, 0, s>>>(items, ta); break;
    case 2: contract_kernel<RN, 2><<<g, b, 0, s>>>(items, ta); break;
    case 3: contract_kernel<RN, 3><<<g, b, 0, s>>>(items, ta); break;
    default: contract_kernel<RN, 4><<<g, b, 0, s>>>(items, ta); break;
  }
}

void launch_contract(int rn, int cu, const CItem* items, int nitems, StepArgs ta, hipStream_t s) {
  if (nitems <= 0) return;
  GLE_BOUNDS_SYNC();
  switch (rn) {
    case 1: launch_rn<1>(cu, items, nitems, ta, s); break;
    case 2: launch_rn<2>(cu, items, nitems, ta, s); break;
    case 4: launch_rn<4>(cu, items, nitems, ta, s); break;
    case 8: launch_rn<8>(cu, items, nitems, ta, s); break;
    default: launch_rn<16>(cu, items, nitems, ta, s); break;
  }
}

// ------------------------------------------------------------------------------------------
// grid (item, chunk): each block sums RED_PER_BLOCK consecutive elements of one tile over all of
// its partial slots in slot order (deterministic).
constexpr int RED_PER_BLOCK = 256;

// s + p[0] + p[st] + ... + p[(n-1)*st], added in slot order; loads issued 8 at a time so their
// latencies overlap (same rounding as the plain loop).
__device__ __forceinline__ double sum_slots(double s, const double* p, int64_t st, int n) {
  int q = 0;
  for (; q + 8 <= n; q += 8) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(q + u) * st];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; q < n; ++q) s += p[q * st];
  return s;
}

__device__ __forceinline__ double max_slots(const double* p, int64_t st, int n, bool& nan) {
  double m = 0.0;
  int q = 0;
  for (; q + 8 <= n; q += 8) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(q + u) * st];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      nan |= (v[u] != v[u]);
      m = fmax(m, v[u]);
    }
  }
  for (; q < n; ++q) {
    const double v = p[q * st];
    nan |= (v != v);
    m = fmax(m, v);
  }
  return m;
}
__global__ __launch_bounds__(256) void reduce_kernel(const RItem* __restrict__ items,
                                                     StepArgs ta) {
  const RItem it = items[blockIdx.x];
  const int n = it.rows * it.cols;
  const int e0 = blockIdx.y * RED_PER_BLOCK;
  (void)ta;
  if (e0 >= n) return;
  for (int e = e0 + threadIdx.x; e < min(n, e0 + RED_PER_BLOCK); e += blockDim.x) {
    const int r = e / it.cols;
    const int c = e - r * it.cols;
    it.dst[(int64_t)r * it.ldd + c] = sum_slots(0.0, it.src + (int64_t)r * it.lds + c, it.slot_stride, it.nslots);
  }
}

void launch_reduce(const RItem* items, int nitems, int max_elems, StepArgs ta,
                   hipStream_t s) {
  if (nitems <= 0) return;
  dim3 g(nitems, (max_elems + RED_PER_BLOCK - 1) / RED_PER_BLOCK);
  reduce_kernel<<<g, 256, 0, s>>>(items, ta);
}

// bath.cur[t] and md.etot[t] (md.py:383, 397) for every step of the run from phase A's per-step
// partial sums, added in fixed DOF-chunk order (deterministic); launched when outputs are read.
__global__ void finalize_kernel(const StepDev* __restrict__ sd) {
  const int B = sd->B, nb = sd->nbath, nmd = sd->nmd, nd = sd->ndblk;
  const int64_t total = (int64_t)nmd * (nb + 1) * B;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(e % B);
    const int qd = (int)((e / B) % (nb + 1));
    const int tn = (int)(e / ((int64_t)B * (nb + 1)));
    const double s = sum_slots(0.0, sd->part + ((int64_t)tn * nd * (nb + 1) + qd) * B + b,
                               (int64_t)(nb + 1) * B, nd);
    if (qd < nb) sd->bath[qd].cur[(int64_t)tn * B + b] = s;
    else sd->etot[(int64_t)tn * B + b] = 0.5 * s;  // md.py:161-165, 383
  }
}

void launch_finalize(const StepDev* sd, int B, int nmd, int nbath, hipStream_t s) {
  const int64_t total = (int64_t)nmd * (nbath + 1) * B;
  const int64_t blocks = std::min<int64_t>((total + 255) / 256, 4096);
  finalize_kernel<<<(unsigned)blocks, 256, 0, s>>>(sd);
}

// ------------------------------------------------------------------------------------------
// Philox4x32-10 counter-based normals: one N(0,1) per (trajectory, frequency, DOF), independent of
// the launch geometry.
__device__ __forceinline__ void philox_round(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
  const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  const uint32_t n0 = hi1 ^ c[1] ^ k0;
  const uint32_t n2 = hi0 ^ c[3] ^ k1;
  c[0] = n0;
  c[1] = lo1;
  c[2] = n2;
  c[3] = lo0;
}

__device__ __forceinline__ double philox_normal(uint64_t seed, uint32_t a, uint32_t b, uint32_t c) {
  uint32_t ctr[4] = {a, b, c, 0x6a09e667u};
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(ctr, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  const uint64_t u0 = ((uint64_t)ctr[0] << 21) ^ (uint64_t)ctr[1];
  const uint64_t u1 = ((uint64_t)ctr[2] << 21) ^ (uint64_t)ctr[3];
  const double x1 = ((double)(u0 & ((1ull << 53) - 1)) + 1.0) * (1.0 / 9007199254740992.0);  // (0,1]
  const double x2 = (double)(u1 & ((1ull << 53) - 1)) * (1.0 / 9007199254740992.0);        // [0,1)
  return sqrt(-2.0 * log(x1)) * cospi(2.0 * x2);
}

__global__ void philox_kernel(double* x, int64_t nfreq, int64_t ncp, int64_t nc, int64_t B,
                              uint64_t seed, uint64_t traj_offset, int64_t w_off) {
  const int64_t n = nfreq * ncp * B;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e % B;
    const int64_t k = (e / B) % ncp;
    const int64_t w = e / (B * ncp) + w_off;
    x[e] = (k < nc) ? philox_normal(seed, (uint32_t)k, (uint32_t)w, (uint32_t)(traj_offset + b)) : 0.0;
  }
}

void launch_philox_normal(double* x, int64_t nfreq, int64_t ncp, int64_t nc, int64_t B,
                          uint64_t seed, uint64_t traj_offset, hipStream_t s, int64_t w_off) {
  philox_kernel<<<2048, 256, 0, s>>>(x, nfreq, ncp, nc, B, seed, traj_offset, w_off);
}

// Streamed noise generation (C5-size baths, whose per-frequency factors do not fit next to the
// spectral kernels): for the frequencies of one chunk, a[w0 + w][row_off + r][b] =
//   sum_k M[w][r][k] x[w][k][b]  with M row-major [nw][nc][kc] (a real factor, or the real or the
// imaginary part of a complex one) and x the chunk's N(0,1) draws [nw][ncp][B].  Setup work
// (once per run), LDS-tiled fp64 FMA: 64 rows x 32 columns per block, k in steps of 32.
constexpr int NG_R = 64, NG_C = 32, NG_K = 32;
// mstride: doubles between the frequencies' factors (0: one shared factor for every frequency of the
// launch); wscale (nullable): a per-frequency scale of the product (a shared factor times sqrt(s_w))
__global__ __launch_bounds__(256) void noise_gemm_kernel(const double* __restrict__ M, int nc, int kc,
                                                         const double* __restrict__ x, int ncp, int B,
                                                         double* __restrict__ a, int rows, int row_off,
                                                         int64_t w0, int64_t mstride,
                                                         const double* __restrict__ wscale) {
  __shared__ double Ms[NG_R][NG_K + 1];
  __shared__ double Xs[NG_K][NG_C + 1];
  const int w = blockIdx.z;
  const int r0 = blockIdx.x * NG_R, c0 = blockIdx.y * NG_C;
  const int tid = threadIdx.x;
  const int ty = tid / 8, tx = tid % 8;  // rows 2 ty, 2 ty + 1; columns 4 tx .. 4 tx + 3
  const double* Mw = M + (int64_t)w * mstride;
  const double* xw = x + (int64_t)w * ncp * B;
  double acc[2][4] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
  for (int k0 = 0; k0 < kc; k0 += NG_K) {
    for (int e = tid; e < NG_R * NG_K; e += 256) {
      const int r = e / NG_K, k = e % NG_K;
      Ms[r][k] = (r0 + r < nc && k0 + k < kc) ? Mw[(int64_t)(r0 + r) * kc + k0 + k] : 0.0;
    }
    for (int e = tid; e < NG_K * NG_C; e += 256) {
      const int k = e / NG_C, c = e % NG_C;
      Xs[k][c] = (k0 + k < kc && c0 + c < B) ? xw[(int64_t)(k0 + k) * B + c0 + c] : 0.0;
    }
    __syncthreads();
#pragma unroll 8
    for (int k = 0; k < NG_K; ++k) {
      const double m0 = Ms[2 * ty][k], m1 = Ms[2 * ty + 1][k];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double xv = Xs[k][4 * tx + j];
        acc[0][j] += m0 * xv;
        acc[1][j] += m1 * xv;
      }
    }
    __syncthreads();
  }
  const double sc = wscale ? wscale[w] : 1.0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = r0 + 2 * ty + i, c = c0 + 4 * tx + j;
      if (r < nc && c < B) a[((w0 + w) * rows + row_off + r) * (int64_t)B + c] = sc * acc[i][j];
    }
}

void launch_noise_gemm(const double* M, int nc, int kc, const double* x, int ncp, int B, double* a, int rows,
                       int row_off, int64_t w0, int nw, hipStream_t s, int64_t mstride, const double* wscale) {
  if (nw <= 0) return;
  const dim3 grid((unsigned)((nc + NG_R - 1) / NG_R), (unsigned)((B + NG_C - 1) / NG_C), (unsigned)nw);
  noise_gemm_kernel<<<grid, 256, 0, s>>>(M, nc, kc, x, ncp, B, a, rows, row_off, w0,
                                         mstride < 0 ? (int64_t)nc * kc : mstride, wscale);
}

// ------------------------------------------------------------------------------------------
// Mirror + FFT of the positive-frequency amplitudes into the time-domain noise, two real series
// per complex transform.  Series s = k*B + b; input a[w][row][b] (rows [0,nc) real part,
// [nc,2nc) imaginary part when complex); output noise[t][k][b].
// The spectrum of noise.py:87-94 has Hermitian part h: h[0] = Re a0, h[N/2] = Re a_{N/2},
// h[w] = a_w, h[N-w] = conj(a_w); real(fft(s)) = fft(h) (real), so fft(h1 + i h2) = x1 + i x2.
__global__ __launch_bounds__(256) void fft_noise_kernel(const double* __restrict__ a,
                                                        double* __restrict__ noise,
                                                        const double2* __restrict__ tw, int logn,
                                                        int nc, int arows, int B, int is_complex,
                                                        double scale, int nseries) {
  extern __shared__ double2 buf[];
  const int N = 1 << logn, h = N >> 1;
  const int s1 = 2 * blockIdx.x, s2 = s1 + 1;
  const bool has2 = s2 < nseries;
  const int k1 = s1 / B, b1 = s1 % B;
  const int k2 = has2 ? s2 / B : 0, b2 = has2 ? s2 % B : 0;
  for (int w = threadIdx.x; w < N; w += blockDim.x) {
    const bool cj = w > h;
    const int src = cj ? N - w : w;
    const bool realonly = (w == 0) || (w == h);
    double r1 = a[((int64_t)src * arows + k1) * B + b1];
    double i1 = (is_complex && !realonly) ? a[((int64_t)src * arows + nc + k1) * B + b1] : 0.0;
    double r2 = 0.0, i2 = 0.0;
    if (has2) {
      r2 = a[((int64_t)src * arows + k2) * B + b2];
      i2 = (is_complex && !realonly) ? a[((int64_t)src * arows + nc + k2) * B + b2] : 0.0;
    }
    if (cj) {
      i1 = -i1;
      i2 = -i2;
    }
    const unsigned rev = __brev((unsigned)w) >> (32 - logn);
    buf[rev] = make_double2(r1 - i2, i1 + r2);
  }
  __syncthreads();
  for (int s = 1; s <= logn; ++s) {
    const int half = 1 << (s - 1);
    const int tstride = N >> s;
    for (int j = threadIdx.x; j < h; j += blockDim.x) {
      const int g = j >> (s - 1);
      const int jj = j & (half - 1);
      const int i0 = (g << s) + jj;
      const int i1 = i0 + half;
      const double2 w = tw[jj * tstride];
      const double2 x0 = buf[i0];
      const double2 x1 = buf[i1];
      const double2 y = make_double2(x1.x * w.x - x1.y * w.y, x1.x * w.y + x1.y * w.x);
      buf[i0] = make_double2(x0.x + y.x, x0.y + y.y);
      buf[i1] = make_double2(x0.x - y.x, x0.y - y.y);
    }
    __syncthreads();
  }
  for (int t = threadIdx.x; t < N; t += blockDim.x) {
    const double2 v = buf[t];
    noise[((int64_t)t * nc + k1) * B + b1] = v.x * scale;
    if (has2) noise[((int64_t)t * nc + k2) * B + b2] = v.y * scale;
  }
}

// ------------------------------------------------------------------------------------------
// Transforms of any length (nmd not a power of two <= 8192: numpy's FFT takes any length, and the
// reference's noise needs only an even nmd, functions.py:47-50; examples/current-induced/rundp.py
// runs nmd = 2 10^5).  Batched complex forward DFT X[k] = sum_n x[n] e^{-2 pi i n k / N} of S
// series (series c at c ld): Stockham autosort passes of radix 8, 4, 2, 3, 5, 7 in global memory --
// the pass of radix R after sub-transforms of length p: thread i < N / R reads x[i + q N / R],
// multiplies by e^{-2 pi i q (i mod p) / (p R)} and writes its R-point DFT to
// (i - i mod p) R + i mod p + m p -- and any other prime factor through Bluestein's chirp-z with a
// power-of-two transform of length M >= 2N - 1 (n k = (n^2 + k^2 - (k - n)^2) / 2).  Setup work,
// once per noise realisation or power spectrum.
namespace {
__device__ __forceinline__ double2 zmul(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

template <int R>
__global__ __launch_bounds__(256) void gfft_pass_kernel(const double2* __restrict__ in, double2* __restrict__ out,
                                                        int64_t N, int64_t ld, int64_t p, int64_t total) {
  const int64_t T = N / R, pr = p * R;
  double2 wr[R];
#pragma unroll
  for (int e = 0; e < R; ++e) {
    double sn, cs;
    sincospi(-2.0 * (double)e / (double)R, &sn, &cs);
    wr[e] = make_double2(cs, sn);
  }
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = g / T, i = g - c * T;
    const double2* x = in + c * ld;
    double2* y = out + c * ld;
    const int64_t k = i % p;
    double2 v[R];
#pragma unroll
    for (int q = 0; q < R; ++q) v[q] = x[i + q * T];
#pragma unroll
    for (int q = 1; q < R; ++q) {
      double sn, cs;
      sincospi(-2.0 * (double)((q * k) % pr) / (double)pr, &sn, &cs);
      v[q] = zmul(v[q], make_double2(cs, sn));
    }
    const int64_t j = (i - k) * R + k;
#pragma unroll
    for (int m = 0; m < R; ++m) {
      double2 acc = v[0];
#pragma unroll
      for (int q = 1; q < R; ++q) {
        const double2 t = zmul(v[q], wr[(q * m) % R]);
        acc.x += t.x;
        acc.y += t.y;
      }
      y[j + m * p] = acc;
    }
  }
}

// chirp w_n = e^{-i pi (n^2 mod 2N) / N}
__device__ __forceinline__ double2 chirp(int64_t n, int64_t N) {
  double sn, cs;
  sincospi(-(double)((n * n) % (2 * N)) / (double)N, &sn, &cs);
  return make_double2(cs, sn);
}

// x[c][n] *= w_n (n < N), 0 for N <= n < M
__global__ void gblue_pre_kernel(double2* x, int64_t N, int64_t M, int64_t S) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < S * M; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = g % M;
    x[g] = n < N ? zmul(x[g], chirp(n, N)) : make_double2(0.0, 0.0);
  }
}

// b[m] = conj(w_m) for m < N, conj(w_{M - m}) for m > M - N, else 0 (the circular kernel)
__global__ void gblue_chirp_kernel(double2* b, int64_t N, int64_t M) {
  for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < M; m += (int64_t)gridDim.x * blockDim.x) {
    double2 v = make_double2(0.0, 0.0);
    if (m < N) v = chirp(m, N);
    else if (m > M - N) v = chirp(M - m, N);
    b[m] = make_double2(v.x, -v.y);
  }
}

// a = conj(a bh): the inverse transform of a bh as a forward one of its conjugate
__global__ void gblue_mid_kernel(double2* a, const double2* __restrict__ bh, int64_t M, int64_t S) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < S * M; g += (int64_t)gridDim.x * blockDim.x) {
    const double2 v = zmul(a[g], bh[g % M]);
    a[g] = make_double2(v.x, -v.y);
  }
}

// X[c][k] = conj(c[k]) w_k / M, k < N
__global__ void gblue_post_kernel(double2* x, int64_t N, int64_t M, int64_t S) {
  const double inv = 1.0 / (double)M;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < S * N; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = g / N, k = g - c * N;
    const double2 v = x[c * M + k];
    const double2 r = zmul(make_double2(v.x, -v.y), chirp(k, N));
    x[c * M + k] = make_double2(r.x * inv, r.y * inv);
  }
}

unsigned grid_of(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 1 << 16)); }

struct Gfft {
  int64_t N = 0, M = 0;  // M > 0: Bluestein with transforms of length M
  std::vector<int> rad, radM;
  double2* bh = nullptr;  // transform of the circular chirp kernel (Bluestein)
  int64_t ld() const { return M ? M : N; }
};

std::vector<int> gfft_radices(int64_t N, int64_t* rest) {
  std::vector<int> r;
  for (int q : {8, 4, 2, 3, 5, 7})
    while (N % q == 0) {
      r.push_back(q);
      N /= q;
    }
  *rest = N;
  return r;
}

// S series of length N at stride ld, x -> (x or y): the buffer holding the result
double2* gfft_mixed(double2* x, double2* y, int64_t S, int64_t N, int64_t ld, const std::vector<int>& rad,
                    hipStream_t s) {
  int64_t p = 1;
  const unsigned grid = grid_of(S * N);
  for (int r : rad) {
    const int64_t total = S * (N / r);
    switch (r) {
      case 8: gfft_pass_kernel<8><<<grid, 256, 0, s>>>(x, y, N, ld, p, total); break;
      case 4: gfft_pass_kernel<4><<<grid, 256, 0, s>>>(x, y, N, ld, p, total); break;
      case 2: gfft_pass_kernel<2><<<grid, 256, 0, s>>>(x, y, N, ld, p, total); break;
      case 3: gfft_pass_kernel<3><<<grid, 256, 0, s>>>(x, y, N, ld, p, total); break;
      case 5: gfft_pass_kernel<5><<<grid, 256, 0, s>>>(x, y, N, ld, p, total); break;
      default: gfft_pass_kernel<7><<<grid, 256, 0, s>>>(x, y, N, ld, p, total); break;
    }
    std::swap(x, y);
    p *= r;
  }
  return x;
}

int gfft_plan(Gfft& g, int64_t N, hipStream_t s) {
  g.N = N;
  int64_t rest = 1;
  g.rad = gfft_radices(N, &rest);
  if (rest == 1) return 0;
  g.M = 1;
  while (g.M < 2 * N - 1) g.M *= 2;
  g.radM = gfft_radices(g.M, &rest);
  double2* tmp = nullptr;
  if (hipMalloc((void**)&g.bh, (size_t)g.M * 2 * sizeof(double2)) != hipSuccess) return -4;
  tmp = g.bh + g.M;
  gblue_chirp_kernel<<<grid_of(g.M), 256, 0, s>>>(g.bh, N, g.M);
  double2* r = gfft_mixed(g.bh, tmp, 1, g.M, g.M, g.radM, s);
  if (r != g.bh) hipMemcpyAsync(g.bh, r, (size_t)g.M * sizeof(double2), hipMemcpyDeviceToDevice, s);
  return 0;
}

// work buffers are plain allocations released after the stream drains (setup paths; stream-ordered
// pool allocations interleaved with the library's other allocations gave wrong noise on some runs)
void gfft_release(Gfft& g, hipStream_t s) {
  if (g.bh) {
    hipStreamSynchronize(s);
    hipFree(g.bh);
  }
  g.bh = nullptr;
}

// forward DFT of the S series in x (stride g.ld(), first N entries); y: scratch of the same size
double2* gfft_exec(const Gfft& g, double2* x, double2* y, int64_t S, hipStream_t s) {
  if (!g.M) return gfft_mixed(x, y, S, g.N, g.N, g.rad, s);
  gblue_pre_kernel<<<grid_of(S * g.M), 256, 0, s>>>(x, g.N, g.M, S);
  double2* a = gfft_mixed(x, y, S, g.M, g.M, g.radM, s);
  gblue_mid_kernel<<<grid_of(S * g.M), 256, 0, s>>>(a, g.bh, g.M, S);
  double2* c = gfft_mixed(a, a == x ? y : x, S, g.M, g.M, g.radM, s);
  gblue_post_kernel<<<grid_of(S * g.N), 256, 0, s>>>(c, g.N, g.M, S);
  return c;
}

// series per pass of a generic transform within a work-buffer budget (two buffers of S ld complex)
int64_t gfft_chunk(const Gfft& g, int64_t nseries) {
  const int64_t budget = (int64_t)1 << 30;
  return std::max<int64_t>(1, std::min<int64_t>(nseries, budget / (2 * g.ld() * (int64_t)sizeof(double2))));
}

// the Hermitian spectra of series pairs (as fft_noise_kernel builds them) for pairs [c0, c0 + S)
__global__ void gnoise_pack_kernel(const double* __restrict__ a, double2* __restrict__ z, int64_t N, int64_t ld,
                                   int nc, int arows, int B, int is_complex, int64_t c0, int64_t S, int64_t nseries) {
  const int64_t h = N / 2;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < S * N; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = g / N, w = g - c * N;
    const int64_t s1 = 2 * (c0 + c), s2 = s1 + 1;
    const bool has2 = s2 < nseries;
    const int64_t k1 = s1 / B, b1 = s1 % B, k2 = has2 ? s2 / B : 0, b2 = has2 ? s2 % B : 0;
    const bool cj = w > h;
    const int64_t src = cj ? N - w : w;
    const bool realonly = (w == 0) || (w == h);
    double r1 = a[(src * arows + k1) * B + b1];
    double i1 = (is_complex && !realonly) ? a[(src * arows + nc + k1) * B + b1] : 0.0;
    double r2 = 0.0, i2 = 0.0;
    if (has2) {
      r2 = a[(src * arows + k2) * B + b2];
      i2 = (is_complex && !realonly) ? a[(src * arows + nc + k2) * B + b2] : 0.0;
    }
    if (cj) {
      i1 = -i1;
      i2 = -i2;
    }
    z[c * ld + w] = make_double2(r1 - i2, i1 + r2);
  }
}

__global__ void gnoise_unpack_kernel(const double2* __restrict__ z, double* __restrict__ noise, int64_t N, int64_t ld,
                                     int nc, int B, double scale, int64_t c0, int64_t S, int64_t nseries) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < S * N; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = g / N, t = g - c * N;
    const int64_t s1 = 2 * (c0 + c), s2 = s1 + 1;
    const double2 v = z[c * ld + t];
    noise[(t * nc + s1 / B) * B + s1 % B] = v.x * scale;
    if (s2 < nseries) noise[(t * nc + s2 / B) * B + s2 % B] = v.y * scale;
  }
}

int launch_fft_noise_generic(const double* a, double* noise, int64_t nmd, int64_t nc, int64_t arows, int64_t B,
                             int is_complex, double scale, hipStream_t s) {
  Gfft g;
  if (gfft_plan(g, nmd, s)) return -4;
  const int64_t nseries = nc * B, npair = (nseries + 1) / 2;
  const int64_t S = gfft_chunk(g, npair);
  double2* buf = nullptr;
  if (hipMalloc((void**)&buf, (size_t)2 * S * g.ld() * sizeof(double2)) != hipSuccess) {
    gfft_release(g, s);
    return -4;
  }
  for (int64_t c0 = 0; c0 < npair; c0 += S) {
    const int64_t n = std::min(S, npair - c0);
    gnoise_pack_kernel<<<grid_of(n * nmd), 256, 0, s>>>(a, buf, nmd, g.ld(), (int)nc, (int)arows, (int)B, is_complex,
                                                         c0, n, nseries);
    const double2* r = gfft_exec(g, buf, buf + S * g.ld(), n, s);
    gnoise_unpack_kernel<<<grid_of(n * nmd), 256, 0, s>>>(r, noise, nmd, g.ld(), (int)nc, (int)B, scale, c0, n,
                                                           nseries);
  }
  const hipError_t e = hipStreamSynchronize(s);
  hipFree(buf);
  gfft_release(g, s);
  if (e != hipSuccess) return -5;
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
}  // namespace

int launch_fft_noise(const double* a, double* noise, const double* tw, int64_t nmd, int64_t nc,
                     int64_t arows, int64_t B, int is_complex, double scale, hipStream_t s) {
  int logn = 0;
  while ((1ll << logn) < nmd) ++logn;
  if ((1ll << logn) != nmd || nmd > 8192)  // any other even length: the global-memory transforms
    return nmd >= 2 && nmd % 2 == 0 ? launch_fft_noise_generic(a, noise, nmd, nc, arows, B, is_complex, scale, s) : -1;
  if (logn < 1) return -1;
  const size_t shmem = (size_t)nmd * sizeof(double2);
  if (shmem > 160 * 1024) return -2;
  if (hipFuncSetAttribute((const void*)fft_noise_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)shmem) != hipSuccess)
    return -3;
  const int64_t nseries = nc * B;
  const int64_t nblk = (nseries + 1) / 2;
  fft_noise_kernel<<<(unsigned)nblk, 256, shmem, s>>>(a, noise, (const double2*)tw, logn, (int)nc,
                                                      (int)arows, (int)B, is_complex, scale,
                                                      (int)nseries);
  return 0;
}

// Velocity power spectrum of recorded series (functions.powerspecp, functions.py:221-236): per DOF
// group g and trajectory b, out[g][b][f] = sum_{k in group} |DFT_t(ps[t][k][b])(f)|^2 (the
// reference's |Fourier1D|^2 = dt^2 |DFT|^2 over dt nmd is applied by the caller).  One block per
// (g, b): the group's DOFs go two at a time through one complex radix-2 FFT in LDS (Z = x1 + i x2,
// |X1(f)|^2 + |X2(f)|^2 = (|Z(f)|^2 + |Z(N-f)|^2) / 2), accumulated per thread in registers over
// the frequencies it owns, in fixed DOF order (deterministic).
template <int NS>
__device__ __forceinline__ void lds_fft(double2* buf, int logn, const double2* tw, double sign);

template <int FPT>
__global__ __launch_bounds__(256) void power_kernel(const double* __restrict__ ps, int64_t nph, int B, int logn,
                                                    const int64_t* __restrict__ goff, const int64_t* __restrict__ dofs,
                                                    const double2* __restrict__ tw_g, int tw_lds,
                                                    double* __restrict__ out) {
  extern __shared__ double2 pbuf[];  // N points (+ N/2 twiddles when tw_lds)
  const int N = 1 << logn;
  const int g = blockIdx.x / B, b = blockIdx.x % B;
  const double2* tw = tw_g;
  if (tw_lds) {
    for (int j = threadIdx.x; j < N / 2; j += blockDim.x) pbuf[N + j] = tw_g[j];
    tw = pbuf + N;
  }
  double acc[FPT];
#pragma unroll
  for (int j = 0; j < FPT; ++j) acc[j] = 0.0;
  const int64_t k0 = goff[g], k1 = goff[g + 1];
  const int64_t rowst = nph * B;
  for (int64_t kk = k0; kk < k1; kk += 2) {
    const int64_t d1 = dofs[kk];
    const bool two = kk + 1 < k1;
    const int64_t d2 = two ? dofs[kk + 1] : d1;
    __syncthreads();  // previous pair's reads of pbuf are done
    for (int t = threadIdx.x; t < N; t += blockDim.x) {
      const double x1 = ps[(int64_t)t * rowst + d1 * B + b];
      const double x2 = two ? ps[(int64_t)t * rowst + d2 * B + b] : 0.0;
      const unsigned rev = __brev((unsigned)t) >> (32 - logn);
      pbuf[rev] = make_double2(x1, x2);
    }
    __syncthreads();
    // (d_tw holds e^{-2 pi i j/N}: with sign -1 this is the inverse-direction transform, whose
    // |.|^2 pair sums equal the forward ones for real series)
    lds_fft<1>(pbuf, logn, tw, -1.0);  // ends with a barrier
#pragma unroll
    for (int j = 0; j < FPT; ++j) {
      const int f = threadIdx.x + 256 * j;
      if (f < N) {
        const double2 z = pbuf[f], zc = pbuf[(N - f) & (N - 1)];
        acc[j] += 0.5 * (z.x * z.x + z.y * z.y + zc.x * zc.x + zc.y * zc.y);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < FPT; ++j) {
    const int f = threadIdx.x + 256 * j;
    if (f < N) out[((int64_t)g * B + b) * N + f] = acc[j];
  }
}

// Power spectra of any length nmd (not a power of two <= 8192): each (DOF entry, trajectory) series
// through the generic transform (gfft_exec) as a complex series with zero imaginary part, then
// out[g][b][f] += |X(f)|^2 over the chunk's entries in entry order (one thread per (b, f):
// deterministic).
__global__ void gpower_pack_kernel(const double* __restrict__ ps, double2* __restrict__ z, int64_t N, int64_t ld,
                                   int64_t nph, int B, const int64_t* __restrict__ dofs, int64_t c0, int64_t S) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < S * N; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = g / N, t = g - c * N;
    const int64_t e = (c0 + c) / B, b = (c0 + c) % B;
    z[c * ld + t] = make_double2(ps[(t * nph + dofs[e]) * B + b], 0.0);
  }
}

__global__ void gpower_acc_kernel(const double2* __restrict__ z, double* __restrict__ out, int64_t N, int64_t ld, int B,
                                  const int64_t* __restrict__ goff, int ngroup, int64_t c0, int64_t S) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < (int64_t)B * N; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = g / N, f = g - b * N;
    int grp = 0;
    for (int64_t c = (b - c0 % B + B) % B; c < S; c += B) {  // the chunk's series of trajectory b
      const int64_t e = (c0 + c) / B;
      while (grp + 1 < ngroup && goff[grp + 1] <= e) ++grp;
      const double2 v = z[c * ld + f];
      out[((int64_t)grp * B + b) * N + f] += v.x * v.x + v.y * v.y;
    }
  }
}

int launch_power_generic(const double* ps, int64_t nph, int B, int64_t nmd, int ngroup, const int64_t* goff,
                         const int64_t* dofs, int64_t nentry, double* out, hipStream_t s) {
  if (hipMemsetAsync(out, 0, (size_t)ngroup * B * nmd * sizeof(double), s) != hipSuccess) return -4;
  const int64_t nseries = nentry * B;
  if (nseries == 0) return 0;
  Gfft g;
  if (gfft_plan(g, nmd, s)) return -4;
  // whole trajectories' worth of series per chunk, so that a chunk's entries stay in order per (b, f)
  const int64_t S = gfft_chunk(g, nseries);
  double2* buf = nullptr;
  if (hipMalloc((void**)&buf, (size_t)2 * S * g.ld() * sizeof(double2)) != hipSuccess) {
    gfft_release(g, s);
    return -4;
  }
  for (int64_t c0 = 0; c0 < nseries; c0 += S) {
    const int64_t n = std::min(S, nseries - c0);
    gpower_pack_kernel<<<grid_of(n * nmd), 256, 0, s>>>(ps, buf, nmd, g.ld(), nph, B, dofs, c0, n);
    const double2* r = gfft_exec(g, buf, buf + S * g.ld(), n, s);
    gpower_acc_kernel<<<grid_of((int64_t)B * nmd), 256, 0, s>>>(r, out, nmd, g.ld(), B, goff, ngroup, c0, n);
  }
  const hipError_t e = hipStreamSynchronize(s);
  hipFree(buf);
  gfft_release(g, s);
  if (e != hipSuccess) return -5;
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_power(const double* ps, int64_t nph, int B, int64_t nmd, int ngroup, const int64_t* goff,
                 const int64_t* dofs, const double* tw, double* out, hipStream_t s, int64_t nentry) {
  int logn = 0;
  while ((1ll << logn) < nmd) ++logn;
  if (nmd < 2) return -1;
  if ((1ll << logn) != nmd || nmd > 8192)
    return launch_power_generic(ps, nph, B, nmd, ngroup, goff, dofs, nentry, out, s);
  const int tw_lds = nmd <= 4096 ? 1 : 0;
  const size_t shm = (size_t)nmd * sizeof(double2) + (tw_lds ? (size_t)nmd / 2 * sizeof(double2) : 0);
  const dim3 grid((unsigned)(ngroup * B));
  if (nmd <= 1024) {
    if (hipFuncSetAttribute((const void*)power_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess) return -3;
    power_kernel<4><<<grid, 256, shm, s>>>(ps, nph, B, logn, goff, dofs, (const double2*)tw, tw_lds, out);
  } else {
    if (hipFuncSetAttribute((const void*)power_kernel<32>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess) return -3;
    power_kernel<32><<<grid, 256, shm, s>>>(ps, nph, B, logn, goff, dofs, (const double2*)tw, tw_lds, out);
  }
  return 0;
}

}  // namespace gle

namespace gle {

// Copy nt time slots between a bath history ring and a dense buffer buf[i][k][b] (i = 0 is time
// tau0, i = 1 is tau0-1, ...).  dir 0: buf -> ring (both mirror copies; buf == nullptr writes
// zeros), dir 1: ring -> buf.
__global__ void ring_copy_kernel(double* H, int64_t ldh, int R, int B, int nc, int64_t tau0, int nt,
                                 double* buf, int dir) {
  const int64_t n = (int64_t)nt * nc * B;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e % B;
    const int64_t k = (e / B) % nc;
    const int64_t i = e / ((int64_t)B * nc);
    const int64_t slot = pmod(tau0 - i, R);
    double* h = H + k * ldh + b;
    if (dir == 0) {
      const double v = buf ? buf[e] : 0.0;
      h[slot * B] = v;
      h[(slot + R) * B] = v;
    } else {
      buf[e] = h[slot * B];
    }
  }
}

void launch_ring_copy(double* H, int64_t ldh, int R, int B, int nc, int64_t tau0, int nt, double* buf,
                      int dir, hipStream_t s) {
  const int64_t n = (int64_t)nt * nc * B;
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  ring_copy_kernel<<<(unsigned)blocks, 256, 0, s>>>(H, ldh, R, B, nc, tau0, nt, buf, dir);
}

// Trajectory-major copy of nt ring slots for trajectories [b0, b0 + nb): out[bb][i][k] =
// src[k ks + ((tau0 - i) mod R) ss + b0 + bb] (i = 0 is time tau0).  Bath rings: ks = ldh, ss = B;
// the recorded full-DOF rings [slot][d][b]: ks = B, ss = nph B.  The host getters copy the chunks
// straight into the caller's arrays (no host-side transpose).
__global__ void hist_out_kernel(const double* __restrict__ src, int64_t ks, int64_t ss, int R, int64_t tau0,
                                int nt, int nk, int b0, int nb, double* __restrict__ out) {
  const int64_t n = (int64_t)nb * nt * nk;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = e % nk;
    const int64_t i = (e / nk) % nt;
    const int64_t bb = e / ((int64_t)nk * nt);
    out[e] = src[k * ks + pmod(tau0 - i, R) * ss + b0 + bb];
  }
}

void launch_hist_out(const double* src, int64_t ks, int64_t ss, int R, int64_t tau0, int nt, int nk, int b0, int nb,
                     double* out, hipStream_t s) {
  const int64_t n = (int64_t)nb * nt * nk;
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
  hist_out_kernel<<<(unsigned)blocks, 256, 0, s>>>(src, ks, ss, R, tau0, nt, nk, b0, nb, out);
}

__global__ void xprime_kernel(XPrimeArgs a) {
  const int64_t n = (int64_t)a.nc * a.B;
  const int64_t t = a.t;
  const int par = (int)(t & 1), par1 = par ^ 1;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = e / a.B, b = e % a.B;
    const double n0 = a.noise[((t % a.nmd) * a.nc + k) * a.B + b];
    const double n1 = a.noise[(((t + 1) % a.nmd) * a.nc + k) * a.B + b];
    const double S = a.S ? a.S[(int64_t)par * a.vs + e] : 0.0;
    double r = 0.0;
    for (int l = 0; l < MAXLVL; ++l)
      if (a.lvl[l]) r += a.lvl[l][k * a.lvl_ld[l] + b + a.lvl_off[l]];
    for (int q = 0; q < a.nqn; ++q) r += a.NP[((int64_t)par1 * a.nqn + q) * a.vs + e];
    a.V0[(int64_t)par * a.vs + e] = n0 - a.c * S;
    a.W1[(int64_t)par * a.vs + e] = n1 - a.c * r;
  }
}

void launch_xprime(const XPrimeArgs& a, hipStream_t s) {
  const int64_t n = (int64_t)a.nc * a.B;
  if (n <= 0) return;
  xprime_kernel<<<(unsigned)std::min<int64_t>((n + 255) / 256, 4096), 256, 0, s>>>(a);
}

// md.potforce cache audit of the run's last step (XCheck in gle_chain.hip: word b / 16, nibble b % 16,
// bit 0 / 1 and 2 / 3: some DOF tile's distance > 0 / >= 1e-9) in every workgroup, then the state
// copy unless the run stopped
__global__ __launch_bounds__(256) void xfinish_kernel(XFinishArgs a) {
  typedef __attribute__((address_space(1))) unsigned long long gull;
  const int nw = (a.B + 15) / 16;
  const unsigned long long* wp = a.xw + ((a.t + 2) % 3) * (int64_t)nw * a.R;
  unsigned long long h = 0ull;
  int st = 0;
  for (int j = threadIdx.x; j <= nw; j += 256) {
    if (j == nw) {
      st = *a.xstop != 0ull;
    } else {
      unsigned long long w = 0ull;
      for (int r = 0; r < a.R; ++r) w |= wp[(int64_t)r * nw + j];
      h |= w & ~(w >> 1) & 0x5555555555555555ull;  // sameq hits (md.py:767-779)
    }
  }
  if (__syncthreads_or(h != 0ull || st)) {
    if (!__syncthreads_or(st) && blockIdx.x == 0) {
      if (h) {
        __hip_atomic_fetch_add((gull*)(a.guard + 0), (unsigned long long)__popcll(h & 0x1111111111111111ull),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add((gull*)(a.guard + 1), (unsigned long long)__popcll(h & 0x4444444444444444ull),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (threadIdx.x == 0) {
        const unsigned long long v = (unsigned long long)a.t + 1ull;
        __hip_atomic_store((gull*)a.xstop, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.xstop_host, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    return;  // a stopped run: the host replays from the buffer of the stop step
  }
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < a.n; e += (int64_t)gridDim.x * blockDim.x) {
    a.P[e] = a.P2[e];
    a.Q[e] = a.Q2[e];
  }
}

// the two-launch path's id0 distance of step t (pmax word per trajectory, a maximum) as the d0 bits
// of the audit nibbles (bits 2 / 3: > 0 / >= 1e-9 or NaN) of slot (t - 1) mod 3
__global__ void xinject_kernel(const unsigned long long* __restrict__ pw, int B, unsigned long long* __restrict__ slot) {
  const int nw = (B + 15) / 16;
  for (int j = threadIdx.x; j < nw; j += blockDim.x) {
    unsigned long long x = 0ull;
    for (int b = 16 * j; b < min(B, 16 * j + 16); ++b) {
      const double m = __longlong_as_double((long long)pw[b]);
      const unsigned long long bits = (m > 0.0 ? 1ull : 0ull) | (!(m < 10e-10) ? 2ull : 0ull);
      x |= bits << (4 * (b % 16) + 2);
    }
    slot[j] = x;
  }
}

void launch_xinject(const unsigned long long* pw, int B, unsigned long long* slot, hipStream_t s) {
  xinject_kernel<<<1, 64, 0, s>>>(pw, B, slot);
}

void launch_xfinish(const XFinishArgs& a, hipStream_t s) {
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((a.n + 255) / 256, 1024));
  xfinish_kernel<<<g, 256, 0, s>>>(a);
}

// md.phis / md.qhis rows (newest first) of trajectories [b0, b0 + nb) into out [nb][nt][nph]: row i
// = slot (tau0 - i) mod R of the full-DOF recording ring rec [R][nph][B] for i < R, zero past the
// ring (or everywhere when rec is null)
__global__ void hist_full_kernel(const double* __restrict__ rec, int B, int R, int64_t tau0, int nt, int nph, int b0,
                                 int nb, double* __restrict__ out) {
  const int64_t n = (int64_t)nb * nt * nph;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = e % nph;
    const int64_t i = (e / nph) % nt;
    const int64_t bb = e / ((int64_t)nph * nt);
    out[e] = (rec && i < R) ? rec[(pmod(tau0 - i, R) * nph + k) * B + b0 + bb] : 0.0;
  }
}

// the bath DOFs' rows i < nrow of the same output from the bath's history ring H (row k of the bath
// at H[k * ldh + slot * B + b]); inv: DOF -> bath row or -1
__global__ void hist_overlay_kernel(const double* __restrict__ H, int64_t ldh, int B, int R, int64_t tau0,
                                    const int32_t* __restrict__ inv, int nrow, int nph, int b0, int nb, int nt,
                                    double* __restrict__ out) {
  const int64_t n = (int64_t)nb * nrow * nph;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = e % nph;
    const int k = inv[c];
    if (k < 0) continue;
    const int64_t i = (e / nph) % nrow;
    const int64_t bb = e / ((int64_t)nph * nrow);
    out[(bb * nt + i) * nph + c] = H[k * ldh + pmod(tau0 - i, R) * B + b0 + bb];
  }
}

void launch_hist_full(const double* rec, int B, int R, int64_t tau0, int nt, int nph, int b0, int nb, double* out,
                      hipStream_t s) {
  const int64_t n = (int64_t)nb * nt * nph;
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
  hist_full_kernel<<<(unsigned)blocks, 256, 0, s>>>(rec, B, R, tau0, nt, nph, b0, nb, out);
}

void launch_hist_overlay(const double* H, int64_t ldh, int B, int R, int64_t tau0, const int32_t* inv, int nrow,
                         int nph, int b0, int nb, int nt, double* out, hipStream_t s) {
  const int64_t n = (int64_t)nb * nrow * nph;
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
  hist_overlay_kernel<<<(unsigned)blocks, 256, 0, s>>>(H, ldh, B, R, tau0, inv, nrow, nph, b0, nb, nt, out);
}

// near ring (slot-major [NRS][vs], the chain's compact copy of the newest p): slots of times
// t, t-1, ..., t-NRS+1 from the history ring
__global__ void near_fill_kernel(const double* __restrict__ H, int64_t ldh, int R, int B, int ncp,
                                 double* __restrict__ NR, int64_t vs, int NRS, int64_t t) {
  const int64_t n = (int64_t)NRS * ncp * B;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e % B;
    const int64_t k = (e / B) % ncp;
    const int64_t s = e / ((int64_t)B * ncp);
    const int64_t tau = t - s;
    NR[pmod(tau, NRS) * vs + k * B + b] = H[k * ldh + pmod(tau, R) * B + b];
  }
}

void launch_near_fill(const double* H, int64_t ldh, int R, int B, int ncp, double* NR, int64_t vs, int NRS,
                      int64_t t, hipStream_t s) {
  const int64_t n = (int64_t)NRS * ncp * B;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  near_fill_kernel<<<(unsigned)blocks, 256, 0, s>>>(H, ldh, R, B, ncp, NR, vs, NRS, t);
}

}  // namespace gle

namespace gle {

// ------------------------------------------------------------------------------------------
// Spectral (overlap-save) levels.  A level of block length P covers the lags of partitions
// m in [m0, m0 + M): k_m[i'] = K_{mP+i'} (i' < P, zero-padded to N = 2P).  Twiddles:
// cstab[q] = (cos(pi q / Pmax), sin(pi q / Pmax)), q < 2 Pmax; a level reads it with stride
// Pmax / P, so e^{-i pi f n / P} = (cs.x, -cs.y) at q = ((f n) mod 2P) * stride.
//
//   Khat_m(f) = sum_i' k_m[i'] e^{-i pi f i'/P}, f = 0..P, stored in fragment-native order
//   [f][plane][rt][m - m0][ks][64] (a wave streams its row tile's k-steps contiguously) as two real
//   planes Re, Im (nplanes = 2: the two-plane Gauss items form Re + Im, Im - Re in registers) or as
//   the three Gauss planes Re, Re + Im, Im - Re (nplanes = 3: one item per Gauss part), read
//   straight out of the fragment-native K already on the device (one-time setup).
// In-place radix-2 FFT of NS complex series of length N = 2^logn held bit-reversed in LDS
// (buf[s * N + i]); sign -1 = forward, +1 = inverse (unscaled).
template <int NS>
__device__ __forceinline__ void lds_fft(double2* buf, int logn, const double2* tw, double sign) {
  // tw: the N/2 twiddles e^{-2 pi i j / N}, j < N/2, staged in LDS by the caller (a twiddle load
  // from global memory in every stage would put logn dependent L2 round trips on the path)
  const int N = 1 << logn, h = N >> 1;
  for (int st = 1; st <= logn; ++st) {
    const int half = 1 << (st - 1);
    const int tstride = N >> st;  // e^{-2 pi i jj / 2^st} = tw[jj * N / 2^st]
    for (int j = threadIdx.x; j < NS * h; j += blockDim.x) {
      const int sidx = j / h, jb = j - sidx * h;
      const int g = jb >> (st - 1);
      const int jj = jb & (half - 1);
      double2* bs = buf + sidx * N;
      const int i0 = (g << st) + jj;
      const int i1 = i0 + half;
      const double2 c = tw[jj * tstride];
      const double wx = c.x, wy = sign * c.y;  // e^{sign i 2 pi jj / 2^st}
      const double2 x0 = bs[i0];
      const double2 x1 = bs[i1];
      const double2 y = make_double2(x1.x * wx - x1.y * wy, x1.x * wy + x1.y * wx);
      bs[i0] = make_double2(x0.x + y.x, x0.y + y.y);
      bs[i1] = make_double2(x0.x - y.x, x0.y - y.y);
    }
    __syncthreads();
  }
}

// twiddles of a length-N transform into LDS: tw[j] = cstab[j * cstride], j < N/2
__device__ __forceinline__ void stage_twiddles(double2* tw, int N, const double2* __restrict__ cstab, int cstride) {
  for (int j = threadIdx.x; j < N / 2; j += blockDim.x) tw[j] = cstab[(int64_t)j * cstride];
}

// xcd != 0 (one pass, grid a multiple of 8): blocks b, b + 8, ... run on one XCD (round-robin
// dispatch), so XCD b % 8 gets the contiguous item range [(b % 8) per, (b % 8 + 1) per): the row
// groups of one (f, g) product, which read the same X window, then share that XCD's L2 instead of
// each fetching the window into a different XCD.
template <int RN, int KC, int AD = CG_AD, int XD = CG_XD, int DBG = 0>
#ifndef CG_WPE
#define CG_WPE 3
#endif
__global__ __launch_bounds__(256, KC <= 4 ? CG_WPE : 2) void cgemm_kernel(const CgItem* __restrict__ items, int nitems, int64_t tseg,
                                                       int xcd, unsigned long long* ts) {
  __shared__ double xs[cg_lds_doubles<RN, KC>()];
  if (ts && threadIdx.x == 0) atomicMin(ts, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  if (xcd) {
    const int per = gridDim.x >> 3;
    const int item = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (item < nitems) cgemm_any<RN, KC, AD, XD, DBG>(items[item], tseg, xs);
  } else {
    for (int item = blockIdx.x; item < nitems; item += gridDim.x) {
      const CgItem it = items[item];
      cgemm_any<RN, KC, AD, XD, DBG>(it, tseg, xs);
      __syncthreads();
    }
  }
  if (ts) {  // launch-uniform
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(ts + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
}
static int g_cg_xcd = -1;  // GLE_CG_XCD=0 switches the XCD grouping off (experiment switch)
static int g_cg_dbg = 0;
static int g_cg_kc = 0;    // k-steps per LDS chunk: 4 (159 VGPRs, 3 waves/SIMD; 23.9 vs 21.6 TF/s in situ), GLE_CG_KC=8: 8
static int g_cg_ring = 0;  // GLE_CG_RING=AD*10+XD (experiment switch): prefetch ring depths
__global__ void empty_kernel(int* p) {
  if (p) p[0] = 0;
}

void launch_cgemm(int rn, const CgItem* items, int nitems, int64_t tseg, hipStream_t s, int max_grid,
                  unsigned long long* ts) {
  if (nitems <= 0) return;
  GLE_BOUNDS_SYNC();
#ifdef GLE_EXPERIMENTS
  g_cg_xcd = -1;  // re-read per launch: variants of one process (scripts/exp_time.py --variants) switch them
#endif
  if (g_cg_xcd < 0) {
    const char* e = gle_env("GLE_CG_XCD");
    g_cg_xcd = (e && atoi(e) == 0) ? 0 : 1;
    const char* k = gle_env("GLE_CG_KC");
    g_cg_kc = (k && atoi(k) == 8) ? 8 : 4;
    // 1: no K-hat loads, 2: no LDS operand reads, 4: no X staging / barrier; 3, 7: combinations
    const char* d = gle_env("GLE_CG_DBG");
    g_cg_dbg = d ? std::max(0, std::min(16, atoi(d))) : 0;
  }
#ifdef GLE_EXPERIMENTS
  if (g_cg_dbg == 16) {  // timing experiment: an empty one-workgroup launch in place of the chunk
    empty_kernel<<<1, 64, 0, s>>>(nullptr);
    return;
  }
#endif
  {  // re-read per launch: variants of one process (scripts/exp_time.py --variants) switch it
    const char* r = gle_env("GLE_CG_RING");
    g_cg_ring = r ? atoi(r) : 0;
  }
  // GLE_CG_LDS_PAD (bytes, experiment switch): unused dynamic LDS per workgroup, capping how many
  // far-field workgroups a CU holds so the per-step chain's workgroups find room beside them
  // (re-read per launch like GLE_CG_RING: variants of one process switch it)
  int lds_pad = 0;
  if (const char* e = gle_env("GLE_CG_LDS_PAD")) lds_pad = std::max(0, std::min(96 * 1024, atoi(e)));
  const size_t shm = (size_t)lds_pad;
  const bool capped = max_grid > 0 && max_grid < nitems;
  const int xcd = (!capped && g_cg_xcd) ? 1 : 0;
  const int grid = capped ? max_grid : (xcd ? (nitems + 7) / 8 * 8 : nitems);
#ifdef GLE_EXPERIMENTS
  if (g_cg_dbg && rn == 4 && g_cg_kc == 4) {  // GLE_CG_DBG timing experiments (results invalid)
    if (g_cg_dbg == 1) cgemm_kernel<4, 4, CG_AD, CG_XD, 1><<<grid, 256, shm, s>>>(items, nitems, tseg, xcd, ts);
    else if (g_cg_dbg == 2) cgemm_kernel<4, 4, CG_AD, CG_XD, 2><<<grid, 256, shm, s>>>(items, nitems, tseg, xcd, ts);
    else if (g_cg_dbg == 3) cgemm_kernel<4, 4, CG_AD, CG_XD, 3><<<grid, 256, shm, s>>>(items, nitems, tseg, xcd, ts);
    else if (g_cg_dbg == 4) cgemm_kernel<4, 4, CG_AD, CG_XD, 4><<<grid, 256, shm, s>>>(items, nitems, tseg, xcd, ts);
    else if (g_cg_dbg == 15) cgemm_kernel<4, 4, CG_AD, CG_XD, 15><<<grid, 256, shm, s>>>(items, nitems, tseg, xcd, ts);
    else cgemm_kernel<4, 4, CG_AD, CG_XD, 7><<<grid, 256, shm, s>>>(items, nitems, tseg, xcd, ts);
    return;
  }
  if (g_cg_ring && rn == 4 && g_cg_kc == 4) {  // prefetch-ring variants
    switch (g_cg_ring) {
      case 31: cgemm_kernel<4, 4, 3, 1><<<grid, 256, shm, s>>>(items, nitems, tseg, xcd, ts); return;
      case 32: cgemm_kernel<4, 4, 3, 2><<<grid, 256, shm, s>>>(items, nitems, tseg, xcd, ts); return;
      case 51: cgemm_kernel<4, 4, 5, 1><<<grid, 256, shm, s>>>(items, nitems, tseg, xcd, ts); return;
      case 52: cgemm_kernel<4, 4, 5, 2><<<grid, 256, shm, s>>>(items, nitems, tseg, xcd, ts); return;
      case 72: cgemm_kernel<4, 4, 7, 2><<<grid, 256, shm, s>>>(items, nitems, tseg, xcd, ts); return;
      default: break;
    }
  }
#endif
  if (g_cg_kc == 4) {
    switch (rn) {
      case 1: cgemm_kernel<1, 4><<<grid, 256, shm, s>>>(items, nitems, tseg, xcd, ts); break;
      case 2: cgemm_kernel<2, 4><<<grid, 256, shm, s>>>(items, nitems, tseg, xcd, ts); break;
      default: cgemm_kernel<4, 4><<<grid, 256, shm, s>>>(items, nitems, tseg, xcd, ts); break;
    }
    return;
  }
  switch (rn) {
    case 1: cgemm_kernel<1, CG_KC><<<grid, 256, shm, s>>>(items, nitems, tseg, xcd, ts); break;
    case 2: cgemm_kernel<2, CG_KC><<<grid, 256, shm, s>>>(items, nitems, tseg, xcd, ts); break;
    default: cgemm_kernel<4, CG_KC><<<grid, 256, shm, s>>>(items, nitems, tseg, xcd, ts); break;
  }
}

// Segment spectra of the nseg newest segments sigma = T/P - sidx (grid: sidx x DOF k x 8-trajectory
// chunk): x[n] = p at time sigma*P - 2P + 2 + n (n < 2P-1), x[2P-1] = 0;
// Xhat(f) = sum_n x[n] e^{-i pi f n / P}, f = 0..P, written into the frequency-f segment ring as two
// planes  g = 0: Re,  1: Im  (nplanes = 2; the two-plane GEMM items form Re + Im in registers) or the
// three Gauss planes  g = 0: Re + Im,  1: Im,  2: Re  (nplanes = 3), rows [g ncp + k].  Two real
// series per complex FFT.
// BC trajectories per block: 64 for the small transforms (one block per DOF, 512 B rows, every
// thread busy in every butterfly stage), fewer for long transforms (LDS: BC/2 series of 2P points)
__device__ __forceinline__ FftBath pick_bath(const FftBaths& fb, int64_t blk) {
  FftBath r = fb.b[0];
#pragma unroll
  for (int j = 1; j < MAXFB; ++j)
    if (j < fb.n && blk >= fb.b[j].blk0) r = fb.b[j];
  return r;
}

template <int BC>
__global__ __launch_bounds__(256) void seg_fft_kernel(FftBaths fb, int B, int P, int logn, int64_t T,
                                                      const double2* __restrict__ cstab, int cstride,
                                                      int nplanes) {
  extern __shared__ double2 fbuf[];  // BC/2 series of N points, then N/2 twiddles
  const FftBath bt = pick_bath(fb, blockIdx.x);
  const int64_t blk = (int64_t)blockIdx.x - bt.blk0;
  const double* __restrict__ H = bt.H;
  const int64_t ldh = bt.ldh;
  const int R = bt.R, nk = bt.nk, ncp = bt.ncp, Rseg = bt.Rseg;
  double* __restrict__ seg = bt.seg;
  const int64_t seg_fstride = bt.seg_fstride, ldseg = bt.ldseg;
  const int N = 2 * P;
  stage_twiddles(fbuf + (BC / 2) * N, N, cstab, cstride);
  const int nbc = (B + BC - 1) / BC;
  const int bc = (int)(blk % nbc);
  const int k = bt.k0 + (int)((blk / nbc) % nk);
  const int sidx = (int)(blk / ((int64_t)nbc * nk));
  const int64_t sigma = T / P - sidx;
  const int64_t t0 = sigma * P - 2 * P + 2;
  const int b0 = bc * BC;
  const double* hk = H + (int64_t)k * ldh;
  for (int e = threadIdx.x; e < N * BC / 2; e += blockDim.x) {
    const int q = e % (BC / 2);
    const int n = e / (BC / 2);
    double xr = 0.0, xi = 0.0;
    if (n < N - 1) {
      const double* hs = hk + pmod(t0 + n, R) * B;
      const int ba = b0 + 2 * q, bb = ba + 1;
      if (ba < B) xr = hs[ba];
      if (bb < B) xi = hs[bb];
    }
    const unsigned rev = __brev((unsigned)n) >> (32 - logn);
    fbuf[q * N + rev] = make_double2(xr, xi);
  }
  __syncthreads();
  lds_fft<BC / 2>(fbuf, logn, fbuf + (BC / 2) * N, -1.0);
  const int64_t slot = pmod(sigma, Rseg);
  for (int e = threadIdx.x; e < (P + 1) * BC; e += blockDim.x) {
    const int bl = e % BC;
    const int f = e / BC;
    const int b = b0 + bl;
    if (b >= B) continue;
    const int q = bl >> 1;
    const double2 z = fbuf[q * N + f];
    const double2 zc = fbuf[q * N + ((N - f) & (N - 1))];
    // X_even = (Z[f] + conj Z[N-f]) / 2, X_odd = (Z[f] - conj Z[N-f]) / (2i)
    double re, im;
    if ((bl & 1) == 0) {
      re = 0.5 * (z.x + zc.x);
      im = 0.5 * (z.y - zc.y);
    } else {
      re = 0.5 * (z.y + zc.y);
      im = -0.5 * (z.x - zc.x);
    }
    double* sf = seg + (int64_t)f * seg_fstride + b;
    // two planes Re, Im (two-plane Gauss items) or the three Gauss planes Re + Im, Im, Re; straight-line
    // stores (a register array indexed by a runtime plane number goes to scratch)
    // (cgemm addresses ring slots modulo Rseg: no mirrored copy)
    const int64_t pl = (int64_t)ncp * ldseg;
    double* so = sf + (int64_t)k * ldseg + (int64_t)slot * B;
    if (nplanes == 2) {
      so[0] = re;
      so[pl] = im;
    } else {
      so[0] = re + im;
      so[pl] = im;
      so[2 * pl] = re;
    }
  }
}

// raise a kernel's dynamic-LDS limit once per (kernel, device): a per-launch attribute call costs
// host time on the step's critical path at block boundaries
static bool lds_attr_once(const void* fn) {
  constexpr int MAXDEV = 64;
  struct Entry {
    const void* fn;
    int dev;
  };
  static thread_local std::vector<Entry> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev >= MAXDEV) return false;
  for (const Entry& e : done)
    if (e.fn == fn && e.dev == dev) return true;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess) return false;
  done.push_back({fn, dev});
  return true;
}

// trajectories per FFT block: the largest of 64/32/16/8 (not above B rounded to 8) whose LDS
// (BC/2 complex series of 2P points) stays within 64 KiB
static int fft_bc(int B, int P) {
  int bc = 64;
  while (bc > 8 && (bc > ((B + 7) / 8) * 8 || ((size_t)(bc / 2) * 2 * P + P) * 16 > 64 * 1024)) bc /= 2;
  return bc;
}

// K-hat of a spectral level (gle_api.hip freeze): for partition m = m0 + mm and frequency f <= P,
//   Khat(f)[r][k] = sum_{ip < P} K_{m P + ip}[r][k] e^{-i pi f ip / P}
// i.e. the 2P-point transform of the zero-padded P slices of every kernel element, written as the
// planes Re, Im (nplanes 2) or the three Gauss planes Re, Re + Im, Im - Re (nplanes 3) in the
// fragment-native layout [f][plane][rt][mm][ks][64].  A fragment's lane is the element's position in
// the kernel's own fragment layout [rt][ks][i][64], so block (fragment, mm, lane chunk) streams the P
// slices of BC lanes (BC doubles contiguous per slice) into LDS as BC/2 complex series (two real
// series per complex FFT, bit-reversed), transforms them (lds_fft, radix 2) and separates the pairs:
// O(P log P) per element instead of the O(P^2) direct sum (C5's P = 1024 level: 8.8 s of setup).
template <int BC>
__global__ __launch_bounds__(256) void khat_fft_kernel(const double* __restrict__ Kf, int ml, int nks_k,
                                                       double* __restrict__ khat, int P, int logn, int m0, int M,
                                                       int nc, int nrt2, int nks2, const double2* __restrict__ cstab,
                                                       int cstride, int nplanes) {
  extern __shared__ double2 fbuf[];  // BC/2 series of N = 2P points, then N/2 twiddles
  const int N = 2 * P;
  stage_twiddles(fbuf + (BC / 2) * N, N, cstab, cstride);
  constexpr int NLC = 64 / BC;
  int64_t blk = blockIdx.x;
  const int lc = (int)(blk % NLC);
  blk /= NLC;
  const int mm = (int)(blk % M);
  blk /= M;
  const int ks2 = (int)(blk % nks2);
  const int rt2 = (int)(blk / nks2);
  const int l0 = lc * BC;
  const int m = m0 + mm;
  const double* __restrict__ src = Kf + ((int64_t)rt2 * nks_k + ks2) * ml * 64 + l0;
  for (int e = threadIdx.x; e < N * (BC / 2); e += blockDim.x) {
    const int q = e % (BC / 2);
    const int n = e / (BC / 2);
    const int i = m * P + n;
    double xr = 0.0, xi = 0.0;
    if (n < P && i < ml) {
      const int la = 2 * q, lb = la + 1;
      const int ra = 16 * rt2 + ((l0 + la) & 15), ka = 4 * ks2 + ((l0 + la) >> 4);
      const int rb = 16 * rt2 + ((l0 + lb) & 15), kb = 4 * ks2 + ((l0 + lb) >> 4);
      if (ra < nc && ka < nc) xr = src[(int64_t)i * 64 + la];
      if (rb < nc && kb < nc) xi = src[(int64_t)i * 64 + lb];
    }
    const unsigned rev = __brev((unsigned)n) >> (32 - logn);
    fbuf[q * N + rev] = make_double2(xr, xi);
  }
  __syncthreads();
  lds_fft<BC / 2>(fbuf, logn, fbuf + (BC / 2) * N, -1.0);
  const int64_t plane = (int64_t)nrt2 * M * nks2 * 64;
  double* __restrict__ out = khat + (((int64_t)rt2 * M + mm) * nks2 + ks2) * 64 + l0;
  for (int e = threadIdx.x; e < (P + 1) * BC; e += blockDim.x) {
    const int l = e % BC;
    const int f = e / BC;
    const int q = l >> 1;
    const double2 z = fbuf[q * N + f];
    const double2 zc = fbuf[q * N + ((N - f) & (N - 1))];
    // X_even = (Z[f] + conj Z[N-f]) / 2, X_odd = (Z[f] - conj Z[N-f]) / (2i)
    double re, im;
    if ((l & 1) == 0) {
      re = 0.5 * (z.x + zc.x);
      im = 0.5 * (z.y - zc.y);
    } else {
      re = 0.5 * (z.y + zc.y);
      im = -0.5 * (z.x - zc.x);
    }
    double* o = out + (int64_t)f * nplanes * plane + l;
    o[0] = re;
    if (nplanes == 2) {
      o[plane] = im;
    } else {  // three Gauss planes Re, Re + Im, Im - Re
      o[plane] = re + im;
      o[2 * plane] = im - re;
    }
  }
}

template <int BC>
static int khat_fft_launch(const double* Kf, int ml, int nks_k, double* khat, int P, int logn, int m0, int M,
                           int nc, int nrt2, int nks2, const double* cstab, int cstride, hipStream_t s,
                           int nplanes) {
  const size_t shmem = ((size_t)(BC / 2) * 2 * P + P) * sizeof(double2);
  if (shmem > 160 * 1024) return -2;
  if (!lds_attr_once((const void*)khat_fft_kernel<BC>)) return -3;
  const int64_t blocks = (int64_t)nrt2 * nks2 * M * (64 / BC);
  if (blocks <= 0) return 0;
  khat_fft_kernel<BC><<<(unsigned)blocks, 256, shmem, s>>>(Kf, ml, nks_k, khat, P, logn, m0, M, nc, nrt2, nks2,
                                                           (const double2*)cstab, cstride, nplanes);
  return 0;
}

int launch_khat_pack(const double* Kf, int ml, int nks_k, double* khat, int P, int m0, int M, int nc, int nrt2,
                     int nks2, const double* cstab, int cstride, hipStream_t s, int nplanes) {
  int logn = 0;
  while ((1 << logn) < 2 * P) ++logn;
  if ((1 << logn) != 2 * P) return -1;
  // lanes per block: the most whose BC/2 series of 2P points (+ twiddles) fit 160 KiB of LDS
  int bc = 64;
  while (bc > 2 && ((size_t)(bc / 2) * 2 * P + P) * sizeof(double2) > 160 * 1024) bc /= 2;
  switch (bc) {
    case 64: return khat_fft_launch<64>(Kf, ml, nks_k, khat, P, logn, m0, M, nc, nrt2, nks2, cstab, cstride, s, nplanes);
    case 32: return khat_fft_launch<32>(Kf, ml, nks_k, khat, P, logn, m0, M, nc, nrt2, nks2, cstab, cstride, s, nplanes);
    case 16: return khat_fft_launch<16>(Kf, ml, nks_k, khat, P, logn, m0, M, nc, nrt2, nks2, cstab, cstride, s, nplanes);
    case 8: return khat_fft_launch<8>(Kf, ml, nks_k, khat, P, logn, m0, M, nc, nrt2, nks2, cstab, cstride, s, nplanes);
    case 4: return khat_fft_launch<4>(Kf, ml, nks_k, khat, P, logn, m0, M, nc, nrt2, nks2, cstab, cstride, s, nplanes);
    default: return khat_fft_launch<2>(Kf, ml, nks_k, khat, P, logn, m0, M, nc, nrt2, nks2, cstab, cstride, s, nplanes);
  }
}

template <int BC>
static int seg_fft_launch(const FftBaths& fb, int B, int P, int logn, int64_t T, const double* cstab, int cstride,
                          hipStream_t s, int nplanes, int64_t blocks) {
  const size_t shmem = ((size_t)(BC / 2) * 2 * P + P) * sizeof(double2);
  if (shmem > 160 * 1024) return -2;
  // raise the dynamic-LDS limit once per instantiation (a per-launch attribute call costs host
  // time on the step's critical path at block boundaries)
  if (!lds_attr_once((const void*)seg_fft_kernel<BC>)) return -3;
  if (blocks <= 0) return 0;
  seg_fft_kernel<BC><<<(unsigned)blocks, 256, shmem, s>>>(fb, B, P, logn, T, (const double2*)cstab, cstride, nplanes);
  return 0;
}

int launch_seg_fft_multi(FftBaths fb, int B, int P, int64_t T, int nseg, const double* cstab, int cstride,
                         hipStream_t s, int nplanes) {
  int logn = 0;
  while ((1 << logn) < 2 * P) ++logn;
  if ((1 << logn) != 2 * P) return -1;
  const int bc = fft_bc(B, P);
  const int nbc = (B + bc - 1) / bc;
  int64_t blocks = 0;
  for (int j = 0; j < fb.n; ++j) {
    fb.b[j].blk0 = blocks;
    blocks += (int64_t)nseg * std::max(0, fb.b[j].nk) * nbc;
  }
  switch (bc) {
    case 64: return seg_fft_launch<64>(fb, B, P, logn, T, cstab, cstride, s, nplanes, blocks);
    case 32: return seg_fft_launch<32>(fb, B, P, logn, T, cstab, cstride, s, nplanes, blocks);
    case 16: return seg_fft_launch<16>(fb, B, P, logn, T, cstab, cstride, s, nplanes, blocks);
    default: return seg_fft_launch<8>(fb, B, P, logn, T, cstab, cstride, s, nplanes, blocks);
  }
}

int launch_seg_fft(const double* H, int64_t ldh, int R, int B, int nc, int ncp, int P, int64_t T,
                   int nseg, double* seg, int64_t seg_fstride, int64_t ldseg, int Rseg,
                   const double* cstab, int cstride, hipStream_t s, int k0, int k1, int nplanes) {
  if (k1 < 0 || k1 > nc) k1 = nc;
  k0 = k0 < 0 ? 0 : k0;
  if (k1 - k0 <= 0) return 0;
  FftBaths fb{};
  fb.n = 1;
  FftBath& b = fb.b[0];
  b.H = H;
  b.ldh = ldh;
  b.R = R;
  b.nc = nc;
  b.ncp = ncp;
  b.k0 = k0;
  b.nk = k1 - k0;
  b.seg = seg;
  b.seg_fstride = seg_fstride;
  b.ldseg = ldseg;
  b.Rseg = Rseg;
  return launch_seg_fft_multi(fb, B, P, T, nseg, cstab, cstride, s, nplanes);
}

// Block output out(kP + 1 + j) = y[j + P - 1] (j < P) of the real inverse transform of the
// Hermitian spectrum Y(f), f = 0..P (Im Y_0, Im Y_P ignored as by irfft), assembled from the Gauss
// products T_g(f):
//   y[n] = (1/2P) sum_{f<2P} Y(f) e^{+i pi f n / P},  Y(2P - f) = conj Y(f).
// Grid: DOF k x 8-trajectory chunk; two real outputs per complex inverse FFT.
template <int BC>
__global__ __launch_bounds__(256) void far_ifft_kernel(FftBaths fb, int B, int P, int logn,
                                                       const double2* __restrict__ cstab, int cstride) {
  extern __shared__ double2 fbuf[];  // BC/2 series of N points, then N/2 twiddles
  const FftBath bt = pick_bath(fb, blockIdx.x);
  const int64_t blk = (int64_t)blockIdx.x - bt.blk0;
  const double* __restrict__ Y = bt.Y;
  const int64_t yfstride = bt.yfstride, ysplit = bt.ysplit, ldout = bt.ldout;
  double* __restrict__ out = bt.out;
  const int nc = bt.nc;
  const int N = 2 * P;
  stage_twiddles(fbuf + (BC / 2) * N, N, cstab, cstride);
  const int nbc = (B + BC - 1) / BC;
  const int bc = (int)(blk % nbc);
  const int k = bt.k0 + (int)(blk / nbc);
  const int b0 = bc * BC;
  const int64_t pl = (int64_t)nc * B;
  for (int e = threadIdx.x; e < N * BC / 2; e += blockDim.x) {
    const int q = e % (BC / 2);
    const int f = e / (BC / 2);
    const bool cj = f > P;
    const int fs = cj ? N - f : f;
    const bool realonly = (fs == 0) || (fs == P);
    const int ba = b0 + 2 * q, bb = ba + 1;
    const double* yf = Y + (int64_t)fs * yfstride + (int64_t)k * B;
    // Re Y = T_0 - T_1, Im Y = T_0 + T_2 (Gauss products, planes [f][g][nc][B])
    double ar = 0.0, ai = 0.0, br = 0.0, bi = 0.0;
    // split-K levels: the two k-halves of every product, added in fixed order (deterministic)
    auto tg = [&](int g, int b) { return ysplit ? yf[g * pl + b] + yf[ysplit + g * pl + b] : yf[g * pl + b]; };
    if (ba < B) {
      const double t0 = tg(0, ba);
      ar = t0 - tg(1, ba);
      ai = realonly ? 0.0 : t0 + tg(2, ba);
    }
    if (bb < B) {
      const double t0 = tg(0, bb);
      br = t0 - tg(1, bb);
      bi = realonly ? 0.0 : t0 + tg(2, bb);
    }
    if (cj) {
      ai = -ai;
      bi = -bi;
    }
    // Z = A + i B
    const unsigned rev = __brev((unsigned)f) >> (32 - logn);
    fbuf[q * N + rev] = make_double2(ar - bi, ai + br);
  }
  __syncthreads();
  lds_fft<BC / 2>(fbuf, logn, fbuf + (BC / 2) * N, 1.0);
  const double scale = 1.0 / N;
  for (int e = threadIdx.x; e < P * BC; e += blockDim.x) {
    const int bl = e % BC;
    const int j = e / BC;
    const int b = b0 + bl;
    if (b >= B) continue;
    const double2 z = fbuf[(bl >> 1) * N + j + P - 1];
    out[(int64_t)k * ldout + (int64_t)j * B + b] = ((bl & 1) ? z.y : z.x) * scale;
  }
}

template <int BC>
static int far_ifft_launch(const FftBaths& fb, int B, int P, int logn, const double* cstab, int cstride, hipStream_t s,
                           int64_t blocks) {
  const size_t shmem = ((size_t)(BC / 2) * 2 * P + P) * sizeof(double2);
  if (shmem > 160 * 1024) return -2;
  // raise the dynamic-LDS limit once per instantiation (a per-launch attribute call costs host
  // time on the step's critical path at block boundaries)
  if (!lds_attr_once((const void*)far_ifft_kernel<BC>)) return -3;
  if (blocks <= 0) return 0;
  far_ifft_kernel<BC><<<(unsigned)blocks, 256, shmem, s>>>(fb, B, P, logn, (const double2*)cstab, cstride);
  return 0;
}

int launch_far_ifft_multi(FftBaths fb, int B, int P, const double* cstab, int cstride, hipStream_t s) {
  int logn = 0;
  while ((1 << logn) < 2 * P) ++logn;
  if ((1 << logn) != 2 * P) return -1;
  const int bc = fft_bc(B, P);
  const int nbc = (B + bc - 1) / bc;
  int64_t blocks = 0;
  for (int j = 0; j < fb.n; ++j) {
    fb.b[j].blk0 = blocks;
    blocks += (int64_t)std::max(0, fb.b[j].nk) * nbc;
  }
  switch (bc) {
    case 64: return far_ifft_launch<64>(fb, B, P, logn, cstab, cstride, s, blocks);
    case 32: return far_ifft_launch<32>(fb, B, P, logn, cstab, cstride, s, blocks);
    case 16: return far_ifft_launch<16>(fb, B, P, logn, cstab, cstride, s, blocks);
    default: return far_ifft_launch<8>(fb, B, P, logn, cstab, cstride, s, blocks);
  }
}

int launch_far_ifft(const double* Y, int64_t yfstride, int64_t ysplit, int nc, int B, int P, double* out,
                    int64_t ldout, const double* cstab, int cstride, hipStream_t s, int k0, int k1) {
  if (k1 < 0 || k1 > nc) k1 = nc;
  k0 = k0 < 0 ? 0 : k0;
  if (k1 - k0 <= 0) return 0;
  FftBaths fb{};
  fb.n = 1;
  FftBath& b = fb.b[0];
  b.Y = Y;
  b.yfstride = yfstride;
  b.ysplit = ysplit;
  b.nc = nc;
  b.k0 = k0;
  b.nk = k1 - k0;
  b.out = out;
  b.ldout = ldout;
  return launch_far_ifft_multi(fb, B, P, cstab, cstride, s);
}

}  // namespace gle
