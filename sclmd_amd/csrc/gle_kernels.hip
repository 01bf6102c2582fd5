// HIP kernels of the GLE stepper for gfx950 (MI355X).
//
//  contract_kernel<RN>  memory-kernel friction contraction (and every other dense product of the
//                       step) on v_mfma_f64_16x16x4_f64: A = kernel slices streamed from HBM in
//                       fragment-native order straight into registers; X = a sliding window of
//                       the velocity-history ring staged once per k-chunk in LDS and shared by the
//                       4 waves (one 16-row tile each) across all slices of the work item.
//  reduce_kernel        fixed-order sum of split-K / split-slice partial tiles (+ far field).
//  potsel_kernel        md.potforce's cache rule (sameq, md.py:449-450, 767-779) per trajectory.
//  phaseA/B/C_kernel    the elementwise parts of md.vv (md.py:383-411): bath-force assembly
//                       (baths.py:232-255, 452-458), heat current (md.py:397), Verlet kicks,
//                       constraints (md.py:782-794), history push (md.py:386-387).
//  philox / fft_noise   coloured-noise generator (noise.py:50-100, 149-206).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>

#include "gle_internal.h"

namespace gle {

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int64_t pmod(int64_t a, int64_t m) {
  int64_t r = a % m;
  return r < 0 ? r + m : r;
}

__device__ __forceinline__ int64_t load_t(const Clock* clk) {
  return __hip_atomic_load(&clk->t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------------
// contraction
template <int RN>
__global__ __launch_bounds__(WG, 2) void contract_kernel(const CItem* __restrict__ items,
                                                         const Clock* __restrict__ clk) {
  __shared__ double lds[KROWS * LDS_COLS];
  constexpr int NT = 16 * RN;
  const CItem it = items[blockIdx.x];
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int64_t t = load_t(clk);

  d4 acc[RN];
#pragma unroll
  for (int n = 0; n < RN; ++n) acc[n] = d4{0.0, 0.0, 0.0, 0.0};

  const int ns_max = it.ring ? (LDS_WW_MAX - NT) / it.cs + 1 : 1;
  const bool active = wave < it.nrt;
  const double* Aw = it.A + (int64_t)wave * it.a_rt + lane;
  const int brow = lane >> 4;
  const int bcol = lane & 15;

  for (int s0 = 0; s0 < it.ni; s0 += ns_max) {
    const int ns = min(ns_max, it.ni - s0);
    const int ww = (ns - 1) * it.cs + NT;
    const int wwp = ((ww + 31) & ~31) + 16;  // row stride = 16 mod 32 doubles: rows r, r+1 on
                                             // complementary LDS bank halves for ds_read_b64
    int64_t wbase = it.col0;
    if (it.ring) {
      const int64_t tau = t + it.tshift - (int64_t)(it.ia + s0 + ns - 1);
      wbase += pmod(tau, it.ring) * it.cs;
    }
    for (int kc = 0; kc < it.nks; kc += KC) {
      __syncthreads();
      const double* xs = it.X + (int64_t)(4 * kc) * it.ldx + wbase;
#pragma unroll
      for (int r = 0; r < KROWS; ++r) {
        const double* xr = xs + (int64_t)r * it.ldx;
        double* lr = lds + r * wwp;
        for (int c = tid; c < ww; c += WG) lr[c] = xr[c];
      }
      __syncthreads();
      if (active) {
        const double* Ak = Aw + (int64_t)kc * it.a_ks + (int64_t)s0 * 64;
        double a0 = Ak[0];
        double a1 = Ak[it.a_ks];
        for (int ss = 0; ss < ns; ++ss) {
          double n0 = 0.0, n1 = 0.0;
          if (ss + 1 < ns) {
            n0 = Ak[(ss + 1) * 64];
            n1 = Ak[it.a_ks + (ss + 1) * 64];
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
          a0 = n0;
          a1 = n1;
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
        if (row < it.nrows && col < it.ncols) it.out[(int64_t)row * it.ldo + col] = acc[n][r];
      }
    }
  }
}

void launch_contract(int rn, const CItem* items, int nitems, const Clock* clk, hipStream_t s) {
  if (nitems <= 0) return;
  dim3 g(nitems), b(WG);
  switch (rn) {
    case 1: contract_kernel<1><<<g, b, 0, s>>>(items, clk); break;
    case 2: contract_kernel<2><<<g, b, 0, s>>>(items, clk); break;
    case 4: contract_kernel<4><<<g, b, 0, s>>>(items, clk); break;
    case 8: contract_kernel<8><<<g, b, 0, s>>>(items, clk); break;
    default: contract_kernel<16><<<g, b, 0, s>>>(items, clk); break;
  }
}

// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void reduce_kernel(const RItem* __restrict__ items,
                                                     Clock* __restrict__ clk, int set_tfar) {
  const RItem it = items[blockIdx.x];
  const int64_t t = load_t(clk);
  const double* add = nullptr;
  if (it.add) add = it.add + (t - clk->t_far) * it.add_cs;
  const int n = it.rows * it.cols;
  for (int e = threadIdx.x; e < n; e += blockDim.x) {
    const int r = e / it.cols;
    const int c = e - r * it.cols;
    double s = add ? add[(int64_t)r * it.lda + c] : 0.0;
    const double* p = it.src + (int64_t)r * it.lds + c;
    for (int q = 0; q < it.nslots; ++q) s += p[q * it.slot_stride];
    it.dst[(int64_t)r * it.ldd + c] = s;
  }
  if (set_tfar && blockIdx.x == 0 && threadIdx.x == 0) clk->t_far = t;
}

void launch_reduce(const RItem* items, int nitems, const Clock* clk, int set_tfar, hipStream_t s) {
  if (nitems <= 0) return;
  reduce_kernel<<<nitems, 256, 0, s>>>(items, const_cast<Clock*>(clk), set_tfar);
}

// ------------------------------------------------------------------------------------------
// Thread mapping shared by the per-step kernels: a block owns BT = min(B, 64) consecutive
// trajectories (fastest index, so lanes are coalesced) and DL = 256/BT DOF lanes.
struct Lanes {
  int BT, DL, bl, dl, b;
  bool ok;
  __device__ Lanes(int B) {
    BT = B < 64 ? B : 64;
    DL = WG / BT;
    bl = threadIdx.x % BT;
    dl = threadIdx.x / BT;
    b = blockIdx.x * BT + bl;
    ok = (dl < DL) && (b < B);
  }
};

__global__ __launch_bounds__(256) void potsel_kernel(const StepDev* __restrict__ sd,
                                                     const double* __restrict__ Y,
                                                     const double* __restrict__ X) {
  __shared__ double red[WG];
  __shared__ int hit[64];
  const int B = sd->B, nph = sd->nph;
  Lanes L(B);
  double m = 0.0;
  if (L.ok)
    for (int d = L.dl; d < nph; d += L.DL) {
      const int64_t i = (int64_t)d * B + L.b;
      m = fmax(m, fabs(X[i] - sd->Q0[i]));
    }
  red[threadIdx.x] = L.ok ? m : 0.0;
  __syncthreads();
  if (L.dl == 0 && L.ok) {
    double mm = 0.0;
    bool nan = false;
    for (int x = 0; x < L.DL; ++x) {
      const double v = red[x * L.BT + L.bl];
      nan |= (v != v);
      mm = fmax(mm, v);
    }
    // md.py:776: max(abs(dif)) < 10e-10, and md.q0 = [] before the first evaluation
    hit[L.bl] = (sd->qvalid[L.b] != 0) && !nan && (mm < 10e-10);
  }
  __syncthreads();
  if (L.ok && !hit[L.bl]) {
    for (int d = L.dl; d < nph; d += L.DL) {
      const int64_t i = (int64_t)d * B + L.b;
      sd->Fc[i] = -1.0 * Y[i];  // f = -1.0*mdot(dyn, q)  (md.py:467)
      sd->Q0[i] = X[i];
    }
  }
  if (L.ok && L.dl == 0) sd->qvalid[L.b] = 1;
}

void launch_potsel(const StepDev* sd, const double* Y, const double* X, int B, hipStream_t s) {
  const int BT = B < 64 ? B : 64;
  potsel_kernel<<<(B + BT - 1) / BT, WG, 0, s>>>(sd, Y, X);
}

// bath force of bath j at DOF-local index k (baths.py:232-255, 452-458):
//   noise[tn] - c*(K0.x + S) - Kq.q   (Kq = -V(exim - zeta1); V*zeta2 folded into K0)
__device__ __forceinline__ double bath_force(const BathDev& bd, int k, int b, int B, int tn,
                                             int par) {
  const int64_t kb = (int64_t)k * B + b;
  double f = bd.noise[((int64_t)tn * bd.nc + k) * B + b] -
             bd.c * (bd.Y[kb] + bd.S[(int64_t)par * bd.ncp * B + kb]);
  if (bd.has_q) f -= bd.Yq[kb];
  return f;
}

__global__ __launch_bounds__(256) void phaseA_kernel(const StepDev* __restrict__ sd,
                                                     const Clock* __restrict__ clk) {
  __shared__ double red[WG];
  const int B = sd->B, nph = sd->nph, nb = sd->nbath;
  Lanes L(B);
  const int64_t t = load_t(clk);
  const int tn = (int)(t % sd->nmd);
  const int par = (int)(t & 1);
  const double dt = sd->dt, dt2 = dt * dt;
  const int d0 = blockIdx.y * sd->dchunk;
  const int d1 = min(nph, d0 + sd->dchunk);
  double cur[MAXBATH];
#pragma unroll
  for (int j = 0; j < MAXBATH; ++j) cur[j] = 0.0;
  double e = 0.0;
  if (L.ok)
    for (int d = d0 + L.dl; d < d1; d += L.DL) {
      const int64_t i = (int64_t)d * B + L.b;
      const double p = sd->P[i], q = sd->Q[i];
      double f = sd->Fc[i];  // potforce(q_t)
#pragma unroll
      for (int j = 0; j < MAXBATH; ++j) {
        if (j < nb) {
          const BathDev& bd = sd->bath[j];
          const int k = bd.inv[d];
          if (k >= 0) {
            const double fb = bath_force(bd, k, L.b, B, tn, par);
            f += fb;           // pf = pf + fbaths[i]   (md.py:432-434)
            cur[j] += fb * p;  // cur[t] = fbaths[i].p  (md.py:397)
          }
        }
      }
      e += p * p;
      const double ph = p + f * dt / 2.0;            // md.py:391
      const double qt = q + p * dt + f * dt2 / 2.0;  // md.py:392
      sd->Ph[i] = ph;
      sd->Qt[i] = qt;
#pragma unroll
      for (int j = 0; j < MAXBATH; ++j) {
        if (j < nb) {
          const BathDev& bd = sd->bath[j];
          const int k = bd.inv[d];
          if (k >= 0) {
            bd.Xcur[(int64_t)k * B + L.b] = ph;
            if (bd.has_q) bd.Xq[(int64_t)k * B + L.b] = qt;
          }
        }
      }
    }
  for (int qd = 0; qd <= nb; ++qd) {
    double v = e;
#pragma unroll
    for (int j = 0; j < MAXBATH; ++j)
      if (j == qd && j < nb) v = cur[j];
    red[threadIdx.x] = L.ok ? v : 0.0;
    __syncthreads();
    if (L.dl == 0 && L.ok) {
      double s = 0.0;
      for (int x = 0; x < L.DL; ++x) s += red[x * L.BT + L.bl];
      sd->part[((int64_t)blockIdx.y * (nb + 1) + qd) * B + L.b] = s;
    }
    __syncthreads();
  }
}

__device__ __forceinline__ double id1_force(const StepDev* sd, int d, int b, int B, int t1,
                                            int par1) {
  double f = sd->Fc[(int64_t)d * B + b];  // potforce(q~)
#pragma unroll
  for (int j = 0; j < MAXBATH; ++j) {
    if (j < sd->nbath) {
      const BathDev& bd = sd->bath[j];
      const int k = bd.inv[d];
      if (k >= 0) f += bath_force(bd, k, b, B, t1, par1);
    }
  }
  return f;
}

__global__ __launch_bounds__(256) void phaseB_kernel(const StepDev* __restrict__ sd,
                                                     const Clock* __restrict__ clk) {
  const int B = sd->B, nph = sd->nph, nb = sd->nbath;
  Lanes L(B);
  const int64_t t = load_t(clk);
  const int t1 = (int)((t + 1) % sd->nmd);
  const int par1 = (int)((t + 1) & 1);
  const double dt = sd->dt;
  const int d0 = blockIdx.y * sd->dchunk;
  const int d1 = min(nph, d0 + sd->dchunk);
  if (!L.ok) return;
  for (int d = d0 + L.dl; d < d1; d += L.DL) {
    bool inb = false;
#pragma unroll
    for (int j = 0; j < MAXBATH; ++j)
      if (j < nb && sd->bath[j].inv[d] >= 0) inb = true;
    if (!inb) continue;  // p1 only feeds the bath friction terms
    const double f = id1_force(sd, d, L.b, B, t1, par1);
    const double p1 = sd->Ph[(int64_t)d * B + L.b] + dt * f / 2.0;  // md.py:402
#pragma unroll
    for (int j = 0; j < MAXBATH; ++j) {
      if (j < nb) {
        const BathDev& bd = sd->bath[j];
        const int k = bd.inv[d];
        if (k >= 0) bd.Xcur[(int64_t)k * B + L.b] = p1;
      }
    }
  }
}

__global__ __launch_bounds__(256) void phaseC_kernel(const StepDev* __restrict__ sd,
                                                     Clock* __restrict__ clk) {
  const int B = sd->B, nph = sd->nph, nb = sd->nbath;
  Lanes L(B);
  const int64_t t = load_t(clk);
  const int tn = (int)(t % sd->nmd);
  const int t1 = (int)((t + 1) % sd->nmd);
  const int par1 = (int)((t + 1) & 1);
  const double dt = sd->dt;
  const int d0 = blockIdx.y * sd->dchunk;
  const int d1 = min(nph, d0 + sd->dchunk);
  if (L.ok) {
    for (int d = d0 + L.dl; d < d1; d += L.DL) {
      const int64_t i = (int64_t)d * B + L.b;
      const double f = id1_force(sd, d, L.b, B, t1, par1);
      double p2 = sd->Ph[i] + dt * f / 2.0;  // md.py:404
      double qt = sd->Qt[i];
      if (sd->cmask[d]) {  // ApplyConstraint (md.py:407-408, 782-794)
        p2 = 0.0;
        qt = 0.0;
      }
      sd->P[i] = p2;
      sd->Q[i] = qt;
      sd->Flast[i] = f;
#pragma unroll
      for (int j = 0; j < MAXBATH; ++j) {
        if (j < nb) {
          const BathDev& bd = sd->bath[j];
          const int k = bd.inv[d];
          if (k >= 0) {
            // history push of p_{t+1} (rpadleft, md.py:387 of the next step), mirrored slot
            const int64_t slot = pmod(t + 1, bd.R);
            double* h = bd.H + (int64_t)k * bd.ldh + L.b;
            h[slot * B] = p2;
            h[(slot + bd.R) * B] = p2;
            if (bd.has_q) bd.Xq[(int64_t)k * B + L.b] = qt;
          }
        }
      }
    }
    // close step t's heat current and kinetic energy from phase A's partial sums (fixed order)
    if (blockIdx.y == 0) {
      for (int qd = L.dl; qd <= nb; qd += L.DL) {
        double s = 0.0;
        for (int y = 0; y < sd->ndblk; ++y) s += sd->part[((int64_t)y * (nb + 1) + qd) * B + L.b];
        if (qd < nb) {
          sd->bath[qd].cur[(int64_t)tn * B + L.b] = s;
        } else {
          sd->etot[(int64_t)tn * B + L.b] = 0.5 * s;  // md.py:161-165, 383
        }
      }
    }
  }
  // the last block to finish advances the step counter (all blocks read t before arriving)
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned total = gridDim.x * gridDim.y;
    const unsigned old = atomicAdd(&clk->arrive, 1u);
    if (old == total - 1) {
      clk->arrive = 0;
      __hip_atomic_store(&clk->t, t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence();
    }
  }
}

static inline dim3 phase_grid(int B, int ndblk) {
  const int BT = B < 64 ? B : 64;
  return dim3((B + BT - 1) / BT, ndblk);
}

void launch_phaseA(const StepDev* sd, const Clock* clk, int B, int nph, int ndblk, hipStream_t s) {
  (void)nph;
  phaseA_kernel<<<phase_grid(B, ndblk), WG, 0, s>>>(sd, clk);
}
void launch_phaseB(const StepDev* sd, const Clock* clk, int B, int nph, int ndblk, hipStream_t s) {
  (void)nph;
  phaseB_kernel<<<phase_grid(B, ndblk), WG, 0, s>>>(sd, clk);
}
void launch_phaseC(const StepDev* sd, Clock* clk, int B, int nph, int ndblk, hipStream_t s) {
  (void)nph;
  phaseC_kernel<<<phase_grid(B, ndblk), WG, 0, s>>>(sd, clk);
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
                              uint64_t seed, uint64_t traj_offset) {
  const int64_t n = nfreq * ncp * B;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e % B;
    const int64_t k = (e / B) % ncp;
    const int64_t w = e / (B * ncp);
    x[e] = (k < nc) ? philox_normal(seed, (uint32_t)k, (uint32_t)w, (uint32_t)(traj_offset + b)) : 0.0;
  }
}

void launch_philox_normal(double* x, int64_t nfreq, int64_t ncp, int64_t nc, int64_t B,
                          uint64_t seed, uint64_t traj_offset, hipStream_t s) {
  philox_kernel<<<2048, 256, 0, s>>>(x, nfreq, ncp, nc, B, seed, traj_offset);
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

int launch_fft_noise(const double* a, double* noise, const double* tw, int64_t nmd, int64_t nc,
                     int64_t arows, int64_t B, int is_complex, double scale, hipStream_t s) {
  int logn = 0;
  while ((1ll << logn) < nmd) ++logn;
  if ((1ll << logn) != nmd || logn < 1) return -1;
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

}  // namespace gle
