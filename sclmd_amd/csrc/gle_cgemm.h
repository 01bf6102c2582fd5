// Far-field GEMM item of the spectral ladder levels (cgemm_item), shared by the standalone
// far-field kernel (gle_kernels.hip, background schedule and priming) and the per-step chain kernel
// (gle_chain.hip, fused schedule: the items ride in the chain launches below the chain tiles).
#pragma once
#include <hip/hip_runtime.h>

#include "gle_internal.h"

namespace gle {

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int64_t cg_pmod(int64_t a, int64_t m) {
  int64_t r = a % m;
  return r < 0 ? r + m : r;
}

// ------------------------------------------------------------------------------------------
// Spectral level contraction as a batched real GEMM: for every (bath, frequency f, Gauss part g)
//   T_g(f)[nc x B] = sum_{m < M} A_g(f, m)[nc x nc] . X_g(f, sigma - m)[nc x B],   sigma = T / P
// (the Gauss 3-multiplication of the complex per-frequency products: 3 real products, not 4).
// A workgroup owns 64 rows x 16 RN columns of one T_g(f): each of its 4 waves streams its 16-row
// tile's A fragments from HBM into registers one chunk ahead; X moves through a double-buffered
// LDS chunk of CG_KC k-steps shared by the 4 waves.  No split over k: no partials, no reduce.
constexpr int CG_KC = 8;   // k-steps per LDS chunk
constexpr int CG_LD = 80;  // LDS row stride (doubles): 64 columns + 16, ds_read_b64 at most 2-way

typedef const __attribute__((address_space(1))) double gdbl;

// The far-field operand K-hat (GBs, each fragment read once per block) streams through with
// non-temporal loads, so it does not evict the per-step chain's matrices (~2 MB per XCD with the
// XCD-aware chain tile order) from the L2s.  CG_NT=0: default cache policy.
#ifndef CG_NT
#define CG_NT 1
#endif
#if CG_NT
#define CG_ALOAD(p) __builtin_nontemporal_load(p)
#else
#define CG_ALOAD(p) (*(p))
#endif

// Prefetch rings.  A fragments (HBM, the streamed operand) go AD chunks ahead of the MFMAs into a
// ring of AD + 1 register chunks; X (segment ring, L2/MALL) goes XD chunks ahead into a ring of XD
// register chunks and from there into the other LDS buffer at the end of the chunk before its use.
// With one workgroup per CU (one wave per SIMD, the far-field chunking beside the chain) nothing
// else on the SIMD hides a load: the rings have to cover an HBM round trip by themselves.
#ifndef CG_AD
#define CG_AD 2
#endif
#ifndef CG_XD
#define CG_XD 1
#endif
template <int RN, int KC, int AD, int XD, int DBG = 0>
__device__ __forceinline__ void cgemm_item(const CgItem& it, int64_t tseg, double (&xs)[2][4 * KC * CG_LD]) {
  static_assert(XD == 1 || XD == 2, "X ring of one or two chunks");
  static_assert((AD + 1) % XD == 0, "the A ring period carries the X ring's");
  constexpr int NT = 16 * RN;
  constexpr int XPT = 4 * KC * NT / 256;  // X doubles per thread per chunk
  constexpr int TPR = NT / XPT;              // staging threads per X row
  static_assert(4 * KC * TPR == 256, "one X row per TPR threads, every thread stages");
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int brow = lane >> 4, bcol = lane & 15;
  const int S = it.ns;  // k-steps of this item: [it.s0, it.s0 + S) of the M nks of T_g(f)
  const int nch = (S + KC - 1) / KC;
  const bool active = wave < it.nrt;
  // global address space: flat loads would also count on lgkmcnt, and every LDS-read wait before an
  // MFMA would then drain the HBM prefetches in flight
  gdbl* Aw = (gdbl*)(it.A + (int64_t)(active ? wave : 0) * it.a_rt + (int64_t)it.s0 * 64 + lane);
  const int xr = tid / TPR, xc = (tid % TPR) * XPT;
  const int tbase = (int)cg_pmod(tseg, it.Rseg);  // ring slot of segment tseg (32-bit from here on)
  // Loads are branch-free (clamped address, zero by multiplication): a branch around a load makes
  // the waitcnt pass drain every load in flight.
  double xv[XD][XPT], av[AD + 1][KC];
  d4 acc[RN];
#pragma unroll
  for (int n = 0; n < RN; ++n) acc[n] = d4{0.0, 0.0, 0.0, 0.0};
#ifdef GLE_BOUNDS
#define CG_BCHK_X(u)                                                                                  \
  GLE_BCHK(it.X + (int64_t)(4 * ks_ + (xr & 3)) * it.ldx + (int64_t)slot_ * it.cs + it.col0 + xc + (u))
#define CG_BCHK_A(s)                                                                                  \
  GLE_BCHK(it.A + (int64_t)(active ? wave : 0) * it.a_rt + (int64_t)it.s0 * 64 + lane + (int64_t)(s) * 64)
#else
#define CG_BCHK_X(u) ((void)0)
#define CG_BCHK_A(s) ((void)0)
#endif
#define CG_LOAD_X(c, XV)                                                                              \
  do {                                                                                                \
    const int s0_ = (c) * KC + (xr >> 2);                                                          \
    const int sc_ = it.s0 + (s0_ < S ? s0_ : S - 1);                                                  \
    const int i_ = (int)((unsigned)sc_ / (unsigned)it.nks), ks_ = sc_ - i_ * it.nks;                  \
    int slot_ = tbase - i_;                                                                           \
    slot_ += slot_ < 0 ? it.Rseg : 0; /* i < M < Rseg */                                              \
    gdbl* xp_ = (gdbl*)(it.X + (int64_t)(4 * ks_ + (xr & 3)) * it.ldx + (int64_t)slot_ * it.cs +      \
                        it.col0 + xc);                                                                \
    _Pragma("unroll") for (int u = 0; u < XPT; ++u) {                                               \
      CG_BCHK_X(u);                                                                                   \
      XV[u] = xp_[u];                                                                                 \
    }                                                                                                 \
  } while (0)
  /* rows past S are stored as zeros (the multiply waits for the load only here, at the store) */
#define CG_STORE_X(c, buf, XV)                                                                        \
  do {                                                                                                \
    const double m_ = (c) * KC + (xr >> 2) < S ? 1.0 : 0.0;                                        \
    _Pragma("unroll") for (int u = 0; u < XPT; ++u) xs[buf][xr * CG_LD + xc + u] = XV[u] * m_;        \
  } while (0)
#define CG_LOAD_A(c, AV)                                                                              \
  do {                                                                                                \
    _Pragma("unroll") for (int u = 0; u < KC; ++u) {                                               \
      const int s0_ = (c) * KC + u;                                                                \
      CG_BCHK_A(s0_ < S ? s0_ : S - 1);                                                               \
      AV[u] = (DBG & 1) ? 1e-3 * (s0_ + 1) : CG_ALOAD(&Aw[(int64_t)(s0_ < S ? s0_ : S - 1) * 64]); /* masked */ \
    }                                                                                                 \
  } while (0)
  // chunk c (ring position r = c mod (AD + 1), a compile-time constant inside the unrolled period):
  // X chunk c + XD into the X ring, A chunk c + AD into the A registers chunk c - 1 used, MFMAs on
  // A chunk c and the LDS buffer c & 1, then X chunk c + 1 into the other LDS buffer.  X is issued
  // first: vmcnt retires in order, so the X store at the end waits for X (and older loads) only.
  CG_LOAD_A(0, av[0]);
  if (AD > 1) CG_LOAD_A(1, av[1 % (AD + 1)]);
  if (AD > 2) CG_LOAD_A(2, av[2 % (AD + 1)]);
  if (AD > 3) CG_LOAD_A(3, av[3 % (AD + 1)]);
  if (AD > 4) CG_LOAD_A(4, av[4 % (AD + 1)]);
  if (AD > 5) CG_LOAD_A(5, av[5 % (AD + 1)]);
  if (AD > 6) CG_LOAD_A(6, av[6 % (AD + 1)]);
  static_assert(AD <= 7, "prologue covers AD <= 7");
  CG_LOAD_X(0, xv[0]);
  if (XD > 1) CG_LOAD_X(1, xv[1 % XD]);
  CG_STORE_X(0, 0, xv[0]);
  __syncthreads();
  for (int c0 = 0; c0 < nch; c0 += AD + 1) {
#pragma unroll
    for (int r = 0; r <= AD; ++r) {
      const int c = c0 + r;
      if (c >= nch) break;
      if (!(DBG & 4)) CG_LOAD_X(c + XD, xv[r % XD]);
      CG_LOAD_A(c + AD, av[(r + AD) % (AD + 1)]);
      const double* xb_ = xs[c & 1] + brow * CG_LD + bcol;
      if constexpr ((DBG & 8) != 0) {
        // timing experiment: hold the workgroup for the chunk's MFMA time without using the pipe
        __builtin_amdgcn_s_sleep(KC * RN);
        acc[0][0] += av[r][0];
      } else {
#pragma unroll
      for (int u = 0; u < KC; ++u) {
        const double a_ = av[r][u] * ((active && c * KC + u < S) ? 1.0 : 0.0);
#pragma unroll
        for (int n = 0; n < RN; ++n)
          acc[n] = __builtin_amdgcn_mfma_f64_16x16x4f64(a_, (DBG & 2) ? a_ * (n + 1) : xb_[4 * u * CG_LD + 16 * n],
                                                        acc[n], 0, 0, 0);
      }
      }
      if (!(DBG & 4)) {
        CG_STORE_X(c + 1, (c & 1) ^ 1, xv[(r + 1) % XD]);
        __syncthreads();
      }
    }
  }
#undef CG_LOAD_A
#undef CG_STORE_X
#undef CG_LOAD_X
#undef CG_BCHK_X
#undef CG_BCHK_A
  if (active) {
    // f64 MFMA C/D map: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
    for (int n = 0; n < RN; ++n)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * wave + brow + 4 * q, col = 16 * n + bcol;
        if (row < it.nrows && col < it.ncols) {
          GLE_BCHK(&it.out[(int64_t)row * it.ldo + col]);
          // global address space (a flat access would count on lgkmcnt: see Aw)
          __attribute__((address_space(1))) double* o =
              (__attribute__((address_space(1))) double*)&it.out[(int64_t)row * it.ldo + col];
          // fused schedule: later k-splits of a product add to the earlier ones' sum (one writer
          // per element per launch, splits in launch order: deterministic)
          *o = it.accum ? *o + acc[n][q] : acc[n][q];
        }
      }
  }
}

// Two-plane Gauss item (it.g3 = 1, 0 < f < P): the three real products of one output tile from
// Khat's two planes (Kr, Ki: each fragment streamed from HBM once, 2/3 of the three-plane bytes) and
// the segment spectra's two planes (Xr, Xi), with the Gauss sums formed in registers:
//   T_0 += Kr (Xr + Xi),  T_1 += (Kr + Ki) Xi,  T_2 += (Ki - Kr) Xr
// (the same fp64 sums the three-plane layout stored, so the same results bit for bit).  X moves
// through a double-buffered LDS chunk of both planes (row stride 16 RN + 16 doubles); three
// accumulator sets per wave.
template <int RN, int KC>
struct Cg3 {
  static constexpr int NT = 16 * RN;
  static constexpr int LD = NT + 16;
  static constexpr int PLANE = 4 * KC * LD;      // doubles of one X plane chunk in LDS
  static constexpr int LDS = 2 * 2 * PLANE;      // two buffers x two planes
};

template <int RN, int KC, int AD>
__device__ __forceinline__ void cgemm_item3(const CgItem& it, int64_t tseg, double* xs) {
  using C = Cg3<RN, KC>;
  constexpr int NT = C::NT, LD = C::LD, PL = C::PLANE;
  constexpr int XPT = 2 * 4 * KC * NT / 256;  // X doubles per thread per chunk (both planes)
  constexpr int TPR = NT / XPT;                // staging threads per X row
  static_assert(2 * 4 * KC * TPR == 256, "one X row of one plane per TPR threads, every thread stages");
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int brow = lane >> 4, bcol = lane & 15;
  const int S = it.ns;
  const int nch = (S + KC - 1) / KC;
  const bool active = wave < it.nrt;
  gdbl* Aw = (gdbl*)(it.A + (int64_t)(active ? wave : 0) * it.a_rt + (int64_t)it.s0 * 64 + lane);
  const int64_t apl = it.a_pl;
  const int xpl = tid / (4 * KC * TPR);                 // plane this thread stages (0: Xr, 1: Xi)
  const int xr = (tid % (4 * KC * TPR)) / TPR, xc = (tid % TPR) * XPT;
  const double* Xp = it.X + (xpl ? it.x_pl : 0);
  const int tbase = (int)cg_pmod(tseg, it.Rseg);
  double xv[XPT], ar[AD + 1][KC], ai[AD + 1][KC];
  d4 acc[3][RN];
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int n = 0; n < RN; ++n) acc[g][n] = d4{0.0, 0.0, 0.0, 0.0};
#ifdef GLE_BOUNDS
#define CG3_BCHK_X(u) GLE_BCHK(Xp + (int64_t)(4 * ks_ + (xr & 3)) * it.ldx + (int64_t)slot_ * it.cs + it.col0 + xc + (u))
#define CG3_BCHK_A(s, o) GLE_BCHK(it.A + (int64_t)(active ? wave : 0) * it.a_rt + (int64_t)it.s0 * 64 + lane + (int64_t)(s) * 64 + (o))
#else
#define CG3_BCHK_X(u) ((void)0)
#define CG3_BCHK_A(s, o) ((void)0)
#endif
#define CG3_LOAD_X(c)                                                                                 \
  do {                                                                                                \
    const int s0_ = (c) * KC + (xr >> 2);                                                          \
    const int sc_ = it.s0 + (s0_ < S ? s0_ : S - 1);                                                  \
    const int i_ = (int)((unsigned)sc_ / (unsigned)it.nks), ks_ = sc_ - i_ * it.nks;                  \
    int slot_ = tbase - i_;                                                                           \
    slot_ += slot_ < 0 ? it.Rseg : 0;                                                                 \
    gdbl* xp_ = (gdbl*)(Xp + (int64_t)(4 * ks_ + (xr & 3)) * it.ldx + (int64_t)slot_ * it.cs + it.col0 + xc); \
    _Pragma("unroll") for (int u = 0; u < XPT; ++u) {                                               \
      CG3_BCHK_X(u);                                                                                  \
      xv[u] = xp_[u];                                                                                 \
    }                                                                                                 \
  } while (0)
#define CG3_STORE_X(c, buf)                                                                           \
  do {                                                                                                \
    const double m_ = (c) * KC + (xr >> 2) < S ? 1.0 : 0.0;                                        \
    _Pragma("unroll") for (int u = 0; u < XPT; ++u) xs[(buf) * 2 * PL + xpl * PL + xr * LD + xc + u] = xv[u] * m_; \
  } while (0)
#define CG3_LOAD_A(c, R)                                                                              \
  do {                                                                                                \
    _Pragma("unroll") for (int u = 0; u < KC; ++u) {                                               \
      const int s0_ = (c) * KC + u;                                                                \
      const int64_t o_ = (int64_t)(s0_ < S ? s0_ : S - 1) * 64;                                       \
      CG3_BCHK_A(s0_ < S ? s0_ : S - 1, 0);                                                           \
      CG3_BCHK_A(s0_ < S ? s0_ : S - 1, apl);                                                         \
      ar[R][u] = CG_ALOAD(&Aw[o_]);                                                                   \
      ai[R][u] = CG_ALOAD(&Aw[o_ + apl]);                                                             \
    }                                                                                                 \
  } while (0)
  CG3_LOAD_A(0, 0);
  if (AD > 1) CG3_LOAD_A(1, 1 % (AD + 1));
  if (AD > 2) CG3_LOAD_A(2, 2 % (AD + 1));
  if (AD > 3) CG3_LOAD_A(3, 3 % (AD + 1));
  static_assert(AD <= 4, "prologue covers AD <= 4");
  CG3_LOAD_X(0);
  CG3_STORE_X(0, 0);
  __syncthreads();
  for (int c0 = 0; c0 < nch; c0 += AD + 1) {
#pragma unroll
    for (int r = 0; r <= AD; ++r) {
      const int c = c0 + r;
      if (c >= nch) break;
      CG3_LOAD_X(c + 1);
      CG3_LOAD_A(c + AD, (r + AD) % (AD + 1));
      const double* xb_ = xs + (c & 1) * 2 * PL + brow * LD + bcol;
#pragma unroll
      for (int u = 0; u < KC; ++u) {
        const double m_ = (active && c * KC + u < S) ? 1.0 : 0.0;
        const double kr = ar[r][u] * m_, ki = ai[r][u] * m_;
        const double k1 = kr + ki, k2 = ki - kr;
#pragma unroll
        for (int n = 0; n < RN; ++n) {
          const double xre = xb_[4 * u * LD + 16 * n], xim = xb_[PL + 4 * u * LD + 16 * n];
          acc[0][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(kr, xre + xim, acc[0][n], 0, 0, 0);
          acc[1][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(k1, xim, acc[1][n], 0, 0, 0);
          acc[2][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(k2, xre, acc[2][n], 0, 0, 0);
        }
      }
      CG3_STORE_X(c + 1, (c & 1) ^ 1);
      __syncthreads();
    }
  }
#undef CG3_LOAD_A
#undef CG3_STORE_X
#undef CG3_LOAD_X
#undef CG3_BCHK_X
#undef CG3_BCHK_A
  if (active) {
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int n = 0; n < RN; ++n)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = 16 * wave + brow + 4 * q, col = 16 * n + bcol;
          if (row < it.nrows && col < it.ncols) {
            __attribute__((address_space(1))) double* o =
                (__attribute__((address_space(1))) double*)&it.out[g * it.o_pl + (int64_t)row * it.ldo + col];
            GLE_BCHK(o);
            *o = it.accum ? *o + acc[g][n][q] : acc[g][n][q];
          }
        }
  }
}

// k-steps per LDS chunk of the two-plane items: 64-column tiles take chunks of 2 (three accumulator
// sets of 4 tiles fit the kernel's register budget without spilling, and the two X planes of a
// chunk the LDS of the one-plane item's chunk of 4)
template <int RN, int KC>
constexpr int cg3_kc() {
  return RN == 4 ? 2 : KC;
}

// doubles of LDS a far-field workgroup needs for either item kind
template <int RN, int KC>
constexpr int cg_lds_doubles() {
  return Cg3<RN, cg3_kc<RN, KC>()>::LDS > 2 * 4 * KC * CG_LD ? Cg3<RN, cg3_kc<RN, KC>()>::LDS : 2 * 4 * KC * CG_LD;
}

// one item of either kind (the kind is item-uniform)
// (the planner gives two-plane items only to levels of <= 32-column items: the 64-column kernel
// carries the one-plane path alone and keeps its register budget)
template <int RN, int KC, int AD, int XD, int DBG = 0>
__device__ __forceinline__ void cgemm_any(const CgItem& it, int64_t tseg, double* lds) {
  if constexpr (RN <= 2) {
    if (it.g3) {
      cgemm_item3<RN, cg3_kc<RN, KC>(), (AD < 4 ? AD : 4)>(it, tseg, lds);
      return;
    }
  }
  cgemm_item<RN, KC, AD, XD, DBG>(it, tseg, *reinterpret_cast<double(*)[2][4 * KC * CG_LD]>(lds));
}

}  // namespace gle
