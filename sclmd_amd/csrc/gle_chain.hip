// Per-step chain of one md.vv (md.py:367-411) on gfx950: three launches A, B, C.
//
//   A  CH_DOF  Y0 = K0.p_t (+ Kq.q_t, + dyn.q_t when md.potforce's cache may miss), then for the
//              tile's DOFs: F0 = Fpot(q_t) + sum_b bforce_b(t) (baths.py:232-255, 452-458), heat
//              current (md.py:397), kinetic energy (md.py:383), p_half, q~ (md.py:391-392)
//      CH_SFIN S(t+1) = K_1.p_t + near-field partials (lags >= 2) + ladder levels
//   B  CH_DOF  Y1 = K0.p_half, Kq.q~, dyn.q~; F1(p_half) and p1 (md.py:401-402)
//      CH_RAW  near-field partials for target t+2
//   C  CH_DOF  Y2 = K0.p1; F1(p1), p2, constraints (md.py:403-408, 782-794), history push
//              (rpadleft, md.py:386-387), cache distances for the next step's id0 call
//      CH_RAW  near-field partials for target t+2
//
// A workgroup owns a whole output tile (no split over workgroups): its NW waves split the tile's
// k-steps, each wave keeps a batch of operand loads in flight at once, the partial tiles meet in
// LDS and are added in a fixed order (deterministic).  Everything the epilogue reads that does not
// depend on the products is loaded before the products start.  The newest p of every bath lives in
// a small slot-major near ring, so per-step operands are contiguous (no TLB walk per k-step as in
// the 2R-slot history ring the ladder reads).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <vector>

#include "gle_internal.h"
#include "gle_cgemm.h"

namespace gle {

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) double gdouble;

// global-address-space view of a pointer: loads and stores become global_* instructions (flat ones
// also count on lgkmcnt and would make every scalar-load wait drain the vector loads in flight)
#ifndef GLE_BOUNDS
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* G(T* p) {
  return (__attribute__((address_space(1))) T*)p;
}
#else
// audit build: every G(p)[i] / *G(p) access is checked against the live allocations
template <class T>
struct BndPtr {
  T* p;
  int site;
  __device__ T& operator[](int64_t i) const {
    bcheck(p + i, (int)sizeof(T), site);
    return p[i];
  }
  __device__ T& operator*() const {
    bcheck(p, (int)sizeof(T), site);
    return *p;
  }
};
template <class T>
__device__ __forceinline__ BndPtr<T> Gb(T* p, int site) {
  return BndPtr<T>{p, site};
}
#define G(p) Gb((p), __LINE__)
#endif

__device__ __forceinline__ int64_t cmod(int64_t a, int64_t m) {
  int64_t r = a % m;
  return r < 0 ? r + m : r;
}

// k-steps a wave keeps in flight per batch (16-wave workgroups have 128 registers per lane).
// The batch sets the kernel's register count: 8/4/2 k-steps with 4 waves per SIMD (128 VGPRs)
// keeps every tile of a stage resident at once, even beside the background ladder kernels; a
// deeper batch (24/12/8: 190 VGPRs, 2 waves per SIMD) left a third of stage A's tiles waiting for
// a slot and measured 900k vs 1.04M traj-steps/s at C3.
#ifndef CH_U1
#define CH_U1 8
#endif
#ifndef CH_U2
#define CH_U2 4
#endif
#ifndef CH_U4
#define CH_U4 2
#endif
#ifndef CH_WPE
#define CH_WPE 4
#endif
// CH_PRIO: wave issue priority of the chain kernels (s_setprio 0..3; the ladder kernels run at 0)
#ifndef CH_PRIO
#define CH_PRIO 3
#endif
// CH_PRIO_RAW: issue priority of the near-field partial tiles (default: that of the whole chain)
#ifndef CH_PRIO_RAW
#define CH_PRIO_RAW CH_PRIO
#endif
// FPOT_PRIO: the potential-force launch at the chain's issue priority
#ifndef FPOT_PRIO
#define FPOT_PRIO 0
#endif
// CH_DB: double-buffered operand batches (the next batch of a task in flight during this one's MFMAs)
#ifndef CH_DB
#define CH_DB 0
#endif
template <int RN, int NW>
struct Batch {
  static constexpr int U = NW >= 16 ? (RN == 1 ? 16 : (RN == 2 ? 6 : 3)) : (RN == 1 ? CH_U1 : (RN == 2 ? CH_U2 : CH_U4));
};

// GLE_CHAIN_DBG timeline: stamp 0 entry, 1 descriptor read, 2 products done, 3 end (100 MHz)
__device__ __forceinline__ void stamp(const StepDev* __restrict__ sd, int stage, int k, const StepArgs& ta) {
  if (stage > 2) stage = 2;  // the fused B+C and composed stages record into stage C's rows
  if (ta.dbg && threadIdx.x == 0 && (int)blockIdx.x < sd->dbg_ntile)
    G(sd->dbg)[((int64_t)stage * sd->dbg_ntile + blockIdx.x) * 4 + k] = __builtin_amdgcn_s_memrealtime();
}

// The wave's tasks: acc += A_s . X rows 4s..4s+3 over each task's k-steps; a task run ends in its
// LDS slot (16 x 16 RN doubles, row-major).  A task's k-steps are loaded in batches of U,
// double-buffered: the loads of batch j+1 are in flight while the MFMAs of batch j run, so a wave
// waits for about one memory round trip per task (<= CH_TPW) plus its MFMA chain instead of one
// round trip per batch.  skip: bit 0 drops the tasks of cond CH_HIT (no trajectory of the tile
// takes the potential-cache hit branch), bit 1 those of cond CH_MISS; their slots read as zeros.
//
// Accumulator sets (CH_NA, compile-time experiment): k-step u of a batch goes into set u mod NA,
// the NA x RN independent accumulators keep several MFMAs of a wave in flight, and the sets are
// added in fixed order when a run ends.  At C3 four sets measured 0.5-0.9 % slower per step than
// one: a launch is bound by the matrix pipes' throughput (~115k f64 MFMAs per fused launch over
// 1024 SIMDs, 73 % of them near-field tiles), not by one wave's accumulator chain.
#ifndef CH_NA
#define CH_NA 1
#endif
// md.potforce cache audit of a composed-step launch (StepArgs::xw).  Per trajectory b, nibble b % 16
// of word b / 16 of the step's audit slot collects, over the DOF tiles, bit 0: some tile's
// max|q~ - q_t| > 0, bit 1: some tile's is >= 1e-9 (or NaN), bits 2 / 3: the same for max|q_{t+1} -
// q~_t| -- so the step's maximum over all DOFs lies in (0, 1e-9), where md.potforce would reuse a force
// computed at another point (md.py:449-450, 767-779), iff bit 0 and not bit 1 (or 2 and not 3).
// Lanes 0 .. nw - 1 of wave 0 load the previous step's words and lane nw the stop word, with the tile
// descriptor; they are looked at after the tile's products, at the barrier those end with (the
// load's latency hides behind the products).  A hit or a set stop word makes a DOF tile return
// before any store (its state, ring and recordings; the S and near tiles write only the composed
// step's own buffers, which the replay rebuilds); the first stopping launch counts the trajectories
// and publishes the stop (the host replays from step t - 1 on the two-launch path, gle_api.hip
// xresolve).
__device__ __forceinline__ unsigned long long xw_hits(unsigned long long w) {
  return w & ~(w >> 1) & 0x5555555555555555ull;  // bit 4j: d1 hit of trajectory j, bit 4j + 2: d0 hit
}

struct XCheck {
  unsigned long long w = 0ull;
  int lane = -1;    // wave-0 lane holding a word: < nw nr word lane % nw of replica lane / nw, == nw nr
                    // the stop word
  int nw = 0;       // audit words (ceil(B / 16)) per replica
  int nr = 1;       // replicas (StepArgs::xR)
  bool on = false;  // a DOF tile of a composed-step launch of gle_run
  int* flags = nullptr;  // LDS: wave 0's vote
  // the barrier after the products; true: the tile stores nothing
  __device__ bool stop(const StepDev* __restrict__ sd, const StepArgs& ta) {
#if defined(XC_DBG) && (XC_DBG & 1)  // timing diagnostics only: no vote
    __syncthreads();
    return false;
#endif
    if (!on) {
      __syncthreads();
      return false;
    }
    const int nl = nw * nr;
    unsigned long long h = 0ull;
    int st = 0;
    if (threadIdx.x < 64) {
      // lane j < nw: word j ORed over the replicas (lanes r nw + j), then its hits
      unsigned long long x = 0ull;
      for (int r = 0; r < nr; ++r) x |= __shfl(w, r * nw + ((int)threadIdx.x % max(nw, 1)));
      h = (int)threadIdx.x < nw ? xw_hits(x) : 0ull;
      st = (lane == nl && w != 0ull) ? 1 : 0;
    }
    if (threadIdx.x < 64) {
      const int any = __any(h != 0ull || st);
      const int was = __any(st);
      if (threadIdx.x == 0) {
        flags[0] = any;
        flags[1] = was;
      }
    }
    __syncthreads();
    if (!flags[0]) return false;
    if (!flags[1] && blockIdx.x == 0 && threadIdx.x < 64) {  // the first stopping launch: count, publish
      typedef __attribute__((address_space(1))) unsigned long long gull;
      if (h) {
        __hip_atomic_fetch_add((gull*)(sd->guard + 0), (unsigned long long)__popcll(h & 0x1111111111111111ull),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add((gull*)(sd->guard + 1), (unsigned long long)__popcll(h & 0x4444444444444444ull),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (threadIdx.x == 0) {
        const unsigned long long v = (unsigned long long)ta.t + 1ull;
        __hip_atomic_store((gull*)ta.xstop, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ta.xstop_host, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    return true;
  }
};

template <int RN, int NW, bool GEMV = false>
__device__ __forceinline__ void products(const ChTile* __restrict__ T, int wave, int lane, int64_t t,
                                         double* lds, int skip) {
  // GEMV (one-trajectory plans, chain stage 5 = stage 4 at B = 1): a 16x16x4 MFMA would use 1 of its
  // 16 columns; each lane instead multiplies its own A element by the X value of its k row on the VALU
  static_assert(!GEMV || RN == 1, "GEMV tiles have one column tile");
  constexpr int U = Batch<RN, NW>::U;
  constexpr int NT = 16 * RN;
  constexpr int NA = (CH_NA / RN) > 1 ? (CH_NA / RN) : 1;  // independent accumulators: NA * RN
  static_assert(U % NA == 0, "a batch fills every accumulator set equally");
  const int nt = T->ntw[wave];
  const int brow = lane >> 4, bcol = lane & 15;
  d4 acc[NA][RN];
#pragma unroll
  for (int j = 0; j < NA; ++j)
#pragma unroll
    for (int n = 0; n < RN; ++n) acc[j][n] = d4{0.0, 0.0, 0.0, 0.0};
  // X columns past the tile's valid ones (trajectories >= B) read the last valid column: their
  // products land in output columns nobody stores, and no read leaves the operand's rows
  int xc[RN];
#pragma unroll
  for (int n = 0; n < RN; ++n) xc[n] = min(bcol + 16 * n, max(T->ncols - 1, 0));
  int cur = -1;
  double gacc = 0.0;  // GEMV: lane l's partial of row l % 16 over the k rows 4 s + l / 16
  auto flush = [&]() {
    if constexpr (GEMV) {
      // the four k-groups of a row are lanes l, l + 16, l + 32, l + 48: row sums in fixed order
      double v = gacc;
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (lane < 16) lds[cur * 16 * NT + lane * NT] = v;
      gacc = 0.0;
      return;
    }
#pragma unroll
    for (int n = 0; n < RN; ++n)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        double v = acc[0][n][q];
#pragma unroll
        for (int j = 1; j < NA; ++j) v += acc[j][n][q];
        lds[cur * 16 * NT + (brow + 4 * q) * NT + 16 * n + bcol] = v;
#pragma unroll
        for (int j = 0; j < NA; ++j) acc[j][n][q] = 0.0;
      }
  };
  for (int i = 0; i < CH_TPW; ++i) {
    if (i >= nt) break;
    const ChTask tk = T->task[wave][i];
    const bool off = (tk.cond == CH_HIT && (skip & 1)) || (tk.cond == CH_MISS && (skip & 2));
    if (tk.slot != cur) {
      if (cur >= 0) flush();
      cur = tk.slot;
    }
    if (off) continue;  // contributes nothing: a slot of skipped tasks only is flushed as zeros
    int64_t col = T->c0;
    if (tk.ring) col += cmod(t + tk.tshift, tk.ring) * (int64_t)tk.sst;
    gdouble* A = (gdouble*)(tk.A + lane);
    gdouble* X = (gdouble*)(tk.X + col);
    const int64_t ldx = tk.ldx;
    const int xr = tk.xrows - 1;  // < 0 when the task starts past the rows: all read the last row
    const int nks = tk.nks, aks = tk.a_ks;
    // Loads are branch-free (index clamped to the task's last k-step) and MFMAs past the end
    // multiply a zero A operand: a load under a branch makes the waitcnt pass drain every load in
    // flight at the join, which turned each batch into one round trip per k-step.
    double a0[U], b0[U][RN], a1[U], b1[U][RN];
    auto fetch = [&](int s0, double (&a)[U], double (&b)[U][RN]) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int s = min(s0 + u, nks - 1);
        const int64_t xo = (int64_t)min(4 * s + brow, xr) * ldx;
#ifdef GLE_BOUNDS
        bcheck(tk.A + lane + (int64_t)s * aks, 8, __LINE__);
        for (int n = 0; n < RN; ++n) bcheck(tk.X + col + xo + xc[n], 8, __LINE__);
#endif
#if defined(CH_DBG) && (CH_DBG & 1)  // timing diagnostics only (wrong results): no A loads
        a[u] = 1e-3 * (s + 1);
#else
        a[u] = A[(int64_t)s * aks];
#endif
#pragma unroll
        for (int n = 0; n < RN; ++n)
#if defined(CH_DBG) && (CH_DBG & 2)  // no X loads
          b[u][n] = 1e-3 * (xo + n);
#elif defined(CH_DBG) && (CH_DBG & 4)  // no X loads in the 64-column (near-field) tiles only
          b[u][n] = RN == 4 ? 1e-3 * (xo + n) : X[xo + xc[n]];
#else
          b[u][n] = X[xo + xc[n]];
#endif
      }
    };
    auto compute = [&](int s0, double (&a)[U], double (&b)[U][RN]) {
      if constexpr (GEMV) {
#pragma unroll
        for (int u = 0; u < U; ++u) gacc = fma(s0 + u < nks ? a[u] : 0.0, b[u][0], gacc);
        return;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const double av = s0 + u < nks ? a[u] : 0.0;
#pragma unroll
        for (int n = 0; n < RN; ++n)
          acc[u % NA][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b[u][n], acc[u % NA][n], 0, 0, 0);
      }
    };
    if constexpr (CH_DB != 0 && RN == 1) {  // CH_DB: the one-column-tile tasks only (registers)
      fetch(0, a0, b0);
      for (int s0 = 0; s0 < nks; s0 += 2 * U) {
        fetch(min(s0 + U, nks - 1), a1, b1);
        compute(s0, a0, b0);
        if (s0 + U >= nks) break;
        fetch(min(s0 + 2 * U, nks - 1), a0, b0);
        compute(s0 + U, a1, b1);
      }
    } else {
      (void)a1;
      (void)b1;
      for (int s0 = 0; s0 < nks; s0 += U) {
        fetch(s0, a0, b0);
        compute(s0, a0, b0);
      }
    }
  }
  if (cur >= 0) flush();
}

// DOF and S(t+1) tiles have the kernel's DRN columns (T->rn == DRN): products of that width only,
// so the 64-column near-field variant is not instantiated beside the DOF prologue's live values
// (it made the register allocator spill the DOF stages)
template <int NW, int RN, bool GV = false>
__device__ __forceinline__ void run_products_rn(const ChTile* __restrict__ T, int64_t t, double* lds, int skip = 0) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  products<RN, NW, GV && RN == 1>(T, wave, lane, t, lds, skip);
}

template <int NW, bool GV = false>
__device__ __forceinline__ void run_products(const ChTile* __restrict__ T, int64_t t, double* lds, int skip = 0) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  switch (T->rn) {
    case 1: products<1, NW, GV>(T, wave, lane, t, lds, skip); break;
    case 2: products<2, NW>(T, wave, lane, t, lds, skip); break;
    default: products<4, NW>(T, wave, lane, t, lds, skip); break;
  }
}

// output o at element e of a tile with slots of ss doubles, added in slot order.  An output has at
// most one slot per wave (fill_tasks*), so the NW slot reads are issued together (clamped to the
// output's slots, the extra ones masked): one LDS latency per output instead of one per slot.  The
// sum is 0 + v_0 + v_1 + ... in slot order as before (a masked +0.0 leaves every partial sum
// unchanged: none of them is -0.0), so the results are the same bits.
template <int NW>
__device__ __forceinline__ double out_sum(const ChTile* __restrict__ T, const double* lds, int o, int e, int ss) {
  const int b0 = T->ob[o], n = T->ob[o + 1] - b0;
  if constexpr (NW > 4) {  // 8-wave tiles (large baths): one slot at a time, within the register budget
    double r = 0.0;
    for (int s = 0; s < n; ++s) r += lds[(b0 + s) * ss + e];
    return r;
  }
  double v[NW];
#pragma unroll
  for (int s = 0; s < NW; ++s) v[s] = lds[(n > 0 ? b0 + min(s, n - 1) : 0) * ss + e];  // >= 1 slot (launch_nd)
  double r = 0.0;
#pragma unroll
  for (int s = 0; s < NW; ++s) r += s < n ? v[s] : 0.0;
  return r;
}

__device__ __forceinline__ unsigned long long* pmax_word(const StepDev* sd, int id, int par, int b) {
  return sd->pmax + ((int64_t)(id * 2 + par)) * sd->B + b;
}

// atomicMax through the global address space: HIP's atomicMax on a generic pointer is a flat atomic,
// which also counts on lgkmcnt, so the next LDS-read wait of the wave (the stamps' and the epilogue's
// descriptor reads) waited for the atomic's round trip through L2
__device__ __forceinline__ void gmax(unsigned long long* p, unsigned long long v) {
#ifdef GLE_BOUNDS
  bcheck(p, 8, __LINE__);
#endif
  __hip_atomic_fetch_max((__attribute__((address_space(1))) unsigned long long*)p, v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
}

// md.potforce's cache rule (sameq, md.py:449-450, 767-779) per trajectory: hit iff the cache is
// valid and max_d |q - q0| < 1e-9.  The max is one word per trajectory, accumulated with atomicMax
// on the bit pattern (non-negative doubles order like their bits; NaN exceeds every finite value).
__device__ __forceinline__ bool word_hit(unsigned long long w) {
  const double m = __longlong_as_double((long long)w);
  return m == m && m < 10e-10;
}

// ------------------------------------------------------------------------------------------
// DOF tiles: 16 DOFs x NT = 16 DRN trajectories; thread element i is e = threadIdx.x + i NW 64
// (row e / NT, column e % NT).
template <int NW, int DRN>
struct DofGeo {
  static constexpr int NT = 16 * DRN;
  static constexpr int NE = 16 * NT;
  static constexpr int EPT = (NE + NW * 64 - 1) / (NW * 64);
};

struct Elem {
  int r, d, b;
  int64_t i;
  bool ok, in;  // in: inside the tile's element range; ok: a real (DOF, trajectory)
};

template <int NW, int DRN>
__device__ __forceinline__ Elem elem_of(const ChTile* __restrict__ T, const StepDev* __restrict__ sd, int k) {
  using Geo = DofGeo<NW, DRN>;
  Elem E;
  const int e = threadIdx.x + k * NW * 64;
  E.in = e < Geo::NE;
  E.r = e / Geo::NT;
  E.d = T->row0 + E.r;
  E.b = T->c0 + (e % Geo::NT);
  E.ok = E.in && E.d < sd->nph && E.b < sd->B;
  E.i = (int64_t)E.d * sd->B + E.b;
  return E;
}

// bath-local row of the element's DOF in tile bath bd, or -1 (the inv load, for tiles whose bath
// rows are not an affine image of their DOFs, is under a tile-uniform branch only)
__device__ __forceinline__ int bath_row(const ChBath& bd, const Elem& E) {
  const bool in = bd.bath >= 0 && E.ok && ((bd.bmask >> E.r) & 1u);
  int k;
  if (bd.boff == CH_INV) k = G(bd.inv)[in ? E.d : 0];
  else k = E.d + bd.boff;
  return in ? k : -1;
}

// Prologue loads are unconditional (clamped indices; unused tile-bath slots point at a zero row)
// and their values are masked afterwards: a load under a divergent branch makes the waitcnt pass
// drain every load in flight at the join, so the loads would not overlap the products.
__device__ __forceinline__ int64_t bath_idx(const Elem& E, int k, int B) {
  return k >= 0 ? (int64_t)k * B + E.b : 0;
}

// Per-trajectory reductions over the tile's 16 rows, one LDS pass: quantity q of element e at
// red[q * NE + e]; column sums (fixed row order) / maxima by threads < NT.
template <int NW, int DRN>
__device__ __forceinline__ double col_red(const double* red, int q, int c, bool max, bool& nan) {
  using Geo = DofGeo<NW, DRN>;
  double v = 0.0;
  nan = false;
  for (int r = 0; r < 16; ++r) {
    const double w = red[q * Geo::NE + r * Geo::NT + c];
    if (max) {
      nan |= (w != w);
      v = fmax(v, w);
    } else {
      v += w;
    }
  }
  return v;
}

// stage A, DOF tile
template <int NW, int DRN>
__device__ __forceinline__ void dof_A(const ChTile* __restrict__ T, const StepDev* __restrict__ sd,
                                      const StepArgs& ta, int mode, double* lds) {
  using Geo = DofGeo<NW, DRN>;
  constexpr int EPT = Geo::EPT;
  const int B = sd->B, nb = sd->nbath;
  const int64_t t = ta.t;
  const int tn = (int)(t % sd->nmd);
  const int par = (int)(t & 1);
  const double dt = sd->dt, dt2 = dt * dt;
  const bool harm = (mode & 1) != 0, diff1 = (mode & 2) != 0;
  // ---- loads that do not depend on the products
  Elem E[EPT];
  double p[EPT], q[EPT], fc[EPT], q0[EPT];
  unsigned long long w0[EPT];
  int qv[EPT];
  int kk[EPT][CH_TB];
  double nz[EPT][CH_TB], sv[EPT][CH_TB];
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    E[x] = elem_of<NW, DRN>(T, sd, x);
    const int64_t ii = E[x].ok ? E[x].i : 0;
    const int bb = E[x].ok ? E[x].b : 0;
    p[x] = G(sd->P)[ii];
    q[x] = G(sd->Q)[ii];
    fc[x] = G(sd->Fc)[ii];
    q0[x] = G(sd->Q0)[ii];
    qv[x] = G(sd->qvalid)[bb];
    w0[x] = *G(pmax_word(sd, 0, par, bb));
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) {
      const ChBath& bd = T->tb[u];
      kk[x][u] = bath_row(bd, E[x]);
      const int64_t kb = bath_idx(E[x], kk[x][u], B);
      nz[x][u] = G(bd.noise)[(int64_t)tn * bd.nc * B + kb];
      sv[x][u] = G(bd.S)[(int64_t)par * bd.vs + kb];
    }
  }
  if (T->first && threadIdx.x < Geo::NT && T->c0 + (int)threadIdx.x < B)
    *G(pmax_word(sd, 0, par ^ 1, T->c0 + threadIdx.x)) = 0ull;
  run_products_rn<NW, DRN>(T, t, lds);
  __syncthreads();
  stamp(sd, 0, 2, ta);
  // ---- epilogue (md.vv id0, md.py:383-397).  Every output sum is read first (unconditionally, the
  // masked ones are not used): their LDS reads are in flight together.
  double cur[EPT][CH_TB], ee[EPT], dq[EPT];
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    const int e = min((int)threadIdx.x + x * NW * 64, Geo::NE - 1);
    const double yd = out_sum<NW>(T, lds, 2 * CH_TB, e, Geo::NE);
    double y[CH_TB];
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) y[u] = out_sum<NW>(T, lds, u, e, Geo::NE);
    const bool hit = harm ? (qv[x] != 0 && word_hit(w0[x])) : true;
    double f = fc[x];  // potforce(q_t)
    if (!hit && E[x].in) {
      f = -1.0 * yd;  // f = -1.0*mdot(dyn, q)  (md.py:467)
      if (E[x].ok) {
        G(sd->Fc)[E[x].i] = f;
        G(sd->Q0)[E[x].i] = q[x];
      }
    }
    // fused B+C: the cached force on the bath rows, the X of K0.Fc (the id1 cache-hit case)
#pragma unroll
    for (int u = 0; u < CH_TB; ++u)
      if (kk[x][u] >= 0 && T->tb[u].Xf) G(T->tb[u].Xf)[(int64_t)kk[x][u] * B + E[x].b] = f;
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) {
      cur[x][u] = 0.0;
      if (kk[x][u] >= 0) {
        const ChBath& bd = T->tb[u];
        double fb = nz[x][u] - bd.c * (y[u] + sv[x][u]);
        if (bd.has_q) fb -= out_sum<NW>(T, lds, CH_TB + u, e, Geo::NE);
        f += fb;                 // pf = pf + fbaths[i]  (md.py:432-434)
        cur[x][u] = fb * p[x];   // cur[t] = fbaths[i].p (md.py:397)
        if (double* rf = sd->rec_f[bd.bath])  // fhis[i][t] = fbaths[i] (md.py:398), bath rows
          G(rf)[((int64_t)tn * bd.nc + kk[x][u]) * B + E[x].b] = fb;
      }
    }
    const double ph = p[x] + f * dt / 2.0;               // md.py:391
    const double qt = q[x] + p[x] * dt + f * dt2 / 2.0;  // md.py:392
    if (E[x].ok) {
      G(sd->Ph)[E[x].i] = ph;
      G(sd->Qt)[E[x].i] = qt;
      // recordings (pointers are launch-uniform): ps / qs at slot t mod nmd, histories at t mod ml
      const int64_t rs = (int64_t)tn * sd->nph * B + E[x].i;
      if (sd->rec_p) G(sd->rec_p)[rs] = p[x];
      if (sd->rec_q) G(sd->rec_q)[rs] = q[x];
      if (sd->rec_hp) {
        const int64_t hs = (int64_t)(t % sd->rec_ml) * sd->nph * B + E[x].i;
        G(sd->rec_hp)[hs] = p[x];
        G(sd->rec_hq)[hs] = q[x];
      }
    }
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) {
      if (kk[x][u] >= 0) {
        const ChBath& bd = T->tb[u];
        const int64_t kb = (int64_t)kk[x][u] * B + E[x].b;
        G(bd.Xcur)[kb] = ph;
        if (bd.has_q) G(bd.Xq)[bd.vs + kb] = qt;
      }
    }
    ee[x] = E[x].ok ? p[x] * p[x] : 0.0;
    dq[x] = E[x].ok ? fabs(qt - (hit ? q0[x] : q[x])) : 0.0;
  }
  // per-trajectory sums over the tile's DOFs (fixed row order): one row of the step's partial table
  // [tile][bath | energy]; baths that miss the tile get zeros
  __syncthreads();
  double* red = lds;
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    const int e = threadIdx.x + x * NW * 64;
    if (E[x].in) {
#pragma unroll
      for (int u = 0; u < CH_TB; ++u) red[u * Geo::NE + e] = cur[x][u];
      red[CH_TB * Geo::NE + e] = ee[x];
      red[(CH_TB + 1) * Geo::NE + e] = dq[x];
    }
  }
  __syncthreads();
  auto prow = G(sd->part + (((int64_t)tn * sd->ndblk + T->tile) * (nb + 1)) * B);
  {
    // one thread per (quantity, column): the tile baths' currents, the kinetic energy, the cache
    // distance (one column sum each, side by side instead of one after another in 16 threads)
    static_assert((CH_TB + 2) * Geo::NT <= NW * 64, "one thread per column reduction");
    const int qn = threadIdx.x / Geo::NT, c = threadIdx.x % Geo::NT;
    const int b = T->c0 + c;
    if (qn < CH_TB + 2 && b < B) {
      bool nan;
      const double v = col_red<NW, DRN>(red, qn, c, qn == CH_TB + 1, nan);
      if (qn < CH_TB) {
        const int j = T->tb[qn].bath;
        if (j >= 0) prow[(int64_t)j * B + b] = v;
      } else if (qn == CH_TB) {
        prow[(int64_t)nb * B + b] = v;
      } else if (diff1) {
        const unsigned long long bits = nan ? 0x7FF8000000000000ull : (unsigned long long)__double_as_longlong(v);
        gmax(pmax_word(sd, 1, par, b), bits);
      }
    }
  }
  for (int z = threadIdx.x; z < nb * Geo::NT; z += NW * 64) {  // baths that miss the tile
    const int j = z / Geo::NT, b = T->c0 + z % Geo::NT;
    bool meets = false;
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) meets |= T->tb[u].bath == j;
    if (!meets && b < B) prow[(int64_t)j * B + b] = 0.0;
  }
}

// stage B, DOF tile
template <int NW, int DRN>
__device__ __forceinline__ void dof_B(const ChTile* __restrict__ T, const StepDev* __restrict__ sd,
                                      const StepArgs& ta, int mode, double* lds) {
  using Geo = DofGeo<NW, DRN>;
  constexpr int EPT = Geo::EPT;
  const int B = sd->B;
  const int64_t t = ta.t;
  const int t1 = (int)((t + 1) % sd->nmd);
  const int par = (int)(t & 1), par1 = par ^ 1;
  const double dt = sd->dt;
  const bool harm = mode != 0;
  Elem E[EPT];
  double ph[EPT], qt[EPT], fc[EPT];
  unsigned long long w1[EPT];
  int kk[EPT][CH_TB];
  double nz[EPT][CH_TB], sv[EPT][CH_TB];
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    E[x] = elem_of<NW, DRN>(T, sd, x);
    const int64_t ii = E[x].ok ? E[x].i : 0;
    ph[x] = G(sd->Ph)[ii];
    qt[x] = G(sd->Qt)[ii];
    fc[x] = G(sd->Fc)[ii];
    w1[x] = *G(pmax_word(sd, 1, par, E[x].ok ? E[x].b : 0));
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) {
      const ChBath& bd = T->tb[u];
      kk[x][u] = bath_row(bd, E[x]);
      const int64_t kb = bath_idx(E[x], kk[x][u], B);
      nz[x][u] = G(bd.noise)[(int64_t)t1 * bd.nc * B + kb];
      sv[x][u] = G(bd.S)[(int64_t)par1 * bd.vs + kb];
    }
  }
  run_products_rn<NW, DRN>(T, t, lds);
  __syncthreads();
  stamp(sd, 1, 2, ta);
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    const int e = threadIdx.x + x * NW * 64;
    const bool hit1 = harm ? word_hit(w1[x]) : true;
    double f = fc[x];  // potforce(q~)
    if (!hit1 && E[x].in) {
      f = -1.0 * out_sum<NW>(T, lds, 2 * CH_TB, e, Geo::NE);
      if (E[x].ok) {  // md.potforce miss at q~: evaluate and cache (md.py:472-473)
        G(sd->Fc)[E[x].i] = f;
        G(sd->Q0)[E[x].i] = qt[x];
      }
    }
    bool inb = false;
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) {
      if (kk[x][u] >= 0) {
        const ChBath& bd = T->tb[u];
        const int64_t kb = (int64_t)kk[x][u] * B + E[x].b;
        double fb = nz[x][u] - bd.c * (out_sum<NW>(T, lds, u, e, Geo::NE) + sv[x][u]);
        if (bd.has_q) {
          const double yq = out_sum<NW>(T, lds, CH_TB + u, e, Geo::NE);
          fb -= yq;
          G(bd.Yq)[kb] = yq;  // Kq.q~ is the same in both id1 calls
        }
        f += fb;
        inb = true;
      }
    }
    if (inb) {
      const double p1 = ph[x] + dt * f / 2.0;  // md.py:402 (p1 only feeds the bath friction terms)
#pragma unroll
      for (int u = 0; u < CH_TB; ++u)
        if (kk[x][u] >= 0) {
          const ChBath& bd = T->tb[u];
          G(bd.Xcur)[bd.vs + (int64_t)kk[x][u] * B + E[x].b] = p1;
        }
    }
  }
}

// stage C, DOF tile
template <int NW, int DRN>
__device__ __forceinline__ void dof_C(const ChTile* __restrict__ T, const StepDev* __restrict__ sd,
                                      const StepArgs& ta, int mode, double* lds) {
  using Geo = DofGeo<NW, DRN>;
  constexpr int EPT = Geo::EPT;
  const int B = sd->B;
  const int64_t t = ta.t;
  const int t1 = (int)((t + 1) % sd->nmd);
  const int par = (int)(t & 1), par1 = par ^ 1;
  const double dt = sd->dt;
  const bool harm = mode != 0;
  Elem E[EPT];
  double ph[EPT], qt[EPT], fc[EPT], q0[EPT];
  int cons[EPT];
  int kk[EPT][CH_TB];
  double nz[EPT][CH_TB], sv[EPT][CH_TB], yq[EPT][CH_TB];
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    E[x] = elem_of<NW, DRN>(T, sd, x);
    const int64_t ii = E[x].ok ? E[x].i : 0;
    ph[x] = G(sd->Ph)[ii];
    qt[x] = G(sd->Qt)[ii];
    fc[x] = G(sd->Fc)[ii];
    cons[x] = G(sd->cmask)[E[x].ok ? E[x].d : 0];
    q0[x] = G(sd->Q0)[ii];
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) {
      const ChBath& bd = T->tb[u];
      kk[x][u] = bath_row(bd, E[x]);
      const int64_t kb = bath_idx(E[x], kk[x][u], B);
      nz[x][u] = G(bd.noise)[(int64_t)t1 * bd.nc * B + kb];
      sv[x][u] = G(bd.S)[(int64_t)par1 * bd.vs + kb];
      yq[x][u] = G(bd.Yq)[bd.has_q ? kb : 0];
    }
  }
  if (T->first && threadIdx.x < Geo::NT && T->c0 + (int)threadIdx.x < B) {
    *G(pmax_word(sd, 1, par1, T->c0 + threadIdx.x)) = 0ull;
    G(sd->qvalid)[T->c0 + threadIdx.x] = 1;
  }
  run_products_rn<NW, DRN>(T, t, lds);
  __syncthreads();
  stamp(sd, 2, 2, ta);
  double dq[EPT];
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    const int e = threadIdx.x + x * NW * 64;
    double f = fc[x];
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) {
      if (kk[x][u] >= 0) {
        const ChBath& bd = T->tb[u];
        f += nz[x][u] - bd.c * (out_sum<NW>(T, lds, u, e, Geo::NE) + sv[x][u]) - yq[x][u];
      }
    }
    double p2 = ph[x] + dt * f / 2.0;  // md.py:404
    double qn = qt[x];
    if (cons[x] != 0) {  // ApplyConstraint (md.py:407-408, 782-794)
      p2 = 0.0;
      qn = 0.0;
    }
    if (E[x].ok) {
      G(sd->P)[E[x].i] = p2;
      G(sd->Q)[E[x].i] = qn;
      G(sd->Flast)[E[x].i] = f;
      // a host force at q~ (gle_step_end with fpot): md.potforce's cache now holds (q~, Fc)
      if (!harm) G(sd->Q0)[E[x].i] = qt[x];
    }
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) {
      if (kk[x][u] >= 0) {
        const ChBath& bd = T->tb[u];
        // history push of p_{t+1} (rpadleft, md.py:387 of the next step): mirrored slot of the
        // ladder's ring and the chain's near ring
        const int64_t kb = (int64_t)kk[x][u] * B + E[x].b;
        const int64_t slot = cmod(t + 1, bd.R);
        auto h = G(bd.H + (int64_t)kk[x][u] * bd.ldh + E[x].b);
        h[slot * B] = p2;
        h[(slot + bd.R) * B] = p2;
        G(bd.NR)[cmod(t + 1, bd.NRS) * bd.vs + kb] = p2;
        if (bd.has_q) G(bd.Xq)[kb] = qn;
      }
    }
    dq[x] = E[x].ok ? fabs(qn - (harm ? q0[x] : qt[x])) : 0.0;
  }
  {  // cache distance of q_{t+1} for the next step's id0 call (after a host force too: the next step
     // may evaluate the force on the device, with md.potforce's rule against q~)
    __syncthreads();
#pragma unroll
    for (int x = 0; x < EPT; ++x) {
      const int e = threadIdx.x + x * NW * 64;
      if (E[x].in) lds[e] = dq[x];
    }
    __syncthreads();
    const int c = threadIdx.x;
    const int b = T->c0 + c;
    if (c < Geo::NT && b < B) {
      bool nan;
      const double m = col_red<NW, DRN>(lds, 0, c, true, nan);
      const unsigned long long bits = nan ? 0x7FF8000000000000ull : (unsigned long long)__double_as_longlong(m);
      gmax(pmax_word(sd, 0, par1, b), bits);
    }
  }
}

// stages B + C fused (md.py:401-408 in one launch; harmonic force, pairwise disjoint baths).  With
// g = Fpot(q~) + sum_u (V - Kq q~), V = n1 - c S1 (the bath part of F1 that does not depend on the
// velocity argument) and F1(x) = g - sum_u c K0 x on the bath rows:
//   p1 = p_half + h F1(p_half),  h = dt/2
//   K0 p1 = M1 p_half + h K0 (V + Fpot_b) - h (K0 Kq) q~,   M1 = K0 - (c h) K0^2
//   K0 Fpot_b = K0 Fc (potential cache hit at q~) or -(K0 P dyn) q~ (miss)
//   p2 = p_half + h F1(p1) = p_half + h (g - c K0 p1)
// so every product reads only stage A's outputs: one dependent launch instead of two, and three
// nc x nc products per bath row instead of the six of B + C.  K0 p1 is re-associated (rounding
// only).  Products of the branch no trajectory of the tile takes are skipped.
template <int NW, int DRN>
__device__ __forceinline__ void dof_BC(const ChTile* __restrict__ T, const StepDev* __restrict__ sd,
                                       const StepArgs& ta, int mode, double* lds) {
  using Geo = DofGeo<NW, DRN>;
  constexpr int EPT = Geo::EPT;
  const int B = sd->B;
  const int64_t t = ta.t;
  const int t1 = (int)((t + 1) % sd->nmd);
  const int par = (int)(t & 1), par1 = par ^ 1;
  const double dt = sd->dt;
  const bool harm = mode != 0;
  const bool pre = (mode & 4) != 0;  // Fpot(q~) evaluated by the fpot launch: Fc / Q0 current, V + Fpot_b
  Elem E[EPT];
  double ph[EPT], qt[EPT], fc[EPT], q0[EPT];
  bool hit1[EPT];
  int cons[EPT];
  int kk[EPT][CH_TB];
  double nz[EPT][CH_TB], sv[EPT][CH_TB];
  int anyhit = 0, anymiss = 0;
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    E[x] = elem_of<NW, DRN>(T, sd, x);
    const int64_t ii = E[x].ok ? E[x].i : 0;
    ph[x] = G(sd->Ph)[ii];
    qt[x] = G(sd->Qt)[ii];
    fc[x] = G(sd->Fc)[ii];
    cons[x] = G(sd->cmask)[E[x].ok ? E[x].d : 0];
    q0[x] = G(sd->Q0)[ii];
    const unsigned long long w1 = *G(pmax_word(sd, 1, par, E[x].ok ? E[x].b : 0));
    hit1[x] = (harm && !pre) ? word_hit(w1) : true;
    anyhit |= (E[x].ok && hit1[x]) ? 1 : 0;
    anymiss |= (E[x].ok && !hit1[x]) ? 1 : 0;
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) {
      const ChBath& bd = T->tb[u];
      kk[x][u] = bath_row(bd, E[x]);
      const int64_t kb = bath_idx(E[x], kk[x][u], B);
      nz[x][u] = G(bd.noise)[(int64_t)t1 * bd.nc * B + kb];
      sv[x][u] = G(bd.S)[(int64_t)par1 * bd.vs + kb];
    }
  }
  // which potential-cache branches at q~ any trajectory of the tile takes (workgroup-uniform)
  anyhit = __syncthreads_or(anyhit);
  anymiss = __syncthreads_or(anymiss);
  run_products_rn<NW, DRN>(T, t, lds, (anyhit ? 0 : 1) | (anymiss ? 0 : 2));
  __syncthreads();
  // the words this launch reads (w1) are read above: only now may the first tile reset them
  if (T->first && threadIdx.x < Geo::NT && T->c0 + (int)threadIdx.x < B) {
    *G(pmax_word(sd, 1, par1, T->c0 + threadIdx.x)) = 0ull;
    if (harm) G(sd->qvalid)[T->c0 + threadIdx.x] = 1;
  }
  stamp(sd, 3, 2, ta);
  double dq[EPT];
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    const int e = min((int)threadIdx.x + x * NW * 64, Geo::NE - 1);
    // the output sums first, unconditionally (their LDS reads in flight together)
    const double yd = out_sum<NW>(T, lds, 2 * CH_TB, e, Geo::NE);
    double yb[CH_TB], ye[CH_TB];
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) {
      yb[u] = out_sum<NW>(T, lds, CH_OYB + u, e, Geo::NE);
      ye[u] = out_sum<NW>(T, lds, (hit1[x] ? CH_OYE : CH_OYD) + u, e, Geo::NE);
    }
    double fpot = fc[x];  // potforce(q~)
    if (!hit1[x] && E[x].in) {
      fpot = -1.0 * yd;
      if (E[x].ok) {  // md.potforce miss at q~: evaluate and cache (md.py:472-473)
        G(sd->Fc)[E[x].i] = fpot;
        G(sd->Q0)[E[x].i] = qt[x];
      }
    }
    double f2 = fpot;  // F1(p1) (md.py:403) = g - sum_u c K0 p1
#pragma unroll
    for (int u = 0; u < CH_TB; ++u)
      if (kk[x][u] >= 0) {
        const ChBath& bd = T->tb[u];
        f2 += nz[x][u] - bd.c * sv[x][u];
        if (bd.has_q) f2 -= out_sum<NW>(T, lds, CH_TB + u, e, Geo::NE);
        const double k0p1 = yb[u] + ye[u];
        f2 -= bd.c * k0p1;
      }
    double p2 = ph[x] + dt * f2 / 2.0;  // md.py:404
    double qn = qt[x];
    if (cons[x] != 0) {  // ApplyConstraint (md.py:407-408, 782-794)
      p2 = 0.0;
      qn = 0.0;
    }
    if (E[x].ok) {
      G(sd->P)[E[x].i] = p2;
      G(sd->Q)[E[x].i] = qn;
      G(sd->Flast)[E[x].i] = f2;
    }
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) {
      if (kk[x][u] >= 0) {
        const ChBath& bd = T->tb[u];
        const int64_t kb = (int64_t)kk[x][u] * B + E[x].b;
        const int64_t slot = cmod(t + 1, bd.R);
        auto hh = G(bd.H + (int64_t)kk[x][u] * bd.ldh + E[x].b);
        hh[slot * B] = p2;
        hh[(slot + bd.R) * B] = p2;
        G(bd.NR)[cmod(t + 1, bd.NRS) * bd.vs + kb] = p2;
        if (bd.has_q) G(bd.Xq)[kb] = qn;
      }
    }
    dq[x] = E[x].ok ? fabs(qn - (hit1[x] ? q0[x] : qt[x])) : 0.0;
  }
  if (harm) {  // cache distance of q_{t+1} for the next step's id0 call
    __syncthreads();
#pragma unroll
    for (int x = 0; x < EPT; ++x) {
      const int e = threadIdx.x + x * NW * 64;
      if (E[x].in) lds[e] = dq[x];
    }
    __syncthreads();
    const int c = threadIdx.x;
    const int b = T->c0 + c;
    if (c < Geo::NT && b < B) {
      bool nan;
      const double m = col_red<NW, DRN>(lds, 0, c, true, nan);
      const unsigned long long bits = nan ? 0x7FF8000000000000ull : (unsigned long long)__double_as_longlong(m);
      gmax(pmax_word(sd, 0, par1, b), bits);
    }
  }
}

// A stage-4 DOF tile split over T->xnsub workgroups (k-ranges of its products): this workgroup's
// output sums go to its slab with write-through (sc1) stores, drained by every wave before the
// workgroup's barrier; lane 0 then adds to the tile's arrival counter (agent scope).  The last
// arriver reads every slab with sc1 loads (no stale L1 / L2 line of another XCD can serve them) and
// sums them in slab order, so the result does not depend on the arrival order.  The counter is
// never reset: every launch adds exactly xnsub per tile (zeroed with the plan).
// CH_XSUB_ORDER 1: the counter add is a release and the last arriver issues an acquire fence
// before its slab loads (the happens-before edge of the HIP / C++ model; on gfx950 an L2 write-back
// and invalidate per tile and launch); 0: relaxed, ordered by the slab stores' completion wait and
// the loads' issue after the counter's return (ISA-level ordering only)
#ifndef CH_XSUB_ORDER
#define CH_XSUB_ORDER 0
#endif
template <int NW, int NE, int EPT>
__device__ __forceinline__ bool xsub_combine(const ChTile* __restrict__ T, double (&ov)[EPT][CH_XO], double* lds) {
  typedef __attribute__((address_space(1))) unsigned long long gull;
  gull* slab = (gull*)T->xslab;
  const int ns = T->xnsub;
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    const int e = threadIdx.x + x * NW * 64;
    if (e < NE) {
#pragma unroll
      for (int o = 0; o < CH_XO; ++o)
        __hip_atomic_store(slab + ((int64_t)T->xsub * CH_XO + o) * NE + e,
                           (unsigned long long)__double_as_longlong(ov[x][o]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave's slab stores have completed; the LDS partial slots are read
  if (threadIdx.x == 0) {
    const unsigned long long old = __hip_atomic_fetch_add((gull*)T->xcnt, 1ull,
                                                          CH_XSUB_ORDER ? __ATOMIC_RELEASE : __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
    lds[0] = (old + 1) % (unsigned long long)ns == 0 ? 1.0 : 0.0;
  }
  __syncthreads();
  if (lds[0] == 0.0) return false;
#if CH_XSUB_ORDER
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every other slab's stores happen-before the loads
#endif
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    const int e = min((int)threadIdx.x + x * NW * 64, NE - 1);
#pragma unroll
    for (int o = 0; o < CH_XO; ++o) ov[x][o] = 0.0;
    // slabs four at a time, all loads of a group in flight together; masked slabs add 0.0
    for (int s0 = 0; s0 < ns; s0 += 4) {
      double v[4][CH_XO];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int sl = min(s0 + k, ns - 1);
#pragma unroll
        for (int o = 0; o < CH_XO; ++o)
          v[k][o] = __longlong_as_double((long long)__hip_atomic_load(slab + ((int64_t)sl * CH_XO + o) * NE + e,
                                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int o = 0; o < CH_XO; ++o) ov[x][o] += s0 + k < ns ? v[k][o] : 0.0;
    }
  }
  return true;
}

// stage 4 (composed one-launch step, gle_internal.h), DOF tile: p_{t+1} is the composed product
// (output CH_OYB); K0.p_t (u), Kq.q_t (CH_TB + u) and dyn.q_t (2 CH_TB) give md.vv's id0 phase for the
// tile's elements: F0, heat current, kinetic energy, recordings, q_{t+1} = q~ (md.py:383-398);
// constraints zero p_{t+1} and q_{t+1} (md.py:407-408); history push of p_{t+1}.
template <int NW, int DRN, bool GV = false>
__device__ __forceinline__ void dof_X(const ChTile* __restrict__ T, const StepDev* __restrict__ sd,
                                      const StepArgs& ta, double* lds, XCheck& xc) {
  using Geo = DofGeo<NW, DRN>;
  constexpr int EPT = Geo::EPT;
  const int B = sd->B, nb = sd->nbath;
  const int64_t t = ta.t;
  const int tn = (int)(t % sd->nmd);
  const int par = (int)(t & 1), par1 = par ^ 1;
  const double dt = sd->dt, dt2 = dt * dt;
  // ---- loads that do not depend on the products
  Elem E[EPT];
  double p[EPT], q[EPT];
  int cons[EPT];
  int kk[EPT][CH_TB];
  double v0[EPT][CH_TB];
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    E[x] = elem_of<NW, DRN>(T, sd, x);
    const int64_t ii = E[x].ok ? E[x].i : 0;
    p[x] = G(T->xp_in)[ii];
    q[x] = G(T->xq_in)[ii];
    cons[x] = G(sd->cmask)[E[x].ok ? E[x].d : 0];
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) {
      const ChBath& bd = T->tb[u];
      kk[x][u] = bath_row(bd, E[x]);
      v0[x][u] = G(bd.V)[(int64_t)par * bd.vs + bath_idx(E[x], kk[x][u], B)];
    }
  }
  const int part = T->xpart;  // 1: p_{t+1} only, 2: id0 phase and q_{t+1} only, 0: both
  run_products_rn<NW, DRN, GV>(T, t, lds);
  if (xc.stop(sd, ta)) return;
  stamp(sd, 4, 2, ta);
  // the tile's output sums: K0.p_t of tile bath u (u), dyn.q_t (CH_TB), p_{t+1} (CH_TB + 1)
  double ov[EPT][CH_XO];
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    const int e = min((int)threadIdx.x + x * NW * 64, Geo::NE - 1);
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) ov[x][u] = out_sum<NW>(T, lds, u, e, Geo::NE);
    ov[x][CH_TB] = out_sum<NW>(T, lds, 2 * CH_TB, e, Geo::NE);
    ov[x][CH_TB + 1] = out_sum<NW>(T, lds, CH_OYB, e, Geo::NE);
  }
  if (T->xnsub > 1 && !xsub_combine<NW, Geo::NE, EPT>(T, ov, lds)) return;
  double cur[EPT][CH_TB], ee[EPT], d1[EPT], d0[EPT];
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    const int e = min((int)threadIdx.x + x * NW * 64, Geo::NE - 1);
    const double yd = ov[x][CH_TB];
    const double xp = ov[x][CH_TB + 1];
    double y[CH_TB];
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) y[u] = ov[x][u];
    double f = -1.0 * yd;  // potforce(q_t) = -1.0*mdot(dyn, q) (md.py:467)
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) {
      cur[x][u] = 0.0;
      if (kk[x][u] >= 0) {
        const ChBath& bd = T->tb[u];
        double fb = v0[x][u] - bd.c * y[u];  // noise - c (K0.p + S(t))
        if (bd.has_q) fb -= out_sum<NW>(T, lds, CH_TB + u, e, Geo::NE);
        f += fb;                 // md.py:432-434
        cur[x][u] = fb * p[x];   // md.py:397
        if (double* rf = sd->rec_f[bd.bath])  // md.py:398
          G(rf)[((int64_t)tn * bd.nc + kk[x][u]) * B + E[x].b] = fb;
      }
    }
    const double ph = p[x] + f * dt / 2.0;               // md.py:391
    const double qt = q[x] + p[x] * dt + f * dt2 / 2.0;  // md.py:392
    double p2 = xp, qn = qt;
    if (cons[x] != 0) {  // ApplyConstraint (md.py:407-408, 782-794)
      p2 = 0.0;
      qn = 0.0;
    }
    if (E[x].ok && part != 2) G(T->xp_out)[E[x].i] = p2;
    if (E[x].ok && part == 0)
      G(sd->Flast)[E[x].i] = (xp - ph) * (2.0 / dt);  // F1(p1): p2 = p_half + dt F1(p1) / 2 (md.py:403-404)
    if (E[x].ok && part != 1) {
      G(T->xq_out)[E[x].i] = qn;
      const int64_t rs = (int64_t)tn * sd->nph * B + E[x].i;
      if (sd->rec_p) G(sd->rec_p)[rs] = p[x];
      if (sd->rec_q) G(sd->rec_q)[rs] = q[x];
      if (sd->rec_hp) {
        const int64_t hs = (int64_t)(t % sd->rec_ml) * sd->nph * B + E[x].i;
        G(sd->rec_hp)[hs] = p[x];
        G(sd->rec_hq)[hs] = q[x];
      }
    }
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) {
      if (kk[x][u] >= 0) {
        const ChBath& bd = T->tb[u];
        const int64_t kb = (int64_t)kk[x][u] * B + E[x].b;
        const int64_t slot = cmod(t + 1, bd.R);  // history push of p_{t+1} (md.py:386-387)
        if (part != 2) {
          auto hh = G(bd.H + (int64_t)kk[x][u] * bd.ldh + E[x].b);
          hh[slot * B] = p2;
          hh[(slot + bd.R) * B] = p2;
          G(bd.NR)[cmod(t + 1, bd.NRS) * bd.vs + kb] = p2;
        }
        if (bd.has_q && part != 1) G(bd.Xq)[(int64_t)par1 * bd.vs + kb] = qn;
      }
    }
    ee[x] = E[x].ok ? p[x] * p[x] : 0.0;
    d1[x] = E[x].ok ? fabs(qt - q[x]) : 0.0;   // |q~ - q0| of the id1 call (q0 = q_t)
    d0[x] = E[x].ok ? fabs(qn - qt) : 0.0;     // |q_{t+1} - q0| of the next id0 call (q0 = q~)
  }
  if (part == 1) return;  // the p_{t+1} half of a split tile: no reductions
  // per-trajectory sums over the tile's DOFs (fixed row order): currents and energy into the step's
  // partial table, the two cache distances as maxima into the audit words of slot t mod 3
  __syncthreads();
  double* red = lds;
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    const int e = threadIdx.x + x * NW * 64;
    if (E[x].in) {
#pragma unroll
      for (int u = 0; u < CH_TB; ++u) red[u * Geo::NE + e] = cur[x][u];
      red[CH_TB * Geo::NE + e] = ee[x];
      red[(CH_TB + 1) * Geo::NE + e] = d1[x];
      red[(CH_TB + 2) * Geo::NE + e] = d0[x];
    }
  }
  __syncthreads();
  auto prow = G(sd->part + (((int64_t)tn * sd->ndblk + T->tile) * (nb + 1)) * B);
  {
    static_assert((CH_TB + 3) * Geo::NT <= NW * 64, "one thread per column reduction");
    const int qn = threadIdx.x / Geo::NT, c = threadIdx.x % Geo::NT;
    const int b = T->c0 + c;
    if (qn <= CH_TB && b < B) {
      bool nan;
      const double v = col_red<NW, DRN>(red, qn, c, false, nan);
      if (qn < CH_TB) {
        const int j = T->tb[qn].bath;
        if (j >= 0) prow[(int64_t)j * B + b] = v;
      } else {
        prow[(int64_t)nb * B + b] = v;
      }
    }
#if defined(XC_DBG) && (XC_DBG & 2)  // timing diagnostics only: no audit words written
    if (false) {
#else
    if (ta.xw) {
#endif
      // the two cache distances as audit nibbles (XCheck): the (quantity, column) threads of the two
      // distances are lanes of one wave; OR over them, one atomic per audit word of the tile's columns
      const int q0 = (CH_TB + 1) * Geo::NT;  // first thread of the distances (wave q0 / 64)
      static_assert(((CH_TB + 1) * Geo::NT) / 64 == ((CH_TB + 3) * Geo::NT - 1) / 64, "one wave");
      if ((int)threadIdx.x / 64 == q0 / 64) {
        unsigned long long nib = 0ull;
        if (qn > CH_TB && qn < CH_TB + 3 && b < B) {
          bool nan;
          const double v = col_red<NW, DRN>(red, qn, c, true, nan);
          const unsigned long long m = (v > 0.0 ? 1ull : 0ull) | ((nan || !(v < 10e-10)) ? 2ull : 0ull);
          nib = m << (4 * (b % 16) + 2 * (qn - CH_TB - 1));
        }
        typedef __attribute__((address_space(1))) unsigned long long gull;
        const int lane = threadIdx.x & 63;
        // replica tile % xR of the step's words: a word takes the atomics of ~ntile / xR tiles (one word
        // line for every tile's atomic measured +2 us/step at C3)
        const int nw = (B + 15) / 16;
        gull* wrep = (gull*)(ta.xw + ((t % 3) * (int64_t)ta.xR + T->tile % ta.xR) * nw);
#pragma unroll 1
        for (int j = 0; j < Geo::NT / 16; ++j) {  // the tile's columns c0 .. c0 + NT - 1: NT / 16 words
          unsigned long long x = (c / 16 == j) ? nib : 0ull;
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) x |= __shfl_xor(x, o);
          if (lane == 0 && x != 0ull)
            __hip_atomic_fetch_or(wrep + (T->c0 / 16 + j), x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
  for (int z = threadIdx.x; z < nb * Geo::NT; z += NW * 64) {  // baths that miss the tile
    const int j = z / Geo::NT, b = T->c0 + z % Geo::NT;
    bool meets = false;
#pragma unroll
    for (int u = 0; u < CH_TB; ++u) meets |= T->tb[u].bath == j;
    if (!meets && b < B) prow[(int64_t)j * B + b] = 0.0;
  }
}

// stage 4 S tile, bath rows [row0, row0+16): V0(t+1) = W1(t) - c K1.p_t and W1(t+1) = n_{t+2} -
// c (K2.p_t + near partials (lags >= 3, written by launch t-1) + levels at target t+2)
template <int NW, int DRN, bool GV = false>
__device__ __forceinline__ void sfin_X(const ChTile* __restrict__ T, const StepDev* __restrict__ sd,
                                       const StepArgs& ta, double* lds) {
  const int B = sd->B;
  const int64_t t = ta.t;
  const int par = (int)(t & 1), par1 = par ^ 1;  // target t+2 has parity par
  const ChSfin& sf = T->sf;
  constexpr int NT = 16 * DRN, NE = 16 * NT;
  constexpr int EPT = (NE + NW * 64 - 1) / (NW * 64);
  double pre[EPT], nz2[EPT], w1[EPT];
  int64_t kb[EPT];
  bool ok[EPT];
  const int t2 = (int)((t + 2) % sd->nmd);
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    const int e = threadIdx.x + x * NW * 64;
    const int k = T->row0 + e / NT;
    const int b = T->c0 + e % NT;
    ok[x] = e < NE && k < sf.nc && b < B;
    kb[x] = (int64_t)k * B + b;
    double v[CH_NPMAX], lv[MAXLVL];
    auto np = G(sf.NP + (sf.nqn > 0 ? (int64_t)par * sf.nqn * sf.vs + (ok[x] ? kb[x] : 0) : 0));
#pragma unroll
    for (int q = 0; q < CH_NPMAX; ++q) v[q] = np[(int64_t)min(q, max(sf.nqn - 1, 0)) * sf.vs];
#pragma unroll
    for (int l = 0; l < MAXLVL; ++l)
      lv[l] = G(sf.lvl[l])[(ok[x] ? (int64_t)k * sf.lvl_ld[l] + b : 0) + ta.lvl_off[l]];
    nz2[x] = G(sf.noise)[ok[x] ? ((int64_t)t2 * sf.nc + k) * B + b : 0];
    w1[x] = G(sf.W1)[(int64_t)par * sf.vs + (ok[x] ? kb[x] : 0)];
    double sn = 0.0, lvs = 0.0;
#pragma unroll
    for (int q = 0; q < CH_NPMAX; ++q) sn += (q < sf.nqn) ? v[q] : 0.0;
#pragma unroll
    for (int l = 0; l < MAXLVL; ++l) lvs += lv[l];
    pre[x] = lvs + sn;
  }
  run_products_rn<NW, DRN, GV>(T, t, lds);
  __syncthreads();  // (only DOF tiles audit: this tile writes the composed step's own buffers)
  stamp(sd, 4, 2, ta);
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    const int e = threadIdx.x + x * NW * 64;
    if (ok[x]) {
      const double y1 = out_sum<NW>(T, lds, 0, e, NE), y2 = out_sum<NW>(T, lds, 1, e, NE);
      G(sf.V)[(int64_t)par1 * sf.vs + kb[x]] = w1[x] - sf.c * y1;              // n_{t+1} - c S(t+1)
      G(sf.W1)[(int64_t)par1 * sf.vs + kb[x]] = nz2[x] - sf.c * (y2 + pre[x]);  // n_{t+2} - c R(t+2)
    }
  }
}

// S(t+1) of bath rows [row0, row0+16) x 16 rn columns: K_1.p_t (the products) + near-field
// partials + levels
template <int NW, int DRN>
__device__ __forceinline__ void sfin(const ChTile* __restrict__ T, const StepDev* __restrict__ sd,
                                     const StepArgs& ta, double* lds, int stage) {
  const int B = sd->B;
  const int64_t t = ta.t;
  const int par1 = (int)((t + 1) & 1);
  const ChSfin& sf = T->sf;
  constexpr int NT = 16 * DRN, NE = 16 * NT;  // S(t+1) tiles have the DOF tiles' width
  constexpr int EPT = (NE + NW * 64 - 1) / (NW * 64);
  double pre[EPT], nzv[EPT];
  int64_t kb[EPT];
  bool ok[EPT];
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    const int e = threadIdx.x + x * NW * 64;
    const int k = T->row0 + e / NT;
    const int b = T->c0 + e % NT;
    ok[x] = e < NE && k < sf.nc && b < B;
    kb[x] = (int64_t)k * B + b;
    // near-field partials and level blocks, all loads in flight together, added in slot / level
    // order
    double v[CH_NPMAX], lv[MAXLVL];
    auto np = G(sf.NP + (sf.nqn > 0 ? (int64_t)par1 * sf.nqn * sf.vs + (ok[x] ? kb[x] : 0) : 0));
    // unconditional loads (slot min(q, nqn-1); nqn == 0 reads the zero row), masked in the sum
#pragma unroll
    for (int q = 0; q < CH_NPMAX; ++q) v[q] = np[(int64_t)min(q, max(sf.nqn - 1, 0)) * sf.vs];
#pragma unroll
    for (int l = 0; l < MAXLVL; ++l)
      lv[l] = G(sf.lvl[l])[(ok[x] ? (int64_t)k * sf.lvl_ld[l] + b : 0) + ta.lvl_off[l]];
    // fused B+C: noise(t+1) of the V row, loaded with the prologue (not after the products)
    nzv[x] = sf.V ? G(sf.noise)[(ok[x] ? ((int64_t)((t + 1) % sd->nmd) * sf.nc + k) * B + b : 0)] : 0.0;
    double sn = 0.0, lvs = 0.0;
#pragma unroll
    for (int q = 0; q < CH_NPMAX; ++q) sn += (q < sf.nqn) ? v[q] : 0.0;
#pragma unroll
    for (int l = 0; l < MAXLVL; ++l) lvs += lv[l];
    pre[x] = lvs + sn;
  }
  run_products_rn<NW, DRN>(T, t, lds);
  __syncthreads();
  stamp(sd, stage, 2, ta);
#pragma unroll
  for (int x = 0; x < EPT; ++x) {
    const int e = threadIdx.x + x * NW * 64;
    if (ok[x]) {
      const double s1 = out_sum<NW>(T, lds, 0, e, NE) + pre[x];
      G(sf.S)[(int64_t)par1 * sf.vs + kb[x]] = s1;
      if (sf.V)  // fused B+C: V = noise(t+1) - c S(t+1), the bath part of F1 that K0 acts on
        G(sf.V)[kb[x]] = nzv[x] - sf.c * s1;
    }
  }
}

// near-field partial tile: rows [0, nrows) x columns [0, ncols) of the parity buffer of t + par_shift
template <int NW, bool GV = false>
__device__ __forceinline__ void raw(const ChTile* __restrict__ T, const StepDev* __restrict__ sd, const StepArgs& ta,
                                    double* lds, int stage) {
  const int64_t t = ta.t;
  run_products<NW, GV>(T, t, lds);
  __syncthreads();
  stamp(sd, stage, 2, ta);
  const int NT = 16 * T->rn;
  double* dst = T->dst + ((t + T->par_shift) & 1) * T->par_stride;
  // every element's slot reads in flight together (at most 16 x 64 elements per tile)
  constexpr int EMAX = (16 * 64 + NW * 64 - 1) / (NW * 64);
  double v[EMAX];
#pragma unroll
  for (int x = 0; x < EMAX; ++x) v[x] = out_sum<NW>(T, lds, 0, min((int)threadIdx.x + x * NW * 64, 16 * NT - 1), 16 * NT);
#pragma unroll
  for (int x = 0; x < EMAX; ++x) {
    const int e = threadIdx.x + x * NW * 64;
    const int row = e / NT, col = e - row * NT;
    if (e < 16 * NT && row < T->nrows && col < T->ncols) G(dst)[(int64_t)row * T->ldd + col] = v[x];
  }
}

// Far-field GEMM item of the fused schedule: workgroup nstatic + j runs item j of the launch's far
// ranges (the spectral levels' current blocks), at the lowest issue priority, in the launch's
// dynamic LDS (>= CH_FAR_LDS bytes).  4-wave launches only (the item's 4 waves own its 64 rows).
// The HBM stream of K-hat goes 3 chunks ahead (119 VGPRs for this path alone, within the chain
// kernel's 128).
constexpr size_t CH_FAR_LDS = sizeof(double) * 2 * 4 * 4 * CG_LD;
#ifndef CH_FAR_PATH
#define CH_FAR_PATH 1
#endif
template <int NW>
__device__ __forceinline__ void far_tile(const StepArgs& ta, double* lds) {
  if constexpr (NW == 4 && CH_FAR_PATH) {
    __builtin_amdgcn_s_setprio(0);
    int j = (int)blockIdx.x - ta.nstatic;
    const CgItem* items = nullptr;
    int64_t tseg = 0;
    int idx = 0;
    bool found = false;
    // constant indices into the kernel-argument ranges (a runtime index would copy StepArgs to
    // scratch)
#pragma unroll
    for (int r = 0; r < MAXLVL; ++r) {
      if (r < ta.nfar && !found) {
        if (j < ta.far[r].count) {
          items = ta.far[r].items;
          tseg = ta.far[r].tseg;
          idx = ta.far[r].first + j;
          found = true;
        } else {
          j -= ta.far[r].count;
        }
      }
    }
    if (!found) return;
    const CgItem it = items[idx];
    // one-plane items only (the planner keeps two-plane levels out of the fused schedule): the
    // two-plane path's three accumulator sets would set the whole chain kernel's register budget
    auto& xs = *reinterpret_cast<double(*)[2][4 * 4 * CG_LD]>(lds);
    switch (it.ncols > 32 ? 4 : (it.ncols > 16 ? 2 : 1)) {
      case 4: cgemm_item<4, 4, 3, 1>(it, tseg, xs); break;
      case 2: cgemm_item<2, 4, 3, 1>(it, tseg, xs); break;
      default: cgemm_item<1, 4, 3, 1>(it, tseg, xs); break;
    }
  }
}

template <int STAGE, int NW, int DRN>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(DRN == 1 && NW <= 8 ? CH_WPE : (NW == 8 ? 4 : 1), 8))) void chain_kernel(const ChTile* __restrict__ tiles, const StepDev* sd,
                                                        StepArgs ta, int mode) {
  extern __shared__ double lds[];
  if ((int)blockIdx.x >= ta.nstatic) {  // far-field item (fused schedule), launch-uniform ranges
    const unsigned long long t_far = __builtin_amdgcn_s_memrealtime();
    far_tile<NW>(ta, lds);
    if (ta.ts) {
      __syncthreads();
      if (threadIdx.x == 0) {
        G(ta.ts)[2 * blockIdx.x] = t_far;
        G(ta.ts)[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
      }
    }
    return;
  }
  // The chain is the step's latency-bound critical path and shares SIMDs with the background
  // ladder's GEMM waves: its waves take issue priority (MFMA pipe and memory issue go to the
  // highest-priority ready wave first, then the oldest)
  __builtin_amdgcn_s_setprio(CH_PRIO);
  // profiling: per-workgroup start / end stamps with plain stores (one device-scope counter that
  // every workgroup hits would serialise ~600 arrivals per launch and stretch the chain)
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  // The tile descriptor and the step descriptor's header are copied into LDS with one round of
  // coalesced vector loads: every later field access is an LDS read instead of a chain of
  // dependent scalar loads.  Only the task lists of this launch's NW waves are copied (task[] is
  // the descriptor's last member, wave-major): with 4 waves the copy is one word per thread, all
  // loads issued before the first LDS store.
  static_assert(offsetof(ChTile, task) + sizeof(ChTask) * CH_NW * CH_TPW == sizeof(ChTile), "task[] last");
  constexpr int NTW = (int)((offsetof(ChTile, task) + sizeof(ChTask) * NW * CH_TPW) / 8);
  constexpr int NSW = (offsetof(StepDev, bath) + 7) / 8;
  constexpr int NCP = NTW + NSW, NIT = (NCP + NW * 64 - 1) / (NW * 64);
  __shared__ unsigned long long tdw[sizeof(ChTile) / 8], sdw[NSW];
  stamp(sd, STAGE, 0, ta);
  XCheck xc;
  __shared__ int xflags[2];
  xc.flags = xflags;
  {
    typedef const __attribute__((address_space(1))) unsigned long long gull;
    gull* tsrc = (gull*)(tiles + blockIdx.x);
    gull* ssrc = (gull*)sd;
    unsigned long long v[NIT];
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int j = min((int)threadIdx.x + k * NW * 64, NCP - 1);
      v[k] = *(j < NTW ? tsrc + j : ssrc + (j - NTW));
    }
    if constexpr (STAGE >= 4) {
      // md.potforce cache audit of the previous step (XCheck), DOF tiles only (the launch's first
      // xndof workgroups): wave 0 loads the words in the descriptor's round trip (loaded after it,
      // the products' first wait included them: +0.5-0.9 us/step at C3, profiles/r06/audit_ab)
      if (ta.xw) {
        xc.nw = (ta.xB + 15) / 16;
        xc.nr = ta.xR;
        const int nl = xc.nw * xc.nr;  // lane r nw + j: word j of replica r; lane nl: the stop word
#if defined(XC_DBG) && (XC_DBG & 4)  // timing diagnostics only: no audit loads
        if (false) {
#else
        if ((int)blockIdx.x < ta.xndof && (int)threadIdx.x <= nl) {
#endif
          xc.lane = threadIdx.x;
          xc.w = xc.lane < nl ? *G(ta.xw + ((ta.t + 2) % 3) * (int64_t)nl + xc.lane) : *G(ta.xstop);
        }
        if (blockIdx.x == 0 && (int)threadIdx.x < nl)  // slot (t + 1) mod 3 for launch t + 1 (read by t - 1)
          *G(ta.xw + ((ta.t + 1) % 3) * (int64_t)nl + threadIdx.x) = 0ull;
      }
    }
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int i = threadIdx.x + k * NW * 64;
      if (i < NTW) tdw[i] = v[k];
      else if (i < NCP) sdw[i - NTW] = v[k];
    }
  }
  __syncthreads();
  const ChTile* T = (const ChTile*)tdw;
  sd = (const StepDev*)sdw;  // header only: bath[] is not copied (tiles carry their baths)
  const int kind = T->kind;
#if CH_PRIO_RAW != CH_PRIO
  // near-field partial tiles (consumed one step later) below the DOF / S(t+1) tiles of the stage
  if (kind == CH_RAW) __builtin_amdgcn_s_setprio(CH_PRIO_RAW);
#endif
  stamp(sd, STAGE, 1, ta);
  constexpr bool GV = STAGE == 5;  // stage 5: the composed stage with one-column (VALU) products
  if (kind == CH_DOF) {
    if (STAGE == 0) dof_A<NW, DRN>(T, sd, ta, mode, lds);
    else if (STAGE == 1) dof_B<NW, DRN>(T, sd, ta, mode, lds);
    else if (STAGE == 2) dof_C<NW, DRN>(T, sd, ta, mode, lds);
    else if (STAGE == 3) dof_BC<NW, DRN>(T, sd, ta, mode, lds);
    else {
      xc.on = ta.xw != nullptr;
      dof_X<NW, DRN, GV>(T, sd, ta, lds, xc);
    }
  } else if (kind == CH_SFIN) {
    if (STAGE >= 4) sfin_X<NW, DRN, GV>(T, sd, ta, lds);
    else sfin<NW, DRN>(T, sd, ta, lds, STAGE);
  } else {
    raw<NW, GV>(T, sd, ta, lds, STAGE);
  }
  stamp(sd, STAGE, 3, ta);
  if (ta.ts) {  // launch-uniform
    __syncthreads();
    if (threadIdx.x == 0) {
      G(ta.ts)[2 * blockIdx.x] = t_start;
      G(ta.ts)[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

// dynamic LDS above the 64 KiB default needs the kernel's limit raised (once per kernel and device;
// every chain_kernel instantiation has the same function type, so the record is keyed by address)
template <class K>
bool lds_limit(K* fn, size_t lds) {
  if (lds <= 64 * 1024) return true;
  struct Entry {
    const void* fn;
    int dev;
  };
  static thread_local std::vector<Entry> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  for (const Entry& e : done)
    if (e.fn == (const void*)fn && e.dev == dev) return true;
  if (hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
    return false;
  done.push_back({(const void*)fn, dev});
  return true;
}

template <int STAGE, int NW>
void launch_nd(int drn, size_t lds, const ChTile* tiles, int ntiles, const StepDev* sd, StepArgs ta, int mode,
               hipStream_t s) {
  int grid = ntiles;
  for (int r = 0; r < ta.nfar; ++r) grid += ta.far[r].count;
  if (ta.nfar > 0) lds = std::max(lds, CH_FAR_LDS);
  // at least one 64-column partial slot: the epilogues' masked slot reads stay inside the launch's LDS
  lds = std::max(lds, (size_t)16 * 64 * sizeof(double));
  if (drn == 2) {
    lds_limit(chain_kernel<STAGE, NW, 2>, lds);
    chain_kernel<STAGE, NW, 2><<<grid, NW * 64, lds, s>>>(tiles, sd, ta, mode);
  } else {
    lds_limit(chain_kernel<STAGE, NW, 1>, lds);
    chain_kernel<STAGE, NW, 1><<<grid, NW * 64, lds, s>>>(tiles, sd, ta, mode);
  }
}

template <int STAGE>
void launch_st(int nw, int drn, size_t lds, const ChTile* tiles, int ntiles, const StepDev* sd, StepArgs ta,
               int mode, hipStream_t s) {
  if (nw == 8) launch_nd<STAGE, 8>(drn, lds, tiles, ntiles, sd, ta, mode, s);
  else launch_nd<STAGE, 4>(drn, lds, tiles, ntiles, sd, ta, mode, s);
}

}  // namespace

void launch_chain(int stage, int nw, int drn, size_t lds_bytes, const ChTile* tiles, int ntiles, const StepDev* sd,
                  StepArgs ta, int mode, hipStream_t s) {
  if (ntiles <= 0) return;
  GLE_BOUNDS_SYNC();
  ta.nstatic = ntiles;
  if (nw != 4) ta.nfar = 0;  // far items need 4-wave workgroups (the planner never gives them others)
  if (stage == 0) launch_st<0>(nw, drn, lds_bytes, tiles, ntiles, sd, ta, mode, s);
  else if (stage == 1) launch_st<1>(nw, drn, lds_bytes, tiles, ntiles, sd, ta, mode, s);
  else if (stage == 2) launch_st<2>(nw, drn, lds_bytes, tiles, ntiles, sd, ta, mode, s);
  else if (stage == 3) launch_st<3>(nw, drn, lds_bytes, tiles, ntiles, sd, ta, mode, s);
  else if (stage == 4) launch_st<4>(nw, drn, lds_bytes, tiles, ntiles, sd, ta, mode, s);
  else launch_st<5>(nw, drn, lds_bytes, tiles, ntiles, sd, ta, mode, s);
}

namespace {
// md.potforce at q~ for every (DOF, trajectory) before the fused velocity stage.  With dyn as ELL
// (EW > 0 nonzeros per row, slot-major) every load of a thread goes out in two rounds: the cache
// word, Fc, q~, the bath row and the row's column / value slots first, then the q~ gathers and the
// V row; CSR (EW = 0) keeps the row-pointer round trip.
template <int EW>
__global__ __launch_bounds__(256) void fpot_kernel(FpotArgs a) {
#if FPOT_PRIO
  __builtin_amdgcn_s_setprio(CH_PRIO);  // on the main stream's critical path, like the chain stages
#endif
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)a.nph * a.B) return;
  const int d = (int)(i / a.B), b = (int)(i - (int64_t)d * a.B);
  const unsigned long long w = *G(a.pmax + ((int64_t)(1 * 2 + a.par)) * a.B + b);
  const double fc = G(a.Fc)[i], qt = G(a.Qt)[i];
  const int vb = G(a.vb)[d];
  int cl[EW > 0 ? EW : 1];
  double vl[EW > 0 ? EW : 1];
#pragma unroll
  for (int k = 0; k < EW; ++k) {
    cl[k] = G(a.col)[(int64_t)k * a.nph + d];
    vl[k] = G(a.val)[(int64_t)k * a.nph + d];
  }
  // the V row (or the noise row of a bath without memory sum), loaded beside the gathers
  double* V = a.V[0];
  const double* nz = a.noise[0];
  int nc = a.nc[0];
#pragma unroll
  for (int j = 1; j < MAXBATH; ++j)
    if ((vb >> 24) == j) {
      V = a.V[j];
      nz = a.noise[j];
      nc = a.nc[j];
    }
  const int k = vb & 0xFFFFFF;
  const int64_t o = vb >= 0 ? (int64_t)k * a.B + b : 0;
  const double v0 = vb < 0 ? 0.0 : (nz ? G(nz)[((int64_t)a.t1 * nc + k) * a.B + b] : G(V)[o]);
  double f;
  if (word_hit(w)) {  // md.potforce cache hit at q~ (md.py:449-450, 767-779)
    f = fc;
  } else {            // miss: f = -1.0*mdot(dyn, q~) and cache it (md.py:467-473)
    double acc = 0.0;
    if constexpr (EW > 0) {
      double x[EW];
#pragma unroll
      for (int s = 0; s < EW; ++s) x[s] = G(a.Qt)[(int64_t)cl[s] * a.B + b];
#pragma unroll
      for (int s = 0; s < EW; ++s) acc = vl[s] != 0.0 ? fma(vl[s], x[s], acc) : acc;  // padding: val 0.0
    } else {
      const int r0 = G(a.rp)[d], r1 = G(a.rp)[d + 1];
      for (int r = r0; r < r1; ++r) acc += G(a.val)[r] * G(a.Qt)[(int64_t)G(a.col)[r] * a.B + b];
    }
    f = -1.0 * acc;
    G(a.Fc)[i] = f;
    G(a.Q0)[i] = qt;
  }
  // V = n1 - c S1 (S(t+1) tiles of stage A) or n1 (no memory sum), plus the bath rows' Fpot(q~)
  if (vb >= 0) G(V)[o] = v0 + f;
}
}  // namespace

void launch_fpot(const FpotArgs& a, hipStream_t s) {
  const int64_t n = (int64_t)a.nph * a.B;
  if (n <= 0) return;
  GLE_BOUNDS_SYNC();
  const unsigned g = (unsigned)((n + 255) / 256);
  if (a.ew <= 0) fpot_kernel<0><<<g, 256, 0, s>>>(a);
  else if (a.ew <= 4) fpot_kernel<4><<<g, 256, 0, s>>>(a);
  else if (a.ew <= 8) fpot_kernel<8><<<g, 256, 0, s>>>(a);
  else fpot_kernel<FPOT_ELL><<<g, 256, 0, s>>>(a);
}

void bounds_publish_chain(const BoundsTab& t) {
#ifdef GLE_BOUNDS
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_btab), &t, sizeof(t));
#else
  (void)t;
#endif
}

}  // namespace gle
