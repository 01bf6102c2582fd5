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
// A workgroup owns a whole output tile (no split over workgroups): its 4 waves split the tile's
// k-steps, each wave keeps all of its operand loads in flight at once, the partial tiles meet in LDS
// and are added in a fixed order (deterministic).  Everything the epilogue reads that does not
// depend on the products is loaded before the products start, so a launch costs one descriptor
// round trip, one operand round trip, the MFMAs and the stores.
#include <hip/hip_runtime.h>

#include "gle_internal.h"

namespace gle {

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int64_t cmod(int64_t a, int64_t m) {
  int64_t r = a % m;
  return r < 0 ? r + m : r;
}

// k-steps a wave keeps in flight per batch
template <int RN>
struct Batch {
  static constexpr int U = RN == 1 ? 16 : (RN == 2 ? 8 : 4);
};

// The wave's tasks: acc += A_s . X rows 4s..4s+3 over each task's k-steps; a task run ends in its
// LDS slot (16 x 16 RN doubles, row-major).
template <int RN>
__device__ __forceinline__ void products(const ChTile* __restrict__ T, int wave, int lane, int64_t t, int B,
                                         double* lds) {
  constexpr int U = Batch<RN>::U;
  constexpr int NT = 16 * RN;
  const int nt = T->ntw[wave];
  const int brow = lane >> 4, bcol = lane & 15;
  d4 acc[RN];
#pragma unroll
  for (int n = 0; n < RN; ++n) acc[n] = d4{0.0, 0.0, 0.0, 0.0};
  int cur = -1;
  for (int i = 0; i < CH_TPW; ++i) {
    if (i >= nt) break;
    const ChTask tk = T->task[wave][i];
    if (tk.slot != cur) {
      if (cur >= 0) {
#pragma unroll
        for (int n = 0; n < RN; ++n)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            lds[cur * 16 * NT + (brow + 4 * q) * NT + 16 * n + bcol] = acc[n][q];
            acc[n][q] = 0.0;
          }
      }
      cur = tk.slot;
    }
    int64_t col = T->c0;
    if (tk.ring) col += cmod(t + tk.tshift, tk.ring) * (int64_t)B;
    const double* A = tk.A + lane;
    const double* X = tk.X + col + (int64_t)brow * tk.ldx + bcol;
    const int64_t xs = 4 * (int64_t)tk.ldx;
    for (int s0 = 0; s0 < tk.nks; s0 += U) {
      double a[U], b[U][RN];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int s = s0 + u;
        if (s < tk.nks) {
          a[u] = A[(int64_t)s * tk.a_ks];
#pragma unroll
          for (int n = 0; n < RN; ++n) b[u][n] = X[(int64_t)s * xs + 16 * n];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (s0 + u < tk.nks) {
#pragma unroll
          for (int n = 0; n < RN; ++n) acc[n] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], b[u][n], acc[n], 0, 0, 0);
        }
      }
    }
  }
  if (cur >= 0) {
#pragma unroll
    for (int n = 0; n < RN; ++n)
#pragma unroll
      for (int q = 0; q < 4; ++q) lds[cur * 16 * NT + (brow + 4 * q) * NT + 16 * n + bcol] = acc[n][q];
  }
}

__device__ __forceinline__ void run_products(const ChTile* __restrict__ T, int64_t t, int B, double* lds) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  switch (T->rn) {
    case 1: products<1>(T, wave, lane, t, B, lds); break;
    case 2: products<2>(T, wave, lane, t, B, lds); break;
    default: products<4>(T, wave, lane, t, B, lds); break;
  }
}

// output o of a 16 x 16 tile at element e (slots of 256 doubles), added in slot order
__device__ __forceinline__ double out_sum(const ChTile* __restrict__ T, const double* lds, int o, int e) {
  double v = 0.0;
  for (int s = T->ob[o]; s < T->ob[o + 1]; ++s) v += lds[s * 256 + e];
  return v;
}

__device__ __forceinline__ unsigned long long* pmax_word(const StepDev* sd, int id, int par, int b) {
  return sd->pmax + ((int64_t)(id * 2 + par)) * sd->B + b;
}

// md.potforce's cache rule (sameq, md.py:449-450, 767-779) per trajectory: hit iff the cache is
// valid and max_d |q - q0| < 1e-9.  The max is one word per trajectory, accumulated with atomicMax
// on the bit pattern (non-negative doubles order like their bits; NaN exceeds every finite value).
__device__ __forceinline__ bool word_hit(unsigned long long w) {
  const double m = __longlong_as_double((long long)w);
  return m == m && m < 10e-10;
}

// per-trajectory reductions over the 16 rows of a DOF tile: thread e = r*16 + c holds row r,
// column c.  red: 16 x 16 doubles of LDS scratch.
__device__ __forceinline__ double col_sum(double v, double* red) {
  __syncthreads();
  red[threadIdx.x] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x < 16)
    for (int r = 0; r < 16; ++r) s += red[r * 16 + threadIdx.x];
  return s;
}
__device__ __forceinline__ double col_max(double v, double* red, bool& nan) {
  __syncthreads();
  red[threadIdx.x] = v;
  __syncthreads();
  double m = 0.0;
  nan = false;
  if (threadIdx.x < 16)
    for (int r = 0; r < 16; ++r) {
      const double w = red[r * 16 + threadIdx.x];
      nan |= (w != w);
      m = fmax(m, w);
    }
  return m;
}

struct Elem {
  int r, d, b;
  int64_t i;
  bool ok;
};

__device__ __forceinline__ Elem elem_of(const ChTile* __restrict__ T, const StepDev* __restrict__ sd) {
  Elem E;
  E.r = threadIdx.x >> 4;
  E.d = T->row0 + E.r;
  E.b = T->c0 + (threadIdx.x & 15);
  E.ok = E.d < sd->nph && E.b < sd->B;
  E.i = (int64_t)E.d * sd->B + E.b;
  return E;
}

// bath-local row of the element's DOF in tile bath u (bath bd), or -1
__device__ __forceinline__ int bath_row(const ChTile* __restrict__ T, const BathDev& bd, int u, const Elem& E) {
  if (!E.ok || !((T->bmask[u] >> E.r) & 1u)) return -1;
  const int off = T->boff[u];
  return off == CH_INV ? bd.inv[E.d] : E.d + off;
}

// ------------------------------------------------------------------------------------------
// stage A, DOF tile
__device__ __forceinline__ void dof_A(const ChTile* __restrict__ T, const StepDev* __restrict__ sd,
                                      const StepArgs& ta, int mode, double* lds) {
  const int B = sd->B, nb = sd->nbath;
  const int64_t t = ta.t;
  const int tn = (int)(t % sd->nmd);
  const int par = (int)(t & 1);
  const double dt = sd->dt, dt2 = dt * dt;
  const bool harm = (mode & 1) != 0, diff1 = (mode & 2) != 0;
  const Elem E = elem_of(T, sd);
  // ---- loads that do not depend on the products
  double p = 0.0, q = 0.0, fc = 0.0, q0 = 0.0;
  unsigned long long w0 = 0;
  if (E.ok) {
    p = sd->P[E.i];
    q = sd->Q[E.i];
    fc = sd->Fc[E.i];
    if (harm || diff1) q0 = sd->Q0[E.i];
    if (harm) w0 = (sd->qvalid[E.b] != 0) ? *pmax_word(sd, 0, par, E.b) : 0x7FF8000000000000ull;
  }
  int kk[CH_TB];
  double nz[CH_TB], sv[CH_TB];
#pragma unroll
  for (int u = 0; u < CH_TB; ++u) {
    kk[u] = -1;
    nz[u] = sv[u] = 0.0;
    const int j = T->tb[u];
    if (j >= 0) {
      const BathDev& bd = sd->bath[j];
      kk[u] = bath_row(T, bd, u, E);
      if (kk[u] >= 0) {
        nz[u] = bd.noise[((int64_t)tn * bd.nc + kk[u]) * B + E.b];
        sv[u] = bd.S[(int64_t)par * bd.vs + (int64_t)kk[u] * B + E.b];
      }
    }
  }
  if (T->first && threadIdx.x < 16 && E.b < B) *pmax_word(sd, 0, par ^ 1, E.b) = 0ull;
  run_products(T, t, B, lds);
  __syncthreads();
  // ---- epilogue (md.vv id0, md.py:383-397)
  const int e = threadIdx.x;
  const bool hit = harm ? word_hit(w0) : true;
  double f = fc;  // potforce(q_t)
  if (!hit) {
    f = -1.0 * out_sum(T, lds, 2 * CH_TB, e);  // f = -1.0*mdot(dyn, q)  (md.py:467)
    if (E.ok) {
      sd->Fc[E.i] = f;
      sd->Q0[E.i] = q;
    }
  }
  double cur[CH_TB];
#pragma unroll
  for (int u = 0; u < CH_TB; ++u) {
    cur[u] = 0.0;
    if (kk[u] >= 0) {
      const BathDev& bd = sd->bath[T->tb[u]];
      double fb = nz[u] - bd.c * (out_sum(T, lds, u, e) + sv[u]);
      if (bd.has_q) fb -= out_sum(T, lds, CH_TB + u, e);
      f += fb;           // pf = pf + fbaths[i]  (md.py:432-434)
      cur[u] = fb * p;   // cur[t] = fbaths[i].p (md.py:397)
    }
  }
  const double ph = p + f * dt / 2.0;            // md.py:391
  const double qt = q + p * dt + f * dt2 / 2.0;  // md.py:392
  if (E.ok) {
    sd->Ph[E.i] = ph;
    sd->Qt[E.i] = qt;
  }
#pragma unroll
  for (int u = 0; u < CH_TB; ++u) {
    if (kk[u] >= 0) {
      const BathDev& bd = sd->bath[T->tb[u]];
      const int64_t kb = (int64_t)kk[u] * B + E.b;
      bd.Xcur[kb] = ph;
      if (bd.has_q) bd.Xq[bd.vs + kb] = qt;
    }
  }
  // per-trajectory sums over the tile's DOFs (fixed order), one row of the step's partial table
  // [tile][bath | energy]; baths that miss the tile get zeros
  double* red = lds;
  double* prow = sd->part + (((int64_t)tn * sd->ndblk + T->tile) * (nb + 1)) * B;
  const bool wcol = threadIdx.x < 16 && E.b < B;
  for (int j = 0; j < nb; ++j) {
    int uj = -1;
#pragma unroll
    for (int u = 0; u < CH_TB; ++u)
      if (T->tb[u] == j) uj = u;
    double s = 0.0;
    if (uj >= 0) {
      double cj = 0.0;
#pragma unroll
      for (int u = 0; u < CH_TB; ++u)
        if (u == uj) cj = cur[u];
      s = col_sum(cj, red);
    }
    if (wcol) prow[(int64_t)j * B + E.b] = s;
  }
  {
    const double s = col_sum(E.ok ? p * p : 0.0, red);
    if (wcol) prow[(int64_t)nb * B + E.b] = s;
  }
  if (diff1) {
    const double dq = E.ok ? fabs(qt - (hit ? q0 : q)) : 0.0;
    bool nan;
    const double m = col_max(dq, red, nan);
    if (wcol) {
      const unsigned long long bits = nan ? 0x7FF8000000000000ull : (unsigned long long)__double_as_longlong(m);
      atomicMax(pmax_word(sd, 1, par, E.b), bits);
    }
  }
}

// stage B, DOF tile
__device__ __forceinline__ void dof_B(const ChTile* __restrict__ T, const StepDev* __restrict__ sd,
                                      const StepArgs& ta, int mode, double* lds) {
  const int B = sd->B;
  const int64_t t = ta.t;
  const int t1 = (int)((t + 1) % sd->nmd);
  const int par = (int)(t & 1), par1 = par ^ 1;
  const double dt = sd->dt;
  const bool harm = mode != 0;
  const Elem E = elem_of(T, sd);
  double ph = 0.0, qt = 0.0, fc = 0.0;
  unsigned long long w1 = 0;
  if (E.ok) {
    ph = sd->Ph[E.i];
    qt = sd->Qt[E.i];
    fc = sd->Fc[E.i];
    if (harm) w1 = *pmax_word(sd, 1, par, E.b);
  }
  int kk[CH_TB];
  double nz[CH_TB], sv[CH_TB];
#pragma unroll
  for (int u = 0; u < CH_TB; ++u) {
    kk[u] = -1;
    nz[u] = sv[u] = 0.0;
    const int j = T->tb[u];
    if (j >= 0) {
      const BathDev& bd = sd->bath[j];
      kk[u] = bath_row(T, bd, u, E);
      if (kk[u] >= 0) {
        nz[u] = bd.noise[((int64_t)t1 * bd.nc + kk[u]) * B + E.b];
        sv[u] = bd.S[(int64_t)par1 * bd.vs + (int64_t)kk[u] * B + E.b];
      }
    }
  }
  run_products(T, t, B, lds);
  __syncthreads();
  const int e = threadIdx.x;
  const bool hit1 = harm ? word_hit(w1) : true;
  double f = fc;  // potforce(q~)
  if (!hit1) {
    f = -1.0 * out_sum(T, lds, 2 * CH_TB, e);
    if (E.ok) {  // md.potforce miss at q~: evaluate and cache (md.py:472-473)
      sd->Fc[E.i] = f;
      sd->Q0[E.i] = qt;
    }
  }
  bool inb = false;
#pragma unroll
  for (int u = 0; u < CH_TB; ++u) {
    if (kk[u] >= 0) {
      const BathDev& bd = sd->bath[T->tb[u]];
      const int64_t kb = (int64_t)kk[u] * B + E.b;
      double fb = nz[u] - bd.c * (out_sum(T, lds, u, e) + sv[u]);
      if (bd.has_q) {
        const double yq = out_sum(T, lds, CH_TB + u, e);
        fb -= yq;
        bd.Yq[kb] = yq;  // Kq.q~ is the same in both id1 calls
      }
      f += fb;
      inb = true;
    }
  }
  if (inb) {
    const double p1 = ph + dt * f / 2.0;  // md.py:402 (p1 only feeds the bath friction terms)
#pragma unroll
    for (int u = 0; u < CH_TB; ++u)
      if (kk[u] >= 0) {
        const BathDev& bd = sd->bath[T->tb[u]];
        bd.Xcur[bd.vs + (int64_t)kk[u] * B + E.b] = p1;
      }
  }
}

// stage C, DOF tile
__device__ __forceinline__ void dof_C(const ChTile* __restrict__ T, const StepDev* __restrict__ sd,
                                      const StepArgs& ta, int mode, double* lds) {
  const int B = sd->B;
  const int64_t t = ta.t;
  const int t1 = (int)((t + 1) % sd->nmd);
  const int par = (int)(t & 1), par1 = par ^ 1;
  const double dt = sd->dt;
  const bool harm = mode != 0;
  const Elem E = elem_of(T, sd);
  double ph = 0.0, qt = 0.0, fc = 0.0, q0 = 0.0;
  bool cons = false;
  if (E.ok) {
    ph = sd->Ph[E.i];
    qt = sd->Qt[E.i];
    fc = sd->Fc[E.i];
    cons = sd->cmask[E.d] != 0;
    if (harm) q0 = sd->Q0[E.i];
  }
  int kk[CH_TB];
  double nz[CH_TB], sv[CH_TB], yq[CH_TB];
#pragma unroll
  for (int u = 0; u < CH_TB; ++u) {
    kk[u] = -1;
    nz[u] = sv[u] = yq[u] = 0.0;
    const int j = T->tb[u];
    if (j >= 0) {
      const BathDev& bd = sd->bath[j];
      kk[u] = bath_row(T, bd, u, E);
      if (kk[u] >= 0) {
        const int64_t kb = (int64_t)kk[u] * B + E.b;
        nz[u] = bd.noise[((int64_t)t1 * bd.nc + kk[u]) * B + E.b];
        sv[u] = bd.S[(int64_t)par1 * bd.vs + kb];
        if (bd.has_q) yq[u] = bd.Yq[kb];
      }
    }
  }
  if (T->first && threadIdx.x < 16 && E.b < B) {
    *pmax_word(sd, 1, par1, E.b) = 0ull;
    if (harm) sd->qvalid[E.b] = 1;
  }
  run_products(T, t, B, lds);
  __syncthreads();
  const int e = threadIdx.x;
  double f = fc;
#pragma unroll
  for (int u = 0; u < CH_TB; ++u) {
    if (kk[u] >= 0) {
      const BathDev& bd = sd->bath[T->tb[u]];
      f += nz[u] - bd.c * (out_sum(T, lds, u, e) + sv[u]) - yq[u];
    }
  }
  double p2 = ph + dt * f / 2.0;  // md.py:404
  double qn = qt;
  if (cons) {  // ApplyConstraint (md.py:407-408, 782-794)
    p2 = 0.0;
    qn = 0.0;
  }
  if (E.ok) {
    sd->P[E.i] = p2;
    sd->Q[E.i] = qn;
    sd->Flast[E.i] = f;
  }
#pragma unroll
  for (int u = 0; u < CH_TB; ++u) {
    if (kk[u] >= 0) {
      const BathDev& bd = sd->bath[T->tb[u]];
      // history push of p_{t+1} (rpadleft, md.py:387 of the next step), mirrored slot
      const int64_t slot = cmod(t + 1, bd.R);
      double* h = bd.H + (int64_t)kk[u] * bd.ldh + E.b;
      h[slot * B] = p2;
      h[(slot + bd.R) * B] = p2;
      if (bd.has_q) bd.Xq[(int64_t)kk[u] * B + E.b] = qn;
    }
  }
  if (harm) {  // cache distance of q_{t+1} for the next step's id0 call
    const double dq = E.ok ? fabs(qn - q0) : 0.0;
    bool nan;
    const double m = col_max(dq, lds, nan);
    if (threadIdx.x < 16 && E.b < B) {
      const unsigned long long bits = nan ? 0x7FF8000000000000ull : (unsigned long long)__double_as_longlong(m);
      atomicMax(pmax_word(sd, 0, par1, E.b), bits);
    }
  }
}

// S(t+1) of bath rows [row0, row0+16): K_1.p_t (the products) + near-field partials + levels
__device__ __forceinline__ void sfin(const ChTile* __restrict__ T, const StepDev* __restrict__ sd,
                                     const StepArgs& ta, double* lds) {
  const int B = sd->B;
  const int64_t t = ta.t;
  const int par1 = (int)((t + 1) & 1);
  const BathDev& bd = sd->bath[T->tile];
  const int r = threadIdx.x >> 4;
  const int k = T->row0 + r;
  const int b = T->c0 + (threadIdx.x & 15);
  const bool ok = k < bd.nc && b < B;
  const int64_t kb = (int64_t)k * B + b;
  // near-field partials and level blocks, added in slot / level order (8 loads in flight)
  double sn = 0.0, pre = 0.0;
  if (ok) {
    const double* np = bd.NP + (int64_t)par1 * bd.nqn * bd.vs + kb;
    for (int q0 = 0; q0 < bd.nqn; q0 += 8) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = (q0 + u < bd.nqn) ? np[(int64_t)(q0 + u) * bd.vs] : 0.0;
#pragma unroll
      for (int u = 0; u < 8; ++u) sn += v[u];
    }
    double lv[MAXLVL];
#pragma unroll
    for (int l = 0; l < MAXLVL; ++l)
      lv[l] = (l < bd.nlvl && bd.lvl[l]) ? bd.lvl[l][(int64_t)k * bd.lvl_ld[l] + ta.lvl_off[l] + b] : 0.0;
#pragma unroll
    for (int l = 0; l < MAXLVL; ++l) pre += lv[l];
  }
  run_products(T, t, B, lds);
  __syncthreads();
  const double s = out_sum(T, lds, 0, threadIdx.x) + sn;
  if (ok) bd.S[(int64_t)par1 * bd.vs + kb] = pre + s;
}

// near-field partial tile: rows [0, nrows) x columns [0, ncols) of the parity buffer of t + par_shift
__device__ __forceinline__ void raw(const ChTile* __restrict__ T, const StepDev* __restrict__ sd, const StepArgs& ta, double* lds) {
  const int64_t t = ta.t;
  run_products(T, t, sd->B, lds);
  __syncthreads();
  const int rn = T->rn, NT = 16 * rn;
  double* dst = T->dst + ((t + T->par_shift) & 1) * T->par_stride;
  for (int e = threadIdx.x; e < 16 * NT; e += CH_NW * 64) {
    double v = 0.0;
    for (int s = T->ob[0]; s < T->ob[1]; ++s) v += lds[s * 16 * NT + e];
    const int row = e / NT, col = e - row * NT;
    if (row < T->nrows && col < T->ncols) dst[(int64_t)row * T->ldd + col] = v;
  }
}

template <int STAGE>
__global__ __launch_bounds__(CH_NW * 64) void chain_kernel(const ChTile* __restrict__ tiles,
                                                           const StepDev* __restrict__ sd, StepArgs ta,
                                                           int mode) {
  __shared__ double lds[CH_LDS];
  const ChTile* T = tiles + blockIdx.x;
  const int kind = T->kind;
  if (kind == CH_DOF) {
    if (STAGE == 0) dof_A(T, sd, ta, mode, lds);
    else if (STAGE == 1) dof_B(T, sd, ta, mode, lds);
    else dof_C(T, sd, ta, mode, lds);
  } else if (kind == CH_SFIN) {
    sfin(T, sd, ta, lds);
  } else {
    raw(T, sd, ta, lds);
  }
}

}  // namespace

void launch_chain(int stage, const ChTile* tiles, int ntiles, const StepDev* sd, StepArgs ta, int mode,
                  hipStream_t s) {
  if (ntiles <= 0) return;
  switch (stage) {
    case 0: chain_kernel<0><<<ntiles, CH_NW * 64, 0, s>>>(tiles, sd, ta, mode); break;
    case 1: chain_kernel<1><<<ntiles, CH_NW * 64, 0, s>>>(tiles, sd, ta, mode); break;
    default: chain_kernel<2><<<ntiles, CH_NW * 64, 0, s>>>(tiles, sd, ta, mode); break;
  }
}

}  // namespace gle
