// Memory-kernel construction on gfx950: phbath.gmem / gamt (baths.py:19-52, 412-445).
//
// The reference evaluates K(t_i) = scale * mean_w flinterp(w, gwl, Gamma) * c(w, t_i) in a Python
// loop over (t, w).  flinterp is linear in Gamma (two weights per w, functions.py:117-134), so the
// whole kernel is one contraction over the ngw nodes of the friction spectrum:
//
//     K[i][e] = sum_g W[i][g] * G[g][e],   W = scale * C(t, w) . I(w -> gwl)   (ml x ngw, host)
//
// with e over the nc*nc matrix elements.  kgen_kernel does it on v_mfma_f64_16x16x4_f64:
//   * a workgroup owns one 64-element block of e (for the stepper: one 16x4 MFMA A-fragment of
//     every kernel slice, i.e. the fragment-native layout the contractions stream) and stages the
//     block's G rows [g0, g0 + 4 nkc) in LDS once;
//   * its 4 waves take interleaved 16-slice row tiles i; per tile the W^T columns (A operand, L2
//     resident, shared by every workgroup) are loaded into registers in one batch, the 4 MFMA
//     column tiles read B from LDS, and the 16 x 64 result is written straight to its final place
//     (fragment-native: 16 slices x 512 B contiguous), so the kernel is written to HBM exactly once
//     and never crosses PCIe.
// ngw > 4*KC_MAX is handled in chunks that accumulate into the output (setup only).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gle_internal.h"

namespace gle {

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int KC_MAX = 32;  // k-steps (4 g each) per chunk: 128 g rows, 64 KiB of LDS

// out block b (64 lanes), slice i:  out[b * o_blk + i * o_row + lane]
// G  block b, row g:                G[b * g_blk + g * g_row + lane]   (lane < nvalid(b), g < ngw)
__global__ __launch_bounds__(256) void kgen_kernel(const double* __restrict__ WT, int64_t mlp, int g0, int nkc,
                                                   int ngw, const double* __restrict__ G, int64_t g_blk,
                                                   int64_t g_row, double* __restrict__ out, int64_t o_blk,
                                                   int64_t o_row, int ml, int64_t nblk, int nvalid_last,
                                                   int accumulate) {
  __shared__ double gs[4 * KC_MAX * 64];
  // XCD-aware order: consecutive blocks of e land on one XCD, so each XCD writes contiguous HBM
  const int64_t nb = gridDim.x;
  const int64_t b = (nb & 7) ? (int64_t)blockIdx.x : (int64_t)(blockIdx.x & 7) * (nb >> 3) + (blockIdx.x >> 3);
  if (b >= nblk) return;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int nvalid = (b == nblk - 1) ? nvalid_last : 64;
  // stage G rows g0 .. g0 + 4 nkc of this block (zero beyond ngw or the valid lanes)
  for (int r = wave; r < 4 * nkc; r += 4) {
    const int g = g0 + r;
    double v = 0.0;
    if (g < ngw && lane < nvalid) v = G[b * g_blk + (int64_t)g * g_row + lane];
    gs[r * 64 + lane] = v;
  }
  __syncthreads();
  const int brow = lane >> 4, bcol = lane & 15;
  const int ntile = (int)(mlp >> 4);
  double* ob = out + b * o_blk;
  for (int it = wave; it < ntile; it += 4) {
    double a[KC_MAX];
    // A operand: lane holds W[i = 16 it + (lane & 15)][g = g0 + 4 s + (lane >> 4)] = WT[g][i]
    const double* wp = WT + (int64_t)(g0 + brow) * mlp + 16 * it + bcol;
#pragma unroll
    for (int s = 0; s < KC_MAX; ++s)
      if (s < nkc) a[s] = wp[(int64_t)4 * s * mlp];
    d4 acc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[n] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < KC_MAX; ++s) {
      if (s < nkc) {
        // B operand: lane holds G[g = 4 s + (lane >> 4)][e = 16 n + (lane & 15)]
        const double* gp = gs + (4 * s + brow) * 64 + bcol;
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[n] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], gp[16 * n], acc[n], 0, 0, 0);
      }
    }
    // D: lane holds rows (lane >> 4) + 4 q, column lane & 15 of each 16 x 16 column tile
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = 16 * it + brow + 4 * q;
      if (i >= ml) continue;
      double* op = ob + (int64_t)i * o_row + bcol;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        if (16 * n + bcol >= nvalid) continue;
        const double v = acc[n][q];
        op[16 * n] = accumulate ? op[16 * n] + v : v;
      }
    }
  }
}

// gamma [ngw][nc][nc] -> fragment-native GF[frag][ngwp][64], frag = rt * nks + ks, lane l holds
// element (16 rt + (l & 15), 4 ks + (l >> 4)); zero padding outside nc
__global__ void gamma_pack_kernel(const double* __restrict__ gam, int ngw, int ngwp, int nc, int nrt, int nks,
                                  double* __restrict__ gf) {
  const int64_t n = (int64_t)nrt * nks * ngwp * 64;
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n; x += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)(x & 63);
    const int64_t y = x >> 6;
    const int g = (int)(y % ngwp);
    const int64_t frag = y / ngwp;
    const int rt = (int)(frag / nks), ks = (int)(frag % nks);
    const int r = 16 * rt + (l & 15), c = 4 * ks + (l >> 4);
    gf[x] = (g < ngw && r < nc && c < nc) ? gam[((int64_t)g * nc + r) * nc + c] : 0.0;
  }
}

}  // namespace

int launch_kgen(const double* WT, int64_t mlp, int ngw, const double* G, int64_t g_blk, int64_t g_row,
                double* out, int64_t o_blk, int64_t o_row, int ml, int64_t nblk, int nvalid_last, hipStream_t s) {
  if (nblk <= 0 || ml <= 0 || ngw <= 0 || (mlp & 15) || mlp < ml || nvalid_last < 1 || nvalid_last > 64) return -1;
  const int64_t grid = (nblk + 7) / 8 * 8;  // multiple of 8 for the XCD-aware order
  if (grid > INT32_MAX) return -1;
  const int ngwp = (ngw + 3) / 4 * 4;
  for (int g0 = 0; g0 < ngwp; g0 += 4 * KC_MAX) {
    const int nkc = (ngwp - g0) / 4 < KC_MAX ? (ngwp - g0) / 4 : KC_MAX;
    hipLaunchKernelGGL(kgen_kernel, dim3((unsigned)grid), dim3(256), 0, s, WT, mlp, g0, nkc, ngw, G, g_blk, g_row,
                       out, o_blk, o_row, ml, nblk, nvalid_last, g0 > 0 ? 1 : 0);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

void launch_gamma_pack(const double* gam, int ngw, int ngwp, int nc, int nrt, int nks, double* gf, hipStream_t s) {
  const int64_t n = (int64_t)nrt * nks * ngwp * 64;
  int64_t grid = (n + 255) / 256;
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(gamma_pack_kernel, dim3((unsigned)grid), dim3(256), 0, s, gam, ngw, ngwp, nc, nrt, nks, gf);
}

}  // namespace gle
