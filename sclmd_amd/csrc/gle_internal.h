// Internal data structures of the hipgle library (device layouts, work descriptors).
//
// Device layout (DOF-major, trajectory-fastest: every per-step array is [rows][B]):
//   state        P, Q, Ph (p half), Qt (q~), G, Fc (cached potential force), Flast   [nph][B]
//   bath ring    H_b [ncp][2R*B + slack] : p restricted to the bath's cids; time slot
//                tau lives at columns (tau mod R)*B + b AND (tau mod R + R)*B + b (mirror), so
//                any window of <= R consecutive slots is one contiguous column range.
//   noise        [nmd][nc][B]
//   kernel K     MFMA-fragment-native: frag(rt, ks, i) = 64 doubles, lane l holds
//                K_i[16*rt + (l&15)][4*ks + (l>>4)] (the A-operand map of v_mfma_f64_16x16x4_f64),
//                stored [rt][ks][i][64] so a wave streams consecutive slices contiguously.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace gle {

constexpr int WG = 256;            // threads per workgroup of the contraction kernel (4 waves)
constexpr int KC = 2;              // k-steps (4 rows each) staged per LDS stage
constexpr int KROWS = 4 * KC;      // 8 staged X rows
constexpr int LDS_COLS = 1000;     // padded staged row length (doubles): 8*1000*8 = 62.5 KB
constexpr int LDS_WW_MAX = 960;    // usable window width: roundup32(960) + 16 <= LDS_COLS
constexpr int MAXBATH = 8;
constexpr int MAXLVL = 12;         // levels of the memory-sum ladder
constexpr int CPLX_WW_CAP = 512;   // contract_cplx_kernel window (doubles per staged row)
constexpr int ROWS_PER_WG = 64;    // 4 waves x 16 rows

// One workgroup's share of a contraction  out[r][c] = sum_{i in slices} sum_k A_i[r][k] X_i[k][c]
// where X_i is either a static matrix or a window of a bath history ring ending at the target time.
struct CItem {
  const double* A;   // fragment base for (row tile rt0, k-step ks0, slice ia)
  const double* X;   // X base at row 4*ks0 (ring: the ring buffer; static: column 0 of the window)
  double* out;       // output tile: rows [0, nrows) of this group, columns [0, ncols)
  int64_t a_rt;      // doubles between consecutive row tiles in A
  int64_t a_ks;      // doubles between consecutive k-steps in A
  int32_t nks;       // k-steps in this item (even)
  int32_t ia;        // first slice (absolute index, used for the window time)
  int32_t ni;        // number of slices
  int32_t nrt;       // row tiles present (1..4)
  int32_t ldx;       // X row stride (doubles)
  int32_t ldo;       // out row stride (doubles)
  int32_t ring;      // R (ring slots) for history windows, 0 for a static X
  int32_t cs;        // columns per time slot (= B) for ring windows
  int32_t tshift;    // window target time = clock.t + tshift; slice i starts at target - i
  int32_t col0;      // column offset of this tile inside the window
  int32_t ncols;     // valid columns to store
  int32_t nrows;     // valid rows to store (<= 64)
  int32_t tdiv;      // ring index = floor(clock.t / tdiv) + tshift - slice (1: steps, P: segments)
  int32_t pad;
  // complex items (contract_cplx_kernel): imaginary parts at these offsets (doubles) from A, X, out
  int64_t a_im, x_im, o_im;
};

// One share of a 16-row output tile of a latency-bound per-step product.  The tile's slice x
// k-step space is split over ngrp workgroups of 4 waves; waves reduce through LDS, groups through
// partial slots summed in fixed order by the last group to arrive (far / mid addends in its
// epilogue).  Same operand conventions as CItem.
struct TItem {
  double* part;        // [ngrp][256*RN] partial slots of this tile (ngrp > 1)
  unsigned* cnt;       // arrival counter of this tile (ngrp > 1)
  const double* A;     // fragment base for (row tile, k-step 0, slice ia)
  const double* X;     // X base (row 0)
  double* out;         // tile output (row 0 of the tile, column 0)
  const double* add[MAXLVL];  // level block buffers (row 0 of the tile; the step's column
                              // offset is StepArgs::lvl_off), first nadd used
  int64_t a_ks;        // doubles between k-steps in A (slice stride is 64)
  int64_t ldx;
  int32_t add_ld[MAXLVL];
  int32_t nadd;
  int32_t ldo;
  int32_t ia, ni, nks; // slices [ia, ia+ni), k-steps
  int32_t ring, cs, tshift;
  int32_t nrows, ncols;
  int32_t grp, ngrp;   // this workgroup's share, number of shares
};

// Deterministic fixed-order sum of split partial tiles (+ optional far-field addend).
struct RItem {
  double* dst;
  const double* src;   // first partial slot
  int32_t ldd;         // dst row stride
  int32_t lds;         // partial row stride
  int32_t nslots;
  int32_t pad;
  int64_t slot_stride; // doubles between partial slots
  int32_t rows, cols;
};


struct BathDev {
  const int32_t* inv;  // [nph] -> bath-local index k or -1
  const double* noise; // [nmd][nc][B]
  double* Y;           // K0 . x       [ncp][B]
  double* S;           // memory sums S(t) double buffer [2][ncp][B]
  double* Yq;          // q-channel K . q (biased ebath) [ncp][B] or nullptr
  double* Xcur;        // gathered x (p half / p1) [ncp][B]
  double* Xq;          // gathered q [ncp][B]
  double* H;           // history ring
  double* cur;         // heat current [nmd][B]
  double c;            // dt factor (dt if ml > 1 else 1, baths.py:454-457)
  int32_t nc, ncp;
  int32_t ldh, R;
  int32_t has_q;
  int32_t pad;
};

struct StepDev {
  int32_t nph, B, nmd, nbath;
  double dt;
  double *P, *Q, *Ph, *Qt, *G, *Fc, *Flast, *etot;
  double* Q0;             // last q the potential force was evaluated at (md.q0)
  int32_t* qvalid;        // [B] md.q0 != [] flag
  double* Ypot;           // dyn . x of the latest potential product [nph][B]
  unsigned long long* pmax;  // [2 (id0,id1)][2 (parity)][B] max |x - q0| as ordered bit patterns
  double* part;           // [nmd][ndblk][nbath+1][B] current / energy partial sums per step
  const uint8_t* cmask;   // [nph] constraint mask
  int32_t ndblk;          // DOF chunks of the phase kernels
  int32_t dchunk;         // DOFs per chunk
  BathDev bath[MAXBATH];
};

// launchers (gle_kernels.hip)
// Every kernel takes the step counter by value: the host knows md.t and the steps at which the
// current far / mid blocks were computed, so no kernel starts with a dependent load of a clock
struct StepArgs {
  int64_t t;                 // md.t of this step
  int64_t lvl_off[MAXLVL];   // per level: offset (doubles) of target t+1 in its block buffer
};
void launch_contract(int rn, int cu, const CItem* items, int nitems, StepArgs ta, hipStream_t s);
void launch_reduce(const RItem* items, int nitems, int max_elems, StepArgs ta,
                   hipStream_t s);
void launch_phaseA(const StepDev* sd, StepArgs ta, int B, int ndblk, int mode0, int diff1,
                   hipStream_t s);
void launch_phaseB(const StepDev* sd, StepArgs ta, int B, int ndblk, int mode1, hipStream_t s);
void launch_phaseC(const StepDev* sd, StepArgs ta, int B, int ndblk, int mode1, int diff0,
                   hipStream_t s);
void launch_finalize(const StepDev* sd, int B, int nmd, int nbath, hipStream_t s);
void launch_philox_normal(double* x, int64_t nfreq, int64_t ncp, int64_t nc, int64_t B,
                          uint64_t seed, uint64_t traj_offset, hipStream_t s);
void launch_ring_copy(double* H, int64_t ldh, int R, int B, int nc, int64_t tau0, int nt, double* buf,
                      int dir, hipStream_t s);
void launch_tile(int rn, const TItem* items, int nitems, StepArgs ta, hipStream_t s);
void launch_contract_cplx(int rn, const CItem* items, int nitems, StepArgs ta, hipStream_t s);
void launch_khat_pack(const double* Kf, int ml, int nks_k, double* khat, int P, int m0, int M,
                      int nc, int nrt2, int nks2, const double* cstab, int cstride, hipStream_t s);
int launch_seg_fft(const double* H, int64_t ldh, int R, int B, int nc, int ncp, int P, int64_t T,
                   int nseg, double* seg, int64_t seg_fstride, int64_t ldseg, int Rseg,
                   const double* cstab, int cstride, hipStream_t s);
int launch_far_ifft(const double* Y, int64_t yfstride, int nc, int B, int P, double* out,
                    int64_t ldout, const double* cstab, int cstride, hipStream_t s);
int launch_fft_noise(const double* a, double* noise, const double* tw, int64_t nmd, int64_t nc,
                     int64_t arows, int64_t B, int is_complex, double scale, hipStream_t s);

}  // namespace gle
