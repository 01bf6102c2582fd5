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
#include <cstdlib>

namespace gle {

// Experiment switches (GLE_* environment variables: plan variants, timing-only variants that skip
// work and give wrong results, timelines) exist only in a -DGLE_EXPERIMENTS build
// (`make experiments`).  The release library reads no environment at all.
inline const char* gle_env(const char* name) {
#ifdef GLE_EXPERIMENTS
  return std::getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

// -DGLE_BOUNDS audit build (`make experiments EXPNAME=bounds EXPFLAGS=-DGLE_BOUNDS`): the chain,
// cgemm and contraction operand loads and the chain's stores check their address against the
// live allocations, each with its LOGICAL extent (without the slack some allocations carry).  A
// miss never faults: it is counted and the first BND_KEEP (address, site) pairs kept; gle_sync
// and gle_run then fail with them.  Sites are source lines.
struct BoundsTab {
  int n = 0;
  unsigned long long* viol = nullptr;  // [0] count, then (address, site) pairs
  const uint64_t* lo = nullptr;        // sorted allocation starts
  const uint64_t* hi = nullptr;        // logical ends
};
constexpr int BND_KEEP = 32;
#ifdef GLE_BOUNDS
static __device__ BoundsTab g_btab;  // one copy per translation unit, set by its bounds_publish_*
__device__ inline void bcheck(const void* p, int bytes, int site) {
  const BoundsTab& T = g_btab;
  if (!T.viol) return;
  const uint64_t a = (uint64_t)p;
  int lo = 0, hi = T.n;  // last allocation starting at or below a
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (T.lo[mid] <= a) lo = mid;
    else hi = mid;
  }
  if (T.n > 0 && a >= T.lo[lo] && a + (uint64_t)bytes <= T.hi[lo]) return;
  const unsigned long long k = atomicAdd(&T.viol[0], 1ull);
  if (k < BND_KEEP) {
    T.viol[1 + 2 * k] = a;
    T.viol[2 + 2 * k] = (unsigned long long)site;
  }
}
#define GLE_BCHK(p) ::gle::bcheck((const void*)(p), (int)sizeof(*(p)), __LINE__)
#else
#define GLE_BCHK(p) ((void)0)
#endif
#define BLD(p) (GLE_BCHK(p), *(p))  // checked load (a plain load outside the audit build)
#ifdef GLE_BOUNDS
void bounds_sync();  // publishes the allocation table if it changed (called by every checked launch)
#define GLE_BOUNDS_SYNC() ::gle::bounds_sync()
#else
#define GLE_BOUNDS_SYNC() ((void)0)
#endif
void bounds_publish_chain(const BoundsTab& t);
void bounds_publish_kernels(const BoundsTab& t);

constexpr int WG = 256;            // threads per workgroup of the contraction kernel (4 waves)
constexpr int KC = 2;              // k-steps (4 rows each) staged per LDS stage
constexpr int KROWS = 4 * KC;      // 8 staged X rows
constexpr int LDS_COLS = 1000;     // padded staged row length (doubles): 8*1000*8 = 62.5 KB
constexpr int LDS_WW_MAX = 960;    // usable window width: roundup32(960) + 16 <= LDS_COLS
constexpr int MAXBATH = 8;
constexpr int MAXLVL = 12;         // levels of the memory-sum ladder
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
};

// One workgroup of a spectral level's batched GEMM (gle_kernels.hip cgemm_kernel): 64 rows x 16 RN
// columns of the Gauss products of Y(f) = sum_m Khat(f, m) Xhat(f, sigma - m), from the two real
// planes of Khat (Kr, Ki) and of the segment spectra (Xr, Xi):
//   g3 = 1 (0 < f < P)  T_0 = Kr (Xr + Xi),  T_1 = (Kr + Ki) Xi,  T_2 = (Ki - Kr) Xr   (one item, all
//                       three parts: Kr and Ki streamed once, the Gauss sums formed in registers)
//   g3 = 0 (f = 0, P)   T_0 = Kr Xr  (real spectra; T_1 = T_2 = 0 are never written)
struct CgItem {
  const double* A;   // Kr plane of f at row tile 4 rg, k-step 0: [rt][m][ks][64] (Ki at + a_pl)
  const double* X;   // segment-ring Xr plane of f, row 0 (Xi at + x_pl)
  double* out;       // T_0(f) at row 64 rg, column col0 (T_1, T_2 at + o_pl, + 2 o_pl)
  int64_t a_rt;      // doubles between row tiles of A (M nks 64)
  int32_t ldx, cs;   // X row stride, columns per ring slot (B)
  int32_t Rseg, M, nks;
  int32_t nrt;       // row tiles present (<= 4)
  int32_t nrows, ncols;  // valid rows (<= 64), columns
  int32_t ldo, col0;
  int32_t s0, ns;    // k-step range [s0, s0 + ns) of this item (split-K halves write separate planes)
  int32_t accum;     // 1: add the item's partial to out (fused schedule: the k-splits of one product
                     // run in successive launches, first one stores); 0: store
  int32_t g3;        // 1: the three Gauss parts from (Kr, Ki) x (Xr, Xi); 0: T_0 = Kr Xr only
  int64_t a_pl;      // doubles from the Kr plane to the Ki plane
  int64_t x_pl;      // doubles from the Xr plane to the Xi plane
  int64_t o_pl;      // doubles between the T_g planes
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
  double* S;           // memory sums S(t) double buffer [2][ncp][B] (parity of t)
  double* Yq;          // Kq . q~ (biased ebath) [ncp][B], chain B -> C
  double* Xcur;        // gathered p half (buffer 0) / p1 (buffer 1), [2][ncp][B]
  double* Xq;          // gathered q_t (buffer 0) / q~ (buffer 1), [2][ncp][B]
  double* H;           // history ring
  double* cur;         // heat current [nmd][B]
  double* NP;          // near-field partial slots [2 parity][nqn][ncp][B] (lags [2, nn))
  double* NR;          // near ring: p of the newest NRS steps, slot-major [NRS][vs] (slot = t mod NRS)
  const double* lvl[MAXLVL];  // ladder level block buffers [ncp][2 P B] (nullptr: inactive)
  int32_t lvl_ld[MAXLVL];
  double c;            // dt factor (dt if ml > 1 else 1, baths.py:454-457)
  int64_t vs;          // doubles between the buffers of S / Xcur / Xq and between NP slots
  int32_t nc, ncp;
  int32_t ldh, R;
  int32_t has_q;
  int32_t nqn;         // near-field partial slots per parity
  int32_t nlvl;
  int32_t NRS;         // near-ring slots
};

struct StepDev {
  int32_t nph, B, nmd, nbath;
  double dt;
  double *P, *Q, *Ph, *Qt, *Fc, *Flast, *etot;
  double* Q0;             // last q the potential force was evaluated at (md.q0)
  int32_t* qvalid;        // [B] md.q0 != [] flag
  unsigned long long* pmax;  // [2 (id0,id1)][2 (parity)][B] max |x - q0| as ordered bit patterns
  double* part;           // [nmd][ndblk][nbath+1][B] current / energy partial sums per step
  const uint8_t* cmask;   // [nph] constraint mask
  int32_t ndblk;          // DOF tiles (16 DOFs each) = current partial rows per step
  int32_t dbg_ntile;      // stamp slots per stage
  unsigned long long* dbg;   // GLE_CHAIN_DBG: [3 stages][dbg_ntile][4] s_memrealtime stamps, or nullptr
  int64_t dbg_t;          // step whose launches record stamps
  // per-step recording (gle_record; nullptr: off), written by stage A at step t for slot t mod nmd:
  double* rec_p;          // md.ps  [nmd][nph][B] (md.py:374-375)
  double* rec_q;          // md.qs  [nmd][nph][B] (md.py:376-377)
  double* rec_hp;         // md.phis / md.qhis as rings of rec_ml slots [rec_ml][nph][B] (slot t mod
  double* rec_hq;         //   rec_ml holds p_t / q_t, md.py:386-387)
  double* rec_f[MAXBATH]; // md.fhis[i] bath-local [nmd][nc][B] (md.py:398)
  int32_t rec_ml, rec_pad;
  // composed one-launch step (stage 4): trajectories found by a stopping launch (StepArgs::xw) whose
  // md.potforce cache would have hit at a point other than q0: [0] at q~ (0 < max|q~ - q_t| < 1e-9,
  // the reference then reuses the force at q_t), [1] at q_{t+1} after a constraint (0 < max|q_{t+1}
  // - q~_t| < 1e-9)
  unsigned long long* guard;
  BathDev bath[MAXBATH];
};

// ---- per-step chain (gle_chain.hip) ------------------------------------------------------
// Composed one-launch step (STAGE 4, small-bath harmonic plans): md.vv is linear in (p_t, q_t) and
// the bath vectors V0 = n_t - c S(t), W1 = n_{t+1} - c R(t+1), R(t+1) = sum_{i>=2} K_i p_{t+1-i}, so
// with Ck = c K0, C1 = c K1, Dq = dyn + Kq (bath blocks scattered), h = dt/2, A1 = I - hCk + h^2 Ck^2,
// A2 = hI - h^2 Ck:
//   p_{t+1} = Mpp p_t + Mpq q_t + Up P V0 + A2 P W1,                     (DOF tiles, output CH_OYB)
//     Mpp = A1 (I - hCk) - dt A2 Dq + (dt^2/2) A2 Dq Ck - A2 C1,
//     Mpq = -h A1 Dq - A2 Dq + (dt^2/2) A2 Dq^2,   Up = h A1 - (dt^2/2) A2 Dq
//   q_{t+1} = q_t + dt p_t + (dt^2/2) F0, F0 = -dyn q_t + P (V0 - c K0 p_t - Kq q_t)   (md.py:392)
// The DOF tiles also form K0 p_t, Kq q_t, dyn q_t for F0 (current, energy, recordings), the
// S tiles V0(t+1) = W1(t) - c K1 p_t and W1(t+1) = n_{t+2} - c (K2 p_t + near(t+2) + levels), the
// near tiles the partials of lags >= 3 for target t+3.  One dependent launch per step instead of
// two (A, BC); the potential force is evaluated fresh, which equals md.potforce unless its 1e-9 cache
// reuse applies at a point q != q0: such a step is detected by the next launch (StepArgs::xw), which
// stops the composed launches, and the host replays from that step on the two-launch path.
// One md.vv is three launches A, B, C.  Every workgroup is one ChTile: a 16-row x 16*rn-column
// output tile whose products are split over the 4 waves by k-steps (each wave's run of tasks
// accumulates into an LDS partial slot; the epilogue adds the slots of an output in fixed order),
// followed by an epilogue of its kind:
//   CH_DOF   16 DOFs x 16 trajectories: the phase of md.vv for those elements (A: bath forces at
//            t, heat current, half kick, drift; B: first velocity iteration; C: second iteration,
//            constraints, history push)
//   CH_SFIN  16 bath rows: S(t+1) = K_1 p_t + near-field partials + ladder levels
//   CH_RAW   16 bath rows x 16*rn columns of a near-field partial (lags >= 2, target t+2)
constexpr int CH_NW = 16;       // waves per chain workgroup (max)
constexpr int CH_TPW = 4;       // tasks per wave
constexpr int CH_TB = 3;        // baths a DOF tile may intersect
// DOF-tile outputs: Y = K0.x of tile bath u (u), YQ = Kq.q (CH_TB + u), YD = dyn.q (2 CH_TB); the
// fused velocity-iteration stage (STAGE 3) uses per tile bath u (h = dt/2, a = c dt/2):
//   CH_OYB + u   M1.p_half + h K0.V - h (K0 Kq).q~        M1 = K0 - a K0^2   (always)
//   CH_OYD + u   -h (K0 P dyn).q~                                           (potential-cache miss)
//   CH_OYE + u   h K0.Fc                                                    (potential-cache hit)
// so K0.p1 = OYB + (hit ? OYE : OYD); CH_OYC / CH_OYF are unused
constexpr int CH_OYB = 2 * CH_TB + 1;
constexpr int CH_OYC = CH_OYB + CH_TB;
constexpr int CH_OYD = CH_OYC + CH_TB;
constexpr int CH_OYE = CH_OYD + CH_TB;
constexpr int CH_OYF = CH_OYE + CH_TB;
constexpr int CH_NOUT = CH_OYF + CH_TB;
constexpr int CH_LDS_PER_WAVE = 1024;  // doubles of LDS partial slots per wave
constexpr int CH_NPMAX = 16;    // near-field partial slots read by one SFIN element
constexpr int CH_XO = CH_TB + 2;  // split stage-4 DOF tile slab outputs: K0.p_t of tile bath u, dyn.q_t, p_{t+1}
constexpr int CH_XSUB_MAX = 8;    // workgroups one stage-4 DOF tile may be split over
enum { CH_DOF = 0, CH_SFIN = 1, CH_RAW = 2 };

struct ChTask {
  const double* A;   // fragment of the first k-step (lane offset added in the kernel)
  const double* X;   // X at row 4 * (first k-step), column 0
  int32_t a_ks;      // doubles between consecutive k-steps of A
  int32_t ldx;       // X row stride (doubles)
  int32_t nks;       // k-steps
  int32_t ring;      // ring slots of a ring X (0: static X)
  int32_t tshift;    // ring: slot pmod(t + tshift, ring)
  int32_t sst;       // ring: doubles between slots
  int32_t slot;      // LDS partial slot
  int32_t cond;      // 0: always; CH_HIT / CH_MISS: only when some trajectory of the tile takes the
                     // potential-cache hit / miss branch at q~ (the fused velocity stage)
  int32_t xrows;     // rows of X that exist from the task's first row, <= 0 when it starts past them
                     // (operand rows past them, the zero-padded k of A, read the last existing
                     // row instead of leaving the operand)
  int32_t pad;
};
constexpr int32_t CH_HIT = 1;
constexpr int32_t CH_MISS = 2;

// One bath of a DOF tile, copied out of BathDev so the epilogue's operands are one descriptor
// round trip away.  DOF row0 + r is in the bath iff bit r of bmask; bath-local k = DOF + boff
// (CH_INV: k from inv).
struct ChBath {
  const double* noise;
  double *S, *Xcur, *Xq, *Yq, *H, *NR;
  double* Xf;        // fused B+C: bath-local copy of the cached potential force after stage A
  double* V;         // fused B+C: noise(t+1) - c S(t+1), bath-local (written by the S(t+1) tiles)
  const int32_t* inv;
  double c;
  int64_t vs;
  int32_t nc, ldh, R, NRS, has_q;
  int32_t bath;      // StepDev bath index, -1: none
  uint32_t bmask;
  int32_t boff;
};

// The bath of an S(t+1) tile: near-field partial slots and ladder level blocks (unused levels
// point at a zero row with ld 0, so every load is unconditional)
struct ChSfin {
  const double* NP;  // parity-0 slot 0 of the bath's near-field partials
  double* S;
  const double* noise;  // fused B+C: V = noise(t+1) - c S(t+1) into V (nullptr: not fused)
  double* V;
  double* W1;           // stage 4: W1 parity buffers [2][vs] (read t & 1, written (t + 1) & 1); V holds V0
  double c;
  const double* lvl[MAXLVL];
  int32_t lvl_ld[MAXLVL];
  int64_t vs;
  int32_t nqn, nc;
};

struct ChTile {
  int32_t kind;      // CH_DOF / CH_SFIN / CH_RAW
  int32_t rn;        // 16-column MFMA tiles (1, 2 or 4)
  int32_t row0;      // CH_DOF: first DOF; otherwise first bath-local row
  int32_t c0;        // first trajectory column
  int32_t tile;      // CH_DOF: DOF-tile index (current partial row); otherwise the bath
  int32_t nrows, ncols;  // valid rows / columns of the tile
  int32_t par_shift; // CH_RAW: destination parity buffer ((t + par_shift) & 1)
  int64_t par_stride;// CH_RAW: doubles between the parity buffers of dst
  double* dst;       // CH_RAW: row 0, column 0 of the tile in parity buffer 0
  int32_t ldd;
  int32_t first;     // CH_DOF: the tile that zeroes the other-parity cache words
  // stage 4 CH_DOF: the state buffers it reads (p_t, q_t) and writes (p_{t+1}, q_{t+1})
  const double* xp_in;
  const double* xq_in;
  double* xp_out;
  double* xq_out;
  int32_t xpart;     // stage 4 CH_DOF: 0 the whole tile, 1 p_{t+1} only, 2 the id0 phase and q_{t+1} only
  // stage 4 CH_DOF split over xnsub workgroups (k-ranges of the tile's products, xsub = this one's):
  // each stores its output sums to slab xsub of xslab ([xnsub][CH_XO][16 x 16 rn], write-through),
  // adds to the tile's arrival counter xcnt, and the last arriver sums the slabs in slab order and
  // runs the epilogue
  int32_t xsub, xnsub;
  double* xslab;
  unsigned long long* xcnt;
  int32_t ntw[CH_NW]; // tasks of wave w (32-bit: read with scalar loads)
  int32_t ob[CH_NOUT + 1];  // output o adds LDS slots [ob[o], ob[o+1]); outputs: Y of tile bath u
                            // (u < CH_TB), YQ of tile bath u (CH_TB + u), YD (2 CH_TB);
                            // CH_SFIN / CH_RAW use output 0
  ChBath tb[CH_TB];  // CH_DOF: the baths meeting the tile
  ChSfin sf;         // CH_SFIN
  ChTask task[CH_NW][CH_TPW];
};
constexpr int32_t CH_INV = -0x40000000;

// launchers (gle_kernels.hip)
// Every kernel takes the step counter by value: the host knows md.t and the steps at which the
// current far / mid blocks were computed, so no kernel starts with a dependent load of a clock
// A range of far-field GEMM items (one spectral level's current block) riding in a chain launch
// (fused schedule): items[first, first + count) with segment index tseg.
struct FarRange {
  const CgItem* items;
  int64_t tseg;
  int32_t first, count;
};
struct StepArgs {
  int64_t t;                 // md.t of this step
  int32_t dbg;               // GLE_CHAIN_DBG: record this launch's timeline
  int32_t pad;
  int64_t lvl_off[MAXLVL];   // per level: offset (doubles) of target t+1 in its block buffer
  unsigned long long* ts;    // chain launches under GLE_PROFILE_CHAIN: workgroup b stores its start /
                             // end (s_memrealtime) at ts[2b], ts[2b+1] (plain stores), else nullptr
  // chain launches: workgroups [0, nstatic) are the launch's chain tiles, the following ones the
  // far-field items of far[0..nfar) in order (fused schedule; nfar = 0 otherwise)
  int32_t nstatic, nfar;
  FarRange far[MAXLVL];
  // composed step (stage 4/5) launches of gle_run, else nullptr: md.potforce's cache audit words
  // xw [3][xR][ceil(xB / 16)] (launch t reads slot (t - 1) mod 3, zeroes
  // (t + 1) mod 3, writes t mod 3;
  // per trajectory a nibble of bits "some DOF tile's distance > 0 / >= 1e-9" for max |q~ - q_t| (id1
  // call) and max |q_{t+1} - q~_t| (next id0 call), XCheck in gle_chain.hip) and the stop words: a
  // launch that finds a distance in (0, 1e-9) -- where md.potforce would reuse a force at another
  // point (md.py:449-450, 767-779) -- or a set xstop stores nothing from its DOF tiles; the first such
  // launch sets *xstop = *xstop_host = t + 1 (device word / host-mapped word), and the host replays
  // from step t - 1 on the two-launch path, which applies the cache rule (gle_api.hip xresolve)
  unsigned long long* xw;
  unsigned long long* xstop;
  unsigned long long* xstop_host;
  int32_t xB, xR;  // trajectories; replicas of a slot's words (DOF tile % xR writes replica tile % xR)
  int32_t xndof;   // the launch's DOF tiles are its first xndof workgroups (they alone read the words)
  int32_t xpad;
};
void launch_contract(int rn, int cu, const CItem* items, int nitems, StepArgs ta, hipStream_t s);
void launch_reduce(const RItem* items, int nitems, int max_elems, StepArgs ta,
                   hipStream_t s);
// stage 0/1/2 = A/B/C, 3 = fused B + C, 4 = the composed step, 5 = the composed step with one-column
// (VALU) products, for one-trajectory plans.  mode: A: 1 = harmonic id0 potential with md.potforce's cache rule (YD = dyn.q_t
// present), 0 = potential force at q_t already in Fc; bit 1: write the id1 cache distance.
// B / C: 1 = harmonic force at q~ (B computes YD = dyn.q~), 0 = host force in Fc.
void launch_chain(int stage, int nw, int drn, size_t lds_bytes, const ChTile* tiles, int ntiles, const StepDev* sd,
                  StepArgs ta, int mode, hipStream_t s);
void launch_finalize(const StepDev* sd, int B, int nmd, int nbath, hipStream_t s);
// md.potforce at q~ for every DOF and trajectory before the fused velocity stage (bc_fpot): the
// cache rule per trajectory (pmax word id1 of parity par), on a miss f = -dyn.q~ (CSR rows) with
// Fc, Q0 updated; f added to the owning bath's V row (vb: bath << 24 | row, -1 outside the baths)
// dyn is held as ELL when its rows have at most FPOT_ELL nonzeros (ew > 0: col / val [ew][nph],
// slot-major, padded with (row, 0.0)), as CSR (rp, col, val) otherwise (ew = 0)
constexpr int FPOT_ELL = 16;
struct FpotArgs {
  int32_t nph, B, par, t1;  // t1 = (t + 1) mod nmd: noise slot of a bath without memory sum
  int32_t ew;               // ELL width, 0: CSR
  const int32_t *rp, *col, *vb;
  const double* val;
  const double* Qt;
  double *Fc, *Q0;
  const unsigned long long* pmax;
  double* V[MAXBATH];
  const double* noise[MAXBATH];  // baths with ml < 2 (no S(t+1) tiles): V = noise(t+1) + Fpot_b
  int32_t nc[MAXBATH];
};
void launch_fpot(const FpotArgs& a, hipStream_t s);
// composed one-launch step, priming one bath from the two-launch path's state at step t:
// V0[t & 1] = n_t - c S[t & 1] (S: nullptr for a bath without memory sum), W1[t & 1] = n_{t+1} -
// c (sum of the nqn near partials of target t+1 at parity (t + 1) & 1 + the levels at target t+1)
struct XPrimeArgs {
  const double* noise;
  const double* S;
  const double* NP;
  const double* lvl[MAXLVL];
  int32_t lvl_ld[MAXLVL];
  int64_t lvl_off[MAXLVL];
  double *V0, *W1;
  double c;
  int64_t vs, t;
  int32_t nc, B, nmd, nqn;
};
void launch_xprime(const XPrimeArgs& a, hipStream_t s);
// end of a gle_run of composed steps at step t: the audit of step t - 1's words as launch t would do
// it (StepArgs::xw), then, at odd t, the state moves from the odd-parity buffers (P2, Q2) to P / Q
// unless the run stopped (the state of the step to replay from stays in the buffer its parity names)
struct XFinishArgs {
  double *P, *Q;
  const double *P2, *Q2;
  int64_t n;  // doubles per state array to move (0: even t, audit only)
  unsigned long long *xw, *xstop, *xstop_host, *guard;
  int64_t t;
  int32_t B, R;  // trajectories, audit replicas (StepArgs::xR)
};
void launch_xfinish(const XFinishArgs& a, hipStream_t s);
// the two-launch path's id0 distances of step t (pmax words of B trajectories) into replica 0 of the
// audit slot of step t - 1 (composed-step entry, x_prime_buffers)
void launch_xinject(const unsigned long long* pw, int B, unsigned long long* slot, hipStream_t s);
void launch_philox_normal(double* x, int64_t nfreq, int64_t ncp, int64_t nc, int64_t B,
                          uint64_t seed, uint64_t traj_offset, hipStream_t s, int64_t w_off = 0);
// streamed noise: a[w0 + w][row_off + r][b] = wscale[w] sum_k M[w][r][k] x[w][k][b] for w < nw (M of
// frequency w at M + w mstride, mstride < 0: nc kc, 0: one shared factor; wscale nullptr: 1)
void launch_noise_gemm(const double* M, int nc, int kc, const double* x, int ncp, int B, double* a, int rows,
                       int row_off, int64_t w0, int nw, hipStream_t s, int64_t mstride = -1,
                       const double* wscale = nullptr);
void launch_near_fill(const double* H, int64_t ldh, int R, int B, int ncp, double* NR, int64_t vs, int NRS,
                      int64_t t, hipStream_t s);
void launch_ring_copy(double* H, int64_t ldh, int R, int B, int nc, int64_t tau0, int nt, double* buf,
                      int dir, hipStream_t s);
void launch_hist_full(const double* rec, int B, int R, int64_t tau0, int nt, int nph, int b0, int nb, double* out,
                      hipStream_t s);
void launch_hist_overlay(const double* H, int64_t ldh, int B, int R, int64_t tau0, const int32_t* inv, int nrow,
                         int nph, int b0, int nb, int nt, double* out, hipStream_t s);
void launch_hist_out(const double* src, int64_t ks, int64_t ss, int R, int64_t tau0, int nt, int nk, int b0, int nb,
                     double* out, hipStream_t s);
// ts (profiling, may be null): [0] <- min over workgroups of the start, [1] <- max of the end
// (s_memrealtime, 100 MHz): the launch's kernel duration as a kernel trace reports it
void launch_cgemm(int rn, const CgItem* items, int nitems, int64_t tseg, hipStream_t s, int max_grid = 0,
                  unsigned long long* ts = nullptr);
// nplanes: 2 (Re, Im: two-plane Gauss items) or 3 (the three Gauss planes, one item per part)
int launch_khat_pack(const double* Kf, int ml, int nks_k, double* khat, int P, int m0, int M,
                     int nc, int nrt2, int nks2, const double* cstab, int cstride, hipStream_t s, int nplanes);
// One bath's operands of a ladder level's transform launch: the baths of a piece go out as ONE
// launch (blocks [blk0, next bath's blk0) are this bath's), not one launch per bath
struct FftBath {
  const double* H;       // seg_fft: history ring, row stride ldh, R slots
  int64_t ldh;
  int32_t R, nc, ncp, k0, nk, Rseg;
  double* seg;           // seg_fft: segment-spectra ring
  int64_t seg_fstride, ldseg;
  const double* Y;       // far_ifft: Gauss products, block output out (row stride ldout)
  int64_t yfstride, ysplit;
  double* out;
  int64_t ldout;
  int64_t blk0;
};
constexpr int MAXFB = 4;
struct FftBaths {
  FftBath b[MAXFB];
  int32_t n, pad;
};
// the baths' transforms of one level piece in one launch (nbath <= MAXFB; k ranges per bath)
int launch_seg_fft_multi(FftBaths fb, int B, int P, int64_t T, int nseg, const double* cstab, int cstride,
                         hipStream_t s, int nplanes);
int launch_far_ifft_multi(FftBaths fb, int B, int P, const double* cstab, int cstride, hipStream_t s);
int launch_seg_fft(const double* H, int64_t ldh, int R, int B, int nc, int ncp, int P, int64_t T,
                   int nseg, double* seg, int64_t seg_fstride, int64_t ldseg, int Rseg,
                   const double* cstab, int cstride, hipStream_t s, int k0, int k1, int nplanes);
// [k0, k1): the DOF range of this launch (the background schedule issues a long level's transforms
// as several DOF-range pieces); k1 < 0: up to nc
int launch_far_ifft(const double* Y, int64_t yfstride, int64_t ysplit, int nc, int B, int P, double* out,
                    int64_t ldout, const double* cstab, int cstride, hipStream_t s, int k0 = 0, int k1 = -1);
// velocity power spectra of recorded series (functions.powerspecp): out [ngroup][B][nmd]
int launch_power(const double* ps, int64_t nph, int B, int64_t nmd, int ngroup, const int64_t* goff,
                 const int64_t* dofs, const double* tw, double* out, hipStream_t s, int64_t nentry);
int launch_fft_noise(const double* a, double* noise, const double* tw, int64_t nmd, int64_t nc,
                     int64_t arows, int64_t B, int is_complex, double scale, hipStream_t s);
// memory-kernel construction (gle_gmem.hip): out[b o_blk + i o_row + l] = sum_g W[i][g] G[b g_blk + g g_row + l]
// over 64-lane blocks b < nblk (the last has nvalid_last lanes), WT = W^T zero padded [ngwp][mlp]
int launch_kgen(const double* WT, int64_t mlp, int ngw, const double* G, int64_t g_blk, int64_t g_row,
                double* out, int64_t o_blk, int64_t o_row, int ml, int64_t nblk, int nvalid_last, hipStream_t s);
void launch_gamma_pack(const double* gam, int ngw, int ngwp, int nc, int nrt, int nks, double* gf, hipStream_t s);

}  // namespace gle
