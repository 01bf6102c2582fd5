// Host side of the hipgle C-ABI: handle, device buffers, work planner, step orchestration.
//
// Step schedule (one md.vv, md.py:367-411): three launches on the handle's stream (gle_chain.hip)
//   A : K0.p_t (+Kq.q_t, +dyn.q_t) and the id0 phase per DOF tile; S(t+1) = K_1.p_t + near-field
//       partials + ladder levels per bath row tile
//   B : K0.p_half, Kq.q~, dyn.q~ and the first velocity iteration; near-field partials for t+2
//   C : K0.p1, second iteration, constraints, history push; near-field partials for t+2
// plus, at block boundaries, the ladder blocks on background streams (one block ahead).
// The memory sum S is computed once per step (the reference recomputes the whole history sum in
// each of its three md.force calls, baths.py:453-457; the i>=1 tail is identical in all three).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/hipgle.h"
#include "gle_internal.h"

using namespace gle;

namespace {

thread_local std::string g_create_error;

struct Op {
  int rn = 1;
  int cu = 1;          // staged X columns per thread per row (contract_kernel template)
  int max_elems = 0;   // largest reduce tile
  std::vector<CItem> items;
  std::vector<RItem> ritems;
  CItem* d_items = nullptr;
  RItem* d_ritems = nullptr;
  double* partial = nullptr;
  size_t partial_doubles = 0;
  double flops = 0, bytes = 0;  // algorithmic, per launch
  bool empty() const { return items.empty() && ritems.empty(); }
};

// One launch of the per-step chain (gle_chain.hip).
struct Chain {
  std::vector<ChTile> tiles;
  ChTile* d = nullptr;
  double flops = 0;  // algorithmic flops of the launch's products
  int nw = 4;        // waves per workgroup
  size_t lds = 0;    // dynamic LDS bytes per workgroup
  int ndof = 0;      // leading DOF tiles (upload_chain)
};

struct Bath {
  int kind = 0;
  int nc = 0, ncp = 0, nrt = 0, nks = 0, ml = 1;
  double c = 1.0;
  bool has_q = false;
  std::vector<int64_t> cids;
  std::vector<int32_t> inv;  // [nph] DOF -> k or -1
  std::vector<double> K;  // host copy [ml][nc][nc] of the p-channel kernel (bias folded)
  std::vector<double> K0; // host copy of slice 0 (bias folded)
  std::vector<double> Kq; // [nc][nc] q-channel
  double* d_K = nullptr;
  double* d_Kn = nullptr;  // compact fragment copy of the per-step slices [0, nn): [rt][ks][i][64]
  int nn = 1;
  double* d_Kq = nullptr;
  // fused B+C stage: bath-local Fc copy, V = n1 - c S1, packed K0^2, K0 Kq and K0 P dyn (runs per
  // DOF tile)
  // (fused stage: d_K0sqd = M1 = K0 - a K0^2, d_hK0d = h K0, d_KKqd = -h K0 Kq, d_KDd = -h K0 P dyn)
  double *d_Xf = nullptr, *d_V = nullptr, *d_K0sqd = nullptr, *d_KKqd = nullptr, *d_KDd = nullptr;
  double* d_hK0d = nullptr;
  std::vector<std::vector<std::pair<int, int>>> kd_rng;
  std::vector<int64_t> kd_tofs;
  // K0 / Kq rows in DOF order for the chain's DOF tiles: tile rt at [tofs[rt]][ks][64]
  double *d_K0d = nullptr, *d_Kqd = nullptr;
  std::vector<int64_t> tofs;
  int64_t tofs_n = 0;
  int32_t* d_inv = nullptr;
  double *d_noise = nullptr, *d_S = nullptr, *d_Yq = nullptr;
  double *d_Xcur = nullptr, *d_Xq = nullptr, *d_H = nullptr, *d_cur = nullptr;
  double* d_NP = nullptr;  // near-field partial slots [2][nqn][vs]
  int nqn = 0;
  double* d_NR = nullptr;  // near ring [NRS][vs]: p of the newest NRS steps (slot t mod NRS)
  int NRS = 2;
  // composed one-launch step: V0 = n_t - c S(t) and W1 = n_{t+1} - c R(t+1) parity buffers [2][vs],
  // near-field partials of lags [3, nn) [2][nqn3][vs]
  double *d_V0 = nullptr, *d_W1 = nullptr, *d_NP3 = nullptr;
  int nqn3 = 0;
  int64_t vs = 0;          // doubles per bath-local [ncp][B] buffer (with slack)
  int64_t ldh = 0;
  int R = 1;
  bool noise_set = false;
  // noise generator
  int64_t nfreq = 0;
  bool fac_complex = false;
  int fac_rows = 0, fac_nrt = 0;
  double* d_fac = nullptr;
  // streamed noise generation (gle_noise_stream_*): spectrum a [nfreq][rows][B], per-chunk draws
  // [cap][ncp][B] and factor chunk [cap][nc][nc] (x2 when complex); scratch between begin and end
  double *d_sa = nullptr, *d_sx = nullptr, *d_sm = nullptr;
  int64_t s_cap = 0;
  bool s_complex = false;
  // factors of the last complete streamed plan kept on the device (gle_noise_stream_retain): a
  // later run replays them with new draws (gle_noise_stream_replay) instead of handing GBs of
  // factors over PCIe again.  s_ret_ok: every segment of the plan in progress found room.
  struct RetSeg {
    bool shared;
    int64_t w0, nw;
    double* d_m;   // factor planes (Re then Im): nw x nc x nc per dense chunk, one nc x nc when shared
    double* d_sc;  // shared: per-frequency scales (inside d_m's allocation)
  };
  std::vector<RetSeg> s_ret;
  bool s_retain = false, s_ret_ok = false, s_ret_complete = false, s_ret_complex = false;
  int64_t s_ret_cap = 0;
  size_t s_ret_bytes = 0;
};

// One level of the memory-sum ladder for one bath.
struct LevelBath {
  bool active = false;  // the bath's kernel reaches this level's lags
  int lag1 = 0;         // lags [lag0, lag1) of this bath
  double* d_out = nullptr;  // block double buffer [ncp][2 P B]: block k at columns (k&1) P B
  // spectral: partitions m in [2, 2+M), segment-spectra ring of Rseg slots
  int M = 0, Rseg = 0;
  int64_t ldseg = 0, khat_fstride = 0, seg_fstride = 0, yfstride = 0;
  double *d_khat = nullptr, *d_seg = nullptr, *d_Yspec = nullptr;
};

// Level l of the ladder: block length P; lags [2P, lag1).  Block k (targets kP+1..kP+P) only needs
// p up to (k-1)P, so it is computed one block ahead on the background stream.
struct Level {
  int P = 1, lag0 = 2, lag1 = 2;
  bool spectral = false;
  // spectral: 2 = K-hat and segment spectra as Re / Im planes, one item forming all three Gauss
  // products (items of <= 32 columns: the HBM-bound K-hat stream of large baths, C5); 3 = the three
  // Gauss planes, one item per product (64-column items: past the fp64 ridge, where the two-plane
  // item's three accumulator sets leave its prefetch ring too shallow, C3)
  int nplanes = 3;
  int cstride = 1;             // twiddle-table stride (Pspec / P)
  int sidx = 0;                // background stream
  std::vector<LevelBath> lb;   // per bath
  Op op[2];                    // direct: per output parity
  std::vector<CgItem> cg;      // spectral: the batched GEMM of the per-frequency products
  CgItem* d_cg = nullptr;
  int cg_rn = 4;
  int cg_split = 1;            // split-K halves per product (small levels: 2 workgroups per CU)
  double cg_flops = 0, cg_bytes = 0;  // algorithmic, per block
  double cg_units = 0;                 // Gauss products of the block's items (3 per two-plane item)
  hipEvent_t ev[2] = {nullptr, nullptr};
  int64_t last_block = INT64_MIN;
  int64_t bg_block[2] = {INT64_MIN, INT64_MIN};  // block launched on the background stream
  // a block is issued in pieces spread over the P / P0 first-level boundaries of its window, so a
  // long block never sits in front of the next small-level block on the in-order stream:
  // spectral: [segment transform] [cgemm item chunk]... [inverse transform + event]
  int ncg_chunk = 1;
  int nfs = 1, nif = 1;        // segment / inverse transform pieces (DOF ranges of every bath)
  int npiece = 1;
  int64_t ev_seq[2] = {0, 0};      // enqueue order of ev[] (merged main-stream waits)
  int64_t pend_block = INT64_MIN;  // block whose pieces are still being issued
  int64_t pend_t0 = 0;
  int next_piece = 0;
  // fused schedule (spectral levels of 4-wave chain plans): block k+1's GEMM items ride in the
  // chain launches of the steps kP .. kP+P-1 (split-major item order, k-splits accumulate in
  // place), its newest segment is transformed by a launch before A(kP), its inverse transform
  // runs before A((k+1)P)
  bool fused = false;
  bool bg_split = false;         // background schedule walking the k-split item list (fcg)
  std::vector<CgItem> fcg;       // fused items: nsplit k-splits x nout products, split-major
  CgItem* d_fcg = nullptr;
  int64_t nout = 0;              // products (bath, f, g, row group, column tile) per split
  int nsplit = 1;
  double fcg_flops = 0;          // algorithmic flops per block (= cg_flops)
  int64_t fblock = INT64_MIN;    // block whose items are in flight in the fused schedule
  int64_t fT = 0;                // first step of its window
};

void free_retained(Bath& b, hipStream_t s);  // retained streamed-noise factors (gle_noise_stream_*)

}  // namespace

struct gle_handle {
  gle_config cfg{};
  std::string err;
  hipStream_t stream = nullptr;
  int64_t nph = 0, B = 0, nmd = 0, nphp = 0;
  double dt = 0;
  int L = 1;
  std::vector<Bath> baths;
  bool has_dyn = false;
  int dyn_nrt = 0, dyn_nks = 0;
  double* d_dyn = nullptr;
  std::vector<double> dyn_h;   // host copy [nph][nph] (roundoff entries dropped, gle_set_dyn)
  int64_t dyn_dropped = 0;
  int dbg_a = 1;               // GLE_CHAIN_DBG: stage-A chain launched at the recorded step
  bool bc_balance = true;      // fused stage: branch classes split over the waves separately     // entries gle_set_dyn dropped as eigen-reconstruction roundoff
  double* d_dynd = nullptr;    // block-sparse DOF-tile fragments of dyn
  std::vector<std::vector<std::pair<int, int>>> dyn_rng;  // per DOF tile: (first k-step, count)
  std::vector<int64_t> dyn_tofs;
  std::vector<int64_t> constr;
  uint8_t* d_cmask = nullptr;
  double *d_P = nullptr, *d_Q = nullptr, *d_Ph = nullptr, *d_Qt = nullptr, *d_Fc = nullptr;
  double *d_Flast = nullptr, *d_etot = nullptr, *d_Q0 = nullptr, *d_part = nullptr;
  unsigned long long* d_pmax = nullptr;
  int32_t* d_qvalid = nullptr;
  StepDev* d_sd = nullptr;
  unsigned long long* d_dbg = nullptr;  // GLE_CHAIN_DBG stamps
  double* d_zero = nullptr;            // zero row (chain S(t+1) tiles' unused level slots)
  bool dbg_no_ladder = false;  // GLE_DBG_NO_LADDER: skip the ladder blocks (timing experiments only)
  // GLE_EXP_ONE=n (timing only, wrong results): one chain launch per step -- stage A's DOF tiles carry
  // n extra nc x nc products per tile bath, its S(t+1) tiles a second product, no velocity-stage
  // launch -- to price a one-launch step built from composed operators
  int exp_one = 0;
  int bg_grid = 0;             // GLE_BG_GRID: cap of the far-field GEMM grid (grid-stride over items)
  // device timestamps of the profiled far-field launches ([start, end] pairs, s_memrealtime)
  unsigned long long* d_tst = nullptr;
  size_t tst_cap = 4096, tst_used = 0;
  bool prof_ch = false;                  // GLE_PROFILE_CHAIN: per-workgroup stamps of the chain launches
  unsigned long long* d_ctst = nullptr;  // [launch slot][workgroup][start, end]
  size_t ctst_cap = 1024, ctst_tiles = 0, ctst_used = 0;
  std::vector<int> ctst_n;               // workgroups of each used slot
  int64_t prof_ch_n = 0;                 // chain launches timed on the device
  double prof_ch_ms = 0, prof_ch_flops = 0;
  int64_t prof_n_dev = 0;
  double prof_ms_dev = 0.0;
  int piece_g = 1;              // steps per piece slot (P0 once planned; GLE_PIECE_STEP=1: every step)
  bool prof_ev = false;         // gle_profile: HIP events around the dominant kernel's launches
  bool bg_serial = false;      // GLE_BG_SERIAL=1: ladder pieces on the main stream (time-sliced, experiment)
  int piece_slack = 1;         // first-level blocks left between a block's last piece and its use (plan)
  int piece_slack_env = -1;    // GLE_PIECE_SLACK (experiment build) overrides the plan's value
  bool merge_waits = true;     // GLE_MERGE_WAITS=0: one main-stream wait per level
  int wait_early = 0;          // GLE_WAIT_EARLY: steps before a block's first use at which the main stream waits for it
  int64_t ev_seq_counter = 0;
  bool dbg_no_chain = false;   // GLE_DBG_NO_CHAIN (experiment): no chain launches
  int dbg_skip = 0;            // GLE_DBG_SKIP bits (timing experiments only, wrong results):
                               // 1 cgemm, 2 seg_fft, 4 far_ifft, 8 direct level ops
  int dbg_ntile = 0;
  int64_t dbg_t = -1;
  double* d_tw = nullptr;
  int ndblk = 1;
  int64_t t = 0;
  bool frozen = false, state_set = false;
  bool need_prime = true;
  bool pot_cache_exact = false;  // q_t == q~_{t-1} bitwise (no constraints): id0 cache hit
  bool host_force_step = false;
  Op op_prime;
  Chain chA[2], chB[2], chC, chNear;  // [with dyn.q]; chNear: all near-field partial tiles (priming)
  Chain chBC;                          // stages B + C fused (harmonic force, disjoint baths)
  bool fuse_bc = false;
  // composed one-launch step (STAGE 4, gle_internal.h): small-bath harmonic plans; variant t & 1
  // reads state buffer t & 1 (d_P / d_Q or d_P2 / d_Q2) and writes the other; between gle_run calls
  // the state is in d_P / d_Q.  x_live: V0 / W1 / NP3 hold step t's values (else x_prime first);
  // std_stale: the two-launch path's S / NP buffers are behind (composed steps ran since)
  bool xstep = false, x_live = false, std_stale = false;
  Chain chX[2], chNear3;
  double *d_P2 = nullptr, *d_Q2 = nullptr;
  double* d_xfrag = nullptr;           // composed-operator DOF-tile fragments
  unsigned long long* d_guard = nullptr;
  // md.potforce's cache rule on the composed path (StepArgs::xw): audit words [3][ceil(B / 16)], the device
  // stop word and its host-mapped copy; a gle_run of composed steps leaves x_pend set until xresolve
  // has read the stop word (and replayed from the stop step on the two-launch path)
  unsigned long long *d_xw = nullptr, *d_xstop = nullptr, *h_xstop = nullptr, *d_xstop_h = nullptr;
  bool x_pend = false;
  int64_t x_call_t0 = 0;               // first step of the last gle_run of composed steps
  int64_t x_replays = 0;               // composed runs stopped and replayed (gle_cache_audit)
  bool std_words_live = false;         // d_pmax holds the two-launch path's id0 distance of step t
  int64_t ret_cap = -1;                // retained streamed-noise factors: byte cap over all baths (< 0: none)
  int x_rep = 1;                       // composed-step audit word replicas (StepArgs::xR)
  double* d_xslab = nullptr;           // split stage-4 DOF tiles: slabs and arrival counters
  unsigned long long* d_xcnt = nullptr;
  int64_t xslab_n = 0;
  bool x_split = false;                // the composed plan splits DOF tiles
  double x_alg_flops = 0, x_alg_bytes = 0;  // algorithmic chain work per composed step
  // fused stage with the potential force at q~ evaluated before it (bc_fpot): a small launch between
  // A and BC computes md.potforce at q~ for every DOF (cache rule included) and adds it to the bath
  // rows of V, so the velocity stage needs M1.p_half + hK0.(V + Fpot_b) only (two products per bath
  // row instead of three: no K0 P dyn product)
  bool bc_fpot = false;
  int32_t *d_dyn_rp = nullptr, *d_dyn_col = nullptr;  // dyn as CSR (rows of nph), for the fpot launch
  double* d_dyn_val = nullptr;
  int32_t* d_fpot_vb = nullptr;                       // per DOF: bath * 2^24 + bath-local row, or -1
  int fpot_ew = 0;                                    // > 0: dyn held as ELL of that width (FpotArgs::ew)
  int ch_nw[3] = {4, 8, 4};            // chain workgroup waves per stage (A, B / fused BC, C)
  bool small_baths = false;            // every bath has nc <= 512 (the chain is latency-bound)
  bool far_fused = false;              // spectral levels ride in the chain launches (fused schedule)
  double far_afrac = 0.5;              // share of a step's far items in its first chain launch
  int64_t far_max_items = 0;           // most far items one chain launch can carry
  int plan_class = GLE_PLAN_AUTO;      // gle_set_plan_class: forces small_baths either way
  double cg_per_cu = 1.25;             // far-field GEMM workgroups per CU per chunk (set by the plan)
  int ch_drn = 1;                      // DOF-tile 16-column MFMA tiles
  int P0 = 1;          // first level block; near field = lags [1, 2 P0)
  int near_end = 1;
  std::vector<Level> levels;
  int far_mode = GLE_FAR_DIRECT;  // GLE_FAR_SPECTRAL if any level is spectral
  double* d_cstab = nullptr;
  static constexpr int NBG = 3;    // background streams: ladder blocks, levels grouped by P so a
                                   // small level never queues behind a much larger level's block
  hipStream_t bg[NBG] = {};
  hipEvent_t ev_step = nullptr;    // end of the latest block-boundary step on the main stream
  hipEvent_t ev_bg[NBG] = {};      // join points of the background streams
  std::vector<void*> allocs;
  size_t dev_bytes = 0;
  // profiling of the dominant contraction
  bool prof = false;
  std::vector<hipEvent_t> ev;
  size_t ev_used = 0;
  int64_t prof_n = 0;
  double prof_ms = 0, prof_flops = 0, prof_bytes = 0;
  double prof_blocks[MAXLVL] = {};  // ladder blocks issued per level since profiling was enabled
  // per-step recording (gle_record): flags, buffers, host copy of the device step descriptor
  StepDev sdh{};
  int32_t rec_flags = 0;
  double *d_rec_p = nullptr, *d_rec_q = nullptr, *d_rec_hp = nullptr, *d_rec_hq = nullptr;
  double* d_rec_f[MAXBATH] = {};
  int rec_ml = 1;
};

namespace {

#define HIPCHK(h, x)                                                                       \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) return fail(h, GLE_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

int fail(gle_handle* h, int code, const std::string& msg) {
  if (h) h->err = msg;
  else g_create_error = msg;
  return code;
}

// ---- -DGLE_BOUNDS audit: process-wide table of live allocations with their logical extents
#ifdef GLE_BOUNDS
namespace {
std::mutex g_bmu;
std::map<uint64_t, std::pair<uint64_t, int>> g_blive;  // start -> (logical end, allocating line)
bool g_bdirty = true;
uint64_t* g_dlo = nullptr;
uint64_t* g_dhi = nullptr;
unsigned long long* g_dviol = nullptr;
size_t g_bcap = 0;
}  // namespace
void bounds_add(void* p, size_t logical, int line) {
  std::lock_guard<std::mutex> lk(g_bmu);
  g_blive[(uint64_t)p] = {(uint64_t)p + logical, line};
  g_bdirty = true;
}
void bounds_del(void* p) {
  std::lock_guard<std::mutex> lk(g_bmu);
  g_blive.erase((uint64_t)p);
  g_bdirty = true;
}
// upload the table before kernels that check against it (audit build: synchronises the device)
void bounds_table_sync() {
  std::lock_guard<std::mutex> lk(g_bmu);
  if (!g_bdirty) return;
  hipDeviceSynchronize();
  const size_t n = g_blive.size();
  if (n > g_bcap) {
    if (g_dlo) hipFree(g_dlo);
    if (g_dhi) hipFree(g_dhi);
    g_bcap = std::max<size_t>(2 * n, 1024);
    hipMalloc((void**)&g_dlo, g_bcap * 8);
    hipMalloc((void**)&g_dhi, g_bcap * 8);
  }
  if (!g_dviol) {
    hipMalloc((void**)&g_dviol, (1 + 2 * BND_KEEP) * 8);
    hipMemset(g_dviol, 0, (1 + 2 * BND_KEEP) * 8);
  }
  std::vector<uint64_t> lo, hi;
  for (auto& kv : g_blive) {
    lo.push_back(kv.first);
    hi.push_back(kv.second.first);
  }
  hipMemcpy(g_dlo, lo.data(), n * 8, hipMemcpyHostToDevice);
  hipMemcpy(g_dhi, hi.data(), n * 8, hipMemcpyHostToDevice);
  BoundsTab t;
  t.n = (int)n;
  t.viol = g_dviol;
  t.lo = g_dlo;
  t.hi = g_dhi;
  bounds_publish_chain(t);
  bounds_publish_kernels(t);
  hipDeviceSynchronize();
  g_bdirty = false;
}
// reads out-of-allocation accesses recorded so far (after a device synchronisation)
int bounds_report(gle_handle* h) {
  std::lock_guard<std::mutex> lk(g_bmu);
  if (!g_dviol) return GLE_OK;
  unsigned long long v[1 + 2 * BND_KEEP];
  hipMemcpy(v, g_dviol, sizeof(v), hipMemcpyDeviceToHost);
  if (v[0] == 0) return GLE_OK;
  std::string msg = "bounds audit: " + std::to_string(v[0]) + " accesses outside their allocation;";
  for (unsigned long long k = 0; k < std::min<unsigned long long>(v[0], BND_KEEP); ++k) {
    const uint64_t a = v[1 + 2 * k];
    auto it = g_blive.upper_bound(a);
    std::string where = "no allocation";
    if (it != g_blive.begin()) {
      --it;
      where = "alloc@" + std::to_string(it->second.second) + "+" + std::to_string((int64_t)(a - it->first)) +
              " (logical " + std::to_string((int64_t)(it->second.first - it->first)) + " B)";
    }
    msg += " [line " + std::to_string(v[2 + 2 * k]) + ": " + where + "]";
  }
  fprintf(stderr, "%s\n", msg.c_str());
  hipMemset(g_dviol, 0, (1 + 2 * BND_KEEP) * 8);
  return fail(h, GLE_ERR_HIP, msg);
}
#else
inline void bounds_add(void*, size_t, int) {}
inline void bounds_del(void*) {}
inline void bounds_table_sync() {}
inline int bounds_report(gle_handle*) { return GLE_OK; }
#endif

// scratch / stream buffers outside the handle's allocation list (registered with the audit too)
template <class T>
hipError_t tmalloc(T** p, size_t bytes, int line = __builtin_LINE()) {
  const hipError_t e = hipMalloc((void**)p, bytes);
  if (e == hipSuccess) bounds_add((void*)*p, bytes, line);
  return e;
}
inline hipError_t tfree(void* p) {
  bounds_del(p);
  return hipFree(p);
}

// slack: bytes past the logical extent that the audit build treats as out of bounds
int dalloc(gle_handle* h, void** p, size_t bytes, size_t slack = 0, int line = __builtin_LINE()) {
  if (bytes == 0) bytes = 16;
  bytes += slack;
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) {
    *p = nullptr;
    return fail(h, GLE_ERR_NOMEM, "hipMalloc(" + std::to_string(bytes) + "): " + hipGetErrorString(e));
  }
  e = hipMemsetAsync(*p, 0, bytes, h->stream);
  if (e != hipSuccess) return fail(h, GLE_ERR_HIP, std::string("hipMemset: ") + hipGetErrorString(e));
  h->allocs.push_back(*p);
  h->dev_bytes += bytes;
  bounds_add(*p, bytes - slack, line);
  return GLE_OK;
}

template <class T>
int dalloc_n(gle_handle* h, T** p, size_t n, size_t slack_n = 0, int line = __builtin_LINE()) {
  return dalloc(h, (void**)p, n * sizeof(T), slack_n * sizeof(T), line);
}

inline int64_t rup(int64_t a, int64_t m) { return (a + m - 1) / m * m; }

// Pack A slices [nsl][M][Kd] (row-major, optionally two real blocks stacked for complex) into
// the fragment-native layout [rt][ks][i][64] with zero padding; rows padded to 16*nrt, k to 4*nks.
std::vector<double> pack_frags(const double* a, int64_t nsl, int64_t M, int64_t Kd, int nrt, int nks,
                               const double* a2 = nullptr) {
  // a2: optional second block stacked below a (rows M..2M-1), used for complex factors
  const int64_t Mtot = a2 ? 2 * M : M;
  std::vector<double> f((size_t)nrt * nks * nsl * 64, 0.0);
  for (int rt = 0; rt < nrt; ++rt)
    for (int ks = 0; ks < nks; ++ks)
      for (int64_t i = 0; i < nsl; ++i) {
        double* dst = &f[(((size_t)rt * nks + ks) * nsl + i) * 64];
        for (int l = 0; l < 64; ++l) {
          const int64_t r = 16 * rt + (l & 15);
          const int64_t k = 4 * ks + (l >> 4);
          if (r >= Mtot || k >= Kd) continue;
          const double* src = (r < M) ? a : a2;
          const int64_t rr = (r < M) ? r : r - M;
          dst[l] = src[(i * M + rr) * Kd + k];
        }
      }
  return f;
}

int upload(gle_handle* h, void* d, const void* s, size_t bytes) {
  HIPCHK(h, hipMemcpyAsync(d, s, bytes, hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return GLE_OK;
}

int rn_for(int64_t ncols) {
  int need = (int)((ncols + 15) / 16);
  int rn = 1;
  while (rn < need && rn < 16) rn *= 2;
  return rn;
}

// One dense product  dst[M][N] (+)= sum_{i in [i0,i1)} A_i . X_i  planned as work items.
struct Gemm {
  const double* A;
  int64_t a_rt, a_ks;
  int nrt_total, nks_total;
  int i0, i1;
  const double* X;
  int64_t ldx;
  int ring, cs, tshift;
  int M, N;
  double* dst;
  int64_t ldd;
  bool force_reduce = false;
  int Kd = 0;  // true (unpadded) reduction length, for the algorithmic flop/byte count
  int tdiv = 1;
  bool lat = false;  // per-step product: minimise sequential LDS stages per item
};

// Split policy: target ~target_items work items in total for this product, each with at least
// min_work (slice x k-step) units; split slices first (history windows share LDS staging across
// slices only within an item, so long slice runs per item are kept), then k.
void plan_gemm(Op& op, const Gemm& g, int target_items, int min_work) {
  const int NT = 16 * op.rn;
  const int ngroups = (g.nrt_total + 3) / 4;
  const int ncol = (int)((g.N + NT - 1) / NT);
  const int ni = g.i1 - g.i0;
  const int nkp = g.nks_total / 2;  // k-step pairs
  const int base = ngroups * ncol;
  int si = 1, sk = 1, chunk = 0;  // chunk > 0: fixed slices per item (last one shorter)
  if (g.lat && ni > 0) {
    // latency-bound per-step product: each item stages ONE window of slices (as many as fit the
    // LDS row) for ONE or a few k-stages, so an item is a couple of LDS round trips long
    const int ns_cap = g.ring ? std::max(1, (LDS_WW_MAX - NT) / std::max(1, g.cs) + 1) : 1;
    si = (ni + ns_cap - 1) / ns_cap;
    int kp_per = 1;
    while ((int64_t)base * si * ((nkp + kp_per - 1) / kp_per) > target_items && kp_per < nkp) kp_per *= 2;
    sk = (nkp + kp_per - 1) / kp_per;
  } else {
    int split = std::max(1, target_items / std::max(1, base));
    const int64_t work = (int64_t)std::max(ni, 0) * g.nks_total;
    split = (int)std::min<int64_t>(split, std::max<int64_t>(1, work / std::max(1, min_work)));
    if (ni > 0) {
      if (g.ring) {
        // slice chunks are whole multiples of what one LDS window holds, so no item runs its
        // k-stages with a short remainder window
        const int wcap = std::min(LDS_WW_MAX, 256 * (op.rn >= 16 ? 3 : 4));
        const int ns_cap = std::max(1, (wcap - NT) / std::max(1, g.cs) + 1);
        const int q = std::max(1, (int)((double)ni / ((double)split * ns_cap) + 0.5));
        chunk = ns_cap * q;
        si = (ni + chunk - 1) / chunk;
        sk = std::max(1, std::min(nkp, split / si));
      } else {
        sk = std::min(split, nkp);
        si = std::max(1, std::min(ni, split / sk));
      }
    }
  }
  const int nsplit = (ni > 0) ? si * sk : 0;
  const bool use_partial = g.force_reduce || nsplit > 1;
  // item order: (column tile, slice range, k range) outer, row group inner -- consecutive items
  // share the staged history window (and, with the kernel's XCD-aware mapping, one L2)
  std::vector<size_t> slot0s((size_t)ngroups * ncol, 0);
  std::vector<int> nslot((size_t)ngroups * ncol, 0);
  for (int gi = 0; gi < ngroups; ++gi)
    for (int ct = 0; ct < ncol; ++ct) {
      slot0s[(size_t)gi * ncol + ct] = op.partial_doubles;
      if (use_partial) op.partial_doubles += (size_t)nsplit * 64 * NT;
    }
  for (int ct = 0; ct < ncol; ++ct) {
    const int col0 = ct * NT;
    const int ncols = std::min<int>(NT, g.N - col0);
    for (int a = 0; a < si && ni > 0; ++a) {
      const int ia = g.i0 + (chunk ? std::min(ni, a * chunk) : (int)((int64_t)ni * a / si));
      const int ib = g.i0 + (chunk ? std::min(ni, (a + 1) * chunk) : (int)((int64_t)ni * (a + 1) / si));
      if (ib <= ia) continue;
      for (int b = 0; b < sk; ++b) {
        const int kp0 = (int)((int64_t)nkp * b / sk), kp1 = (int)((int64_t)nkp * (b + 1) / sk);
        if (kp1 <= kp0) continue;
        for (int gi = 0; gi < ngroups; ++gi) {
          const int nrows = std::min(64, g.M - 64 * gi);
          if (nrows <= 0) continue;
          const size_t key = (size_t)gi * ncol + ct;
          CItem it{};
          it.A = g.A + (int64_t)(4 * gi) * g.a_rt + (int64_t)(2 * kp0) * g.a_ks + (int64_t)ia * 64;
          it.X = g.X + (int64_t)(8 * kp0) * g.ldx;
          it.a_rt = g.a_rt;
          it.a_ks = g.a_ks;
          it.nks = 2 * (kp1 - kp0);
          it.ia = ia;
          it.ni = ib - ia;
          it.nrt = std::min(4, g.nrt_total - 4 * gi);
          it.ldx = (int32_t)g.ldx;
          it.ring = g.ring;
          it.cs = g.cs;
          it.tshift = g.tshift;
          it.tdiv = g.tdiv;
          it.col0 = col0;
          it.ncols = ncols;
          it.nrows = nrows;
          const size_t slot_sz = (size_t)64 * NT;
          if (use_partial) {
            // offset into the op's partial buffer, fixed up in materialize()
            it.out = (double*)(uintptr_t)((slot0s[key] + (size_t)nslot[key] * slot_sz) * sizeof(double));
            it.ldo = NT;
          } else {
            it.out = g.dst + (int64_t)(64 * gi) * g.ldd + col0;
            it.ldo = (int32_t)g.ldd;
          }
          op.items.push_back(it);
          ++nslot[key];
        }
      }
    }
  }
  if (use_partial)
    for (int gi = 0; gi < ngroups; ++gi)
      for (int ct = 0; ct < ncol; ++ct) {
        const int col0 = ct * NT;
        const int nrows = std::min(64, g.M - 64 * gi);
        if (nrows <= 0) continue;
        const size_t key = (size_t)gi * ncol + ct;
        RItem r{};
        r.dst = g.dst + (int64_t)(64 * gi) * g.ldd + col0;
        r.src = (const double*)(uintptr_t)(slot0s[key] * sizeof(double));  // offset, fixed up in materialize()
        r.ldd = (int32_t)g.ldd;
        r.lds = NT;
        r.nslots = nslot[key];
        r.slot_stride = (int64_t)64 * NT;
        r.rows = nrows;
        r.cols = std::min<int>(NT, g.N - col0);
        op.ritems.push_back(r);
      }
  // algorithmic work of this product: each kernel entry read once, X read
  // once, output written once.
  if (ni > 0) {
    const double kd = g.Kd > 0 ? g.Kd : 4.0 * g.nks_total;
    op.flops += 2.0 * g.M * kd * g.N * ni;
    op.bytes += 8.0 * ((double)ni * g.M * kd + kd * (g.ring ? (double)(ni + (g.N + g.cs - 1) / std::max(1, g.cs) - 1) * g.cs : g.N) + (double)g.M * g.N);
  }
}

// Fix up partial-slot offsets once the partial buffer exists.  Items that write partials were
// tagged with ldo == NT and an offset pointer smaller than the partial size.
int materialize(gle_handle* h, Op& op, const std::vector<bool>& is_partial) {
  // staged window width -> registers per thread for the next-stage prefetch
  int maxww = 16 * op.rn;
  for (const auto& it : op.items) {
    const int ww = it.ring ? (it.ni - 1) * it.cs + 16 * op.rn : 16 * op.rn;
    maxww = std::max(maxww, std::min(ww, LDS_WW_MAX));
  }
  const int cap = op.rn >= 16 ? 3 : 4;
  op.cu = std::max(1, std::min(cap, (maxww + 255) / 256));
  for (const auto& r : op.ritems) op.max_elems = std::max(op.max_elems, r.rows * r.cols);
  if (op.partial_doubles) {
    int rc = dalloc_n(h, &op.partial, op.partial_doubles);
    if (rc) return rc;
  }
  for (size_t i = 0; i < op.items.size(); ++i)
    if (is_partial[i]) op.items[i].out = op.partial + (uintptr_t)op.items[i].out / sizeof(double);
  // pad the grid to a multiple of 8 (XCD-aware block mapping) with empty items
  while (op.items.size() % 8) {
    CItem e{};
    e.A = op.items.empty() ? nullptr : op.items[0].A;
    e.X = op.items.empty() ? nullptr : op.items[0].X;
    e.out = nullptr;
    e.nks = 0;
    e.ni = 0;
    e.nrt = 0;
    e.ldx = 1;
    e.ldo = 1;
    e.cs = 1;
    e.tdiv = 1;
    op.items.push_back(e);
  }
  for (auto& r : op.ritems) r.src = op.partial + (uintptr_t)r.src / sizeof(double);
  if (!op.items.empty()) {
    int rc = dalloc_n(h, &op.d_items, op.items.size());
    if (rc) return rc;
    rc = upload(h, op.d_items, op.items.data(), op.items.size() * sizeof(CItem));
    if (rc) return rc;
  }
  if (!op.ritems.empty()) {
    int rc = dalloc_n(h, &op.d_ritems, op.ritems.size());
    if (rc) return rc;
    rc = upload(h, op.d_ritems, op.ritems.data(), op.ritems.size() * sizeof(RItem));
    if (rc) return rc;
  }
  return GLE_OK;
}

// Wrapper that records which items are partial writers while planning.
struct Planner {
  gle_handle* h;
  Op& op;
  std::vector<bool> partial;
  bool lat;
  Planner(gle_handle* hh, Op& o, int rn, bool latency = false) : h(hh), op(o), lat(latency) { op.rn = rn; }
  void add(const Gemm& g0, int target, int min_work) {
    Gemm g = g0;
    if (lat) g.lat = true;
    const size_t n0 = op.items.size();
    const size_t r0 = op.ritems.size();
    plan_gemm(op, g, target, min_work);
    const bool use_partial = op.ritems.size() > r0;
    for (size_t i = n0; i < op.items.size(); ++i) partial.push_back(use_partial);
  }
  int done() { return materialize(h, op, partial); }
};

inline int64_t floordiv(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

// Step arguments of step t: per level, the column offset of target t+1 in its block buffer
// (block floor(t/P), parity half of the buffer, column (t mod P) * B).
StepArgs step_args(const gle_handle* h, int64_t t) {
  StepArgs a{};
  a.t = t;
  a.dbg = (h->d_dbg && t == h->dbg_t) ? 1 : 0;
  for (size_t l = 0; l < h->levels.size(); ++l) {
    const int64_t P = h->levels[l].P;
    const int64_t k = floordiv(t, P);
    a.lvl_off[l] = ((k & 1) * P + (t - k * P)) * h->B;
  }
  return a;
}
StepArgs step_args(const gle_handle* h) { return step_args(h, h->t); }

// [start, end] pairs ready for atomicMin / atomicMax
void reset_tst(gle_handle* h, size_t n, hipStream_t s) {
  std::vector<unsigned long long> init(2 * n);
  for (size_t i = 0; i < n; ++i) {
    init[2 * i] = ~0ull;
    init[2 * i + 1] = 0ull;
  }
  hipMemcpyAsync(h->d_tst, init.data(), init.size() * 8, hipMemcpyHostToDevice, s);
  hipStreamSynchronize(s);
}

void drain_profile(gle_handle* h) {
  hipStreamSynchronize(h->stream);
  for (int i = 0; i < gle_handle::NBG; ++i)
    if (h->bg[i]) hipStreamSynchronize(h->bg[i]);
  for (size_t i = 0; i + 1 < h->ev_used; i += 2) {
    float ms = 0;
    hipEventElapsedTime(&ms, h->ev[i], h->ev[i + 1]);
    h->prof_ms += ms;
  }
  h->ev_used = 0;
  if (h->d_tst && h->tst_used > 0) {
    std::vector<unsigned long long> v(2 * h->tst_used);
    hipMemcpy(v.data(), h->d_tst, v.size() * 8, hipMemcpyDeviceToHost);
    for (size_t i = 0; i < h->tst_used; ++i)
      if (v[2 * i + 1] >= v[2 * i] && v[2 * i] != ~0ull) {
        h->prof_ms_dev += (double)(v[2 * i + 1] - v[2 * i]) * 1e-5;  // 100 MHz ticks -> ms
        h->prof_n_dev += 1;
      }
    reset_tst(h, h->tst_used, h->stream);
    h->tst_used = 0;
  }
  if (h->d_ctst && h->ctst_used > 0) {  // chain launches: first workgroup start to last end
    std::vector<unsigned long long> v(2 * h->ctst_used * h->ctst_tiles);
    hipMemcpy(v.data(), h->d_ctst, v.size() * 8, hipMemcpyDeviceToHost);
    for (size_t i = 0; i < h->ctst_used; ++i) {
      unsigned long long t0 = ~0ull, t1 = 0;
      for (int b = 0; b < h->ctst_n[i]; ++b) {
        t0 = std::min(t0, v[2 * (i * h->ctst_tiles + b)]);
        t1 = std::max(t1, v[2 * (i * h->ctst_tiles + b) + 1]);
      }
      if (t1 >= t0 && t0 != 0) {
        h->prof_ch_ms += (double)(t1 - t0) * 1e-5;
        h->prof_ch_n += 1;
      }
    }
    h->ctst_used = 0;
    h->ctst_n.clear();
  }
}

// Launch one op on stream s; profile: HIP events around the contraction launch (the dominant
// kernel) on that same stream.
void run_op(gle_handle* h, Op& op, hipStream_t s, const StepArgs& ta, bool profile) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (profile && h->prof_ev && !op.items.empty()) {
    if (h->ev_used + 2 > h->ev.size() || (h->d_tst && h->tst_used >= h->tst_cap)) drain_profile(h);
    e0 = h->ev[h->ev_used];
    e1 = h->ev[h->ev_used + 1];
    h->ev_used += 2;
    hipEventRecord(e0, s);
  }
  StepArgs tc = ta;
  if (e0 && h->d_tst) tc.ts = h->d_tst + 2 * h->tst_used++;  // device stamps: first start, last end
  launch_contract(op.rn, op.cu, op.d_items, (int)op.items.size(), tc, s);
  if (e1) {
    hipEventRecord(e1, s);
    h->prof_n += 1;
    h->prof_flops += op.flops;
    h->prof_bytes += op.bytes;
  }
  launch_reduce(op.d_ritems, (int)op.ritems.size(), op.max_elems, ta, s);
}

// The fused schedule's far-field items for chain launch `part` of step t (0: the step's first
// launch, 1: its velocity-stage launch, 2: none): per fused level with a block in flight, step
// i = t - fT of its window carries items [i n / P, (i + 1) n / P), the first far_afrac of them in
// part 0.  Returns the algorithmic flops of the items (block flops x their share).
double far_ranges(gle_handle* h, int64_t t, int part, StepArgs& ta) {
  ta.nfar = 0;
  double fl = 0.0;
  if (!h->far_fused || h->dbg_no_ladder || part > 1) return fl;
  for (size_t l = 0; l < h->levels.size(); ++l) {
    Level& lv = h->levels[l];
    if (!lv.fused || lv.fblock == INT64_MIN) continue;
    const int64_t i = t - lv.fT;
    if (i < 0 || i >= lv.P) continue;
    const int64_t n = (int64_t)lv.fcg.size();
    const int64_t lo = i * n / lv.P, hi = (i + 1) * n / lv.P;
    const int64_t mid = lo + (int64_t)((double)(hi - lo) * h->far_afrac + 0.5);
    const int64_t first = part == 0 ? lo : mid, count = part == 0 ? mid - lo : hi - mid;
    if (count <= 0) continue;
    FarRange& f = ta.far[ta.nfar++];
    f.items = lv.d_fcg;
    f.tseg = lv.fT / lv.P;
    f.first = (int32_t)first;
    f.count = (int32_t)count;
    const double share = (double)count / (double)n;
    fl += lv.fcg_flops * share;
    if (h->prof) h->prof_blocks[l] += share;
  }
  return fl;
}

// One chain launch (with the fused schedule's far items of its part); profiled (HIP events, same
// stream) when the ladder has no levels.
void run_chain(gle_handle* h, int stage, Chain& c, const StepArgs& ta, int mode, bool profile, int part) {
  hipEvent_t e1 = nullptr;
  if (profile && h->prof_ev && !c.tiles.empty()) {
    if (h->ev_used + 2 > h->ev.size()) drain_profile(h);
    hipEventRecord(h->ev[h->ev_used], h->stream);
    e1 = h->ev[h->ev_used + 1];
    h->ev_used += 2;
  }
  StepArgs tc = ta;
  const double far_flops = far_ranges(h, ta.t, c.nw == 4 ? part : 2, tc);
  int64_t nfar = 0;
  for (int r = 0; r < tc.nfar; ++r) nfar += tc.far[r].count;
  if (h->prof_ch && h->d_ctst && !c.tiles.empty() && c.tiles.size() + nfar <= h->ctst_tiles) {
    if (h->ctst_used >= h->ctst_cap) drain_profile(h);
    tc.ts = h->d_ctst + 2 * h->ctst_used * h->ctst_tiles;
    h->ctst_used += 1;
    h->ctst_n.push_back((int)(c.tiles.size() + nfar));
    h->prof_ch_flops += c.flops + far_flops;
  }
  // GLE_DBG_NO_CHAIN (experiment, timing only: wrong results): the ladder without the per-step chain,
  // to time the far-field launches isolated against the same launches beside the chain
  if (!h->dbg_no_chain)
    launch_chain(stage, c.nw, h->ch_drn, c.lds, c.d, (int)c.tiles.size(), h->d_sd, tc, mode, h->stream);
  if (e1) {
    hipEventRecord(e1, h->stream);
    h->prof_n += 1;
    h->prof_flops += c.flops;
  }
}

// Make the main stream wait for everything queued on the background stream.
void join_bg(gle_handle* h) {
  for (int i = 0; i < gle_handle::NBG; ++i)
    if (h->bg[i]) {
      hipEventRecord(h->ev_bg[i], h->bg[i]);
      hipStreamWaitEvent(h->stream, h->ev_bg[i], 0);
    }
}

int sync_bg(gle_handle* h) {
  for (int i = 0; i < gle_handle::NBG; ++i)
    if (h->bg[i]) HIPCHK(h, hipStreamSynchronize(h->bg[i]));
  return GLE_OK;
}

int check_bath(gle_handle* h, int32_t b) {
  if (!h) return GLE_ERR_ARG;
  if (b < 0 || b >= (int)h->baths.size()) return fail(h, GLE_ERR_ARG, "bad bath id");
  return GLE_OK;
}

// Build every work plan once the system is fixed (first state / step call).
// ---- per-step chain planning (gle_chain.hip) ---------------------------------------------

// A run of k-steps of one chain output: acc_o += sum_s A[s * a_ks] . X rows 4s..4s+3.
struct Seg {
  int o;
  const double* A;
  int a_ks;
  const double* X;
  int ldx, ring, tshift, nks;
  int sst;       // ring: doubles between slots
  int cond = 0;  // 0 / CH_HIT / CH_MISS (ChTask::cond)
  int xrows = 0; // rows of X that exist from its row 0 (0: all 4 nks)
};

// Split the k-steps [g_begin, g_end) of the concatenated segments evenly over the CH_NW waves of
// tile T; every (wave, output) run gets its own LDS slot, slots of one output are contiguous.
int fill_tasks(gle_handle* h, ChTile& T, const std::vector<Seg>& segs, int nout, int64_t g_begin,
               int64_t g_end, Chain& c) {
  int slot = 0;
  const int NW = c.nw;
  double* flops = &c.flops;
  std::vector<int> nsl(nout, 0), first(nout, -1);
  // wave w takes [bnd[w], bnd[w + 1]): the even split point, cut short at a segment end if it would
  // need more than CH_TPW runs (the following waves take the rest); when that leaves work past the
  // last wave (many short segments: small baths, several baths in one tile), each wave instead takes
  // whole runs up to CH_TPW of them
  std::vector<int64_t> bnd(NW + 1, g_begin);
  auto cut = [&](int64_t g0, int64_t g1, bool greedy) {
    int64_t pos = 0;
    int runs = 0;
    for (const Seg& sg : segs) {
      const int64_t s0 = std::max(g0, pos), s1 = std::min(greedy ? g_end : g1, pos + sg.nks);
      if (s1 > s0 && ++runs == CH_TPW) return greedy ? pos + sg.nks : std::min(g1, pos + sg.nks);
      pos += sg.nks;
    }
    return greedy ? g_end : g1;
  };
  for (int pass = 0; pass < 2; ++pass) {
    for (int w = 0; w < NW; ++w) {
      const int64_t g0 = bnd[w];
      bnd[w + 1] = pass == 0 ? cut(g0, std::max(g0, g_begin + (g_end - g_begin) * (w + 1) / NW), false)
                             : cut(g0, g_end, true);
    }
    if (bnd[NW] >= g_end) break;
    if (pass == 1) return fail(h, GLE_ERR_UNSUP, "chain plan: too many k-step runs per wave");
  }
  int64_t g0 = g_begin;
  for (int w = 0; w < NW; ++w) {
    const int64_t g1 = std::min(bnd[w + 1], g_end);
    int64_t pos = 0;
    int cur_o = -1, cnt = 0, cur_slot = -1;
    for (const Seg& sg : segs) {
      const int64_t s0 = std::max(g0, pos), s1 = std::min(g1, pos + sg.nks);
      if (s1 > s0) {
        if (sg.o != cur_o) {
          cur_o = sg.o;
          cur_slot = slot++;
          if (first[cur_o] < 0) first[cur_o] = cur_slot;
          ++nsl[cur_o];
        }
        if (cnt >= CH_TPW) return fail(h, GLE_ERR_UNSUP, "chain plan: too many k-step runs per wave");
        ChTask& tk = T.task[w][cnt++];
        const int64_t kl = s0 - pos;
        tk.A = sg.A + kl * sg.a_ks;
        tk.a_ks = sg.a_ks;
        tk.X = sg.X + 4 * kl * sg.ldx;
        tk.ldx = sg.ldx;
        tk.ring = sg.ring;
        tk.tshift = sg.tshift;
        tk.sst = sg.sst;
        tk.nks = (int32_t)(s1 - s0);
        tk.slot = cur_slot;
        tk.cond = sg.cond;
        tk.xrows = (int32_t)((sg.xrows > 0 ? sg.xrows : 4 * sg.nks) - 4 * kl);
        *flops += 128.0 * T.ncols * (double)(s1 - s0);  // 2 x 16 rows x 4 k x valid columns
      }
      pos += sg.nks;
    }
    T.ntw[w] = (int8_t)cnt;
    g0 = g1;
  }
  c.lds = std::max(c.lds, (size_t)slot * 256 * T.rn * 8);
  if (c.lds > 150 * 1024) return fail(h, GLE_ERR_UNSUP, "chain plan: LDS slots");
  int run = 0;
  for (int o = 0; o < nout; ++o) {
    if (nsl[o] && first[o] != run) return fail(h, GLE_ERR_UNSUP, "chain plan: slot order");
    T.ob[o] = (int8_t)run;
    run += nsl[o];
  }
  T.ob[nout] = (int8_t)run;
  for (int o = nout + 1; o <= CH_NOUT; ++o) T.ob[o] = (int8_t)run;
  return GLE_OK;
}

// Fused velocity stage: the k-steps of each branch class (always / potential-cache hit / miss) are
// split evenly over the waves on their own, so whichever of hit and miss the tile takes at run
// time, every wave carries 1/NW of the products (the plain even split of the concatenation left
// the wave holding the skipped branch idle: 75 k-steps per busy wave at C3 instead of ~57).
// Returns 1 (nothing changed) when a wave would need more than CH_TPW runs; the caller then
// uses fill_tasks.
int fill_tasks_balanced(ChTile& T, const std::vector<Seg>& segs, int nout, Chain& c) {
  const int NW = c.nw;
  struct Run {
    int seg;
    int64_t kl, n;
  };
  std::vector<std::vector<Run>> runs(NW);
  for (int cond : {0, CH_MISS, CH_HIT}) {
    int64_t G = 0;
    for (const Seg& sg : segs)
      if (sg.cond == cond) G += sg.nks;
    for (int w = 0; w < NW; ++w) {
      const int64_t g0 = G * w / NW, g1 = G * (w + 1) / NW;
      int64_t pos = 0;
      for (size_t i = 0; i < segs.size(); ++i) {
        if (segs[i].cond != cond) continue;
        const int64_t s0 = std::max(g0, pos), s1 = std::min(g1, pos + segs[i].nks);
        if (s1 > s0) runs[w].push_back(Run{(int)i, s0 - pos, s1 - s0});
        pos += segs[i].nks;
      }
    }
  }
  for (int w = 0; w < NW; ++w) {
    std::stable_sort(runs[w].begin(), runs[w].end(),
                     [&](const Run& a, const Run& b) { return segs[a.seg].o < segs[b.seg].o; });
    if ((int)runs[w].size() > CH_TPW) return 1;
  }
  // one LDS slot per (wave, output), the slots of an output contiguous (output order, then waves)
  std::vector<std::vector<int>> slot_of(NW, std::vector<int>(nout, -1));
  int slot = 0;
  for (int o = 0; o < nout; ++o) {
    T.ob[o] = (int8_t)slot;
    for (int w = 0; w < NW; ++w)
      for (const Run& r : runs[w])
        if (segs[r.seg].o == o) {
          slot_of[w][o] = slot++;
          break;
        }
  }
  for (int o = nout; o <= CH_NOUT; ++o) T.ob[o] = (int8_t)slot;
  for (int w = 0; w < CH_NW; ++w) T.ntw[w] = 0;
  for (int w = 0; w < NW; ++w) {
    int cnt = 0;
    for (const Run& r : runs[w]) {
      const Seg& sg = segs[r.seg];
      ChTask& tk = T.task[w][cnt++];
      tk = ChTask{};
      tk.A = sg.A + r.kl * sg.a_ks;
      tk.a_ks = sg.a_ks;
      tk.X = sg.X + 4 * r.kl * sg.ldx;
      tk.ldx = sg.ldx;
      tk.ring = sg.ring;
      tk.tshift = sg.tshift;
      tk.sst = sg.sst;
      tk.nks = (int32_t)r.n;
      tk.slot = slot_of[w][sg.o];
      tk.cond = sg.cond;
      tk.xrows = (int32_t)((sg.xrows > 0 ? sg.xrows : 4 * sg.nks) - 4 * r.kl);
      c.flops += 128.0 * T.ncols * (double)r.n;  // 2 x 16 rows x 4 k x valid columns
    }
    T.ntw[w] = cnt;
  }
  c.lds = std::max(c.lds, (size_t)slot * 256 * T.rn * 8);
  return 0;
}

// XCD-aware tile order.  Workgroups are dispatched round-robin over the 8 XCDs (block b on XCD
// b mod 8, observed, not guaranteed: speed only, never correctness), each with its own L2.  Tiles
// that read the same matrix rows (the column tiles of one DOF row tile; the near-field and S(t+1)
// tiles of one bath row tile) are given one XCD, groups balanced by work (largest first onto the
// least-loaded XCD), so each XCD's L2 holds ~1/8 of the chain's ~17 MB of matrices instead of
// every XCD streaming all of them from the MALL each step.  Short XCD lists are padded with empty
// tiles so that position p of the launch is on XCD p mod 8.
void xcd_order(gle_handle* h, Chain& c) {
  constexpr int NX = 8;
  if (c.tiles.size() < 2 * NX) return;
  // off by default: measured 1.5-2 % slower per step at C3 than plan order (r02, 3 interleaved
  // rounds), the L2 locality not paying for the imbalance; GLE_XCD_ORDER=1 (experiment build) on
  const char* e = gle_env("GLE_XCD_ORDER");
  if (!e || atoi(e) == 0) return;
  // mode 1: DOF tiles grouped by row tile (shared K rows), near-field tiles by (bath, row tile);
  // mode 2: near-field tiles grouped by (bath, k-range, columns) -- the 19 row tiles that read the
  // same history operand X share an L2 -- every other tile on its own; mode 3: 2 + DOF by row
  const int mode = atoi(e);
  // a tile costs a fixed latency (descriptor, prologue loads, epilogue, ~ the time of 48 k-steps of
  // 16-column MFMAs) plus its products: with the products alone, light tiles (DOFs outside every
  // bath) piled up on a few XCDs and the padding to equal list lengths tripled the launch
  double tile_cost = 48.0;
  if (const char* e = gle_env("GLE_XCD_TILE_COST")) tile_cost = std::max(0.0, atof(e));
  std::vector<std::pair<int64_t, std::vector<size_t>>> groups;  // (key, tiles)
  std::vector<double> gwork;
  for (size_t i = 0; i < c.tiles.size(); ++i) {
    const ChTile& T = c.tiles[i];
    int64_t key = T.kind == CH_DOF ? (int64_t)(T.row0 / 16) : ((int64_t)(T.tile + 1) << 32) + T.row0 / 16;
    if (mode >= 2) {
      if (T.kind == CH_RAW) key = (int64_t)(uintptr_t)(T.dst - (int64_t)T.row0 * T.ldd);  // (bath, q, c0)
      else if (T.kind != CH_DOF || mode == 2) key = -1 - (int64_t)i;                       // ungrouped
    }
    double w = 1.0 + tile_cost;
    for (int wv = 0; wv < CH_NW; ++wv)
      for (int k = 0; k < T.ntw[wv] && k < CH_TPW; ++k) w += (double)T.task[wv][k].nks * T.rn;
    size_t g = 0;
    for (; g < groups.size(); ++g)
      if (groups[g].first == key) break;
    if (g == groups.size()) {
      groups.push_back({key, {}});
      gwork.push_back(0.0);
    }
    groups[g].second.push_back(i);
    gwork[g] += w;
  }
  std::vector<size_t> ord(groups.size());
  for (size_t g = 0; g < ord.size(); ++g) ord[g] = g;
  std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return gwork[a] > gwork[b]; });
  std::vector<std::vector<size_t>> lists(NX);
  std::vector<double> load(NX, 0.0);
  for (size_t g : ord) {
    int x = 0;
    for (int y = 1; y < NX; ++y)
      if (load[y] < load[x] || (load[y] == load[x] && lists[y].size() < lists[x].size())) x = y;
    load[x] += gwork[g];
    for (size_t i : groups[g].second) lists[x].push_back(i);
  }
  size_t n = 0;
  for (auto& l : lists) n = std::max(n, l.size());
  ChTile empty{};
  empty.kind = CH_RAW;  // no tasks, no rows: products and stores are empty
  empty.rn = 1;
  empty.dst = h->d_zero;
  empty.ldd = 1;
  std::vector<ChTile> out;
  out.reserve(n * NX);
  for (size_t m = 0; m < n; ++m)
    for (int x = 0; x < NX; ++x) out.push_back(m < lists[x].size() ? c.tiles[lists[x][m]] : empty);
  c.tiles.swap(out);
}

// Experiment (GLE_CH_ORDER=1): tiles in decreasing order of their longest wave's dependent operand
// round trips (batches of k-steps), so the longest tiles are dispatched first.
void lpt_order(gle_handle* h, Chain& c) {
  const char* e = gle_env("GLE_CH_ORDER");
  if (!e || atoi(e) == 0) return;
  auto rts = [&](const ChTile& T) {
    const int U = c.nw >= 16 ? (T.rn == 1 ? 16 : (T.rn == 2 ? 6 : 3)) : (T.rn == 1 ? 8 : (T.rn == 2 ? 4 : 2));
    int best = 0;
    for (int w = 0; w < c.nw && w < CH_NW; ++w) {
      int n = 0;
      for (int k = 0; k < T.ntw[w] && k < CH_TPW; ++k) n += (T.task[w][k].nks + U - 1) / U;
      best = std::max(best, n);
    }
    return best;
  };
  std::stable_sort(c.tiles.begin(), c.tiles.end(), [&](const ChTile& a, const ChTile& b) { return rts(a) > rts(b); });
}

int upload_chain(gle_handle* h, Chain& c) {
  if (c.tiles.empty()) return GLE_OK;
  lpt_order(h, c);
  xcd_order(h, c);
  // DOF tiles first (plan order): the composed step's audit words are read by them alone; any other
  // order (experiment tile orders) makes every workgroup read them
  int nd = 0, ndof = 0;
  while (nd < (int)c.tiles.size() && c.tiles[nd].kind == CH_DOF) ++nd;
  for (const ChTile& T : c.tiles) ndof += T.kind == CH_DOF ? 1 : 0;
  c.ndof = nd == ndof ? nd : (int)c.tiles.size();
  int rc = dalloc_n(h, &c.d, c.tiles.size());
  if (!rc) rc = upload(h, c.d, c.tiles.data(), c.tiles.size() * sizeof(ChTile));
  return rc;
}

int plan_chain(gle_handle* h) {
  const int64_t B = h->B;
  const int nb = (int)h->baths.size();
  const int ntile = h->ndblk;
  if (const char* e = gle_env("GLE_CHAIN_NW")) {
    int v[3] = {4, 8, 4};
    sscanf(e, "%d,%d,%d", &v[0], &v[1], &v[2]);
    for (int i = 0; i < 3; ++i) h->ch_nw[i] = v[i] >= 8 ? 8 : 4;  // (16-wave groups spill)
  }
  if (const char* e = gle_env("GLE_CHAIN_DRN")) h->ch_drn = atoi(e) >= 2 ? 2 : 1;
  if (const char* e = gle_env("GLE_BC_BALANCE")) h->bc_balance = atoi(e) != 0;
  const char* near_in = gle_env("GLE_NEAR_IN");
  if (!near_in) near_in = "AC";
  const int drn = (int)std::min<int64_t>(h->ch_drn, (B + 15) / 16);
  h->ch_drn = drn;
  const int ncol1 = (int)((B + 16 * drn - 1) / (16 * drn));
  // K0 / Kq rows in DOF order: DOF tile rt of bath j at tofs[rt], [ks][64] fragments
  auto pack_dof_b = [&](const Bath& b, const std::vector<double>& M) {
    std::vector<double> f((size_t)b.tofs_n, 0.0);
    for (int rt = 0; rt < ntile; ++rt) {
      if (b.tofs[rt] < 0) continue;
      for (int ks = 0; ks < b.nks; ++ks)
        for (int l = 0; l < 64; ++l) {
          const int64_t d = 16 * rt + (l & 15), kc = 4 * ks + (l >> 4);
          if (d >= h->nph || kc >= b.nc || b.inv[d] < 0) continue;
          f[(size_t)(b.tofs[rt] + ks * 64 + l)] = M[(size_t)b.inv[d] * b.nc + kc];
        }
    }
    return f;
  };
  for (auto& b : h->baths) {
    auto pack_dof = [&](const std::vector<double>& M) { return pack_dof_b(b, M); };
    b.tofs.assign(ntile, -1);
    int64_t n = 0;
    for (int rt = 0; rt < ntile; ++rt) {
      bool any = false;
      for (int r = 0; r < 16 && 16 * rt + r < h->nph; ++r) any |= b.inv[16 * rt + r] >= 0;
      if (any) {
        b.tofs[rt] = n;
        n += (int64_t)b.nks * 64;
      }
    }
    b.tofs_n = n;
    std::vector<double> f = pack_dof(b.K0);
    int rc = dalloc_n(h, &b.d_K0d, f.size());
    if (!rc) rc = upload(h, b.d_K0d, f.data(), f.size() * 8);
    if (!rc && b.has_q) {
      f = pack_dof(b.Kq);
      rc = dalloc_n(h, &b.d_Kqd, f.size());
      if (!rc) rc = upload(h, b.d_Kqd, f.data(), f.size() * 8);
    }
    if (rc) return rc;
  }
  // dyn as block-sparse DOF-tile fragments: per tile at most two runs of nonzero 16x4 blocks
  if (h->has_dyn) {
    const int nksd = (int)(h->nphp / 4);
    h->dyn_rng.assign(ntile, {});
    h->dyn_tofs.assign(ntile, 0);
    int64_t n = 0;
    for (int rt = 0; rt < ntile; ++rt) {
      std::vector<std::pair<int, int>> rg;
      for (int ks = 0; ks < nksd; ++ks) {
        bool nz = false;
        for (int r = 0; r < 16 && !nz; ++r) {
          const int64_t d = 16 * rt + r;
          if (d >= h->nph) break;
          for (int c = 4 * ks; c < 4 * ks + 4 && c < h->nph; ++c) nz |= h->dyn_h[(size_t)d * h->nph + c] != 0.0;
        }
        if (!nz) continue;
        if (!rg.empty() && rg.back().first + rg.back().second == ks) ++rg.back().second;
        else rg.push_back({ks, 1});
      }
      while (rg.size() > 2) {  // merge across the smallest gap
        size_t bi = 0;
        int bg = INT32_MAX;
        for (size_t i = 0; i + 1 < rg.size(); ++i) {
          const int gap = rg[i + 1].first - (rg[i].first + rg[i].second);
          if (gap < bg) {
            bg = gap;
            bi = i;
          }
        }
        rg[bi].second = rg[bi + 1].first + rg[bi + 1].second - rg[bi].first;
        rg.erase(rg.begin() + bi + 1);
      }
      h->dyn_tofs[rt] = n;
      for (auto& r : rg) n += (int64_t)r.second * 64;
      h->dyn_rng[rt] = rg;
    }
    std::vector<double> f((size_t)std::max<int64_t>(n, 64), 0.0);
    for (int rt = 0; rt < ntile; ++rt) {
      int64_t o = h->dyn_tofs[rt];
      for (auto& r : h->dyn_rng[rt])
        for (int ks = r.first; ks < r.first + r.second; ++ks, o += 64)
          for (int l = 0; l < 64; ++l) {
            const int64_t d = 16 * rt + (l & 15), c = 4 * ks + (l >> 4);
            if (d < h->nph && c < h->nph) f[(size_t)(o + l)] = h->dyn_h[(size_t)d * h->nph + c];
          }
    }
    int rc = dalloc_n(h, &h->d_dynd, f.size());
    if (!rc) rc = upload(h, h->d_dynd, f.data(), f.size() * 8);
    if (rc) return rc;
  }
  // fused B+C stage (dof_BC in gle_chain.hip): harmonic force and pairwise disjoint baths
  {
    bool disjoint = true;
    std::vector<int> owner(h->nph, -1);
    for (int j = 0; j < nb && disjoint; ++j)
      for (int64_t d : h->baths[j].cids) {
        if (owner[d] >= 0) disjoint = false;
        owner[d] = j;
      }
    const char* e = gle_env("GLE_FUSE_BC");
    h->fuse_bc = h->has_dyn && disjoint && nb > 0 && !(e && atoi(e) == 0);
    // large baths: the K0 P dyn product costs the fused stage a third of its nc x nc products, more
    // than the extra launch (C5: 421.6 vs 432.0 us/step; C3: 52.0 vs 50.9, 3 / 2 interleaved
    // rounds, same box, r03)
    const char* ef = gle_env("GLE_BC_FPOT");
    h->bc_fpot = h->fuse_bc && (ef ? atoi(ef) != 0 : !h->small_baths);
  }
  if (h->bc_fpot) {
    std::vector<int32_t> rp(h->nph + 1, 0), col;
    std::vector<double> val;
    for (int64_t d = 0; d < h->nph; ++d) {
      for (int64_t c2 = 0; c2 < h->nph; ++c2) {
        const double v = h->dyn_h[(size_t)(d * h->nph + c2)];
        if (v == 0.0) continue;
        col.push_back((int32_t)c2);
        val.push_back(v);
      }
      rp[d + 1] = (int32_t)col.size();
    }
    if (col.empty()) {
      col.push_back(0);
      val.push_back(0.0);
    }
    std::vector<int32_t> vb(h->nph, -1);
    for (int j = 0; j < nb; ++j)
      for (int64_t k = 0; k < h->baths[j].nc; ++k) vb[h->baths[j].cids[k]] = (j << 24) | (int32_t)k;
    // ELL copy when every row has at most FPOT_ELL nonzeros (the chain junctions: <= 3): slot s of
    // row d at [s][d], padded with (d, 0.0); the kernel skips the zero slots, so the sum is the
    // CSR row's, in the same order
    int ew = 0;
    for (int64_t d = 0; d < h->nph; ++d) ew = std::max(ew, rp[d + 1] - rp[d]);
    h->fpot_ew = ew <= FPOT_ELL ? (ew <= 4 ? 4 : (ew <= 8 ? 8 : FPOT_ELL)) : 0;
    if (h->fpot_ew > 0) {
      const int W = h->fpot_ew;
      std::vector<int32_t> ecol((size_t)W * h->nph);
      std::vector<double> eval((size_t)W * h->nph, 0.0);
      for (int64_t d = 0; d < h->nph; ++d)
        for (int sl = 0; sl < W; ++sl) {
          const int r = rp[d] + sl;
          const bool real = r < rp[d + 1];
          ecol[(size_t)sl * h->nph + d] = real ? col[r] : (int32_t)d;
          eval[(size_t)sl * h->nph + d] = real ? val[r] : 0.0;
        }
      rp.assign(2, 0);  // unused
      col.swap(ecol);
      val.swap(eval);
    }
    int rc = dalloc_n(h, &h->d_dyn_rp, rp.size());
    if (!rc) rc = upload(h, h->d_dyn_rp, rp.data(), rp.size() * 4);
    if (!rc) rc = dalloc_n(h, &h->d_dyn_col, col.size());
    if (!rc) rc = upload(h, h->d_dyn_col, col.data(), col.size() * 4);
    if (!rc) rc = dalloc_n(h, &h->d_dyn_val, val.size());
    if (!rc) rc = upload(h, h->d_dyn_val, val.data(), val.size() * 8);
    if (!rc) rc = dalloc_n(h, &h->d_fpot_vb, vb.size());
    if (!rc) rc = upload(h, h->d_fpot_vb, vb.data(), vb.size() * 4);
    if (rc) return rc;
  }
  if (h->fuse_bc) {
    for (auto& b : h->baths) {
      const int64_t nc = b.nc, nph = h->nph;
      int rc = dalloc_n(h, &b.d_Xf, (size_t)b.vs);
      if (!rc) rc = dalloc_n(h, &b.d_V, (size_t)b.vs);
      if (rc) return rc;
      // M1 = K0 - a K0^2 (a = c dt/2), h K0 and -h K0 Kq (h = dt/2) (nc x nc), -h K0 P dyn (nc x nph):
      // host fp64, row-streaming triple loops.  K0.p1 = M1.p_half + h K0.(V + Fpot_b) - h (K0 Kq).q~
      const double hh = h->dt / 2.0, aa = b.c * h->dt / 2.0;
      std::vector<double> sq((size_t)nc * nc, 0.0);
      for (int64_t r = 0; r < nc; ++r)
        for (int64_t k = 0; k < nc; ++k) {
          const double a = b.K0[(size_t)(r * nc + k)];
          if (a == 0.0) continue;
          const double* src = &b.K0[(size_t)(k * nc)];
          double* dst = &sq[(size_t)(r * nc)];
          for (int64_t c2 = 0; c2 < nc; ++c2) dst[c2] += a * src[c2];
        }
      for (size_t e = 0; e < sq.size(); ++e) sq[e] = b.K0[e] - aa * sq[e];
      std::vector<double> f = pack_dof_b(b, sq);
      rc = dalloc_n(h, &b.d_K0sqd, f.size());  // M1
      if (!rc) rc = upload(h, b.d_K0sqd, f.data(), f.size() * 8);
      if (rc) return rc;
      {
        std::vector<double> hk((size_t)nc * nc);
        for (size_t e = 0; e < hk.size(); ++e) hk[e] = hh * b.K0[e];
        f = pack_dof_b(b, hk);
        rc = dalloc_n(h, &b.d_hK0d, f.size());
        if (!rc) rc = upload(h, b.d_hK0d, f.data(), f.size() * 8);
        if (rc) return rc;
      }
      if (b.has_q) {
        std::vector<double> kq((size_t)nc * nc, 0.0);
        for (int64_t r = 0; r < nc; ++r)
          for (int64_t k = 0; k < nc; ++k) {
            const double a = b.K0[(size_t)(r * nc + k)];
            if (a == 0.0) continue;
            for (int64_t c2 = 0; c2 < nc; ++c2) kq[(size_t)(r * nc + c2)] += a * b.Kq[(size_t)(k * nc + c2)];
          }
        for (double& v : kq) v *= -hh;
        f = pack_dof_b(b, kq);
        rc = dalloc_n(h, &b.d_KKqd, f.size());
        if (!rc) rc = upload(h, b.d_KKqd, f.data(), f.size() * 8);
        if (rc) return rc;
      }
      std::vector<double> kd((size_t)nc * nph, 0.0);
      for (int64_t k = 0; k < nc; ++k) {
        const double* drow = &h->dyn_h[(size_t)(b.cids[k] * nph)];
        std::vector<int64_t> nzc;
        for (int64_t c2 = 0; c2 < nph; ++c2)
          if (drow[c2] != 0.0) nzc.push_back(c2);
        for (int64_t r = 0; r < nc; ++r) {
          const double a = b.K0[(size_t)(r * nc + k)];
          if (a == 0.0) continue;
          for (int64_t c2 : nzc) kd[(size_t)(r * nph + c2)] += a * drow[c2];
        }
      }
      // DOF-tile fragments of K0 P dyn: per tile at most two runs of nonzero 16x4 blocks
      const int nksd = (int)(h->nphp / 4);
      b.kd_rng.assign(ntile, {});
      b.kd_tofs.assign(ntile, 0);
      int64_t n = 0;
      for (int rt = 0; rt < ntile; ++rt) {
        std::vector<std::pair<int, int>> rg;
        for (int ks = 0; ks < nksd; ++ks) {
          bool nz = false;
          for (int r = 0; r < 16 && !nz; ++r) {
            const int64_t d = 16 * rt + r;
            if (d >= nph || b.inv[d] < 0) continue;
            for (int64_t c2 = 4 * ks; c2 < 4 * ks + 4 && c2 < nph; ++c2) nz |= kd[(size_t)(b.inv[d] * nph + c2)] != 0.0;
          }
          if (!nz) continue;
          if (!rg.empty() && rg.back().first + rg.back().second == ks) ++rg.back().second;
          else rg.push_back({ks, 1});
        }
        while (rg.size() > 2) {
          size_t bi = 0;
          int bg = INT32_MAX;
          for (size_t i = 0; i + 1 < rg.size(); ++i) {
            const int gap = rg[i + 1].first - (rg[i].first + rg[i].second);
            if (gap < bg) {
              bg = gap;
              bi = i;
            }
          }
          rg[bi].second = rg[bi + 1].first + rg[bi + 1].second - rg[bi].first;
          rg.erase(rg.begin() + bi + 1);
        }
        b.kd_tofs[rt] = n;
        for (auto& r : rg) n += (int64_t)r.second * 64;
        b.kd_rng[rt] = rg;
      }
      std::vector<double> fk((size_t)std::max<int64_t>(n, 64), 0.0);
      for (int rt = 0; rt < ntile; ++rt) {
        int64_t o = b.kd_tofs[rt];
        for (auto& r : b.kd_rng[rt])
          for (int ks = r.first; ks < r.first + r.second; ++ks, o += 64)
            for (int l = 0; l < 64; ++l) {
              const int64_t d = 16 * rt + (l & 15), c2 = 4 * ks + (l >> 4);
              if (d < nph && c2 < nph && b.inv[d] >= 0) fk[(size_t)(o + l)] = -hh * kd[(size_t)(b.inv[d] * nph + c2)];
            }
      }
      rc = dalloc_n(h, &b.d_KDd, fk.size());
      if (!rc) rc = upload(h, b.d_KDd, fk.data(), fk.size() * 8);
      if (rc) return rc;
    }
  }
  // zero row for the S(t+1) tiles' unused level slots (read at column offsets up to 2 P B + B)
  {
    int Pt = 1;
    for (auto& lv : h->levels) Pt = std::max(Pt, lv.P);
    int rc = dalloc_n(h, &h->d_zero, (size_t)(2 * Pt + 2) * B + 64);
    if (rc) return rc;
  }
  // near-field partial items (lags [2, nn), target t+2) per bath: sizes and slot counts
  // 16, 32 or 64 columns: the product routines have no 48-column form (B in (32, 48] rounds up)
  int rn_raw = std::min(4, rn_for(B));
  if (const char* e = gle_env("GLE_RAW_RN")) rn_raw = std::max(1, std::min(rn_raw, atoi(e) >= 4 ? 4 : (atoi(e) >= 2 ? 2 : 1)));
  const int nt_raw = 16 * rn_raw;
  const int ncolr = (int)((B + nt_raw - 1) / nt_raw);
  const char* env = gle_env("GLE_NEAR_KS");
  const int raw_ks = env ? std::max(4, atoi(env)) : 24;
  for (auto& b : h->baths) {
    b.NRS = std::max(2, b.nn + 1);
    int rc0 = dalloc_n(h, &b.d_NR, (size_t)b.NRS * b.vs, 4096);
    if (rc0) return rc0;
    b.nqn = 0;
    if (b.nn > 2) {
      const int64_t W = (int64_t)(b.nn - 2) * b.nks;
      int q = (int)std::min<int64_t>(CH_NPMAX, (W + raw_ks - 1) / raw_ks);
      // at most CH_TPW - 1 whole slices per wave, so a wave's range spans at most CH_TPW slice runs
      q = std::max(q, (b.nn - 2 + 4 * (CH_TPW - 1) - 1) / (4 * (CH_TPW - 1)));
      q = std::max(1, std::min<int>(q, (int)W));
      if (q > CH_NPMAX) return fail(h, GLE_ERR_UNSUP, "near field too long for the chain (block_len)");
      b.nqn = q;
      int rc = dalloc_n(h, &b.d_NP, (size_t)2 * q * b.vs, 4096);
      if (rc) return rc;
    }
  }
  // ---- tiles
  auto dof_tile = [&](int stage, bool withD, int rt, int ct, Chain& c) -> int {
    ChTile T{};
    T.kind = CH_DOF;
    T.rn = drn;
    T.row0 = 16 * rt;
    T.c0 = 16 * drn * ct;
    T.tile = rt;
    T.nrows = (int)std::min<int64_t>(16, h->nph - 16 * rt);
    T.ncols = (int)std::min<int64_t>(16 * drn, B - T.c0);
    T.first = rt == 0 ? 1 : 0;
    std::vector<Seg> segs;
    std::vector<Seg> qsegs;
    int nu = 0;
    int ubath[CH_TB] = {-1, -1, -1};
    for (int u = 0; u < CH_TB; ++u) {  // unused slots: valid zero rows (the chain loads them unmasked)
      ChBath& cb = T.tb[u];
      cb.bath = -1;
      cb.noise = cb.S = cb.Yq = h->d_zero;
    }
    for (int j = 0; j < nb; ++j) {
      Bath& b = h->baths[j];
      uint32_t m = 0;
      bool affine = true;
      int off = 0;
      for (int r = 0; r < 16; ++r) {
        const int64_t d = 16 * rt + r;
        if (d >= h->nph || b.inv[d] < 0) continue;
        const int o = b.inv[d] - (int)d;
        if (m == 0) off = o;
        else if (o != off) affine = false;
        m |= 1u << r;
      }
      if (!m) continue;
      if (nu == CH_TB) return fail(h, GLE_ERR_UNSUP, "chain plan: more than 3 baths meet one 16-DOF tile");
      const int u = nu++;
      ChBath& cb = T.tb[u];
      cb.noise = b.d_noise;
      cb.S = b.d_S;
      cb.Xcur = b.d_Xcur;
      cb.Xq = b.d_Xq;
      cb.Yq = b.d_Yq ? b.d_Yq : h->d_zero;  // read at row 0 only unless has_q
      cb.H = b.d_H;
      cb.NR = b.d_NR;
      cb.inv = b.d_inv;
      cb.c = b.c;
      cb.vs = b.vs;
      cb.nc = b.nc;
      cb.ldh = (int32_t)b.ldh;
      cb.R = b.R;
      cb.NRS = b.NRS;
      cb.has_q = b.has_q ? 1 : 0;
      cb.bath = j;
      cb.bmask = m;
      cb.boff = affine ? off : CH_INV;
      cb.Xf = h->fuse_bc ? b.d_Xf : nullptr;
      cb.V = h->fuse_bc ? b.d_V : nullptr;
      ubath[u] = j;
      Seg y{u, b.d_K0d + b.tofs[rt], 64, nullptr, (int)B, 0, 0, b.nks, 0};
      if (stage == 0) {
        y.X = b.d_NR;
        y.ring = b.NRS;
        y.sst = (int)b.vs;
      } else {
        y.X = b.d_Xcur + (stage == 2 ? b.vs : 0);
      }
      if (stage != 3) segs.push_back(y);  // the fused stage needs K0.p1 only (CH_OYB + CH_OYD / CH_OYE)
      if (stage == 0)
        for (int x = 0; x < h->exp_one; ++x)  // GLE_EXP_ONE (timing only)
          segs.push_back(Seg{u, b.d_K0d + b.tofs[rt], 64, b.d_Xcur, (int)B, 0, 0, b.nks, 0});
      if (b.has_q && stage != 2)
        qsegs.push_back(Seg{CH_TB + u, b.d_Kqd + b.tofs[rt], 64, b.d_Xq + (stage == 0 ? 0 : b.vs), (int)B, 0, 0,
                            b.nks, 0});
    }
    segs.insert(segs.end(), qsegs.begin(), qsegs.end());
    if (withD && h->has_dyn && stage != 2 && !(stage == 3 && h->bc_fpot)) {
      int64_t o = h->dyn_tofs[rt];
      for (auto& r : h->dyn_rng[rt]) {
        segs.push_back(Seg{2 * CH_TB, h->d_dynd + o, 64, (stage == 0 ? h->d_Q : h->d_Qt) + (int64_t)4 * r.first * B,
                           (int)B, 0, 0, r.second, 0});
        o += (int64_t)r.second * 64;
      }
    }
    if (stage == 3) {  // fused B+C: the composite products (outputs in increasing order)
      // the potential force at q~ enters through dyn.q~ only on a cache miss (md.py:449-473)
      for (auto& sg : segs)
        if (sg.o == 2 * CH_TB) sg.cond = CH_MISS;
      // GLE_EXP_BCLIGHT (experiment, timing only: wrong results): the fused stage without its M1.p_half
      // and h K0.V products (one product per bath row left), to price moving them into stage A
      const bool bclight = gle_env("GLE_EXP_BCLIGHT") != nullptr;
      for (int u = 0; u < nu && !bclight; ++u) {  // OYB: M1.p_half + h K0.V - h (K0 Kq).q~
        const Bath& b = h->baths[ubath[u]];
        segs.push_back(Seg{CH_OYB + u, b.d_K0sqd + b.tofs[rt], 64, b.d_Xcur, (int)B, 0, 0, b.nks, 0});
        if (b.ml >= 2 || h->bc_fpot)  // V = n1 - c S1 from the S(t+1) tiles (+ Fpot_b: the fpot launch,
                                      // which also forms V = n1 + Fpot_b of a bath without memory)
          segs.push_back(Seg{CH_OYB + u, b.d_hK0d + b.tofs[rt], 64, b.d_V, (int)B, 0, 0, b.nks, 0});
        else {          // no memory sum: V = noise(t+1), read from the noise ring (nc rows per slot)
          Seg sg{CH_OYB + u, b.d_hK0d + b.tofs[rt], 64, b.d_noise, (int)B, (int)h->nmd, 1, b.nks, (int)(b.nc * B)};
          sg.xrows = b.nc;
          segs.push_back(sg);
        }
        if (b.has_q)
          segs.push_back(Seg{CH_OYB + u, b.d_KKqd + b.tofs[rt], 64, b.d_Xq + b.vs, (int)B, 0, 0, b.nks, 0});
      }
      for (int u = 0; u < nu && !h->bc_fpot; ++u) {  // OYD: -h (K0 P dyn).q~   (cache miss at q~)
        const Bath& b = h->baths[ubath[u]];
        int64_t o = b.kd_tofs[rt];
        for (auto& r : b.kd_rng[rt]) {
          Seg sg{CH_OYD + u, b.d_KDd + o, 64, h->d_Qt + (int64_t)4 * r.first * B, (int)B, 0, 0, r.second, 0};
          sg.cond = CH_MISS;
          segs.push_back(sg);
          o += (int64_t)r.second * 64;
        }
      }
      for (int u = 0; u < nu && !h->bc_fpot; ++u) {  // OYE: h K0.Fc   (cache hit at q~)
        const Bath& b = h->baths[ubath[u]];
        Seg sg{CH_OYE + u, b.d_hK0d + b.tofs[rt], 64, b.d_Xf, (int)B, 0, 0, b.nks, 0};
        sg.cond = CH_HIT;
        segs.push_back(sg);
      }
    }
    int64_t W = 0;
    for (auto& sg : segs) W += sg.nks;
    const bool bal = stage == 3 && h->bc_balance && c.lds <= 150 * 1024;
    if (!bal || fill_tasks_balanced(T, segs, CH_NOUT, c)) {
      int rc = fill_tasks(h, T, segs, CH_NOUT, 0, W, c);
      if (rc) return rc;
    }
    if (c.lds > 150 * 1024) return fail(h, GLE_ERR_UNSUP, "chain plan: LDS slots");
    c.tiles.push_back(T);
    return GLE_OK;
  };
  for (int v = 0; v < 2; ++v) {
    for (Chain* c : {&h->chA[v], &h->chB[v]}) {
      c->tiles.clear();
      c->flops = 0;
    }
    h->chA[v].nw = h->ch_nw[0];
    h->chB[v].nw = h->ch_nw[1];
    // stage A's DOF epilogue reduces 5 quantities over the tile in LDS
    h->chA[v].lds = (size_t)5 * 256 * drn * 8;
    h->chB[v].lds = 0;
  }
  h->chC.tiles.clear();
  h->chC.flops = 0;
  h->chC.nw = h->ch_nw[2];
  h->chC.lds = (size_t)256 * drn * 8;
  h->chNear.tiles.clear();
  h->chNear.nw = 4;
  h->chNear.lds = 0;
  h->chBC.tiles.clear();
  h->chBC.flops = 0;
  h->chBC.nw = h->ch_nw[1];
  h->chBC.lds = (size_t)256 * drn * 8;
  for (int rt = 0; rt < ntile; ++rt)
    for (int ct = 0; ct < ncol1; ++ct) {
      int rc = 0;
      for (int v = 0; v < 2 && !rc; ++v) {
        rc = dof_tile(0, v == 1, rt, ct, h->chA[v]);
        if (!rc) rc = dof_tile(1, v == 1, rt, ct, h->chB[v]);
      }
      if (!rc) rc = dof_tile(2, false, rt, ct, h->chC);
      if (!rc && h->fuse_bc) rc = dof_tile(3, true, rt, ct, h->chBC);
      if (rc) return rc;
    }
  // S(t+1) tiles (chain A): K_1.p_t + near-field partials + levels, per bath row tile
  for (int j = 0; j < nb; ++j) {
    Bath& b = h->baths[j];
    if (b.ml < 2) continue;
    for (int rt = 0; rt < b.nrt; ++rt)
      for (int ct = 0; ct < ncol1; ++ct) {
        ChTile T{};
        T.kind = CH_SFIN;
        T.rn = drn;
        T.row0 = 16 * rt;
        T.c0 = 16 * drn * ct;
        T.tile = j;
        T.nrows = std::min(16, b.nc - 16 * rt);
        T.ncols = (int)std::min<int64_t>(16 * drn, B - T.c0);
        ChSfin& sf = T.sf;
        sf.NP = b.nqn ? b.d_NP : h->d_zero;
        sf.S = b.d_S;
        sf.vs = b.vs;
        sf.nqn = b.nqn;
        sf.nc = b.nc;
        sf.noise = h->fuse_bc ? b.d_noise : nullptr;
        sf.V = h->fuse_bc ? b.d_V : nullptr;
        sf.c = b.c;
        for (int l = 0; l < MAXLVL; ++l) {
          const bool act = l < (int)h->levels.size() && h->levels[l].lb[j].active;
          sf.lvl[l] = act ? h->levels[l].lb[j].d_out : h->d_zero;
          sf.lvl_ld[l] = act ? 2 * h->levels[l].P * (int32_t)B : 0;
        }
        std::vector<Seg> segs{Seg{0, b.d_Kn + ((int64_t)rt * b.nks * b.nn + 1) * 64, b.nn * 64, b.d_NR, (int)B,
                                  b.NRS, 0, b.nks, (int)b.vs}};
        if (h->exp_one) segs.push_back(segs[0]);  // GLE_EXP_ONE: K_2 p_t beside K_1 p_t (timing only)
        // GLE_EXP_AZ=n (experiment): n extra copies of every S(t+1) tile in stage A (each writes the
        // same values), to price stage-A tiles of one nc x nc product each
        int ncopy = 1;
        if (const char* e = gle_env("GLE_EXP_AZ")) ncopy += std::max(0, atoi(e));
        for (int v = 0; v < 2; ++v)
          for (int cp = 0; cp < ncopy; ++cp) {
            int rc = fill_tasks(h, T, segs, 1, 0, (int64_t)segs.size() * b.nks, h->chA[v]);
            if (rc) return rc;
            h->chA[v].tiles.push_back(T);
          }
      }
  }
  // near-field partial tiles (chains B and C, alternating items)
  for (int j = 0; j < nb; ++j) {
    Bath& b = h->baths[j];
    if (b.nqn == 0) continue;
    std::vector<Seg> base;
    for (int i = 2; i < b.nn; ++i)
      base.push_back(Seg{0, nullptr, b.nn * 64, b.d_NR, (int)B, b.NRS, 2 - i, b.nks, (int)b.vs});
    const int64_t W = (int64_t)(b.nn - 2) * b.nks;
    for (int rt = 0; rt < b.nrt; ++rt) {
      std::vector<Seg> segs = base;
      for (int i = 2; i < b.nn; ++i) segs[i - 2].A = b.d_Kn + ((int64_t)rt * b.nks * b.nn + i) * 64;
      for (int ct = 0; ct < ncolr; ++ct)
        for (int q = 0; q < b.nqn; ++q) {
          ChTile T{};
          T.kind = CH_RAW;
          T.rn = rn_raw;
          T.row0 = 16 * rt;
          T.c0 = nt_raw * ct;
          T.tile = j;
          T.nrows = std::min(16, b.nc - 16 * rt);
          T.ncols = (int)std::min<int64_t>(nt_raw, B - T.c0);
          T.par_shift = 2;
          T.par_stride = (int64_t)b.nqn * b.vs;
          T.dst = b.d_NP + (int64_t)q * b.vs + (int64_t)16 * rt * B + T.c0;
          T.ldd = (int)B;
          // near-field tiles go to the stages named in GLE_NEAR_IN (default A and C), round robin
          const int ns = (int)strlen(near_in);
          const char st = near_in[q % std::max(1, ns)];
          Chain* pair[3] = {nullptr, nullptr, nullptr};
          if (st == 'A') {
            pair[0] = &h->chA[0];
            pair[1] = &h->chA[1];
          } else if (st == 'B') {
            pair[0] = &h->chB[0];
            pair[1] = &h->chB[1];
          } else {
            pair[0] = &h->chC;
          }
          if (st != 'A' && h->fuse_bc) pair[2] = &h->chBC;  // the fused launch replaces B and C
          for (Chain* c : pair) {
            if (!c) continue;
            ChTile Tc = T;
            int rc = fill_tasks(h, Tc, segs, 1, W * q / b.nqn, W * (q + 1) / b.nqn, *c);
            if (rc) return rc;
            c->tiles.push_back(Tc);
          }
          ChTile Tn = T;
          int rc = fill_tasks(h, Tn, segs, 1, W * q / b.nqn, W * (q + 1) / b.nqn, h->chNear);
          if (rc) return rc;
          h->chNear.tiles.push_back(Tn);
        }
    }
  }
  for (Chain* c : {&h->chA[0], &h->chA[1], &h->chB[0], &h->chB[1], &h->chC, &h->chNear, &h->chBC}) {
    int rc = upload_chain(h, *c);
    if (rc) return rc;
  }
  return GLE_OK;
}

// Allocate the buffers of the enabled recordings (zeroed on first use), point the step descriptor
// at them (nullptr: off) and upload it.
int apply_record(gle_handle* h) {
  const int64_t B = h->B, nph = h->nph, nmd = h->nmd;
  int mlmax = 1;
  for (auto& b : h->baths) mlmax = std::max(mlmax, b.ml);
  h->rec_ml = mlmax;
  const int f = h->rec_flags;
  int rc = 0;
  if ((f & GLE_REC_P) && !h->d_rec_p) rc = dalloc_n(h, &h->d_rec_p, (size_t)nmd * nph * B);
  if (!rc && (f & GLE_REC_Q) && !h->d_rec_q) rc = dalloc_n(h, &h->d_rec_q, (size_t)nmd * nph * B);
  if (!rc && (f & GLE_REC_HIST) && !h->d_rec_hp) {
    rc = dalloc_n(h, &h->d_rec_hp, (size_t)mlmax * nph * B);
    if (!rc) rc = dalloc_n(h, &h->d_rec_hq, (size_t)mlmax * nph * B);
  }
  for (size_t j = 0; j < h->baths.size() && !rc; ++j)
    if ((f & GLE_REC_F) && !h->d_rec_f[j]) rc = dalloc_n(h, &h->d_rec_f[j], (size_t)nmd * h->baths[j].nc * B);
  if (rc) return rc;
  StepDev& sd = h->sdh;
  sd.rec_p = (f & GLE_REC_P) ? h->d_rec_p : nullptr;
  sd.rec_q = (f & GLE_REC_Q) ? h->d_rec_q : nullptr;
  sd.rec_hp = (f & GLE_REC_HIST) ? h->d_rec_hp : nullptr;
  sd.rec_hq = (f & GLE_REC_HIST) ? h->d_rec_hq : nullptr;
  for (int j = 0; j < MAXBATH; ++j) sd.rec_f[j] = (f & GLE_REC_F) ? h->d_rec_f[j] : nullptr;
  sd.rec_ml = mlmax;
  HIPCHK(h, hipStreamSynchronize(h->stream));  // launches in flight read the old descriptor
  return upload(h, h->d_sd, &sd, sizeof(sd));
}

// Fused far-field schedule (spectral levels, every chain stage in 4-wave workgroups): per level the
// block's GEMM products (bath, f, Gauss part, 64-row group, column tile) are cut into nsplit k-splits
// of about FAR_KS k-steps, ordered split-major; step i of the block window carries items
// [i n / P, (i + 1) n / P) in its chain launches (A the first part, the velocity stage the rest).
// Every launch's range is at most nout items long (nsplit <= P), so the k-splits of one product fall
// into successive launches: the first stores, the others add (deterministic, no partial planes).
int plan_far_fused(gle_handle* h) {
  h->far_fused = false;
  h->far_max_items = 0;
  bool any = false, two = false;
  for (auto& lv : h->levels) {
    any |= lv.spectral;
    two |= lv.spectral && lv.nplanes == 2;
  }
  if (two) return GLE_OK;  // the chain kernel's far path runs one-plane items only
  const bool nw4 = h->chA[0].nw == 4 && h->chA[1].nw == 4 && h->chB[0].nw == 4 && h->chB[1].nw == 4 &&
                   h->chC.nw == 4 && (!h->fuse_bc || h->chBC.nw == 4);
  // measured r03 (C3, one MI355X, same box): 83 us/step fused vs 50 us background -- the items,
  // HBM-latency-bound at the chain's register budget, finish after the chain tiles and add to
  // every launch; the background schedule overlaps them with the chain across launches.  Off by
  // default (GLE_FAR_FUSED=1 in the experiment build).
  const bool fused = nw4 && gle_env("GLE_FAR_FUSED") != nullptr;
  const bool bg_split = !fused && gle_env("GLE_BG_SPLIT") != nullptr;
  if (!any || (!fused && !bg_split)) return GLE_OK;
  int ks_target = 40;  // k-steps per item: ~4 x 40 MFMAs per wave, about a chain tile's products
  if (const char* e = gle_env("GLE_FAR_KS")) ks_target = std::max(4, atoi(e));
  const int64_t B = h->B;
  for (auto& lv : h->levels) {
    if (!lv.spectral) continue;
    int nsplit = 1;
    for (size_t j = 0; j < h->baths.size(); ++j)
      if (lv.lb[j].active) nsplit = std::max(nsplit, (lv.lb[j].M * h->baths[j].nks + ks_target - 1) / ks_target);
    nsplit = std::min(nsplit, lv.P);
    for (size_t j = 0; j < h->baths.size(); ++j)
      if (lv.lb[j].active) nsplit = std::min(nsplit, lv.lb[j].M * h->baths[j].nks);
    lv.nsplit = std::max(1, nsplit);
    lv.fcg.clear();
    const int NT = 16 * lv.cg_rn;
    for (int sp = 0; sp < lv.nsplit; ++sp) {
      int64_t nout = 0;
      for (size_t j = 0; j < h->baths.size(); ++j) {
        Bath& b = h->baths[j];
        LevelBath& L = lv.lb[j];
        if (!L.active) continue;
        const int64_t a_rt = (int64_t)L.M * b.nks * 64;
        const int64_t plane = (int64_t)b.nrt * a_rt;
        const int S = L.M * b.nks;
        for (int f = 0; f <= lv.P; ++f) {
          const bool real = f == 0 || f == lv.P;  // real spectra: T_1, T_2 stay zero
          const int ng = lv.nplanes == 2 ? 1 : (real ? 1 : 3);
          for (int g = 0; g < ng; ++g) {
            for (int rg = 0; 4 * rg < b.nrt; ++rg)
              for (int c0 = 0; c0 < B; c0 += NT) {
                CgItem it{};
                it.s0 = (int32_t)((int64_t)S * sp / lv.nsplit);
                it.ns = (int32_t)((int64_t)S * (sp + 1) / lv.nsplit) - it.s0;
                it.accum = sp > 0 ? 1 : 0;
                it.g3 = (lv.nplanes == 2 && !real) ? 1 : 0;
                it.A = L.d_khat + (int64_t)f * L.khat_fstride + g * plane + (int64_t)4 * rg * a_rt;
                it.a_pl = plane;
                it.X = L.d_seg + (int64_t)f * L.seg_fstride + (int64_t)g * b.ncp * L.ldseg;
                it.x_pl = (int64_t)b.ncp * L.ldseg;
                it.out = L.d_Yspec + (int64_t)f * L.yfstride + (int64_t)g * b.nc * B + (int64_t)64 * rg * B + c0;
                it.o_pl = (int64_t)b.nc * B;
                it.a_rt = a_rt;
                it.ldx = (int32_t)L.ldseg;
                it.cs = (int32_t)B;
                it.Rseg = L.Rseg;
                it.M = L.M;
                it.nks = b.nks;
                it.nrt = std::min(4, b.nrt - 4 * rg);
                it.nrows = std::min(64, b.nc - 64 * rg);
                it.ncols = (int)std::min<int64_t>(NT, B - c0);
                it.ldo = (int32_t)B;
                it.col0 = c0;
                lv.fcg.push_back(it);
                ++nout;
              }
          }
        }
      }
      lv.nout = nout;
    }
    lv.fcg_flops = lv.cg_flops;
    int rc = dalloc_n(h, &lv.d_fcg, lv.fcg.size());
    if (!rc) rc = upload(h, lv.d_fcg, lv.fcg.data(), lv.fcg.size() * sizeof(CgItem));
    if (rc) return rc;
    if (bg_split) {
      // chunks of ~cg_per_cu workgroups per CU, at least nsplit of them (each at most nout items)
      int ncu = 256;
      hipDeviceProp_t prop;
      if (hipGetDeviceProperties(&prop, h->cfg.device) == hipSuccess) ncu = prop.multiProcessorCount;
      const int64_t want = (int64_t)((double)lv.fcg.size() / (h->cg_per_cu * ncu));
      lv.ncg_chunk = (int)std::max<int64_t>(lv.nsplit, want);
      lv.nfs = lv.nif = 1;
      lv.npiece = lv.ncg_chunk + 2;
      lv.bg_split = true;
      continue;
    }
    lv.fused = true;
    h->far_max_items += ((int64_t)lv.fcg.size() + lv.P - 1) / lv.P + 1;
  }
  h->far_fused = fused;
  if (fused && !gle_env("GLE_FAR_AFRAC")) {
    // a step's items split between its two launches by the workgroup slots each leaves free (4
    // chain-sized workgroups per CU): every item resident from its launch's start, beside the tiles
    int ncu = 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, h->cfg.device) == hipSuccess) ncu = prop.multiProcessorCount;
    const double cap = 4.0 * ncu;
    const double fa = std::max(1.0, cap - (double)h->chA[0].tiles.size());
    const double fb = std::max(1.0, cap - (double)(h->fuse_bc ? h->chBC.tiles.size() : h->chB[0].tiles.size()));
    h->far_afrac = fa / (fa + fb);
  }
  return GLE_OK;
}

// ---- composed one-launch step (STAGE 4): planning -------------------------------------------
// Dense host composition of the step's operators (gle_internal.h, "Composed one-launch step"):
// small-bath plans only (nph <= 4096, every bath nc <= 512), so n^2 matrices and the zero-skipping
// products below stay at a few hundred ms of host fp64 work at C3.
struct Dense {
  int64_t n = 0;
  std::vector<double> a;
  explicit Dense(int64_t n_ = 0) : n(n_), a((size_t)(n_ * n_), 0.0) {}
  double& at(int64_t r, int64_t c) { return a[(size_t)(r * n + c)]; }
  double at(int64_t r, int64_t c) const { return a[(size_t)(r * n + c)]; }
};

// A B, skipping zero entries of A and the zero columns of B's rows
Dense dmul(const Dense& A, const Dense& Bm) {
  const int64_t n = A.n;
  Dense C(n);
  std::vector<std::vector<int32_t>> nzc((size_t)n);
  for (int64_t r = 0; r < n; ++r)
    for (int64_t c = 0; c < n; ++c)
      if (Bm.at(r, c) != 0.0) nzc[(size_t)r].push_back((int32_t)c);
  for (int64_t r = 0; r < n; ++r) {
    double* cr = &C.a[(size_t)(r * n)];
    for (int64_t k = 0; k < n; ++k) {
      const double v = A.at(r, k);
      if (v == 0.0) continue;
      const double* bk = &Bm.a[(size_t)(k * n)];
      for (int32_t c : nzc[(size_t)k]) cr[c] += v * bk[c];
    }
  }
  return C;
}

// Y += alpha X
void daxpy(Dense& Y, double alpha, const Dense& X) {
  for (size_t i = 0; i < Y.a.size(); ++i) Y.a[i] += alpha * X.a[i];
}

// bath-local slice i of a bath's kernel, [nc][nc], from the device's compact near-field copy
int host_slice(gle_handle* h, const Bath& b, int i, std::vector<double>& out) {
  out.assign((size_t)b.nc * b.nc, 0.0);
  if (i >= b.nn) return GLE_OK;  // past the kernel: zero
  const int64_t nfrag = (int64_t)b.nrt * b.nks;
  std::vector<double> f((size_t)nfrag * 64);
  HIPCHK(h, hipMemcpy2DAsync(f.data(), 64 * 8, b.d_Kn + (int64_t)i * 64, (size_t)b.nn * 64 * 8, 64 * 8, (size_t)nfrag,
                             hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  for (int rt = 0; rt < b.nrt; ++rt)
    for (int ks = 0; ks < b.nks; ++ks)
      for (int l = 0; l < 64; ++l) {
        const int64_t r = 16 * rt + (l & 15), c = 4 * ks + (l >> 4);
        if (r < b.nc && c < b.nc) out[(size_t)(r * b.nc + c)] = f[((size_t)rt * b.nks + ks) * 64 + l];
      }
  return GLE_OK;
}

// Rows [16 rt, 16 rt + 16) of an nph x ncols operand (element e(d, k)) as runs of nonzero 16 x 4
// blocks (at most two per tile, merged across the smallest gap), fragments appended to frag:
// (first k-step, k-steps, fragment offset) per run; nnz counts the operand's nonzero entries.
struct XRun {
  int ks0, nks;
  int64_t off;
};
template <class E>
std::vector<XRun> pack_runs(int64_t nph, int64_t ncols, int rt, const E& e, std::vector<double>& frag, double& nnz) {
  const int nks = (int)((ncols + 3) / 4);
  std::vector<std::pair<int, int>> rg;
  for (int ks = 0; ks < nks; ++ks) {
    bool nz = false;
    for (int r = 0; r < 16; ++r) {
      const int64_t d = 16 * (int64_t)rt + r;
      if (d >= nph) break;
      for (int64_t c = 4 * ks; c < 4 * ks + 4 && c < ncols; ++c)
        if (e(d, c) != 0.0) {
          nz = true;
          nnz += 1.0;
        }
    }
    if (!nz) continue;
    if (!rg.empty() && rg.back().first + rg.back().second == ks) ++rg.back().second;
    else rg.push_back({ks, 1});
  }
  while (rg.size() > 2) {
    size_t bi = 0;
    int bg = INT32_MAX;
    for (size_t i = 0; i + 1 < rg.size(); ++i) {
      const int gap = rg[i + 1].first - (rg[i].first + rg[i].second);
      if (gap < bg) {
        bg = gap;
        bi = i;
      }
    }
    rg[bi].second = rg[bi + 1].first + rg[bi + 1].second - rg[bi].first;
    rg.erase(rg.begin() + bi + 1);
  }
  std::vector<XRun> out;
  for (auto& r : rg) {
    out.push_back({r.first, r.second, (int64_t)frag.size()});
    for (int ks = r.first; ks < r.first + r.second; ++ks)
      for (int l = 0; l < 64; ++l) {
        const int64_t d = 16 * (int64_t)rt + (l & 15), c = 4 * ks + (l >> 4);
        frag.push_back(d < nph && c < ncols ? e(d, c) : 0.0);
      }
  }
  return out;
}

// Plan the composed one-launch step when the plan allows it (harmonic potential with disjoint baths,
// small baths, no biased electron bath, first block length >= 2, no fused far-field schedule); any
// planning failure leaves the two-launch plan alone.
int plan_xstep(gle_handle* h) {
  h->xstep = false;
  const int nb = (int)h->baths.size();
  const int64_t nph = h->nph, B = h->B;
  if (const char* e = gle_env("GLE_XSTEP"))
    if (atoi(e) == 0) return GLE_OK;
  // B <= 1008: the audit words (ceil(B / 16)) and the stop word fit the lanes of one wave (XCheck)
  bool ok = h->fuse_bc && !h->bc_fpot && h->small_baths && !h->far_fused && h->P0 >= 2 && nb > 0 && nph <= 4096 &&
            h->exp_one == 0 && B <= 1008;
  for (const Bath& b : h->baths) ok = ok && !b.has_q && b.nc <= 512;
  if (!ok) return GLE_OK;
  const double dt = h->dt, hh = dt / 2.0, h2 = hh * hh, h3 = h2 * hh, dt22 = dt * dt / 2.0;
  // ---- operators
  Dense I(nph), Ck(nph), C1(nph), D(nph);
  for (int64_t d = 0; d < nph; ++d) I.at(d, d) = 1.0;
  D.a = h->dyn_h;
  std::vector<std::vector<double>> K1(nb), K2(nb);
  for (int j = 0; j < nb; ++j) {
    Bath& b = h->baths[j];
    int rc = host_slice(h, b, 1, K1[j]);
    if (!rc) rc = host_slice(h, b, 2, K2[j]);
    if (rc) return rc;
    for (int64_t r = 0; r < b.nc; ++r)
      for (int64_t c = 0; c < b.nc; ++c) {
        Ck.at(b.cids[r], b.cids[c]) = b.c * b.K0[(size_t)(r * b.nc + c)];
        C1.at(b.cids[r], b.cids[c]) = b.c * K1[j][(size_t)(r * b.nc + c)];
      }
  }
  const Dense Ck2 = dmul(Ck, Ck), Ck3 = dmul(Ck2, Ck), CkD = dmul(Ck, D), DCk = dmul(D, Ck);
  const Dense CkDCk = dmul(CkD, Ck), D2 = dmul(D, D), CkD2 = dmul(Ck, D2), Ck2D = dmul(Ck, CkD), CkC1 = dmul(Ck, C1);
  // Mpp = I - 2hCk + 2h^2 Ck^2 - h^3 Ck^3 - dt (hD - h^2 CkD) + (dt^2/2)(hDCk - h^2 CkDCk) - (hC1 - h^2 CkC1)
  Dense Mpp = I;
  daxpy(Mpp, -2.0 * hh, Ck);
  daxpy(Mpp, 2.0 * h2, Ck2);
  daxpy(Mpp, -h3, Ck3);
  daxpy(Mpp, -dt * hh, D);
  daxpy(Mpp, dt * h2, CkD);
  daxpy(Mpp, dt22 * hh, DCk);
  daxpy(Mpp, -dt22 * h2, CkDCk);
  daxpy(Mpp, -hh, C1);
  daxpy(Mpp, h2, CkC1);
  // Mpq = -h (D - hCkD + h^2 Ck^2 D) - (hD - h^2 CkD) + (dt^2/2)(hD^2 - h^2 CkD^2)
  Dense Mpq(nph);
  daxpy(Mpq, -2.0 * hh, D);
  daxpy(Mpq, 2.0 * h2, CkD);
  daxpy(Mpq, -h3, Ck2D);
  daxpy(Mpq, dt22 * hh, D2);
  daxpy(Mpq, -dt22 * h2, CkD2);
  // Up = h (I - hCk + h^2 Ck^2) - (dt^2/2)(hD - h^2 CkD)   (acts on P V0)
  Dense Up(nph);
  daxpy(Up, hh, I);
  daxpy(Up, -h2, Ck);
  daxpy(Up, h3, Ck2);
  daxpy(Up, -dt22 * hh, D);
  daxpy(Up, dt22 * h2, CkD);
  // Wp = hI - h^2 Ck  (acts on P W1)
  Dense Wp(nph);
  daxpy(Wp, hh, I);
  daxpy(Wp, -h2, Ck);
  // ---- buffers
  int rc = 0;
  const size_t nst = (size_t)h->nphp * B, nsl = (size_t)64 * B + 1024;
  if (!h->d_P2) rc = dalloc_n(h, &h->d_P2, nst, nsl);
  if (!rc && !h->d_Q2) rc = dalloc_n(h, &h->d_Q2, nst, nsl);
  for (int j = 0; j < nb && !rc; ++j) {
    Bath& b = h->baths[j];
    rc = dalloc_n(h, &b.d_V0, (size_t)2 * b.vs);
    if (!rc) rc = dalloc_n(h, &b.d_W1, (size_t)2 * b.vs);
  }
  if (rc) return rc;
  // near-field partials of lags [3, nn) for target t+3 (the S tiles of the next launch sum them)
  int rn_raw = std::min(4, rn_for(B));  // 16, 32 or 64 columns (no 48-column product form)
  const int nt_raw = 16 * rn_raw;
  const int ncolr = (int)((B + nt_raw - 1) / nt_raw);
  int raw_ks = 24;
  if (const char* e = gle_env("GLE_NEAR3_KS")) raw_ks = std::max(4, atoi(e));
  for (auto& b : h->baths) {
    b.nqn3 = 0;
    if (b.nn > 3) {
      const int64_t W = (int64_t)(b.nn - 3) * b.nks;
      int q = (int)std::min<int64_t>(CH_NPMAX, (W + raw_ks - 1) / raw_ks);
      q = std::max(q, (b.nn - 3 + 4 * (CH_TPW - 1) - 1) / (4 * (CH_TPW - 1)));
      q = std::max(1, std::min<int>(q, (int)W));
      if (q > CH_NPMAX) return GLE_OK;
      b.nqn3 = q;
      rc = dalloc_n(h, &b.d_NP3, (size_t)2 * q * b.vs, 4096);
      if (rc) return rc;
    }
  }
  // ---- DOF-tile fragments: Mpp (X = p), Mpq (X = q), Up / Wp restricted to each bath's columns
  // (X = V0 / W1 of that bath); the runs are shared by both state-buffer variants
  const int ntile = h->ndblk;
  std::vector<double> frag;
  double nnz = 0.0;
  struct TileOps {
    std::vector<XRun> pp, pq;
    std::vector<std::vector<XRun>> up, wp;
  };
  std::vector<TileOps> ops((size_t)ntile);
  for (int rt = 0; rt < ntile; ++rt) {
    TileOps& o = ops[(size_t)rt];
    o.pp = pack_runs(nph, nph, rt, [&](int64_t d, int64_t c) { return Mpp.at(d, c); }, frag, nnz);
    o.pq = pack_runs(nph, nph, rt, [&](int64_t d, int64_t c) { return Mpq.at(d, c); }, frag, nnz);
    o.up.resize(nb);
    o.wp.resize(nb);
    for (int j = 0; j < nb; ++j) {
      const Bath& b = h->baths[j];
      o.up[j] = pack_runs(nph, b.nc, rt, [&](int64_t d, int64_t k) { return Up.at(d, b.cids[k]); }, frag, nnz);
      o.wp[j] = pack_runs(nph, b.nc, rt, [&](int64_t d, int64_t k) { return Wp.at(d, b.cids[k]); }, frag, nnz);
    }
  }
  if (frag.empty()) frag.assign(64, 0.0);
  rc = dalloc_n(h, &h->d_xfrag, frag.size());
  if (!rc) rc = upload(h, h->d_xfrag, frag.data(), frag.size() * 8);
  if (!rc) rc = dalloc_n(h, &h->d_guard, 2);
  h->x_rep = B <= 112 ? 8 : 1;  // audit replicas: 8 nw + 1 lanes of one wave (XCheck)
  if (!rc) rc = dalloc_n(h, &h->d_xw, (size_t)3 * h->x_rep * ((B + 15) / 16));
  if (!rc) rc = dalloc_n(h, &h->d_xstop, 1);
  if (!rc && !h->h_xstop) {
    void* hp = nullptr;
    if (hipHostMalloc(&hp, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return fail(h, GLE_ERR_NOMEM, "hipHostMalloc (composed-step stop word)");
    h->h_xstop = (unsigned long long*)hp;
    *(volatile unsigned long long*)h->h_xstop = 0ull;
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, hp, 0) != hipSuccess)
      return fail(h, GLE_ERR_HIP, "hipHostGetDevicePointer (composed-step stop word)");
    h->d_xstop_h = (unsigned long long*)dp;
  }
  if (rc) return rc;
  // algorithmic work per step: the composed operators, K0 / K1 / K2 and the near lags [3, nn) on the
  // bath rows, dyn (F0), every matrix entry read once
  double knn = 0.0;
  for (const Bath& b : h->baths) knn += (double)b.nc * b.nc * (double)std::max(0, std::min(b.nn, 3) + std::max(0, b.nn - 3));
  double dyn_nnz = 0.0;
  for (double v : h->dyn_h) dyn_nnz += v != 0.0 ? 1.0 : 0.0;
  h->x_alg_flops = 2.0 * B * (nnz + knn + dyn_nnz);
  h->x_alg_bytes = 8.0 * (nnz + knn + dyn_nnz) + 8.0 * 16.0 * (double)nph * B;
  // ---- tiles
  const int drn = h->ch_drn;
  const int ncol1 = (int)((B + 16 * drn - 1) / (16 * drn));
  const bool xsplit = gle_env("GLE_XSPLIT") != nullptr;
  // DOF tiles split over workgroups by k-steps (xsub_combine, gle_chain.hip) when the plan has few
  // of them (small B): a tile's products are then streamed by up to CH_XSUB_MAX workgroups instead
  // of one CU's four waves
  int xks = ntile * ncol1 < 128 ? 128 : 0;  // C2 (B = 1): 23.3 us/step vs 26.2 unsplit, 24.0 at 32 k-steps; C3 slower split
  if (const char* e = gle_env("GLE_XSUB_KS")) xks = std::max(0, atoi(e));
  const int64_t xne = (int64_t)256 * drn;
  std::vector<int> xns((size_t)ntile * ncol1, 1);
  std::vector<int64_t> xoff((size_t)ntile * ncol1, 0);
  int64_t xslab_n = 0;
  auto err_off = [&](int code) {  // a plan the chain cannot hold: keep the two-launch plan
    h->err.clear();
    (void)code;
    return GLE_OK;
  };
  for (int v = 0; v < 2; ++v) {
    Chain& c = h->chX[v];
    c.tiles.clear();
    c.flops = 0;
    c.nw = 4;
    if (const char* e = gle_env("GLE_XSTEP_NW")) c.nw = atoi(e) >= 8 ? 8 : 4;
    c.lds = (size_t)6 * 256 * drn * 8;  // the DOF epilogue reduces 6 quantities over the tile
    double* pin = v == 0 ? h->d_P : h->d_P2;
    double* qin = v == 0 ? h->d_Q : h->d_Q2;
    double* pout = v == 0 ? h->d_P2 : h->d_P;
    double* qout = v == 0 ? h->d_Q2 : h->d_Q;
    for (int rt = 0; rt < ntile; ++rt)
      for (int ct = 0; ct < ncol1; ++ct) {
        ChTile T{};
        T.kind = CH_DOF;
        T.rn = drn;
        T.row0 = 16 * rt;
        T.c0 = 16 * drn * ct;
        T.tile = rt;
        T.nrows = (int)std::min<int64_t>(16, nph - 16 * rt);
        T.ncols = (int)std::min<int64_t>(16 * drn, B - T.c0);
        T.first = rt == 0 ? 1 : 0;
        T.xp_in = pin;
        T.xq_in = qin;
        T.xp_out = pout;
        T.xq_out = qout;
        for (int u = 0; u < CH_TB; ++u) {
          ChBath& cb = T.tb[u];
          cb.bath = -1;
          cb.noise = cb.S = cb.Yq = cb.V = h->d_zero;
        }
        std::vector<Seg> segs;
        int nu = 0;
        for (int j = 0; j < nb; ++j) {
          Bath& b = h->baths[j];
          uint32_t m = 0;
          bool affine = true;
          int off = 0;
          for (int r = 0; r < 16; ++r) {
            const int64_t d = 16 * rt + r;
            if (d >= nph || b.inv[d] < 0) continue;
            const int o2 = b.inv[d] - (int)d;
            if (m == 0) off = o2;
            else if (o2 != off) affine = false;
            m |= 1u << r;
          }
          if (!m) continue;
          if (nu == CH_TB) return err_off(0);
          const int u = nu++;
          ChBath& cb = T.tb[u];
          cb.noise = b.d_noise;
          cb.S = b.d_S ? b.d_S : h->d_zero;
          cb.Xcur = b.d_Xcur;
          cb.Xq = b.d_Xq;
          cb.Yq = h->d_zero;
          cb.H = b.d_H;
          cb.NR = b.d_NR;
          cb.inv = b.d_inv;
          cb.c = b.c;
          cb.vs = b.vs;
          cb.nc = b.nc;
          cb.ldh = (int32_t)b.ldh;
          cb.R = b.R;
          cb.NRS = b.NRS;
          cb.has_q = 0;
          cb.bath = j;
          cb.bmask = m;
          cb.boff = affine ? off : CH_INV;
          cb.V = b.d_V0;
          // K0.p_t on the tile's bath rows (X: the near ring's slot t)
          segs.push_back(Seg{u, b.d_K0d + b.tofs[rt], 64, b.d_NR, (int)B, b.NRS, 0, b.nks, (int)b.vs});
        }
        {  // dyn.q_t
          int64_t o = h->dyn_tofs[rt];
          for (auto& r : h->dyn_rng[rt]) {
            segs.push_back(Seg{2 * CH_TB, h->d_dynd + o, 64, qin + (int64_t)4 * r.first * B, (int)B, 0, 0, r.second, 0});
            o += (int64_t)r.second * 64;
          }
        }
        const TileOps& o = ops[(size_t)rt];
        for (const XRun& r : o.pp)
          segs.push_back(Seg{CH_OYB, h->d_xfrag + r.off, 64, pin + (int64_t)4 * r.ks0 * B, (int)B, 0, 0, r.nks, 0});
        for (const XRun& r : o.pq)
          segs.push_back(Seg{CH_OYB, h->d_xfrag + r.off, 64, qin + (int64_t)4 * r.ks0 * B, (int)B, 0, 0, r.nks, 0});
        for (int j = 0; j < nb; ++j) {
          const Bath& b = h->baths[j];
          for (const XRun& r : o.up[j])
            segs.push_back(Seg{CH_OYB, h->d_xfrag + r.off, 64, b.d_V0 + (int64_t)v * b.vs + (int64_t)4 * r.ks0 * B,
                               (int)B, 0, 0, r.nks, 0});
          for (const XRun& r : o.wp[j])
            segs.push_back(Seg{CH_OYB, h->d_xfrag + r.off, 64, b.d_W1 + (int64_t)v * b.vs + (int64_t)4 * r.ks0 * B,
                               (int)B, 0, 0, r.nks, 0});
        }
        if (xsplit) {
          // GLE_XSPLIT (experiment): the composed p_{t+1} products in one workgroup, the id0 phase
          // (K0.p_t, dyn.q_t) and q_{t+1} in another (F1 of md.f is not formed)
          std::vector<Seg> sp, sq;
          for (auto& sg : segs) (sg.o == CH_OYB ? sp : sq).push_back(sg);
          for (int part = 1; part <= 2; ++part) {
            ChTile Tp = T;
            Tp.xpart = part;
            Tp.first = part == 2 ? T.first : 0;
            const auto& ss = part == 1 ? sp : sq;
            int64_t W = 0;
            for (auto& sg : ss) W += sg.nks;
            if (fill_tasks(h, Tp, ss, CH_NOUT, 0, W, c)) return err_off(0);
            c.tiles.push_back(Tp);
          }
          continue;
        }
        int64_t W = 0;
        for (auto& sg : segs) W += sg.nks;
        const size_t ti = (size_t)rt * ncol1 + ct;
        if (v == 0 && xks > 0) {
          xns[ti] = (int)std::min<int64_t>(CH_XSUB_MAX, std::max<int64_t>(1, (W + xks - 1) / xks));
          xoff[ti] = xslab_n;
          if (xns[ti] > 1) xslab_n += (int64_t)xns[ti] * CH_XO * xne;
        }
        if (xns[ti] > 1) {
          for (int sub = 0; sub < xns[ti]; ++sub) {
            ChTile Ts = T;
            Ts.xsub = sub;
            Ts.xnsub = xns[ti];
            Ts.first = sub == 0 ? T.first : 0;
            Ts.xslab = (double*)(uintptr_t)(xoff[ti] + 1);  // slab offset + 1, resolved below
            Ts.xcnt = (unsigned long long*)(uintptr_t)(ti + 1);
            if (fill_tasks(h, Ts, segs, CH_NOUT, W * sub / xns[ti], W * (sub + 1) / xns[ti], c)) return err_off(0);
            c.tiles.push_back(Ts);
          }
          continue;
        }
        if (fill_tasks(h, T, segs, CH_NOUT, 0, W, c)) return err_off(0);
        c.tiles.push_back(T);
      }
    // S tiles: V0(t+1), W1(t+1) per bath row tile
    for (int j = 0; j < nb; ++j) {
      Bath& b = h->baths[j];
      for (int rt = 0; rt < b.nrt; ++rt)
        for (int ct = 0; ct < ncol1; ++ct) {
          ChTile T{};
          T.kind = CH_SFIN;
          T.rn = drn;
          T.row0 = 16 * rt;
          T.c0 = 16 * drn * ct;
          T.tile = j;
          T.nrows = std::min(16, b.nc - 16 * rt);
          T.ncols = (int)std::min<int64_t>(16 * drn, B - T.c0);
          ChSfin& sf = T.sf;
          sf.NP = b.nqn3 ? b.d_NP3 : h->d_zero;
          sf.S = nullptr;
          sf.vs = b.vs;
          sf.nqn = b.nqn3;
          sf.nc = b.nc;
          sf.noise = b.d_noise;
          sf.V = b.d_V0;
          sf.W1 = b.d_W1;
          sf.c = b.c;
          for (int l = 0; l < MAXLVL; ++l) {
            const bool act = l < (int)h->levels.size() && h->levels[l].lb[j].active;
            sf.lvl[l] = act ? h->levels[l].lb[j].d_out : h->d_zero;
            sf.lvl_ld[l] = act ? 2 * h->levels[l].P * (int32_t)B : 0;
          }
          std::vector<Seg> segs;
          for (int i = 1; i <= 2 && i < b.nn; ++i)
            segs.push_back(Seg{i - 1, b.d_Kn + ((int64_t)rt * b.nks * b.nn + i) * 64, b.nn * 64, b.d_NR, (int)B, b.NRS, 0,
                               b.nks, (int)b.vs});
          int64_t W = 0;
          for (auto& sg : segs) W += sg.nks;
          if (fill_tasks(h, T, segs, 2, 0, W, c)) return err_off(0);
          c.tiles.push_back(T);
        }
    }
  }
  // near-field partial tiles (lags [3, nn), target t+3): in both variants, and alone for priming
  h->chNear3.tiles.clear();
  h->chNear3.nw = h->chX[0].nw;
  h->chNear3.lds = 0;
  for (auto& b : h->baths) {
    if (b.nqn3 == 0) continue;
    const int64_t W = (int64_t)(b.nn - 3) * b.nks;
    for (int rt = 0; rt < b.nrt; ++rt) {
      std::vector<Seg> segs;
      for (int i = 3; i < b.nn; ++i)
        segs.push_back(Seg{0, b.d_Kn + ((int64_t)rt * b.nks * b.nn + i) * 64, b.nn * 64, b.d_NR, (int)B, b.NRS, 3 - i,
                           b.nks, (int)b.vs});
      for (int ct = 0; ct < ncolr; ++ct)
        for (int q = 0; q < b.nqn3; ++q) {
          ChTile T{};
          T.kind = CH_RAW;
          T.rn = rn_raw;
          T.row0 = 16 * rt;
          T.c0 = nt_raw * ct;
          T.tile = (int)(&b - h->baths.data());
          T.nrows = std::min(16, b.nc - 16 * rt);
          T.ncols = (int)std::min<int64_t>(nt_raw, B - T.c0);
          T.par_shift = 3;
          T.par_stride = (int64_t)b.nqn3 * b.vs;
          T.dst = b.d_NP3 + (int64_t)q * b.vs + (int64_t)16 * rt * B + T.c0;
          T.ldd = (int)B;
          for (Chain* c : {&h->chX[0], &h->chX[1], &h->chNear3}) {
            ChTile Tc = T;
            if (fill_tasks(h, Tc, segs, 1, W * q / b.nqn3, W * (q + 1) / b.nqn3, *c)) return err_off(0);
            c->tiles.push_back(Tc);
          }
        }
    }
  }
  h->x_split = xslab_n > 0;
  if (xslab_n > 0) {  // split DOF tiles: slabs and arrival counters (zeroed: the counters count from 0)
    if (!h->d_xslab || h->xslab_n < xslab_n) {
      rc = dalloc_n(h, &h->d_xslab, (size_t)xslab_n);
      if (!rc) rc = dalloc_n(h, &h->d_xcnt, (size_t)ntile * ncol1);
      if (rc) return rc;
      h->xslab_n = xslab_n;
    } else {
      HIPCHK(h, hipMemsetAsync(h->d_xcnt, 0, (size_t)ntile * ncol1 * 8, h->stream));
    }
    for (int v = 0; v < 2; ++v)
      for (ChTile& T : h->chX[v].tiles)
        if (T.kind == CH_DOF && T.xnsub > 1) {
          T.xslab = h->d_xslab + ((int64_t)(uintptr_t)T.xslab - 1);
          T.xcnt = h->d_xcnt + ((int64_t)(uintptr_t)T.xcnt - 1);
        }
  }
  for (Chain* c : {&h->chX[0], &h->chX[1], &h->chNear3}) {
    if (c->tiles.empty()) continue;
    rc = upload_chain(h, *c);
    if (rc) return rc;
  }
  h->xstep = true;
  h->x_live = false;
  return GLE_OK;
}

int freeze(gle_handle* h) {
  if (h->frozen) return GLE_OK;
  const int64_t B = h->B;
  int mlmax = 1;
  for (auto& b : h->baths) mlmax = std::max(mlmax, b.ml);
  // ---- memory-sum ladder:  S(t+1) = near(t+1) + sum_l level_l(t+1)
  //   near     lags [1, 2 P0), every step, in the step's first product (tile kernel)
  //   level l  block P = P0 2^l, lags [2P, 4P) (the last level: [2P, ml)); block k (targets
  //            kP+1..kP+P) needs p only up to (k-1)P, so it is computed one block AHEAD on the
  //            background stream while the per-step chain runs
  //   a level is SPECTRAL (uniformly partitioned overlap-save, partitions of P lags, transforms of
  //   length 2P: ~4(P+1)/P^2 of the direct flops) or DIRECT (one MFMA contraction per block, each
  //   kernel slice reused for P*B columns)
  const int mode = h->cfg.far_mode;
  const bool spec_ok = mode == GLE_FAR_SPECTRAL || (mode == GLE_FAR_AUTO && B >= 8);
  // first block length: 8 when every bath has nc <= 512 (the chain is latency-bound there, so the
  // near field's extra lags [8, 16) cost it little and one ladder level less pays: C3 -4 %, C2
  // -14 % per step), 4 for the larger baths (C5: +4 % at 8)
  int ncmax = 0;
  for (auto& b : h->baths) ncmax = std::max(ncmax, b.nc);
  h->small_baths = h->plan_class == GLE_PLAN_SMALL_BATHS ? true
                  : h->plan_class == GLE_PLAN_LARGE_BATHS ? false
                                                          : ncmax <= 512;
  h->cg_per_cu = h->small_baths ? 1.25 : 4.0;
  // ladder pieces of a block spread over its whole window (slack 0, small baths: the main stream
  // waits at the block's first use) or end one first-level block early (slack 1, large baths).  C3,
  // with far-field chunks of 1.25 workgroups per CU, 3 interleaved rounds on each of two boxes
  // (r04, `profiles/r04/sched_c3.jsonl`): 512-step window 48.7-48.9 vs 49.5 us/step, 20-step
  // windows over all phases of the largest level mean 51.1 vs 52.5-52.9, max 54.6 vs 62.6-63.4
  h->piece_slack = h->piece_slack_env >= 0 ? h->piece_slack_env : (h->small_baths ? 0 : 1);
  const int P0 = h->cfg.block_len > 0 ? h->cfg.block_len : (h->small_baths ? 8 : 4);
  // fused-stage tile waves: 4 (C3: 53.3 vs 55.3 us/step at 8, r02).  Large baths took 8 until round
  // 5 (C5 r02: 447 vs ~410 us at 4); with the two-plane far field and the ELL potential-force launch
  // 4 waves are faster there too: 255 vs 263.5 us/step (512 steps), 253.4 vs 259.1 (20-step
  // windows), 3 interleaved rounds on one box (`profiles/r05/c5_fused_waves.jsonl`) -- an 8-wave
  // workgroup needs two free wave slots on every SIMD beside the far-field chunks of 4 per CU
  h->ch_nw[1] = 4;
  int Pmax;
  if (h->cfg.max_block > 0) {
    Pmax = std::max(P0, h->cfg.max_block);
  } else if (spec_ok) {
    // spectral levels cost the same per step whatever their P (M = 2 partitions of P lags, K-hat read
    // once per block of P steps), except the last one, whose M = (ml - 2P) / P grows as ml / P: the
    // largest block is the smallest power of two >= 256 with 4P >= ml (at most 1024), so the last
    // level has M = 2 too.  C3 (ml 1024): 256.  C5 (ml 4096): 1024, a third of the K-hat bytes per
    // step that a last level of P = 256 with M = 14 streams.
    int pm = 256;
    while (4 * pm < mlmax && pm < 1024) pm *= 2;
    if (const char* e = gle_env("GLE_PMAX_SPEC")) pm = std::max(8, atoi(e));
    Pmax = std::max(P0, pm);
  } else {
    // direct: enough columns per block for MFMA reuse of each streamed kernel slice, and long
    // enough blocks that the last level's kernel slices stream from HBM rarely: the last level
    // reads (ml - 2 Pmax) slices per Pmax steps.  C2 (one trajectory, ml = 1024): Pmax 64 ran
    // 30.8 us/step against 46.6 at 32 (128: 31.4, 256: 31.9; same box, r03)
    int L = P0;
    while (L * B < 256 && L < 64) L *= 2;
    Pmax = L;
  }
  h->P0 = P0;
  h->wait_early = std::min(h->wait_early, P0 - 1);
  if (h->piece_slack < 1) h->wait_early = 0;
  // pieces go out at every step (GLE_PIECE_STEP=P0: only at first-level boundaries): the same
  // long-window rate, and a short window's background work depends less on its phase (20-step
  // windows over all phases: 55-67 us/step vs 55-79 us at C3)
  h->piece_g = 1;
  if (const char* e = gle_env("GLE_PIECE_STEP")) h->piece_g = std::max(1, std::min(P0, atoi(e)));
  h->near_end = std::min(mlmax, 2 * P0);
  h->levels.clear();
  for (int64_t P = P0; 2 * P < mlmax; P *= 2) {
    Level lv;
    lv.P = (int)P;
    lv.lag0 = (int)(2 * P);
    const bool last = P >= Pmax || 4 * P >= mlmax || (int)h->levels.size() == MAXLVL - 1;
    lv.lag1 = last ? mlmax : (int)(4 * P);
    const bool pow2 = (P & (P - 1)) == 0;
    // auto: spectral from P = 8, and from P = 4 for large baths (C5: 252.7 vs 256.6 us/step at 512
    // steps, 3 interleaved rounds, `profiles/r05/c5_ab/spec_min_ab_c5.jsonl`; its direct form was a
    // 0.39 ms contraction every 4 steps)
    int pmin = mode == GLE_FAR_SPECTRAL ? 2 : (h->small_baths ? 8 : 4);
    if (const char* e = gle_env("GLE_SPEC_MIN")) pmin = std::max(2, atoi(e));
    lv.spectral = spec_ok && pow2 && P >= pmin && 2 * P <= 8192;
    h->levels.push_back(lv);
    if (last) break;
  }
  // device-memory check of the spectral levels (transformed kernels, segment rings, spectra)
  {
    size_t need = 0;
    for (auto& lv : h->levels) {
      if (!lv.spectral) continue;
      for (auto& b : h->baths) {
        if (b.ml <= lv.lag0) continue;
        const int M = (std::min(lv.lag1, b.ml) + lv.P - 1) / lv.P - 2;
        const int npl = B <= 32 ? 2 : 3;  // Level::nplanes
        need += (size_t)(lv.P + 1) * npl * b.nrt * b.nks * M * 64 * 8;
        need += (size_t)(lv.P + 1) * npl * b.ncp * ((M + 4) * B + (npl == 2 ? 8 : 512)) * 8;
        need += (size_t)(lv.P + 1) * 3 * b.nc * B * 8;
      }
    }
    // the spectral buffers are the last big allocations of the plan (the kernels, noise and history
    // rings are already resident): keep a reserve for the remaining per-level buffers and the chain
    size_t fr = 0, tot = 0;
    hipMemGetInfo(&fr, &tot);
    const size_t reserve = std::max<size_t>((size_t)8 << 30, tot / 32);
    if (need + reserve > fr) {
      if (mode == GLE_FAR_SPECTRAL)
        return fail(h, GLE_ERR_NOMEM, "spectral levels need " + std::to_string(need >> 20) + " MiB");
      for (auto& lv : h->levels) lv.spectral = false;
    }
  }
  h->far_mode = GLE_FAR_DIRECT;
  int Pspec = 1, Ptop = P0;
  for (auto& lv : h->levels) {
    Ptop = std::max(Ptop, lv.P);
    if (lv.spectral) {
      h->far_mode = GLE_FAR_SPECTRAL;
      Pspec = std::max(Pspec, lv.P);
    }
  }
  h->L = Ptop;
  const int rn_step = rn_for(B);
  // history rings: ml + the background lookahead (a block may read p P+1 steps older than the
  // newest slot the main stream writes while it runs) + slack
  for (auto& b : h->baths) {
    b.R = b.ml + 3 * Ptop + 2;
    b.ldh = 2 * (int64_t)b.R * B + 512 + 16 * rn_for((int64_t)Ptop * B);
    int rc = dalloc_n(h, &b.d_H, (size_t)b.ncp * b.ldh, 4096);
    if (rc) return rc;
  }
  if (h->far_mode == GLE_FAR_SPECTRAL) {
    // twiddles cstab[q] = (cos(pi q / Pspec), sin(pi q / Pspec)), q < 2 Pspec
    std::vector<double> cst((size_t)4 * Pspec);
    for (int q = 0; q < 2 * Pspec; ++q) {
      const long double a = 3.14159265358979323846264338327950288L * (long double)q / (long double)Pspec;
      cst[2 * q] = (double)cosl(a);
      cst[2 * q + 1] = (double)sinl(a);
    }
    int rc = dalloc_n(h, &h->d_cstab, cst.size());
    if (!rc) rc = upload(h, h->d_cstab, cst.data(), cst.size() * 8);
    if (rc) return rc;
  }
  for (auto& lv : h->levels) {
    lv.cstride = lv.spectral ? Pspec / lv.P : 1;
    lv.cg_rn = std::min(4, rn_for(B));  // 16, 32 or 64 columns (cgemm_kernel has no 48-column form)
    lv.nplanes = lv.cg_rn <= 2 ? 2 : 3;  // (64-column items have no two-plane kernel path)
    lv.cg_split = 1;
    if (lv.spectral) {
      // small levels of large baths: split the k range of every product in two (partial planes
      // added by the inverse transform) so the launch has >= 2 workgroups per CU to hide the HBM
      // latency of the K̂ stream, which is still read once (GLE_CG_NARROW: 32-column tiles
      // instead, reading it once per 32 columns)
      int64_t n4 = 0;
      for (auto& b : h->baths)
        if (b.ml > lv.lag0)
          n4 += (int64_t)(lv.P + 1) * ((b.nrt + 3) / 4) * ((B + 16 * lv.cg_rn - 1) / (16 * lv.cg_rn));
      int ncu = 256;
      hipDeviceProp_t prop;
      if (hipGetDeviceProperties(&prop, h->cfg.device) == hipSuccess) ncu = prop.multiProcessorCount;
      // not with small baths: with 2-workgroup-per-CU chunks the unsplit products ran 49.0 vs 50.3
      // us/step at C3 (3 interleaved rounds, r03); GLE_CG_SPLIT=0/1 forces it off / on
      const char* esp = gle_env("GLE_CG_SPLIT");
      const bool want_split = esp ? atoi(esp) != 0 : !h->small_baths;
      if (n4 < 2 * ncu && want_split) {
        if (gle_env("GLE_CG_NARROW")) lv.cg_rn = 2;
        else lv.cg_split = 2;
      }
    }
    lv.lb.assign(h->baths.size(), LevelBath{});
    for (size_t j = 0; j < h->baths.size(); ++j) {
      Bath& b = h->baths[j];
      LevelBath& L = lv.lb[j];
      if (b.ml <= lv.lag0) continue;
      L.active = true;
      L.lag1 = std::min(lv.lag1, b.ml);
      int rc = dalloc_n(h, &L.d_out, (size_t)b.ncp * 2 * lv.P * B, 4096);
      if (rc) return rc;
      if (!lv.spectral) continue;
      L.M = (L.lag1 + lv.P - 1) / lv.P - 2;
      L.Rseg = L.M + 4;
      // ring slots addressed modulo Rseg (no mirrored copy); rows padded by 512 doubles for
      // 64-column items (C3: 49.8 vs 50.2 us/step at 8, 3 interleaved rounds, r04) and by 32 for the
      // two-plane levels (512 was 73 % of a row at C5's P = 1024 level, ~7 GB per bath).  The pad
      // also bounds the staged X loads: a 16- or 32-column item stages NT columns from col0, so for
      // the last ring slot it reads up to NT - 1 - (B - 1) mod NT doubles past the slot (15 at B = 1);
      // those columns (>= B) feed output columns that are never stored, and with a pad of >= 31 the
      // reads stay inside the row (GLE_SEG_PAD below 31 lets them run into the next row or plane,
      // harmless for the results but outside the row).
      L.ldseg = (int64_t)L.Rseg * B + (lv.nplanes == 2 ? 32 : 512);
      if (const char* e = gle_env("GLE_SEG_PAD")) L.ldseg = (int64_t)L.Rseg * B + std::max(0, atoi(e));
      L.khat_fstride = (int64_t)lv.nplanes * b.nrt * b.nks * L.M * 64;  // Re, Im | the Gauss planes
      L.seg_fstride = (int64_t)lv.nplanes * b.ncp * L.ldseg;             // Re, Im | Re + Im, Im, Re rows
      L.yfstride = (int64_t)3 * b.nc * B;                       // T_0, T_1, T_2
      rc = dalloc_n(h, &L.d_khat, (size_t)(lv.P + 1) * L.khat_fstride);
      if (!rc) rc = dalloc_n(h, &L.d_seg, (size_t)(lv.P + 1) * L.seg_fstride, 4096);
      if (!rc) rc = dalloc_n(h, &L.d_Yspec, (size_t)lv.cg_split * (lv.P + 1) * L.yfstride, 4096);
      if (rc) return rc;
      if (launch_khat_pack(b.d_K, b.ml, b.nks, L.d_khat, lv.P, 2, L.M, b.nc, b.nrt, b.nks, h->d_cstab,
                           lv.cstride, h->stream, lv.nplanes))
        return fail(h, GLE_ERR_UNSUP, "K-hat transform launch failed (P = " + std::to_string(lv.P) + ")");
      HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    // background stream per level group, bounds in units of P0 (GLE_BG_GROUP=g1,g2 in the experiment
    // build): small baths {P0}, {.. 8 P0}, rest (C3: 8 | 16-64 | 128-256: each level's pieces are a
    // chain of small dependent launches, so the ladder is bound by its streams' serial latency, and
    // the first level, due every P0 steps, gets a stream of its own; round 5 with the composed step:
    // 42.4-42.9 vs 46.0 us/step, `profiles/r05/composed/sched_ab_c3.jsonl`; round 4's 4,32 was best
    // beside the two-launch chain; small-bath direct plans too since the composed step: C2 21.1 vs
    // 23.4 us/step, the largest level's 0.56 ms contraction no longer holds up the first level's
    // blocks, `profiles/r05/split/bg_group_ab_c2.jsonl`), large baths {.. 8 P0}, {.. 64 P0}, rest
    const bool g_small = h->small_baths;
    int g1 = g_small ? 1 : 8, g2 = g_small ? 8 : 64;
    if (const char* e = gle_env("GLE_BG_GROUP")) sscanf(e, "%d,%d", &g1, &g2);
    lv.sidx = lv.P <= g1 * P0 ? 0 : (lv.P <= g2 * P0 ? 1 : 2);
    for (int q = 0; q < 2; ++q)
      HIPCHK(h, hipEventCreateWithFlags(&lv.ev[q], hipEventDisableTiming | hipEventReleaseToDevice));
  }
  // DOF tiles of the chain (16 DOFs each) = rows of the per-step current / energy partial table
  h->ndblk = (int)((h->nph + 15) / 16);
  int rc = dalloc_n(h, &h->d_part, (size_t)h->nmd * h->ndblk * (h->baths.size() + 1) * B);
  if (rc) return rc;
  rc = dalloc_n(h, &h->d_pmax, (size_t)4 * B);
  if (rc) return rc;
  // constraint mask
  std::vector<uint8_t> mask(h->nph, 0);
  for (auto d : h->constr) mask[d] = 1;
  rc = dalloc_n(h, &h->d_cmask, h->nph);
  if (rc) return rc;
  rc = upload(h, h->d_cmask, mask.data(), h->nph);
  if (rc) return rc;

  // compact copy of the slices every step reads (K_0 and the near field): the full fragment-native
  // kernel puts consecutive k-steps of one slice ml*512 B apart, so a per-step product touching
  // only a few slices would hit a new page (TLB miss) on nearly every fragment
  for (auto& b : h->baths) {
    b.nn = std::max(1, std::min(b.ml, h->near_end));
    rc = dalloc_n(h, &b.d_Kn, (size_t)b.nrt * b.nks * b.nn * 64);
    if (rc) return rc;
    HIPCHK(h, hipMemcpy2DAsync(b.d_Kn, (size_t)b.nn * 64 * 8, b.d_K, (size_t)b.ml * 64 * 8,
                               (size_t)b.nn * 64 * 8, (size_t)b.nrt * b.nks, hipMemcpyDeviceToDevice,
                               h->stream));
  }

  // ---- plans
  const int TGT_BIG = 512;
  auto kgemm = [&](Bath& b, const double* A, int i0, int i1, const double* X, int64_t ldx, int ring,
                   int tshift, int N, double* dst, int64_t ldd) {
    Gemm g{};
    g.A = A;
    g.a_ks = (int64_t)(A == b.d_K ? b.ml : (A == b.d_Kn ? b.nn : 1)) * 64;
    g.a_rt = (int64_t)b.nks * g.a_ks;
    g.nrt_total = b.nrt;
    g.nks_total = b.nks;
    g.i0 = i0;
    g.i1 = i1;
    g.X = X;
    g.ldx = ldx;
    g.ring = ring;
    g.cs = (int)B;
    g.tshift = tshift;
    g.M = b.nc;
    g.Kd = b.nc;
    g.N = N;
    g.dst = dst;
    g.ldd = ldd;
    return g;
  };
  // LEVEL blocks.  Block k is computed with the step argument t = T = (k-1)P.
  //   direct:   out[c] = sum_{i in [2P, lag1)} K_i p_{T+P+1+c/B-i}, c < P*B (targets T+P+1..T+2P),
  //             one op per output parity (block buffer half k&1)
  //   spectral: per frequency f, Y_f = sum_{m>=2} Khat_m(f) Xhat_{T/P+2-m}(f) on [[Re,-Im],[Im,Re]]
  //             (the segment ring holds Xhat of the segments ending at sigma*P)
  for (auto& lv : h->levels) {
    if (lv.spectral) {
      // one workgroup per (bath, f, Gauss part g, 64-row group, 16 RN-column tile); items of one
      // (f, g) are adjacent, so the row groups that share an X window run together
      lv.cg.clear();  // cg_rn / cg_split were chosen with the level's buffers
      lv.cg_flops = lv.cg_bytes = lv.cg_units = 0;
      const int NT = 16 * lv.cg_rn;
      for (size_t j = 0; j < h->baths.size(); ++j) {
        Bath& b = h->baths[j];
        LevelBath& L = lv.lb[j];
        if (!L.active) continue;
        const int64_t a_rt = (int64_t)L.M * b.nks * 64;
        const int64_t plane = (int64_t)b.nrt * a_rt;
        for (int f = 0; f <= lv.P; ++f) {
          // f = 0 and f = P: K-hat and X-hat are real, so Re Y = T_0 - T_1 = T_0 = Kr Xr and Im Y is
          // dropped (far_ifft realonly): one product, the T_1 / T_2 planes stay zero.  Otherwise one
          // item forms all three Gauss parts from the Re / Im planes of K-hat and X-hat.
          // three-plane layout (nplanes = 3): one item per Gauss part g, reading plane g of K-hat and X
          const bool real = f == 0 || f == lv.P;
          const int ng = lv.nplanes == 2 ? 1 : (real ? 1 : 3);
          for (int g = 0; g < ng; ++g) {
            for (int rg = 0; 4 * rg < b.nrt; ++rg)
              for (int c0 = 0; c0 < B; c0 += NT)
                for (int hk = 0; hk < lv.cg_split; ++hk) {
                CgItem it{};
                const int S = L.M * b.nks;
                it.s0 = S * hk / lv.cg_split;
                it.ns = S * (hk + 1) / lv.cg_split - it.s0;
                it.g3 = (lv.nplanes == 2 && !real) ? 1 : 0;
                it.A = L.d_khat + (int64_t)f * L.khat_fstride + g * plane + (int64_t)4 * rg * a_rt;
                it.a_pl = plane;
                it.X = L.d_seg + (int64_t)f * L.seg_fstride + (int64_t)g * b.ncp * L.ldseg;
                it.x_pl = (int64_t)b.ncp * L.ldseg;
                it.out = L.d_Yspec + (int64_t)hk * (lv.P + 1) * L.yfstride + (int64_t)f * L.yfstride +
                         (int64_t)g * b.nc * B + (int64_t)64 * rg * B + c0;
                it.o_pl = (int64_t)b.nc * B;
                it.a_rt = a_rt;
                it.ldx = (int32_t)L.ldseg;
                it.cs = (int32_t)B;
                it.Rseg = L.Rseg;
                it.M = L.M;
                it.nks = b.nks;
                it.nrt = std::min(4, b.nrt - 4 * rg);
                it.nrows = std::min(64, b.nc - 64 * rg);
                it.ncols = (int)std::min<int64_t>(NT, B - c0);
                it.ldo = (int32_t)B;
                it.col0 = c0;
                lv.cg.push_back(it);
                lv.cg_units += it.g3 ? 3.0 : 1.0;
              }
            // algorithmic work of the products of (f, g): the Gauss parts' MFMA flops;
            // K-hat's planes read once, the X window's planes read once, the T planes written once
            const bool two = lv.nplanes == 2 && !real;
            const double np = two ? 3.0 : 1.0, npl = two ? 2.0 : 1.0;
            lv.cg_flops += np * 2.0 * b.nc * ((double)L.M * b.nc) * B;
            lv.cg_bytes += 8.0 * (npl * (double)b.nc * L.M * b.nc + npl * (double)L.M * b.nc * B + np * (double)b.nc * B);
          }
        }
      }
      rc = dalloc_n(h, &lv.d_cg, lv.cg.size());
      if (!rc) rc = upload(h, lv.d_cg, lv.cg.data(), lv.cg.size() * sizeof(CgItem));
      if (rc) return rc;
      {
        // cgemm chunks of ~cg_per_cu workgroups per CU, at most one chunk per first-level boundary
        int ncu = 256;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, h->cfg.device) == hipSuccess) ncu = prop.multiProcessorCount;
        const int nslot = std::max(1, lv.P / h->P0);
        // workgroups per CU per cgemm chunk (GLE_CG_PER_CU): 1.25 with small baths and the
        // whole-window piece schedule (C3 r04: 1 and 2.5 cost 0.5-2 us/step, 1.5-1.75 within
        // 0.2; with slack 1, 2 was best in r03: 50.0 vs 51.1 us/step at 0.5), 4 for large baths
        // (C5, with the fpot launch: 354 vs 400 us/step at 2, flat from 4 to 32)
        double per_cu = h->small_baths ? 1.25 : 4.0;
        if (const char* e = gle_env("GLE_CG_PER_CU")) per_cu = std::max(0.25, atof(e));
        h->cg_per_cu = per_cu;
        // chunks sized in Gauss products (a two-plane item forms three): the chunk durations the
        // per-CU rates were measured with (GLE_CG_UNITS=0: in items, i.e. workgroups)
        const char* eu = gle_env("GLE_CG_UNITS");
        const double units = (eu && atoi(eu) == 0) ? (double)lv.cg.size() : lv.cg_units;
        const double want = units / (per_cu * ncu);
        const int64_t nch = gle_env("GLE_CG_CEIL") ? (int64_t)std::ceil(want - 1e-9) : (int64_t)want;
        lv.ncg_chunk = (int)std::max<int64_t>(1, std::min<int64_t>(nch, nslot));
        if (const char* e = gle_env("GLE_NO_PIECES")) lv.ncg_chunk = atoi(e) > 0 ? 1 : lv.ncg_chunk;
        // the long levels' transforms go out as DOF-range pieces too (one piece = every bath's
        // range j): a whole-level transform of P = 256 (2 x 2400 workgroups at C3) held the CUs
        // of ~20 steps' chain launches at once, the slowest short windows of the phase scan
        int fdiv = 32;
        if (const char* e = gle_env("GLE_FFT_CHUNK")) fdiv = atoi(e) > 0 ? std::max(1, atoi(e)) : 1 << 30;
        lv.nfs = lv.nif = std::max(1, std::min(lv.P / fdiv, 16));
        lv.npiece = lv.nfs + lv.ncg_chunk + lv.nif;
      }
    } else {
      for (int par = 0; par < 2; ++par) {
        Planner p(h, lv.op[par], rn_for((int64_t)lv.P * B));
        for (size_t j = 0; j < h->baths.size(); ++j) {
          Bath& b = h->baths[j];
          LevelBath& L = lv.lb[j];
          if (!L.active) continue;
          Gemm g = kgemm(b, b.d_K, lv.lag0, L.lag1, b.d_H, b.ldh, b.R, lv.P + 1, (int)(lv.P * B),
                         L.d_out + (int64_t)par * lv.P * B, (int64_t)2 * lv.P * B);
          g.force_reduce = true;
          p.add(g, TGT_BIG, 16);
        }
        rc = p.done();
        if (rc) return rc;
      }
    }
  }
  // PRIME: S(t) = sum_{i>=1} K_i p_{t-i} from the current history (after set_state/history)
  {
    Planner p(h, h->op_prime, rn_step);
    for (auto& b : h->baths)
      if (b.ml > 1) {
        Gemm g = kgemm(b, b.d_K, 1, b.ml, b.d_H, b.ldh, b.R, 0, (int)B, b.d_S, B);  // S[0]; parity fixed at run time
        g.force_reduce = true;
        p.add(g, TGT_BIG, 16);
      }
    rc = p.done();
    if (rc) return rc;
  }
  rc = plan_chain(h);
  if (rc) return rc;
  rc = plan_far_fused(h);
  if (rc) return rc;
  rc = plan_xstep(h);
  if (rc) return rc;
  // device step descriptor
  StepDev sd{};
  sd.nph = (int32_t)h->nph;
  sd.B = (int32_t)B;
  sd.nmd = (int32_t)h->nmd;
  sd.nbath = (int32_t)h->baths.size();
  sd.dt = h->dt;
  sd.P = h->d_P;
  sd.Q = h->d_Q;
  sd.Ph = h->d_Ph;
  sd.Qt = h->d_Qt;
  sd.Fc = h->d_Fc;
  sd.Flast = h->d_Flast;
  sd.etot = h->d_etot;
  sd.Q0 = h->d_Q0;
  sd.qvalid = h->d_qvalid;
  sd.pmax = h->d_pmax;
  sd.part = h->d_part;
  sd.cmask = h->d_cmask;
  sd.ndblk = h->ndblk;
  sd.guard = h->d_guard;
  if (const char* dbg = gle_env("GLE_CHAIN_DBG")) {
    size_t n = 0;
    for (Chain* c : {&h->chA[0], &h->chA[1], &h->chB[1], &h->chC, &h->chBC, &h->chX[0], &h->chX[1]})
      n = std::max(n, c->tiles.size());
    sd.dbg_ntile = (int32_t)n;
    sd.dbg_t = atoll(dbg);
    rc = dalloc_n(h, &h->d_dbg, (size_t)3 * n * 4);
    if (rc) return rc;
    sd.dbg = h->d_dbg;
    h->dbg_ntile = (int)n;
    h->dbg_t = sd.dbg_t;
  }
  for (size_t j = 0; j < h->baths.size(); ++j) {
    Bath& b = h->baths[j];
    BathDev& bd = sd.bath[j];
    bd.inv = b.d_inv;
    bd.noise = b.d_noise;
    bd.S = b.d_S;
    bd.Yq = b.d_Yq;
    bd.Xcur = b.d_Xcur;
    bd.Xq = b.d_Xq;
    bd.H = b.d_H;
    bd.cur = b.d_cur;
    bd.NP = b.d_NP;
    bd.NR = b.d_NR;
    bd.NRS = b.NRS;
    bd.nlvl = (int32_t)h->levels.size();
    for (size_t l = 0; l < h->levels.size(); ++l) {
      const LevelBath& L = h->levels[l].lb[j];
      bd.lvl[l] = L.active ? L.d_out : nullptr;
      bd.lvl_ld[l] = 2 * h->levels[l].P * (int32_t)B;
    }
    bd.c = b.c;
    bd.vs = b.vs;
    bd.nc = b.nc;
    bd.ncp = b.ncp;
    bd.ldh = (int32_t)b.ldh;
    bd.R = b.R;
    bd.has_q = b.has_q ? 1 : 0;
    bd.nqn = b.nqn;
  }
  rc = dalloc_n(h, &h->d_sd, 1);
  if (rc) return rc;
  h->sdh = sd;
  h->frozen = true;
  return apply_record(h);  // uploads the step descriptor
}

// Pieces [j0, j1) of block k of level lv on stream s (see Level::npiece); the last piece records
// the block's event.  Spectral: the newest segment spectrum is transformed first (all M when
// priming), then the cgemm item chunks, then the inverse transform.
int launch_level_pieces(gle_handle* h, Level& lv, int64_t k, hipStream_t s, bool priming, int j0, int j1) {
  const int64_t T = (k - 1) * (int64_t)lv.P;
  const StepArgs ta = step_args(h, T);
  const int par = (int)(k & 1);
  const int li = (int)(&lv - h->levels.data());
  if (lv.spectral && priming) {
    // the whole block at once with the unsplit items (k-halves in separate planes): all M segment
    // transforms, one GEMM launch, the inverse transform
    for (size_t b = 0; b < h->baths.size(); ++b) {
      Bath& bb = h->baths[b];
      LevelBath& L = lv.lb[b];
      if (!L.active) continue;
      if (launch_seg_fft(bb.d_H, bb.ldh, bb.R, (int)h->B, bb.nc, bb.ncp, lv.P, T, L.M, L.d_seg, L.seg_fstride,
                         L.ldseg, L.Rseg, h->d_cstab, lv.cstride, s, 0, -1, lv.nplanes))
        return fail(h, GLE_ERR_UNSUP, "segment transform launch failed (P = " + std::to_string(lv.P) + ")");
    }
    launch_cgemm(lv.cg_rn, lv.d_cg, (int)lv.cg.size(), T / lv.P, s, 0, nullptr);
    for (size_t b = 0; b < h->baths.size(); ++b) {
      Bath& bb = h->baths[b];
      LevelBath& L = lv.lb[b];
      if (!L.active) continue;
      if (launch_far_ifft(L.d_Yspec, L.yfstride, lv.cg_split > 1 ? (int64_t)(lv.P + 1) * L.yfstride : 0, bb.nc,
                          (int)h->B, lv.P, L.d_out + (int64_t)par * lv.P * h->B, (int64_t)2 * lv.P * h->B, h->d_cstab,
                          lv.cstride, s))
        return fail(h, GLE_ERR_UNSUP, "inverse transform launch failed (P = " + std::to_string(lv.P) + ")");
    }
    HIPCHK(h, hipEventRecord(lv.ev[par], s));
    lv.ev_seq[par] = ++h->ev_seq_counter;
    return GLE_OK;
  }
  // background schedule with k-split items (bg_split): the chunks walk the split-major item list in
  // order on the level's in-order stream (each chunk at most nout items: the k-splits of a product
  // land in successive launches, the later ones adding), the inverse transform reads one plane
  const bool split = lv.bg_split;
  const CgItem* d_items = split ? lv.d_fcg : lv.d_cg;
  const int64_t nitems = split ? (int64_t)lv.fcg.size() : (int64_t)lv.cg.size();
  for (int j = j0; j < j1; ++j) {
    if (!lv.spectral) {
      // profiled only when no level is spectral: the roofline then names one kernel class
      if (priming || !(h->dbg_skip & 8)) run_op(h, lv.op[par], s, ta, h->far_mode != GLE_FAR_SPECTRAL);
      if (h->prof && !priming) h->prof_blocks[li] += 1.0;
      continue;
    }
    // pieces: [0, nfs) segment transform DOF ranges, then ncg_chunk GEMM chunks, then [.., npiece)
    // inverse transform DOF ranges
    const int jg = j - lv.nfs + 1;  // 1-based GEMM chunk
    if (j < lv.nfs) {
      // every bath's DOF range j in one launch (up to MAXFB baths per launch)
      FftBaths fb{};
      auto flush = [&]() {
        if (fb.n && launch_seg_fft_multi(fb, (int)h->B, lv.P, T, priming ? lv.lb[0].M : 1, h->d_cstab, lv.cstride, s,
                                         lv.nplanes))
          return fail(h, GLE_ERR_UNSUP, "segment transform launch failed (P = " + std::to_string(lv.P) + ")");
        fb.n = 0;
        return GLE_OK;
      };
      for (size_t b = 0; b < h->baths.size(); ++b) {
        Bath& bb = h->baths[b];
        LevelBath& L = lv.lb[b];
        if (!L.active || (!priming && (h->dbg_skip & 2))) continue;
        const int k0 = (int)((int64_t)bb.nc * j / lv.nfs), k1 = (int)((int64_t)bb.nc * (j + 1) / lv.nfs);
        if (priming && L.M != lv.lb[0].M) {  // (priming transforms all M segments: one bath per launch)
          if (launch_seg_fft(bb.d_H, bb.ldh, bb.R, (int)h->B, bb.nc, bb.ncp, lv.P, T, L.M, L.d_seg, L.seg_fstride,
                             L.ldseg, L.Rseg, h->d_cstab, lv.cstride, s, k0, k1, lv.nplanes))
            return fail(h, GLE_ERR_UNSUP, "segment transform launch failed (P = " + std::to_string(lv.P) + ")");
          continue;
        }
        FftBath& e = fb.b[fb.n++];
        e = FftBath{};
        e.H = bb.d_H;
        e.ldh = bb.ldh;
        e.R = bb.R;
        e.nc = bb.nc;
        e.ncp = bb.ncp;
        e.k0 = k0;
        e.nk = k1 - k0;
        e.seg = L.d_seg;
        e.seg_fstride = L.seg_fstride;
        e.ldseg = L.ldseg;
        e.Rseg = L.Rseg;
        if (fb.n == MAXFB) {
          int rc = flush();
          if (rc) return rc;
        }
      }
      int rc = flush();
      if (rc) return rc;
    } else if (jg <= lv.ncg_chunk) {
      // one chunk of the batched GEMM of the per-frequency products, profiled like run_op
      const int64_t n = nitems;
      const int64_t c0 = n * (jg - 1) / lv.ncg_chunk, c1 = n * jg / lv.ncg_chunk;
      if (c1 <= c0) continue;
      hipEvent_t e1 = nullptr;
      unsigned long long* ts = nullptr;
      if (h->prof_ev) {
        if (h->ev_used + 2 > h->ev.size() || h->tst_used >= h->tst_cap) drain_profile(h);
        hipEventRecord(h->ev[h->ev_used], s);
        e1 = h->ev[h->ev_used + 1];
        h->ev_used += 2;
        if (h->d_tst && !priming) ts = h->d_tst + 2 * h->tst_used++;
      }
      if (priming || !(h->dbg_skip & 1))
        launch_cgemm(lv.cg_rn, d_items + c0, (int)(c1 - c0), T / lv.P, s, priming ? 0 : h->bg_grid, ts);
      if (h->prof && !priming) h->prof_blocks[li] += (double)(c1 - c0) / (double)n;
      if (e1) {
        hipEventRecord(e1, s);
        const double frac = (double)(c1 - c0) / (double)n;
        h->prof_n += 1;
        h->prof_flops += lv.cg_flops * frac;
        h->prof_bytes += lv.cg_bytes * frac;
      }
    } else {
      const int ji = jg - lv.ncg_chunk - 1;  // inverse transform piece: every bath's range in one launch
      FftBaths fb{};
      auto flush = [&]() {
        if (fb.n && launch_far_ifft_multi(fb, (int)h->B, lv.P, h->d_cstab, lv.cstride, s))
          return fail(h, GLE_ERR_UNSUP, "inverse transform launch failed (P = " + std::to_string(lv.P) + ")");
        fb.n = 0;
        return GLE_OK;
      };
      for (size_t b = 0; b < h->baths.size(); ++b) {
        Bath& bb = h->baths[b];
        LevelBath& L = lv.lb[b];
        if (!L.active || (!priming && (h->dbg_skip & 4))) continue;
        const int k0 = (int)((int64_t)bb.nc * ji / lv.nif), k1 = (int)((int64_t)bb.nc * (ji + 1) / lv.nif);
        FftBath& e = fb.b[fb.n++];
        e = FftBath{};
        e.Y = L.d_Yspec;
        e.yfstride = L.yfstride;
        e.ysplit = (!split && lv.cg_split > 1) ? (int64_t)(lv.P + 1) * L.yfstride : 0;
        e.nc = bb.nc;
        e.k0 = k0;
        e.nk = k1 - k0;
        e.out = L.d_out + (int64_t)par * lv.P * h->B;
        e.ldout = (int64_t)2 * lv.P * h->B;
        if (fb.n == MAXFB) {
          int rc = flush();
          if (rc) return rc;
        }
      }
      int rc = flush();
      if (rc) return rc;
    }
  }
  if (j1 >= lv.npiece) {
    HIPCHK(h, hipEventRecord(lv.ev[par], s));
    lv.ev_seq[par] = ++h->ev_seq_counter;
  }
  return GLE_OK;
}

int launch_level_block(gle_handle* h, Level& lv, int64_t k, hipStream_t s, bool priming) {
  return launch_level_pieces(h, lv, k, s, priming, 0, lv.npiece);
}

// After set_state / set_history: S(t) from the whole history and, per level, block k0 = floor(t/P)
// (targets up to the next block boundary) on the main stream.  Block k0 + 1 enters the level's
// piece schedule at once, as if it had been started at the boundary k0 P: its pieces go out on
// the background stream over the first-level boundaries up to (k0 + 1) P (the ones already passed
// at the first step), so every window of steps after a prime carries the steady-state share of
// far-field work.
int prime(gle_handle* h) {
  join_bg(h);  // blocks still in flight read the ring and write the buffers recomputed here
  const StepArgs ta = step_args(h);
  // S(t) into S[t&1]: the prime op writes S[0]; copy when t is odd
  if (!h->op_prime.empty()) {
    run_op(h, h->op_prime, h->stream, ta, false);
    if (h->t & 1)
      for (auto& b : h->baths)
        if (b.ml > 1)
          HIPCHK(h, hipMemcpyAsync(b.d_S + b.vs, b.d_S, (size_t)b.ncp * h->B * 8,
                                   hipMemcpyDeviceToDevice, h->stream));
  }
  for (auto& lv : h->levels) {
    const int64_t k0 = floordiv(h->t, lv.P);
    int rc = launch_level_block(h, lv, k0, h->stream, true);
    if (rc) return rc;
    if (lv.fused) {
      // fused schedule: the next block too (its data ends at k0 P <= t), so the items ride from the
      // next block boundary on with whole windows
      rc = launch_level_block(h, lv, k0 + 1, h->stream, true);
      if (rc) return rc;
      lv.last_block = k0 + 1;
      lv.fblock = INT64_MIN;
      lv.pend_block = INT64_MIN;
      lv.bg_block[0] = lv.bg_block[1] = INT64_MIN;
      continue;
    }
    lv.last_block = k0 + 1;
    lv.bg_block[0] = lv.bg_block[1] = INT64_MIN;
    lv.bg_block[(k0 + 1) & 1] = k0 + 1;  // the main stream waits for it at (k0 + 1) P
    lv.pend_block = k0 + 1;
    lv.pend_t0 = k0 * (int64_t)lv.P;
    lv.next_piece = 0;
  }
  // near-field partials of target t+1 (lags >= 2: p up to t-1), as the chain of step t-1 leaves them
  for (auto& b : h->baths)
    launch_near_fill(b.d_H, b.ldh, b.R, (int)h->B, b.ncp, b.d_NR, b.vs, b.NRS, h->t, h->stream);
  launch_chain(1, h->chNear.nw, h->ch_drn, h->chNear.lds, h->chNear.d, (int)h->chNear.tiles.size(), h->d_sd,
               step_args(h, h->t - 1), 0, h->stream);
  if (!h->levels.empty()) {
    // the pending blocks' pieces read what this prime wrote (segment spectra, ring)
    HIPCHK(h, hipEventRecord(h->ev_step, h->stream));
    for (int i = 0; i < gle_handle::NBG; ++i)
      if (h->bg[i]) HIPCHK(h, hipStreamWaitEvent(h->bg[i], h->ev_step, 0));
  }
  h->need_prime = false;
  return GLE_OK;
}

int ladder_step(gle_handle* h, int early);

int step_begin_impl(gle_handle* h, const double* fpot_host_T) {
  if (!h->state_set) return fail(h, GLE_ERR_STATE, "gle_set_state has not been called");
  bounds_table_sync();
  for (size_t j = 0; j < h->baths.size(); ++j)
    if (!h->baths[j].noise_set) return fail(h, GLE_ERR_STATE, "bath " + std::to_string(j) + " has no noise");
  if (fpot_host_T == nullptr && !h->has_dyn)
    return fail(h, GLE_ERR_STATE, "no potential force: pass fpot or call gle_set_dyn (md.py:468-470)");
  int rc = 0;
  if (h->std_stale) {
    // composed steps ran since the two-launch path's buffers were current: rebuild S(t), the near
    // partials and the blocks from the history, and forget the potential cache (its words held the
    // composed step's audit distances)
    h->std_stale = false;
    h->need_prime = true;
    h->pot_cache_exact = false;
    HIPCHK(h, hipMemsetAsync(h->d_qvalid, 0, (size_t)h->B * sizeof(int32_t), h->stream));
    HIPCHK(h, hipMemsetAsync(h->d_pmax, 0, (size_t)4 * h->B * sizeof(unsigned long long), h->stream));
  }
  h->x_live = false;  // this step does not maintain the composed step's V0 / W1 / NP3
  if (h->need_prime) {
    rc = prime(h);
    if (rc) return rc;
  }
  rc = ladder_step(h, 0);
  if (rc) return rc;
  const bool need_pot = (fpot_host_T == nullptr) && !h->pot_cache_exact;
  const StepArgs ta = step_args(h);
  if (fpot_host_T)
    HIPCHK(h, hipMemcpyAsync(h->d_Fc, fpot_host_T, (size_t)h->nph * h->B * 8, hipMemcpyHostToDevice, h->stream));
  if (h->d_dbg && h->t == h->dbg_t) h->dbg_a = need_pot ? 1 : 0;  // GLE_CHAIN_DBG: the stage-A variant recorded
  run_chain(h, 0, h->chA[need_pot ? 1 : 0], ta, (need_pot ? 1 : 0) | (fpot_host_T ? 0 : 2), h->levels.empty(), 0);
  h->host_force_step = fpot_host_T != nullptr;
  return GLE_OK;
}

// The ladder's work at the start of step t (before its chain launches): fused levels' transforms,
// the background blocks' pieces, and the main stream's waits for the blocks its launches read --
// target t+1 (early = 0) or also target t+2 (early = 1: the composed step's S tiles)
int ladder_step(gle_handle* h, int early) {
  int rc = 0;
  const int64_t t = h->t;
  // ladder: at each block boundary T = kP, start block k+1 (targets T+P+1..T+2P, data up to T) on
  // the level's background stream once step T-1 has closed; consume block k from this step on
  // The block's pieces are issued over the first-level boundaries T, T+P0, ..., T+P-P0 (levels in
  // increasing P, so each boundary's small-level block is queued before the big levels' pieces).
  bool bg_waited[gle_handle::NBG] = {};
  hipEvent_t wait_ev[gle_handle::NBG] = {};
  int64_t wait_seq[gle_handle::NBG] = {};
  const bool boundary = t % h->P0 == 0, tick = t % h->piece_g == 0;
  // fused levels, at their block boundaries t = kP on the main stream: the inverse transform of
  // block k (its items rode in the chain launches of the last P steps; A(t) reads it), then the
  // newest segment's transform for block k + 1, whose items start riding in A(t)
  if (h->far_fused && !h->dbg_no_ladder) {
    for (auto& lv : h->levels) {
      if (!lv.fused || t % lv.P != 0) continue;
      const int64_t k = floordiv(t, lv.P);
      if (lv.fblock == k) {
        for (size_t b = 0; b < h->baths.size(); ++b) {
          Bath& bb = h->baths[b];
          LevelBath& L = lv.lb[b];
          if (!L.active) continue;
          if (launch_far_ifft(L.d_Yspec, L.yfstride, 0, bb.nc, (int)h->B, lv.P, L.d_out + (int64_t)(k & 1) * lv.P * h->B,
                              (int64_t)2 * lv.P * h->B, h->d_cstab, lv.cstride, h->stream))
            return fail(h, GLE_ERR_UNSUP, "inverse transform launch failed (P = " + std::to_string(lv.P) + ")");
        }
        lv.fblock = INT64_MIN;
      }
      if (k + 1 > lv.last_block) {
        for (size_t b = 0; b < h->baths.size(); ++b) {
          Bath& bb = h->baths[b];
          LevelBath& L = lv.lb[b];
          if (!L.active) continue;
          if (launch_seg_fft(bb.d_H, bb.ldh, bb.R, (int)h->B, bb.nc, bb.ncp, lv.P, t, 1, L.d_seg, L.seg_fstride,
                             L.ldseg, L.Rseg, h->d_cstab, lv.cstride, h->stream, 0, -1, lv.nplanes))
            return fail(h, GLE_ERR_UNSUP, "segment transform launch failed (P = " + std::to_string(lv.P) + ")");
        }
        lv.fblock = k + 1;
        lv.fT = t;
        lv.last_block = k + 1;
      }
    }
  }
  if (!h->dbg_no_ladder && (boundary || tick)) {
    for (auto& lv : h->levels) {
      if (lv.fused) continue;
      hipStream_t bs = h->bg_serial ? h->stream : h->bg[lv.sidx];
      const int64_t k = floordiv(t, lv.P);
      if (boundary && t % lv.P == 0 && k + 1 > lv.last_block) {
        if (lv.pend_block != INT64_MIN) {  // (cannot happen: the last piece is due at T + P - P0)
          rc = launch_level_pieces(h, lv, lv.pend_block, bs, false, lv.next_piece, lv.npiece);
          if (rc) return rc;
        }
        if (!bg_waited[lv.sidx]) {
          HIPCHK(h, hipStreamWaitEvent(bs, h->ev_step, 0));
          bg_waited[lv.sidx] = true;
        }
        lv.pend_block = k + 1;
        lv.pend_t0 = t;
        lv.next_piece = 0;
        lv.last_block = k + 1;
        lv.bg_block[(k + 1) & 1] = k + 1;
      }
      if (tick && lv.pend_block != INT64_MIN) {
        // the pieces go out over the first slots (piece_g steps each) of the block's window up to
        // `slack` first-level blocks before the main stream needs the block, which leaves them that
        // long to drain
        const int nslot = std::max(1, (lv.P - h->piece_slack * h->P0) / h->piece_g);
        const int slot = (int)((t - lv.pend_t0) / h->piece_g);
        const int j1 = slot + 1 >= nslot ? lv.npiece : (int)(((int64_t)(slot + 1) * lv.npiece + nslot - 1) / nslot);
        if (j1 > lv.next_piece) {
          rc = launch_level_pieces(h, lv, lv.pend_block, bs, false, lv.next_piece, j1);
          if (rc) return rc;
          lv.next_piece = j1;
        }
        if (lv.next_piece >= lv.npiece) lv.pend_block = INT64_MIN;
      }
      // the main stream waits for block k at the first step within wait_early steps of its first
      // use k P (the block's last piece and event were enqueued >= piece_slack first-level blocks
      // before k P, and wait_early < P0); wait_early = 0: at the boundary k P itself
      const int64_t kw = floordiv(t + h->wait_early + early, lv.P);
      if (lv.bg_block[kw & 1] == kw) {
        const int64_t k = kw;
        // per background stream, waiting for the block enqueued last implies the earlier ones
        // (in-order streams): one barrier packet per stream instead of one per level
        if (h->merge_waits) {
          if (!wait_ev[lv.sidx] || lv.ev_seq[k & 1] > wait_seq[lv.sidx]) {
            wait_ev[lv.sidx] = lv.ev[k & 1];
            wait_seq[lv.sidx] = lv.ev_seq[k & 1];
          }
        } else {
          HIPCHK(h, hipStreamWaitEvent(h->stream, lv.ev[k & 1], 0));
        }
        lv.bg_block[k & 1] = INT64_MIN;
      }
    }
    for (int i = 0; i < gle_handle::NBG; ++i)
      if (wait_ev[i]) HIPCHK(h, hipStreamWaitEvent(h->stream, wait_ev[i], 0));
  }
  return rc;
}

int step_end_impl(gle_handle* h, const double* fpot_host_T) {
  int mode1 = 1;
  const StepArgs ta = step_args(h);
  if (fpot_host_T) {
    HIPCHK(h, hipMemcpyAsync(h->d_Fc, fpot_host_T, (size_t)h->nph * h->B * 8, hipMemcpyHostToDevice, h->stream));
    mode1 = 0;
  } else {
    if (!h->has_dyn) return fail(h, GLE_ERR_STATE, "no potential force at q~");
    if (h->host_force_step) return fail(h, GLE_ERR_STATE, "step begun with a host force must end with one");
  }
  if (h->exp_one && mode1 == 1) {
    // GLE_EXP_ONE: no velocity-stage launch (timing only)
  } else if (h->fuse_bc && mode1 == 1) {
    if (h->bc_fpot) {
      FpotArgs fa{};
      fa.nph = (int32_t)h->nph;
      fa.B = (int32_t)h->B;
      fa.par = (int32_t)(h->t & 1);
      fa.ew = h->fpot_ew;
      fa.rp = h->d_dyn_rp;
      fa.col = h->d_dyn_col;
      fa.val = h->d_dyn_val;
      fa.vb = h->d_fpot_vb;
      fa.Qt = h->d_Qt;
      fa.Fc = h->d_Fc;
      fa.Q0 = h->d_Q0;
      fa.pmax = h->d_pmax;
      fa.t1 = (int32_t)((h->t + 1) % h->nmd);
      for (size_t j = 0; j < h->baths.size() && j < (size_t)MAXBATH; ++j) {
        fa.V[j] = h->baths[j].d_V;
        fa.noise[j] = h->baths[j].ml < 2 ? h->baths[j].d_noise : nullptr;
        fa.nc[j] = h->baths[j].nc;
      }
      launch_fpot(fa, h->stream);
      mode1 |= 4;  // the velocity stage takes Fpot(q~) from Fc, V holds V + Fpot_b
    }
    run_chain(h, 3, h->chBC, ta, mode1, h->levels.empty(), 1);
  } else {
    run_chain(h, 1, h->chB[mode1], ta, mode1, h->levels.empty(), 1);
    run_chain(h, 2, h->chC, ta, mode1, h->levels.empty(), 2);
  }
  // the next step is a block boundary: the background blocks started there wait for this step
  if (!h->levels.empty() && (h->t + 1) % h->P0 == 0) HIPCHK(h, hipEventRecord(h->ev_step, h->stream));
  h->t += 1;
  h->pot_cache_exact = (fpot_host_T == nullptr) && h->constr.empty();
  h->std_words_live = true;  // the velocity stage wrote step t + 1's id0 distances (host force: against q~)
  HIPCHK(h, hipGetLastError());
  return GLE_OK;
}

// Composed one-launch step (STAGE 4): V0[t & 1], W1[t & 1] and the near partials of lags >= 3 for
// target t+2 from the two-launch path's state at step t (S(t), near partials of target t+1, the
// level blocks of target t+1); the caller's ladder_step has made the main stream wait for them.
// the composed stage's kernel: 5 (one-column VALU products) for one-trajectory plans, else 4 (C2:
// 20.6 vs 21.4 us/step, `profiles/r05/split/gemv_ab_c2.jsonl`)
int xstage(const gle_handle* h) { return h->B == 1 ? 5 : 4; }

int x_prime_buffers(gle_handle* h) {
  const StepArgs ta = step_args(h);
  for (auto& b : h->baths) {
    XPrimeArgs a{};
    a.noise = b.d_noise;
    a.S = b.ml > 1 ? b.d_S : nullptr;
    a.NP = b.nqn ? b.d_NP : nullptr;
    a.nqn = b.nqn;
    const int j = (int)(&b - h->baths.data());
    for (size_t l = 0; l < h->levels.size() && l < (size_t)MAXLVL; ++l) {
      const LevelBath& L = h->levels[l].lb[j];
      a.lvl[l] = L.active ? L.d_out : nullptr;
      a.lvl_ld[l] = 2 * h->levels[l].P * (int32_t)h->B;
      a.lvl_off[l] = ta.lvl_off[l];
    }
    a.V0 = b.d_V0;
    a.W1 = b.d_W1;
    a.c = b.c;
    a.vs = b.vs;
    a.t = h->t;
    a.nc = b.nc;
    a.B = (int32_t)h->B;
    a.nmd = (int32_t)h->nmd;
    launch_xprime(a, h->stream);
  }
  if (!h->chNear3.tiles.empty())
    launch_chain(xstage(h), h->chNear3.nw, h->ch_drn, h->chNear3.lds, h->chNear3.d, (int)h->chNear3.tiles.size(),
                 h->d_sd, step_args(h, h->t - 1), 0, h->stream);
  // audit words: zero, except that after a two-launch step the first composed launch audits that
  // step's id0 distance for step t (md.potforce's cache as the two-launch path left it: a distance in
  // (0, 1e-9) stops the composed run before it stores anything, and the two-launch path goes on)
  const size_t nl = (size_t)((h->B + 15) / 16) * h->x_rep;  // words of a slot
  HIPCHK(h, hipMemsetAsync(h->d_xw, 0, 3 * nl * sizeof(unsigned long long), h->stream));
  if (h->std_words_live)
    launch_xinject(h->d_pmax + (h->t & 1) * h->B, (int)h->B, h->d_xw + ((h->t + 2) % 3) * nl, h->stream);
  h->x_live = true;
  return GLE_OK;
}

int run_xstep(gle_handle* h, int64_t nsteps) {
  if (!h->state_set) return fail(h, GLE_ERR_STATE, "gle_set_state has not been called");
  bounds_table_sync();
  for (size_t j = 0; j < h->baths.size(); ++j)
    if (!h->baths[j].noise_set) return fail(h, GLE_ERR_STATE, "bath " + std::to_string(j) + " has no noise");
  if (nsteps == 0) return GLE_OK;
  int rc = 0;
  if (!h->x_live && h->std_stale) h->need_prime = true;  // e.g. new noise after composed steps
  if (h->need_prime) {
    h->x_live = false;
    rc = prime(h);
    if (rc) return rc;
    h->std_stale = false;
  }
  const size_t nst = (size_t)h->nphp * h->B * 8;
  if (h->t & 1) {  // step t reads state buffer t & 1
    HIPCHK(h, hipMemcpyAsync(h->d_P2, h->d_P, nst, hipMemcpyDeviceToDevice, h->stream));
    HIPCHK(h, hipMemcpyAsync(h->d_Q2, h->d_Q, nst, hipMemcpyDeviceToDevice, h->stream));
  }
  h->x_call_t0 = h->t;
  for (int64_t s = 0; s < nsteps; ++s) {
    rc = ladder_step(h, 1);
    if (rc) return rc;
    if (!h->x_live) {
      rc = x_prime_buffers(h);
      if (rc) return rc;
    }
    StepArgs ta = step_args(h);
    const StepArgs t2 = step_args(h, h->t + 1);  // the S tiles read the levels at target t+2
    for (int l = 0; l < MAXLVL; ++l) ta.lvl_off[l] = t2.lvl_off[l];
    ta.xw = h->d_xw;
    ta.xstop = h->d_xstop;
    ta.xstop_host = h->d_xstop_h;
    ta.xB = (int32_t)h->B;
    ta.xR = h->x_rep;
    ta.xndof = h->chX[h->t & 1].ndof;
    run_chain(h, xstage(h), h->chX[h->t & 1], ta, 0, h->levels.empty(), 0);
    h->std_stale = true;
    h->std_words_live = false;
    if (!h->levels.empty() && (h->t + 1) % h->P0 == 0) HIPCHK(h, hipEventRecord(h->ev_step, h->stream));
    h->t += 1;
  }
  // the audit of the last step (as launch t would), and the state into d_P / d_Q between calls unless
  // the run stopped (xresolve replays it)
  {
    XFinishArgs fa{};
    fa.P = h->d_P;
    fa.Q = h->d_Q;
    fa.P2 = h->d_P2;
    fa.Q2 = h->d_Q2;
    fa.n = (h->t & 1) ? (int64_t)h->nphp * h->B : 0;
    fa.xw = h->d_xw;
    fa.xstop = h->d_xstop;
    fa.xstop_host = h->d_xstop_h;
    fa.guard = h->d_guard;
    fa.t = h->t;
    fa.B = (int32_t)h->B;
    fa.R = h->x_rep;
    launch_xfinish(fa, h->stream);
  }
  h->x_pend = true;
  h->pot_cache_exact = false;
  HIPCHK(h, hipGetLastError());
  return GLE_OK;
}

// After a gle_run of composed steps (x_pend): wait for it and read the stop word.  A stopped run
// (a launch found that md.potforce would have reused its cached force at a point other than q0,
// md.py:449-450, 767-779) left the state of the step r before the stopping launch in its parity
// buffer and stored nothing after step r's launch; r's launch itself ran, but the step whose words
// tripped is r, so the run resumes at r on the two-launch path (which applies the cache rule) up to
// the step the caller asked for.  If the stop came from the first launch of the run auditing the
// two-launch path's own distance (x_prime_buffers), nothing composed ran: the run resumes at its
// first step with that path's potential cache as it was.
int xresolve(gle_handle* h) {
  if (!h->x_pend) return GLE_OK;
  h->x_pend = false;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  const unsigned long long v = *(volatile unsigned long long*)h->h_xstop;
  if (v == 0ull) return GLE_OK;
  const int64_t t_end = h->t;
  int64_t r = (int64_t)v - 2;
  const bool entry = r < h->x_call_t0;
  if (entry) r = h->x_call_t0;
  if (r < h->x_call_t0 || r >= t_end) return fail(h, GLE_ERR_STATE, "composed-step stop outside the run");
  const size_t nst = (size_t)h->nphp * h->B * 8;
  if (r & 1) {
    HIPCHK(h, hipMemcpyAsync(h->d_P, h->d_P2, nst, hipMemcpyDeviceToDevice, h->stream));
    HIPCHK(h, hipMemcpyAsync(h->d_Q, h->d_Q2, nst, hipMemcpyDeviceToDevice, h->stream));
  }
  HIPCHK(h, hipMemsetAsync(h->d_xstop, 0, sizeof(unsigned long long), h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  *(volatile unsigned long long*)h->h_xstop = 0ull;
  h->x_replays += 1;
  h->t = r;
  h->x_live = false;
  h->need_prime = true;   // the ladder's schedule and blocks ran ahead to t_end
  h->std_stale = !entry;  // composed steps ran: the two-launch path's cache starts empty at r
  for (int64_t s = r; s < t_end; ++s) {
    int rc = step_begin_impl(h, nullptr);
    if (!rc) rc = step_end_impl(h, nullptr);
    if (rc) return rc;
  }
  return GLE_OK;
}

// transpose host [B][n] <-> device layout [n][B] (row stride ld >= B)
void to_dev_layout(const double* src, std::vector<double>& dst, int64_t B, int64_t n, int64_t rows_alloc) {
  dst.assign((size_t)rows_alloc * B, 0.0);
  for (int64_t b = 0; b < B; ++b)
    for (int64_t i = 0; i < n; ++i) dst[(size_t)i * B + b] = src[(size_t)b * n + i];
}

void from_dev_layout(const std::vector<double>& src, double* dst, int64_t B, int64_t n) {
  for (int64_t b = 0; b < B; ++b)
    for (int64_t i = 0; i < n; ++i) dst[(size_t)b * n + i] = src[(size_t)i * B + b];
}

int download(gle_handle* h, void* dst, const void* src, size_t bytes) {
  HIPCHK(h, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return bounds_report(h);
}

}  // namespace

#ifdef GLE_BOUNDS
void gle::bounds_sync() { bounds_table_sync(); }
#endif

// every entry that reads or changes the state, the noise or the recordings first finishes a pending
// composed run (xresolve: a stopped run is replayed before anything sees the state)
#define XRESOLVE(h)                  \
  do {                               \
    const int xr_ = xresolve(h);     \
    if (xr_) return xr_;             \
  } while (0)

// =========================================================================================
extern "C" {

int gle_abi_version(void) { return GLE_ABI_VERSION; }

const char* gle_last_error(const gle_handle* h) {
  return h ? h->err.c_str() : g_create_error.c_str();
}

int gle_device_mem_info(int32_t device, int64_t* free_bytes, int64_t* total_bytes) {
  if (!free_bytes || !total_bytes) return fail(nullptr, GLE_ERR_ARG, "null argument");
  // the caller's current device (e.g. torch's) is restored on every return path
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  if (hipSetDevice(device) != hipSuccess) {
    if (prev >= 0) (void)hipSetDevice(prev);
    return fail(nullptr, GLE_ERR_HIP, "gle_device_mem_info: no such device");
  }
  size_t fr = 0, tot = 0;
  const hipError_t e = hipMemGetInfo(&fr, &tot);
  if (prev >= 0) (void)hipSetDevice(prev);
  if (e != hipSuccess) return fail(nullptr, GLE_ERR_HIP, std::string("hipMemGetInfo: ") + hipGetErrorString(e));
  *free_bytes = (int64_t)fr;
  *total_bytes = (int64_t)tot;
  return GLE_OK;
}

int gle_device_count(int32_t* count) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    g_create_error = std::string("hipGetDeviceCount: ") + hipGetErrorString(e);
    if (count) *count = 0;
    return GLE_ERR_HIP;
  }
  if (count) *count = n;
  return GLE_OK;
}

int gle_create(const gle_config* cfg, gle_handle** out) {
  if (!cfg || !out) return fail(nullptr, GLE_ERR_ARG, "null argument");
  *out = nullptr;
  if (cfg->nph <= 0 || cfg->ntraj <= 0 || cfg->nmd <= 0 || !(cfg->dt > 0))
    return fail(nullptr, GLE_ERR_ARG, "nph, ntraj, nmd must be > 0 and dt > 0");
  if (cfg->nmd % 2) return fail(nullptr, GLE_ERR_ARG, "nmd must be even (functions.py:47-50 length check)");
  if (cfg->far_mode < GLE_FAR_AUTO || cfg->far_mode > GLE_FAR_SPECTRAL) return fail(nullptr, GLE_ERR_ARG, "bad far_mode");
  if (cfg->block_len < 0 || cfg->block_len > 4096) return fail(nullptr, GLE_ERR_ARG, "bad block_len");
  if (cfg->max_block < 0 || cfg->max_block > 4096) return fail(nullptr, GLE_ERR_ARG, "bad max_block");
  if (cfg->nph > (1 << 24) || cfg->ntraj > (1 << 20)) return fail(nullptr, GLE_ERR_UNSUP, "size too large");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0)
    return fail(nullptr, GLE_ERR_HIP, std::string("no HIP device: ") + (e != hipSuccess ? hipGetErrorString(e) : "count 0"));
  if (cfg->device < 0 || cfg->device >= ndev) return fail(nullptr, GLE_ERR_ARG, "bad device ordinal");
  e = hipSetDevice(cfg->device);
  if (e != hipSuccess) return fail(nullptr, GLE_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
  gle_handle* h = new gle_handle();
  h->cfg = *cfg;
  h->nph = cfg->nph;
  h->B = cfg->ntraj;
  h->nmd = cfg->nmd;
  h->dt = cfg->dt;
  h->nphp = rup(h->nph, 8);
  h->dbg_no_ladder = gle_env("GLE_DBG_NO_LADDER") != nullptr;
  if (const char* e = gle_env("GLE_EXP_ONE")) h->exp_one = std::max(0, atoi(e));
  if (const char* e = gle_env("GLE_FAR_AFRAC")) h->far_afrac = std::max(0.0, std::min(1.0, atof(e)));
  if (const char* e = gle_env("GLE_DBG_SKIP")) h->dbg_skip = atoi(e);
  h->dbg_no_chain = gle_env("GLE_DBG_NO_CHAIN") != nullptr;
  if (const char* e = gle_env("GLE_BG_GRID")) h->bg_grid = std::max(0, atoi(e));
  if (const char* e = gle_env("GLE_PIECE_SLACK")) h->piece_slack_env = std::max(0, atoi(e));
  if (const char* e = gle_env("GLE_BG_SERIAL")) h->bg_serial = atoi(e) != 0;
  if (const char* e = gle_env("GLE_MERGE_WAITS")) h->merge_waits = atoi(e) != 0;
  if (const char* e = gle_env("GLE_WAIT_EARLY")) h->wait_early = std::max(0, atoi(e));
  // main stream (the latency-bound per-step chain) at the highest priority, background streams
  // (ladder blocks) at the lowest
  {
    int lo = 0, hi = 0;
    hipDeviceGetStreamPriorityRange(&lo, &hi);
    // GLE_BG_RESERVE=R: the background streams stay off CU mask bits [0, R), which the per-step
    // chain then finds free at every launch
    int reserve = 0;
    if (const char* r = gle_env("GLE_BG_RESERVE")) reserve = std::max(0, atoi(r));
    // GLE_CU_SPLIT=N (experiment): the background streams on N CUs spread evenly over the mask, the
    // main stream (GLE_CU_SPLIT_MAIN=1, default) on the other ones -- disjoint CU sets
    int split = 0;
    if (const char* r = gle_env("GLE_CU_SPLIT")) split = std::max(0, atoi(r));
    const char* split_main = gle_env("GLE_CU_SPLIT_MAIN");
    // GLE_QUEUE_MODE (experiment): 1 background streams on full-CU-mask streams (dedicated hardware
    // queues outside the per-priority pools), 2 the main stream too
    int qmode = 0;
    if (const char* r = gle_env("GLE_QUEUE_MODE")) qmode = atoi(r);
    std::vector<uint32_t> cumask, mainmask;
    if (qmode > 0 && reserve == 0 && split == 0) {
      hipDeviceProp_t prop;
      hipGetDeviceProperties(&prop, cfg->device);
      const int ncu = prop.multiProcessorCount;
      cumask.assign((ncu + 31) / 32, 0u);
      for (int c = 0; c < ncu; ++c) cumask[c / 32] |= 1u << (c % 32);
      mainmask = cumask;
      if (qmode > 1) split = -1;  // main on the full mask (below)
      reserve = 1;                // background on the full mask (below)
    }
    if (qmode == 0 && (reserve > 0 || split > 0)) {
      hipDeviceProp_t prop;
      hipGetDeviceProperties(&prop, cfg->device);
      const int ncu = prop.multiProcessorCount;
      cumask.assign((ncu + 31) / 32, 0u);
      mainmask.assign((ncu + 31) / 32, 0u);
      if (split > 0) {
        split = std::min(split, ncu - 8);
        for (int c = 0; c < ncu; ++c) {
          const bool far = (int64_t)(c + 1) * split / ncu > (int64_t)c * split / ncu;
          (far ? cumask : mainmask)[c / 32] |= 1u << (c % 32);
        }
      } else {
        for (int c = std::min(reserve, ncu - 8); c < ncu; ++c) cumask[c / 32] |= 1u << (c % 32);
      }
    }
    if ((split > 0 && !(split_main && atoi(split_main) == 0)) || split < 0)
      e = hipExtStreamCreateWithCUMask(&h->stream, (uint32_t)mainmask.size(), mainmask.data());
    else
      e = hipStreamCreateWithPriority(&h->stream, hipStreamNonBlocking, hi);
    reserve = reserve > 0 || split != 0;
    for (int i = 0; i < gle_handle::NBG && e == hipSuccess; ++i) {
      if (reserve > 0)
        e = hipExtStreamCreateWithCUMask(&h->bg[i], (uint32_t)cumask.size(), cumask.data());
      else
        e = hipStreamCreateWithPriority(&h->bg[i], hipStreamNonBlocking, gle_env("GLE_BG_SAMEPRIO") ? hi : lo);
      if (e == hipSuccess)
        e = hipEventCreateWithFlags(&h->ev_bg[i], hipEventDisableTiming | hipEventReleaseToDevice);
    }
  }
  if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_step, hipEventDisableTiming | hipEventReleaseToDevice);
  if (e != hipSuccess) {
    gle_destroy(h);
    return fail(nullptr, GLE_ERR_HIP, std::string("stream/event creation: ") + hipGetErrorString(e));
  }
  const size_t nst = (size_t)h->nphp * h->B, nsl = (size_t)64 * h->B + 1024;  // row slack for static windows
  int rc = 0;
  rc |= dalloc_n(h, &h->d_P, nst, nsl);
  rc |= dalloc_n(h, &h->d_Q, nst, nsl);
  rc |= dalloc_n(h, &h->d_Ph, nst, nsl);
  rc |= dalloc_n(h, &h->d_Qt, nst, nsl);
  rc |= dalloc_n(h, &h->d_Fc, nst, nsl);
  rc |= dalloc_n(h, &h->d_Flast, nst, nsl);
  rc |= dalloc_n(h, &h->d_Q0, nst, nsl);
  rc |= dalloc_n(h, &h->d_etot, (size_t)h->nmd * h->B);
  rc |= dalloc_n(h, &h->d_qvalid, (size_t)h->B);
  if (rc) {
    g_create_error = h->err;
    gle_destroy(h);
    return GLE_ERR_NOMEM;
  }
  // twiddles exp(-2 pi i k / nmd), k < nmd/2 (long double for accuracy)
  {
    std::vector<double> tw((size_t)h->nmd);
    for (int64_t k = 0; k < h->nmd / 2; ++k) {
      const long double ang = -2.0L * 3.14159265358979323846264338327950288L * (long double)k / (long double)h->nmd;
      tw[2 * k] = (double)cosl(ang);
      tw[2 * k + 1] = (double)sinl(ang);
    }
    rc = dalloc_n(h, &h->d_tw, (size_t)h->nmd);
    if (!rc) rc = upload(h, h->d_tw, tw.data(), tw.size() * 8);
    if (rc) {
      g_create_error = h->err;
      gle_destroy(h);
      return rc;
    }
  }
  *out = h;
  return GLE_OK;
}

// GLE_CHAIN_DBG: per-stage timeline of the recorded step's chain launches (stderr)
static void dump_chain_dbg(gle_handle* h) {
  const int n = h->dbg_ntile;
  std::vector<unsigned long long> st((size_t)3 * n * 4);
  if (hipMemcpy(st.data(), h->d_dbg, st.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
  const char* kn[3] = {"DOF", "SFIN", "RAW"};
  for (int g = 0; g < 3; ++g) {
    const Chain& c = g == 0 ? h->chA[h->dbg_a]
                            : (g == 1 ? h->chB[1] : (h->xstep ? h->chX[h->dbg_t & 1] : (h->fuse_bc ? h->chBC : h->chC)));
    unsigned long long t0 = ~0ull, t1 = 0;
    for (size_t i = 0; i < c.tiles.size(); ++i) {
      const unsigned long long* r = &st[((size_t)g * n + i) * 4];
      if (r[0]) t0 = std::min(t0, r[0]);
      t1 = std::max(t1, r[3]);
    }
    if (t0 == ~0ull) continue;
    fprintf(stderr, "[chain dbg] stage %c: %zu tiles, span %.2f us\n", "ABC"[g], c.tiles.size(), (t1 - t0) / 100.0);
    for (int k = 0; k < 3; ++k) {
      std::vector<double> v[5];
      for (size_t i = 0; i < c.tiles.size(); ++i) {
        if (c.tiles[i].kind != k) continue;
        const unsigned long long* r = &st[((size_t)g * n + i) * 4];
        if (!r[0] || !r[3]) continue;
        v[0].push_back((r[0] - t0) / 100.0);
        v[1].push_back((r[1] - r[0]) / 100.0);
        v[2].push_back((r[2] - r[1]) / 100.0);
        v[3].push_back((r[3] - r[2]) / 100.0);
        v[4].push_back((r[3] - t0) / 100.0);
      }
      if (v[0].empty()) continue;
      const char* nm[5] = {"start", "desc", "prod", "epi", "end"};
      fprintf(stderr, "[chain dbg]   %-4s n %4zu", kn[k], v[0].size());
      for (int q = 0; q < 5; ++q) {
        std::sort(v[q].begin(), v[q].end());
        fprintf(stderr, "  %s %.2f/%.2f/%.2f", nm[q], v[q][v[q].size() / 2], v[q][v[q].size() * 9 / 10], v[q].back());
      }
      fprintf(stderr, "\n");
    }
  }
}

int gle_destroy(gle_handle* h) {
  if (!h) return GLE_OK;
  hipSetDevice(h->cfg.device);
  if (h->d_dbg) {
    hipDeviceSynchronize();
    dump_chain_dbg(h);
  }
  for (int i = 0; i < gle_handle::NBG; ++i)
    if (h->bg[i]) hipStreamSynchronize(h->bg[i]);
  if (h->stream) hipStreamSynchronize(h->stream);
  // streamed-noise scratch (tmalloc, not in allocs) of a stream that was begun and never ended
  for (int j = 0; j < (int)h->baths.size(); ++j) {
    gle_noise_stream_abort(h, j);
    free_retained(h->baths[j], h->stream);
  }
  for (void* p : h->allocs) {
    bounds_del(p);
    hipFree(p);
  }
  if (h->h_xstop) hipHostFree(h->h_xstop);
  for (auto e : h->ev) hipEventDestroy(e);
  for (auto& lv : h->levels)
    for (auto e : lv.ev)
      if (e) hipEventDestroy(e);
  if (h->ev_step) hipEventDestroy(h->ev_step);
  for (int i = 0; i < gle_handle::NBG; ++i) {
    if (h->ev_bg[i]) hipEventDestroy(h->ev_bg[i]);
    if (h->bg[i]) hipStreamDestroy(h->bg[i]);
  }
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
  return GLE_OK;
}

}  // extern "C"

namespace {

// shared argument checks of gle_add_bath / gle_add_bath_gmem; fills the bath's shape fields
int new_bath(gle_handle* h, int32_t kind, const int64_t* cids, int64_t nc, int64_t ml, Bath& b) {
  if (h->frozen) return fail(h, GLE_ERR_STATE, "baths must be added before the first state/step call");
  if ((int)h->baths.size() >= MAXBATH) return fail(h, GLE_ERR_UNSUP, "too many baths");
  if (kind != GLE_BATH_PHONON && kind != GLE_BATH_ELECTRON) return fail(h, GLE_ERR_ARG, "bad bath kind");
  if (!cids || nc <= 0 || nc > h->nph || ml <= 0) return fail(h, GLE_ERR_ARG, "bad bath shape");
  if (kind == GLE_BATH_ELECTRON && ml != 1) return fail(h, GLE_ERR_ARG, "electron bath is time-local (ml == 1, baths.py:97)");
  std::vector<int> seen(h->nph, 0);
  for (int64_t k = 0; k < nc; ++k) {
    if (cids[k] < 0 || cids[k] >= h->nph) return fail(h, GLE_ERR_ARG, "cids out of range");
    if (seen[cids[k]]++) return fail(h, GLE_ERR_ARG, "duplicate DOF in cids");
  }
  hipSetDevice(h->cfg.device);
  b.kind = kind;
  b.nc = (int)nc;
  b.ncp = (int)rup(nc, 8);
  b.nrt = (int)((nc + 15) / 16);
  b.nks = b.ncp / 4;
  b.ml = (int)ml;
  b.c = ml > 1 ? h->dt : 1.0;  // baths.py:454-457 (and :235-241)
  b.cids.assign(cids, cids + nc);
  return GLE_OK;
}

// per-bath device buffers and the DOF map; b.d_K and b.K0 are already set
int commit_bath(gle_handle* h, Bath&& b, int32_t* bath_id) {
  const int64_t nc = b.nc;
  const int64_t* cids = b.cids.data();
  int rc = 0;
  b.inv.assign(h->nph, -1);
  for (int64_t k = 0; k < nc; ++k) b.inv[cids[k]] = (int32_t)k;
  const int64_t B = h->B;
  const size_t nbuf = (size_t)(b.ncp + 64) * B + 1024;
  b.vs = (int64_t)nbuf;
  rc |= dalloc_n(h, &b.d_inv, (size_t)h->nph);
  if (!rc) rc = upload(h, b.d_inv, b.inv.data(), b.inv.size() * 4);
  // exact size: the fused stage reads noise(t+1) as an MFMA operand of ncp rows (K0 columns past nc
  // are zero), its tasks clamp the rows past nc to row nc - 1 (ChTask::xrows, GLE_BOUNDS-audited)
  rc |= dalloc_n(h, &b.d_noise, (size_t)h->nmd * nc * B);
  rc |= dalloc_n(h, &b.d_S, 2 * nbuf);
  rc |= dalloc_n(h, &b.d_Xcur, 2 * nbuf);
  rc |= dalloc_n(h, &b.d_Xq, 2 * nbuf);
  rc |= dalloc_n(h, &b.d_cur, (size_t)h->nmd * B);
  if (b.has_q) rc |= dalloc_n(h, &b.d_Yq, nbuf);
  if (rc) return GLE_ERR_NOMEM;
  h->baths.push_back(std::move(b));
  if (bath_id) *bath_id = (int32_t)h->baths.size() - 1;
  return GLE_OK;
}

// W [ml][ngw] -> W^T zero padded to [rup(ngw, 4)][rup(ml, 16)]
std::vector<double> transpose_w(const double* W, int64_t ml, int64_t ngw, int64_t* mlp) {
  *mlp = rup(ml, 16);
  const int64_t ngwp = rup(ngw, 4);
  std::vector<double> wt((size_t)ngwp * *mlp, 0.0);
  for (int64_t i = 0; i < ml; ++i)
    for (int64_t g = 0; g < ngw; ++g) wt[(size_t)(g * *mlp + i)] = W[i * ngw + g];
  return wt;
}

struct DevTmp {  // scratch device buffer freed on scope exit (setup paths)
  void* p = nullptr;
  ~DevTmp() {
    if (p) tfree(p);
  }
};

}  // namespace

extern "C" {

int gle_add_bath(gle_handle* h, int32_t kind, const int64_t* cids, int64_t nc, int64_t ml,
                 const double* kernel, double bias, const double* exim, const double* zeta1,
                 const double* zeta2, int32_t* bath_id) {
  if (!h) return GLE_ERR_ARG;
  if (!kernel) return fail(h, GLE_ERR_ARG, "bad bath shape");
  Bath b;
  int rc0 = new_bath(h, kind, cids, nc, ml, b);
  if (rc0) return rc0;
  b.K.assign(kernel, kernel + ml * nc * nc);
  // electron-bath bias terms, active only if exim, zeta1, zeta2 are all nonzero (baths.py:233)
  auto anynz = [&](const double* m) {
    if (!m) return false;
    for (int64_t i = 0; i < nc * nc; ++i)
      if (m[i] != 0.0) return true;
    return false;
  };
  if (kind == GLE_BATH_ELECTRON && anynz(exim) && anynz(zeta1) && anynz(zeta2)) {
    b.has_q = true;
    b.Kq.assign((size_t)nc * nc, 0.0);
    for (int64_t i = 0; i < nc * nc; ++i) {
      b.K[i] += bias * zeta2[i];                     //  - V zeta2 . p   (baths.py:248-249)
      b.Kq[i] = -(bias * exim[i] - bias * zeta1[i]);  // + V exim . q - V zeta1 . q (:246-247)
    }
  }
  int rc = 0;
  {
    std::vector<double> f = pack_frags(b.K.data(), ml, nc, nc, b.nrt, b.nks);
    rc = dalloc_n(h, &b.d_K, f.size());
    if (!rc) rc = upload(h, b.d_K, f.data(), f.size() * 8);
    if (rc) return rc;
    if (b.has_q) {
      std::vector<double> fq = pack_frags(b.Kq.data(), 1, nc, nc, b.nrt, b.nks);
      rc = dalloc_n(h, &b.d_Kq, fq.size());
      if (!rc) rc = upload(h, b.d_Kq, fq.data(), fq.size() * 8);
      if (rc) return rc;
    }
  }
  b.K0.assign(b.K.begin(), b.K.begin() + nc * nc);
  b.K.clear();
  b.K.shrink_to_fit();
  return commit_bath(h, std::move(b), bath_id);
}

int gle_add_bath_gmem(gle_handle* h, const int64_t* cids, int64_t nc, int64_t ml, const double* W,
                      int64_t ngw, const double* gamma, int32_t* bath_id) {
  if (!h) return GLE_ERR_ARG;
  if (!W || !gamma || ngw <= 0) return fail(h, GLE_ERR_ARG, "gmem: bad coefficient / spectrum shape");
  Bath b;
  int rc = new_bath(h, GLE_BATH_PHONON, cids, nc, ml, b);
  if (rc) return rc;
  const int64_t nfrag = (int64_t)b.nrt * b.nks;
  const int64_t ngwp = rup(ngw, 4);
  int64_t mlp = 0;
  std::vector<double> wt = transpose_w(W, ml, ngw, &mlp);
  DevTmp d_wt, d_gam, d_gf;
  HIPCHK(h, tmalloc(&d_wt.p, wt.size() * 8));
  HIPCHK(h, tmalloc(&d_gam.p, (size_t)ngw * nc * nc * 8));
  HIPCHK(h, tmalloc(&d_gf.p, (size_t)nfrag * ngwp * 64 * 8));
  HIPCHK(h, hipMemcpyAsync(d_wt.p, wt.data(), wt.size() * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(d_gam.p, gamma, (size_t)ngw * nc * nc * 8, hipMemcpyHostToDevice, h->stream));
  launch_gamma_pack((const double*)d_gam.p, (int)ngw, (int)ngwp, b.nc, b.nrt, b.nks, (double*)d_gf.p, h->stream);
  rc = dalloc_n(h, &b.d_K, (size_t)nfrag * ml * 64);
  if (rc) return rc;
  if (launch_kgen((const double*)d_wt.p, mlp, (int)ngw, (const double*)d_gf.p, ngwp * 64, 64, b.d_K, ml * 64, 64,
                  (int)ml, nfrag, 64, h->stream))
    return fail(h, GLE_ERR_HIP, "gmem: kernel-construction launch failed");
  // host copy of slice 0 (the chain's K0 rows are packed on the host in plan_chain)
  std::vector<double> f0((size_t)nfrag * 64);
  HIPCHK(h, hipMemcpy2DAsync(f0.data(), 64 * 8, b.d_K, (size_t)ml * 64 * 8, 64 * 8, (size_t)nfrag,
                             hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  b.K0.assign((size_t)nc * nc, 0.0);
  for (int rt = 0; rt < b.nrt; ++rt)
    for (int ks = 0; ks < b.nks; ++ks)
      for (int l = 0; l < 64; ++l) {
        const int64_t r = 16 * rt + (l & 15), c = 4 * ks + (l >> 4);
        if (r < nc && c < nc) b.K0[(size_t)(r * nc + c)] = f0[((size_t)rt * b.nks + ks) * 64 + l];
      }
  return commit_bath(h, std::move(b), bath_id);
}

int gle_get_kernel(gle_handle* h, int32_t bath, int64_t i0, int64_t n, double* out) {
  if (!h || !out) return GLE_ERR_ARG;
  if (bath < 0 || bath >= (int32_t)h->baths.size()) return fail(h, GLE_ERR_ARG, "bad bath id");
  const Bath& b = h->baths[bath];
  if (i0 < 0 || n < 0 || i0 + n > b.ml) return fail(h, GLE_ERR_ARG, "kernel slice range out of [0, ml)");
  if (n == 0) return GLE_OK;
  hipSetDevice(h->cfg.device);
  const int64_t nfrag = (int64_t)b.nrt * b.nks;
  std::vector<double> f((size_t)nfrag * n * 64);
  HIPCHK(h, hipMemcpy2DAsync(f.data(), (size_t)n * 64 * 8, b.d_K + i0 * 64, (size_t)b.ml * 64 * 8,
                             (size_t)n * 64 * 8, (size_t)nfrag, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  const int64_t nc = b.nc;
  for (int rt = 0; rt < b.nrt; ++rt)
    for (int ks = 0; ks < b.nks; ++ks)
      for (int64_t i = 0; i < n; ++i) {
        const double* src = &f[(((size_t)rt * b.nks + ks) * n + i) * 64];
        for (int l = 0; l < 64; ++l) {
          const int64_t r = 16 * rt + (l & 15), c = 4 * ks + (l >> 4);
          if (r < nc && c < nc) out[(i * nc + r) * nc + c] = src[l];
        }
      }
  return GLE_OK;
}

int gle_gamt(int32_t device, int64_t ml, int64_t ngw, int64_t nel, const double* W, const double* G,
             double* out) {
  if (ml <= 0 || ngw <= 0 || nel <= 0 || !W || !G || !out) return fail(nullptr, GLE_ERR_ARG, "gamt: bad shape");
  if (hipSetDevice(device) != hipSuccess) return fail(nullptr, GLE_ERR_HIP, "gamt: no such device");
  int64_t mlp = 0;
  std::vector<double> wt = transpose_w(W, ml, ngw, &mlp);
  const int64_t nblk = (nel + 63) / 64;
  DevTmp d_wt, d_g, d_o;
  auto ok = [](hipError_t e) { return e == hipSuccess; };
  if (!ok(tmalloc(&d_wt.p, wt.size() * 8)) || !ok(tmalloc(&d_g.p, (size_t)ngw * nel * 8)) ||
      !ok(tmalloc(&d_o.p, (size_t)ml * nel * 8)))
    return fail(nullptr, GLE_ERR_NOMEM, "gamt: device allocation failed");
  if (!ok(hipMemcpy(d_wt.p, wt.data(), wt.size() * 8, hipMemcpyHostToDevice)) ||
      !ok(hipMemcpy(d_g.p, G, (size_t)ngw * nel * 8, hipMemcpyHostToDevice)))
    return fail(nullptr, GLE_ERR_HIP, "gamt: upload failed");
  if (launch_kgen((const double*)d_wt.p, mlp, (int)ngw, (const double*)d_g.p, 64, nel, (double*)d_o.p, 64, nel,
                  (int)ml, nblk, (int)(nel - 64 * (nblk - 1)), nullptr))
    return fail(nullptr, GLE_ERR_HIP, "gamt: launch failed");
  if (!ok(hipMemcpy(out, d_o.p, (size_t)ml * nel * 8, hipMemcpyDeviceToHost)))
    return fail(nullptr, GLE_ERR_HIP, "gamt: download failed");
  return GLE_OK;
}

int gle_set_dyn(gle_handle* h, const double* dyn) {
  if (!h || !dyn) return GLE_ERR_ARG;
  if (h->frozen) return fail(h, GLE_ERR_STATE, "dyn must be set before the first state/step call");
  hipSetDevice(h->cfg.device);
  h->dyn_nrt = (int)((h->nph + 15) / 16);
  h->dyn_nks = (int)(h->nphp / 4);
  // md.setDyn stores U diag(w^2) U^T (md.py:264-292): its eigen-reconstruction leaves roundoff
  // (<= ~10 eps of the row's largest entry at C3 / C5) in every entry the dynamical matrix does not
  // couple, so the block-sparse device copy would turn dense.  Entries at or below DYN_DROP_EPS
  // unit roundoffs of the larger of their two rows' largest magnitudes are dropped, d_ij and d_ji
  // together (the pattern stays symmetric): per row the dropped part is at most
  // nph * 16 eps * max(max|d_i.|, max|d_j.|) * max|q|, the order of the dense product's own
  // rounding bound.  The count is reported by gle_plan_detail.
  constexpr double DYN_DROP_EPS = 16.0;
  const int64_t n = h->nph;
  h->dyn_h.assign(dyn, dyn + n * n);
  h->dyn_dropped = 0;
  std::vector<double> rmax(n, 0.0);
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = 0; j < n; ++j) rmax[i] = std::max(rmax[i], std::fabs(h->dyn_h[(size_t)(i * n + j)]));
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = i; j < n; ++j) {
      double& a = h->dyn_h[(size_t)(i * n + j)];
      double& b = h->dyn_h[(size_t)(j * n + i)];
      if (a == 0.0 && b == 0.0) continue;
      const double thr = DYN_DROP_EPS * 0x1p-52 * std::max(rmax[i], rmax[j]);
      if (std::max(std::fabs(a), std::fabs(b)) > thr) continue;
      h->dyn_dropped += (a != 0.0) + (i != j && b != 0.0);
      a = 0.0;
      b = 0.0;
    }
  std::vector<double> f = pack_frags(h->dyn_h.data(), 1, h->nph, h->nph, h->dyn_nrt, h->dyn_nks);
  int rc = dalloc_n(h, &h->d_dyn, f.size());
  if (!rc) rc = upload(h, h->d_dyn, f.data(), f.size() * 8);
  if (rc) return rc;
  h->has_dyn = true;
  return GLE_OK;
}

int gle_set_constraint(gle_handle* h, const int64_t* dofs, int64_t n) {
  if (!h || (n > 0 && !dofs) || n < 0) return GLE_ERR_ARG;
  if (h->frozen) return fail(h, GLE_ERR_STATE, "constraints must be set before the first state/step call");
  for (int64_t i = 0; i < n; ++i)  // a rejected call leaves the previous constraints in place
    if (dofs[i] < 0 || dofs[i] >= h->nph) return fail(h, GLE_ERR_ARG, "constraint DOF out of range");
  h->constr.assign(dofs, dofs + n);
  return GLE_OK;
}

int gle_set_state(gle_handle* h, const double* p, const double* q, int64_t t) {
  if (!h || !p || !q) return GLE_ERR_ARG;
  if (t < 0) return fail(h, GLE_ERR_ARG, "t must be >= 0");
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  int rc = freeze(h);
  if (rc) return rc;
  rc = sync_bg(h);  // background blocks read the ring rewritten here
  if (rc) return rc;
  const int64_t B = h->B, n = h->nph;
  std::vector<double> tp, tq;
  to_dev_layout(p, tp, B, n, n);
  to_dev_layout(q, tq, B, n, n);
  rc = upload(h, h->d_P, tp.data(), tp.size() * 8);
  if (!rc) rc = upload(h, h->d_Q, tq.data(), tq.size() * 8);
  if (rc) return rc;
  h->t = t;
  HIPCHK(h, hipMemsetAsync(h->d_qvalid, 0, (size_t)B * 4, h->stream));
  HIPCHK(h, hipMemsetAsync(h->d_pmax, 0, (size_t)B * 4 * 8, h->stream));
  // p_t into the history ring slot of t; q_t into the q gather
  for (auto& b : h->baths) {
    std::vector<double> col((size_t)b.nc * B), colq((size_t)b.ncp * B, 0.0);
    for (int64_t k = 0; k < b.nc; ++k)
      for (int64_t j = 0; j < B; ++j) {
        col[(size_t)k * B + j] = p[(size_t)j * n + b.cids[k]];
        colq[(size_t)k * B + j] = q[(size_t)j * n + b.cids[k]];
      }
    double* d_tmp = nullptr;
    HIPCHK(h, tmalloc((void**)&d_tmp, col.size() * 8));
    hipMemcpyAsync(d_tmp, col.data(), col.size() * 8, hipMemcpyHostToDevice, h->stream);
    launch_ring_copy(b.d_H, b.ldh, b.R, (int)B, b.nc, t, 1, d_tmp, 0, h->stream);
    hipMemcpyAsync(b.d_Xq, colq.data(), colq.size() * 8, hipMemcpyHostToDevice, h->stream);
    hipError_t e = hipStreamSynchronize(h->stream);
    tfree(d_tmp);
    if (e != hipSuccess) return fail(h, GLE_ERR_HIP, std::string("set_state: ") + hipGetErrorString(e));
  }
  h->state_set = true;
  h->need_prime = true;
  h->pot_cache_exact = false;
  return GLE_OK;
}

int gle_get_state(gle_handle* h, double* p, double* q, int64_t* t) {
  if (!h) return GLE_ERR_ARG;
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  const int64_t B = h->B, n = h->nph;
  std::vector<double> buf((size_t)n * B);
  if (p) {
    int rc = download(h, buf.data(), h->d_P, buf.size() * 8);
    if (rc) return rc;
    from_dev_layout(buf, p, B, n);
  }
  if (q) {
    int rc = download(h, buf.data(), h->d_Q, buf.size() * 8);
    if (rc) return rc;
    from_dev_layout(buf, q, B, n);
  }
  if (t) *t = h->t;
  return GLE_OK;
}

int gle_set_history(gle_handle* h, int32_t bath, const double* phis) {
  int rc = check_bath(h, bath);
  if (rc) return rc;
  if (!h->state_set) return fail(h, GLE_ERR_STATE, "call gle_set_state first (history slots are relative to t)");
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  rc = sync_bg(h);  // background blocks read the ring rewritten here
  if (rc) return rc;
  Bath& b = h->baths[bath];
  const int64_t B = h->B;
  // phis[i] (newest first) is p at time t-1-i (md.phis between steps, md.py:386-387)
  double* d_tmp = nullptr;
  if (phis) {
    std::vector<double> buf((size_t)b.ml * b.nc * B);
    for (int64_t j = 0; j < B; ++j)
      for (int64_t i = 0; i < b.ml; ++i)
        for (int64_t k = 0; k < b.nc; ++k)
          buf[((size_t)i * b.nc + k) * B + j] = phis[((size_t)j * b.ml + i) * b.nc + k];
    HIPCHK(h, tmalloc((void**)&d_tmp, buf.size() * 8));
    hipMemcpyAsync(d_tmp, buf.data(), buf.size() * 8, hipMemcpyHostToDevice, h->stream);
    launch_ring_copy(b.d_H, b.ldh, b.R, (int)B, b.nc, h->t - 1, b.ml, d_tmp, 0, h->stream);
    hipError_t e = hipStreamSynchronize(h->stream);
    tfree(d_tmp);
    if (e != hipSuccess) return fail(h, GLE_ERR_HIP, std::string("set_history: ") + hipGetErrorString(e));
  } else {
    launch_ring_copy(b.d_H, b.ldh, b.R, (int)B, b.nc, h->t - 1, b.ml, nullptr, 0, h->stream);
    HIPCHK(h, hipStreamSynchronize(h->stream));
  }
  h->need_prime = true;
  return GLE_OK;
}

// Trajectory-major copy of a ring into host memory, in chunks of trajectories through a device
// buffer of at most ~256 MB (C5's histories are GBs beside ~280 GB of resident plan): the transpose
// runs on the device, each chunk lands in its place in the caller's array.
static int hist_to_host(gle_handle* h, const double* src, int64_t ks, int64_t ss, int R, int64_t tau0, int nt,
                        int nk, double* out) {
  const int64_t per = (int64_t)nt * nk;
  if (per <= 0) return GLE_OK;
  const int64_t nbc = std::max<int64_t>(1, std::min<int64_t>(h->B, (256ll << 20) / (per * 8)));
  double* d_tmp = nullptr;
  HIPCHK(h, tmalloc((void**)&d_tmp, (size_t)(nbc * per * 8)));
  hipError_t e = hipSuccess;
  for (int64_t b0 = 0; b0 < h->B && e == hipSuccess; b0 += nbc) {
    const int nb = (int)std::min<int64_t>(nbc, h->B - b0);
    launch_hist_out(src, ks, ss, R, tau0, nt, nk, (int)b0, nb, d_tmp, h->stream);
    e = hipMemcpyAsync(out + b0 * per, d_tmp, (size_t)nb * per * 8, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  }
  tfree(d_tmp);
  if (e != hipSuccess) return fail(h, GLE_ERR_HIP, std::string("history copy: ") + hipGetErrorString(e));
  return GLE_OK;
}

int gle_get_history(gle_handle* h, int32_t bath, double* phis) {
  int rc = check_bath(h, bath);
  if (rc) return rc;
  if (!phis) return fail(h, GLE_ERR_ARG, "null output");
  if (!h->frozen) return fail(h, GLE_ERR_STATE, "no state yet");
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  Bath& b = h->baths[bath];
  // row i (newest first) = time t-1-i of the ring (both mirror copies hold it)
  return hist_to_host(h, b.d_H, b.ldh, h->B, b.R, h->t - 1, b.ml, b.nc, phis);
}

int gle_get_force(gle_handle* h, double* f) {
  if (!h || !f) return GLE_ERR_ARG;
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  std::vector<double> buf((size_t)h->nph * h->B);
  int rc = download(h, buf.data(), h->d_Flast, buf.size() * 8);
  if (rc) return rc;
  from_dev_layout(buf, f, h->B, h->nph);
  return GLE_OK;
}

int gle_set_noise(gle_handle* h, int32_t bath, const double* noise) {
  int rc = check_bath(h, bath);
  if (rc) return rc;
  if (!noise) return fail(h, GLE_ERR_ARG, "null noise");
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  Bath& b = h->baths[bath];
  const int64_t B = h->B, nmd = h->nmd, nc = b.nc;
  std::vector<double> buf((size_t)nmd * nc * B);
  for (int64_t j = 0; j < B; ++j)
    for (int64_t t = 0; t < nmd; ++t)
      for (int64_t k = 0; k < nc; ++k) buf[((size_t)t * nc + k) * B + j] = noise[((size_t)j * nmd + t) * nc + k];
  rc = upload(h, b.d_noise, buf.data(), buf.size() * 8);
  if (rc) return rc;
  b.noise_set = true;
  h->x_live = false;  // V0 / W1 carry the noise
  return GLE_OK;
}

int gle_get_noise(gle_handle* h, int32_t bath, double* noise) {
  int rc = check_bath(h, bath);
  if (rc) return rc;
  if (!noise) return fail(h, GLE_ERR_ARG, "null output");
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  Bath& b = h->baths[bath];
  const int64_t B = h->B, nmd = h->nmd, nc = b.nc;
  std::vector<double> buf((size_t)nmd * nc * B);
  rc = download(h, buf.data(), b.d_noise, buf.size() * 8);
  if (rc) return rc;
  for (int64_t j = 0; j < B; ++j)
    for (int64_t t = 0; t < nmd; ++t)
      for (int64_t k = 0; k < nc; ++k) noise[((size_t)j * nmd + t) * nc + k] = buf[((size_t)t * nc + k) * B + j];
  return GLE_OK;
}

int gle_noise_factors(gle_handle* h, int32_t bath, int64_t nfreq, const double* m_re, const double* m_im) {
  int rc = check_bath(h, bath);
  if (rc) return rc;
  if (!m_re || nfreq != h->nmd / 2 + 1) return fail(h, GLE_ERR_ARG, "factors must cover nmd/2+1 frequencies");
  hipSetDevice(h->cfg.device);
  Bath& b = h->baths[bath];
  b.fac_complex = m_im != nullptr;
  b.fac_rows = b.fac_complex ? 2 * b.nc : b.nc;
  b.fac_nrt = (b.fac_rows + 15) / 16;
  b.nfreq = nfreq;
  std::vector<double> f = pack_frags(m_re, nfreq, b.nc, b.nc, b.fac_nrt, b.nks, m_im);
  if (b.d_fac) {
    tfree(b.d_fac);
    auto it = std::find(h->allocs.begin(), h->allocs.end(), (void*)b.d_fac);
    if (it != h->allocs.end()) h->allocs.erase(it);
    b.d_fac = nullptr;
  }
  rc = dalloc_n(h, &b.d_fac, f.size());
  if (!rc) rc = upload(h, b.d_fac, f.data(), f.size() * 8);
  return rc;
}

int gle_noise_generate(gle_handle* h, int32_t bath, const double* x_host, uint64_t seed, uint64_t traj_offset) {
  int rc = check_bath(h, bath);
  if (rc) return rc;
  Bath& b = h->baths[bath];
  if (!b.d_fac) return fail(h, GLE_ERR_STATE, "gle_noise_factors not set for this bath");
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  const int64_t B = h->B, nf = b.nfreq, ncp = b.ncp, nc = b.nc;
  // x [nfreq][ncp][B]
  double* d_x = nullptr;
  double* d_a = nullptr;
  const size_t nx = (size_t)nf * ncp * B + (size_t)(64 + 16) * B + 4096;
  const size_t na = (size_t)nf * b.fac_rows * B + 4096;
  HIPCHK(h, tmalloc((void**)&d_x, nx * 8));
  if (tmalloc((void**)&d_a, na * 8) != hipSuccess) {
    tfree(d_x);
    return fail(h, GLE_ERR_NOMEM, "noise work buffers");
  }
  auto cleanup = [&]() {
    hipStreamSynchronize(h->stream);
    tfree(d_x);
    tfree(d_a);
  };
  if (hipMemsetAsync(d_x, 0, nx * 8, h->stream) != hipSuccess) {
    cleanup();
    return fail(h, GLE_ERR_HIP, "memset");
  }
  if (x_host) {
    std::vector<double> buf((size_t)nf * ncp * B, 0.0);
    for (int64_t j = 0; j < B; ++j)
      for (int64_t w = 0; w < nf; ++w)
        for (int64_t k = 0; k < nc; ++k) buf[((size_t)w * ncp + k) * B + j] = x_host[((size_t)j * nf + w) * nc + k];
    hipError_t e = hipMemcpyAsync(d_x, buf.data(), buf.size() * 8, hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) {
      cleanup();
      return fail(h, GLE_ERR_HIP, std::string("upload draws: ") + hipGetErrorString(e));
    }
  } else {
    launch_philox_normal(d_x, nf, ncp, nc, B, seed, traj_offset, h->stream);
  }
  // a_w = M_w . x_w  : batched over frequencies (one slice per item)
  Op op;
  {
    Planner p(h, op, rn_for(B));
    for (int64_t w = 0; w < nf; ++w) {
      Gemm g{};
      g.A = b.d_fac + w * 64;
      g.a_ks = nf * 64;
      g.a_rt = (int64_t)b.nks * g.a_ks;
      g.nrt_total = b.fac_nrt;
      g.nks_total = b.nks;
      g.i0 = 0;
      g.i1 = 1;
      g.X = d_x + (size_t)w * ncp * B;
      g.ldx = B;
      g.M = b.fac_rows;
      g.Kd = b.nc;
      g.N = (int)B;
      g.dst = d_a + (size_t)w * b.fac_rows * B;
      g.ldd = B;
      plan_gemm(op, g, 1, 1 << 30);
    }
    op.rn = rn_for(B);
    std::vector<bool> part(op.items.size(), false);
    // direct-write items only: allocate descriptors temporarily
    CItem* d_items = nullptr;
    hipError_t e = tmalloc((void**)&d_items, op.items.size() * sizeof(CItem));
    if (e != hipSuccess) {
      cleanup();
      return fail(h, GLE_ERR_NOMEM, "noise items");
    }
    e = hipMemcpyAsync(d_items, op.items.data(), op.items.size() * sizeof(CItem), hipMemcpyHostToDevice, h->stream);
    // chunk the grid to stay well inside launch limits
    const int CH = 1 << 20;
    for (size_t s = 0; s < op.items.size(); s += CH)
      launch_contract(op.rn, 1, d_items + s, (int)std::min<size_t>(CH, op.items.size() - s), step_args(h), h->stream);
    const double scale = 1.0 / (h->dt * (double)h->nmd);  // dw/2pi (functions.py:51)
    int frc = launch_fft_noise(d_a, b.d_noise, h->d_tw, h->nmd, nc, b.fac_rows, B, b.fac_complex ? 1 : 0, scale, h->stream);
    e = hipStreamSynchronize(h->stream);
    tfree(d_items);
    if (frc) {
      cleanup();
      return fail(h, GLE_ERR_HIP, "device noise FFT: transform launch or work buffers failed (nmd " + std::to_string(h->nmd) + ")");
    }
    if (e != hipSuccess) {
      cleanup();
      return fail(h, GLE_ERR_HIP, std::string("noise generation: ") + hipGetErrorString(e));
    }
  }
  cleanup();
  b.noise_set = true;
  h->x_live = false;  // V0 / W1 carry the noise
  return GLE_OK;
}

namespace {
void free_stream(Bath& b) {
  for (double** p : {&b.d_sa, &b.d_sx, &b.d_sm}) {
    if (*p) tfree(*p);
    *p = nullptr;
  }
  b.s_cap = 0;
}

// retained factors are read by products already queued on `s`: wait for them before freeing
void free_retained(Bath& b, hipStream_t s) {
  if (!b.s_ret.empty()) hipStreamSynchronize(s);
  for (auto& r : b.s_ret) tfree(r.d_m);
  b.s_ret.clear();
  b.s_ret_bytes = 0;
  b.s_ret_complete = false;
}

// device memory for one retained segment of `nd` doubles, or nullptr (then nothing of the plan in
// progress is retained: the stream goes on through the chunk buffer)
// device memory a retention must leave free: every bath's stream scratch at its widest (a later
// bath's stream allocates its own while this bath's factors are kept), the ~256 MB chunk buffer the
// history getters and md.dump's snapshot use, and 256 MB of slack
size_t retain_margin(const gle_handle* h) {
  size_t m = (size_t)512 << 20;
  const int64_t nf = h->nmd / 2 + 1, B = h->B;
  for (const Bath& o : h->baths) {
    const int64_t cap = std::min<int64_t>(std::max<int64_t>(o.s_ret_cap, 64), nf);
    m += (size_t)(nf * 2 * o.nc * B + cap * o.ncp * B + cap * o.nc * o.nc * 2) * 8;
  }
  return m;
}

// device memory for one retained segment of `nd` doubles, or nullptr (then nothing of the plan in
// progress is retained: the stream goes on through the chunk buffer, and md keeps the factors on the
// host).  Retention stops before it leaves less than retain_margin free or exceeds the handle's cap.
double* retain_alloc(gle_handle* h, Bath& b, size_t nd) {
  if (!b.s_retain || !b.s_ret_ok) return nullptr;
  size_t held = 0;
  for (const Bath& o : h->baths) held += o.s_ret_bytes;
  size_t fr = 0, tot = 0;
  bool ok = h->ret_cap < 0 || held + nd * 8 <= (size_t)h->ret_cap;
  if (ok) ok = hipMemGetInfo(&fr, &tot) == hipSuccess && fr >= nd * 8 + retain_margin(h);
  double* p = nullptr;
  if (!ok || tmalloc(&p, nd * 8) != hipSuccess) {
    (void)hipGetLastError();
    b.s_ret_ok = false;
    free_retained(b, h->stream);
    return nullptr;
  }
  b.s_ret_bytes += nd * 8;
  return p;
}

// spectrum rows a_w += M_w x_w for frequencies [w0, w0 + nw) from device factors (one dense chunk,
// nw <= s_cap), draws keyed by (frequency, DOF, global trajectory)
void stream_dense(gle_handle* h, Bath& b, int64_t w0, int64_t nw, const double* dm, uint64_t seed, uint64_t toff) {
  const int64_t B = h->B, nc = b.nc, rows = b.s_complex ? 2 * nc : nc;
  const size_t nm = (size_t)nw * nc * nc;
  hipMemsetAsync(b.d_sx, 0, (size_t)nw * b.ncp * B * 8, h->stream);
  launch_philox_normal(b.d_sx, nw, b.ncp, nc, B, seed, toff, h->stream, w0);
  launch_noise_gemm(dm, (int)nc, (int)nc, b.d_sx, b.ncp, (int)B, b.d_sa, (int)rows, 0, w0, (int)nw, h->stream);
  if (b.s_complex)
    launch_noise_gemm(dm + nm, (int)nc, (int)nc, b.d_sx, b.ncp, (int)B, b.d_sa, (int)rows, (int)nc, w0, (int)nw,
                      h->stream);
}

// the same for nw frequencies sharing one factor F (dm: Re F then Im F) times scale dsc[w]
void stream_shared(gle_handle* h, Bath& b, int64_t w0, int64_t nw, const double* dm, const double* dsc,
                   uint64_t seed, uint64_t toff) {
  const int64_t B = h->B, nc = b.nc, rows = b.s_complex ? 2 * nc : nc;
  const size_t nm = (size_t)nc * nc;
  for (int64_t o = 0; o < nw; o += b.s_cap) {
    const int64_t n = std::min<int64_t>(b.s_cap, nw - o);
    hipMemsetAsync(b.d_sx, 0, (size_t)n * b.ncp * B * 8, h->stream);
    launch_philox_normal(b.d_sx, n, b.ncp, nc, B, seed, toff, h->stream, w0 + o);
    launch_noise_gemm(dm, (int)nc, (int)nc, b.d_sx, b.ncp, (int)B, b.d_sa, (int)rows, 0, w0 + o, (int)n, h->stream,
                      0, dsc + o);
    if (b.s_complex)
      launch_noise_gemm(dm + nm, (int)nc, (int)nc, b.d_sx, b.ncp, (int)B, b.d_sa, (int)rows, (int)nc, w0 + o, (int)n,
                        h->stream, 0, dsc + o);
  }
}

// spectrum / draw scratch of one stream (the factor chunk buffer only when factors arrive from the host)
int stream_scratch(gle_handle* h, Bath& b, bool is_complex, int64_t cap, bool chunk_buffer) {
  free_stream(b);
  const int64_t nf = h->nmd / 2 + 1, B = h->B;
  const int64_t rows = is_complex ? 2 * b.nc : b.nc;
  b.s_complex = is_complex;
  b.s_cap = std::min(cap, nf);
  const size_t na = (size_t)nf * rows * B, nx = (size_t)b.s_cap * b.ncp * B,
               nm = chunk_buffer ? (size_t)b.s_cap * b.nc * b.nc * (is_complex ? 2 : 1) : 0;
  if (tmalloc((void**)&b.d_sa, na * 8) != hipSuccess || tmalloc((void**)&b.d_sx, nx * 8) != hipSuccess ||
      (nm && tmalloc((void**)&b.d_sm, nm * 8) != hipSuccess)) {
    free_stream(b);
    return fail(h, GLE_ERR_NOMEM, "noise stream buffers (" + std::to_string((na + nx + nm) >> 17) + " MiB)");
  }
  HIPCHK(h, hipMemsetAsync(b.d_sa, 0, na * 8, h->stream));
  return GLE_OK;
}

// mirror + FFT of the accumulated spectrum into the bath's noise; releases the scratch
int stream_finish(gle_handle* h, Bath& b) {
  const double scale = 1.0 / (h->dt * (double)h->nmd);  // dw/2pi (functions.py:51)
  const int frc = launch_fft_noise(b.d_sa, b.d_noise, h->d_tw, h->nmd, b.nc, b.s_complex ? 2 * b.nc : b.nc, h->B,
                                   b.s_complex ? 1 : 0, scale, h->stream);
  const hipError_t e = hipStreamSynchronize(h->stream);
  free_stream(b);
  if (frc) return fail(h, GLE_ERR_HIP, "device noise FFT: transform launch or work buffers failed");
  if (e != hipSuccess) return fail(h, GLE_ERR_HIP, std::string("noise stream: ") + hipGetErrorString(e));
  b.noise_set = true;
  h->x_live = false;  // V0 / W1 carry the noise
  return GLE_OK;
}
}  // namespace

int gle_noise_stream_abort(gle_handle* h, int32_t bath) {
  int rc = check_bath(h, bath);
  if (rc) return rc;
  hipSetDevice(h->cfg.device);
  HIPCHK(h, hipStreamSynchronize(h->stream));  // chunks in flight read the scratch
  Bath& b = h->baths[bath];
  if (b.d_sa && !b.s_ret_complete) free_retained(b, h->stream);  // a plan cut short is not kept
  free_stream(b);
  return GLE_OK;
}

int gle_noise_stream_begin(gle_handle* h, int32_t bath, int32_t is_complex, int64_t max_chunk) {
  int rc = check_bath(h, bath);
  if (rc) return rc;
  if (max_chunk < 1) return fail(h, GLE_ERR_ARG, "max_chunk must be >= 1");
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  Bath& b = h->baths[bath];
  free_retained(b, h->stream);  // a new plan replaces the retained one
  b.s_ret_ok = b.s_retain;
  b.s_ret_cap = max_chunk;
  return stream_scratch(h, b, is_complex != 0, max_chunk, true);
}

int gle_noise_stream_chunk(gle_handle* h, int32_t bath, int64_t w0, int64_t nw, const double* m_re,
                           const double* m_im, uint64_t seed, uint64_t traj_offset) {
  int rc = check_bath(h, bath);
  if (rc) return rc;
  Bath& b = h->baths[bath];
  if (!b.d_sa) return fail(h, GLE_ERR_STATE, "gle_noise_stream_begin first");
  const int64_t nf = h->nmd / 2 + 1;
  if (!m_re || w0 < 0 || nw < 1 || nw > b.s_cap || w0 + nw > nf || (b.s_complex && !m_im))
    return fail(h, GLE_ERR_ARG, "bad noise stream chunk");
  hipSetDevice(h->cfg.device);
  const size_t nm = (size_t)nw * b.nc * b.nc;
  double* dm = retain_alloc(h, b, nm * (b.s_complex ? 2 : 1));
  if (dm) b.s_ret.push_back({false, w0, nw, dm, nullptr});
  else dm = b.d_sm;  // the previous chunk's products read it: the copies are stream-ordered after them
  HIPCHK(h, hipMemcpyAsync(dm, m_re, nm * 8, hipMemcpyHostToDevice, h->stream));
  if (b.s_complex) HIPCHK(h, hipMemcpyAsync(dm + nm, m_im, nm * 8, hipMemcpyHostToDevice, h->stream));
  stream_dense(h, b, w0, nw, dm, seed, traj_offset);
  HIPCHK(h, hipStreamSynchronize(h->stream));  // the caller reuses its host chunk buffers
  return GLE_OK;
}

int gle_noise_stream_shared(gle_handle* h, int32_t bath, int64_t w0, int64_t nw, const double* scale,
                            const double* m_re, const double* m_im, uint64_t seed, uint64_t traj_offset) {
  int rc = check_bath(h, bath);
  if (rc) return rc;
  Bath& b = h->baths[bath];
  if (!b.d_sa) return fail(h, GLE_ERR_STATE, "gle_noise_stream_begin first");
  const int64_t nf = h->nmd / 2 + 1;
  if (!m_re || !scale || w0 < 0 || nw < 1 || w0 + nw > nf || (b.s_complex && !m_im))
    return fail(h, GLE_ERR_ARG, "bad shared noise stream range");
  hipSetDevice(h->cfg.device);
  const size_t nm = (size_t)b.nc * b.nc, np = nm * (b.s_complex ? 2 : 1);
  DevTmp d_sc;
  double* dm = retain_alloc(h, b, np + nw);
  double* dsc = nullptr;
  if (dm) {
    dsc = dm + np;
    b.s_ret.push_back({true, w0, nw, dm, dsc});
  } else {
    if (tmalloc(&d_sc.p, (size_t)nw * 8) != hipSuccess) return fail(h, GLE_ERR_NOMEM, "noise stream scales");
    dm = b.d_sm;  // the shared factor takes the chunk buffer's first slot(s), stream-ordered
    dsc = (double*)d_sc.p;
  }
  HIPCHK(h, hipMemcpyAsync(dm, m_re, nm * 8, hipMemcpyHostToDevice, h->stream));
  if (b.s_complex) HIPCHK(h, hipMemcpyAsync(dm + nm, m_im, nm * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(dsc, scale, (size_t)nw * 8, hipMemcpyHostToDevice, h->stream));
  stream_shared(h, b, w0, nw, dm, dsc, seed, traj_offset);
  HIPCHK(h, hipStreamSynchronize(h->stream));  // the caller's host buffers and the scale scratch
  return GLE_OK;
}

int gle_noise_stream_end(gle_handle* h, int32_t bath) {
  int rc = check_bath(h, bath);
  if (rc) return rc;
  Bath& b = h->baths[bath];
  if (!b.d_sa) return fail(h, GLE_ERR_STATE, "gle_noise_stream_begin first");
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  if (b.s_retain && b.s_ret_ok) {
    b.s_ret_complete = true;
    b.s_ret_complex = b.s_complex;
  } else {
    free_retained(b, h->stream);
  }
  return stream_finish(h, b);
}

int gle_noise_stream_retain(gle_handle* h, int32_t bath, int32_t retain) {
  int rc = check_bath(h, bath);
  if (rc) return rc;
  hipSetDevice(h->cfg.device);
  Bath& b = h->baths[bath];
  b.s_retain = retain != 0;
  if (!b.s_retain) free_retained(b, h->stream);
  return GLE_OK;
}

int gle_noise_stream_retain_cap(gle_handle* h, int64_t max_bytes) {
  if (!h) return GLE_ERR_ARG;
  h->ret_cap = max_bytes;
  return GLE_OK;
}

int gle_noise_stream_retained(gle_handle* h, int32_t bath, int64_t* bytes) {
  int rc = check_bath(h, bath);
  if (rc) return rc;
  if (!bytes) return fail(h, GLE_ERR_ARG, "null output");
  const Bath& b = h->baths[bath];
  *bytes = b.s_ret_complete ? (int64_t)b.s_ret_bytes : 0;
  return GLE_OK;
}

int gle_noise_stream_replay(gle_handle* h, int32_t bath, uint64_t seed, uint64_t traj_offset) {
  int rc = check_bath(h, bath);
  if (rc) return rc;
  Bath& b = h->baths[bath];
  if (!b.s_ret_complete) return fail(h, GLE_ERR_STATE, "no retained noise plan (gle_noise_stream_retain)");
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  rc = stream_scratch(h, b, b.s_ret_complex, b.s_ret_cap, false);
  if (rc) return rc;
  for (const auto& r : b.s_ret) {
    if (r.shared) stream_shared(h, b, r.w0, r.nw, r.d_m, r.d_sc, seed, traj_offset);
    else stream_dense(h, b, r.w0, r.nw, r.d_m, seed, traj_offset);
  }
  return stream_finish(h, b);
}

int gle_step_begin(gle_handle* h, const double* fpot, double* q_tilde_out) {
  if (!h) return GLE_ERR_ARG;
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  int rc = 0;
  if (fpot) {
    std::vector<double> tf;
    to_dev_layout(fpot, tf, h->B, h->nph, h->nph);
    rc = step_begin_impl(h, tf.data());
    if (!rc) HIPCHK(h, hipStreamSynchronize(h->stream));  // tf goes out of scope
  } else {
    rc = step_begin_impl(h, nullptr);
  }
  if (rc) return rc;
  if (q_tilde_out) {
    std::vector<double> buf((size_t)h->nph * h->B);
    rc = download(h, buf.data(), h->d_Qt, buf.size() * 8);
    if (rc) return rc;
    from_dev_layout(buf, q_tilde_out, h->B, h->nph);
  }
  return GLE_OK;
}

int gle_step_end(gle_handle* h, const double* fpot_qt) {
  if (!h) return GLE_ERR_ARG;
  hipSetDevice(h->cfg.device);
  if (fpot_qt) {
    std::vector<double> tf;
    to_dev_layout(fpot_qt, tf, h->B, h->nph, h->nph);
    int rc = step_end_impl(h, tf.data());
    if (!rc) HIPCHK(h, hipStreamSynchronize(h->stream));
    return rc;
  }
  return step_end_impl(h, nullptr);
}

int gle_run(gle_handle* h, int64_t nsteps) {
  if (!h || nsteps < 0) return GLE_ERR_ARG;
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  if (h->xstep && h->frozen) return run_xstep(h, nsteps);
  for (int64_t s = 0; s < nsteps; ++s) {
    int rc = step_begin_impl(h, nullptr);
    if (rc) return rc;
    rc = step_end_impl(h, nullptr);
    if (rc) return rc;
  }
  return GLE_OK;
}

int gle_sync(gle_handle* h) {
  if (!h) return GLE_ERR_ARG;
  hipSetDevice(h->cfg.device);
  // one host wait: the main stream joins the background streams, then is synchronised (one
  // wake-up instead of one per stream; GLE_SYNC_JOIN=0: per-stream synchronisation)
  const char* ej = gle_env("GLE_SYNC_JOIN");
  const bool per_stream = ej && atoi(ej) == 0;
  if (per_stream) {
    int rc = sync_bg(h);
    if (rc) return rc;
  } else {
    join_bg(h);
  }
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (h->x_pend) {  // the composed run just waited for: replay it if it stopped (xresolve)
    const int64_t replays = h->x_replays;
    XRESOLVE(h);
    if (h->x_replays != replays) {
      join_bg(h);
      HIPCHK(h, hipStreamSynchronize(h->stream));
    }
  }
  HIPCHK(h, hipGetLastError());
  return bounds_report(h);
}

int gle_get_current(gle_handle* h, double* cur) {
  if (!h || !cur) return GLE_ERR_ARG;
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  if (h->frozen) launch_finalize(h->d_sd, (int)h->B, (int)h->nmd, (int)h->baths.size(), h->stream);
  const int64_t B = h->B, nmd = h->nmd;
  std::vector<double> buf((size_t)nmd * B);
  for (size_t j = 0; j < h->baths.size(); ++j) {
    int rc = download(h, buf.data(), h->baths[j].d_cur, buf.size() * 8);
    if (rc) return rc;
    for (int64_t b = 0; b < B; ++b)
      for (int64_t t = 0; t < nmd; ++t) cur[((size_t)j * B + b) * nmd + t] = buf[(size_t)t * B + b];
  }
  return GLE_OK;
}

int gle_get_energy(gle_handle* h, double* etot) {
  if (!h || !etot) return GLE_ERR_ARG;
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  if (h->frozen) launch_finalize(h->d_sd, (int)h->B, (int)h->nmd, (int)h->baths.size(), h->stream);
  const int64_t B = h->B, nmd = h->nmd;
  std::vector<double> buf((size_t)nmd * B);
  int rc = download(h, buf.data(), h->d_etot, buf.size() * 8);
  if (rc) return rc;
  for (int64_t b = 0; b < B; ++b)
    for (int64_t t = 0; t < nmd; ++t) etot[(size_t)b * nmd + t] = buf[(size_t)t * B + b];
  return GLE_OK;
}

int gle_current_sums(gle_handle* h, double* out) {
  if (!h || !out) return GLE_ERR_ARG;
  const int64_t B = h->B, nmd = h->nmd;
  std::vector<double> cur(h->baths.size() * B * nmd);
  int rc = gle_get_current(h, cur.data());
  if (rc) return rc;
  for (size_t j = 0; j < h->baths.size(); ++j) {
    double s = 0, s2 = 0;
    for (int64_t b = 0; b < B; ++b) {
      double m = 0;
      for (int64_t t = 0; t < nmd; ++t) m += cur[((size_t)j * B + b) * nmd + t];
      m /= (double)nmd;
      s += m;
      s2 += m * m;
    }
    out[3 * j] = s;
    out[3 * j + 1] = s2;
    out[3 * j + 2] = (double)B;
  }
  return GLE_OK;
}

int gle_profile(gle_handle* h, int32_t enable) {
  if (!h) return GLE_ERR_ARG;
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  if ((enable & GLE_PROFILE_EVENTS) && h->ev.empty()) {
    h->ev.resize(4096);
    for (auto& e : h->ev) HIPCHK(h, hipEventCreate(&e));
  }
  if ((enable & GLE_PROFILE_EVENTS) && !h->d_tst) {
    int rc = dalloc_n(h, &h->d_tst, 2 * h->tst_cap);
    if (rc) return rc;
    reset_tst(h, h->tst_cap, h->stream);
  }
  if (h->d_tst && h->tst_used > 0) {
    HIPCHK(h, hipDeviceSynchronize());
    reset_tst(h, h->tst_used, h->stream);
  }
  if ((enable & GLE_PROFILE_CHAIN) && !h->d_ctst) {
    size_t n = 0;
    for (Chain* c : {&h->chA[0], &h->chA[1], &h->chB[0], &h->chB[1], &h->chC, &h->chBC, &h->chX[0], &h->chX[1]})
      n = std::max(n, c->tiles.size());
    n += (size_t)h->far_max_items;  // far items of the fused schedule ride in the same grids
    h->ctst_tiles = n;
    if (n > 0) {
      int rc = dalloc_n(h, &h->d_ctst, 2 * h->ctst_cap * n);
      if (rc) return rc;
    }
  }
  if (h->ctst_used > 0) HIPCHK(h, hipDeviceSynchronize());
  h->ctst_used = 0;
  h->ctst_n.clear();
  h->prof_ch = (enable & GLE_PROFILE_CHAIN) != 0;
  h->tst_used = 0;
  h->prof_n_dev = 0;
  h->prof_ms_dev = 0.0;
  h->prof_ch_n = 0;
  h->prof_ch_ms = h->prof_ch_flops = 0.0;
  h->prof = enable != 0;
  h->prof_ev = (enable & GLE_PROFILE_EVENTS) != 0;
  h->ev_used = 0;
  h->prof_n = 0;
  h->prof_ms = h->prof_flops = h->prof_bytes = 0;
  for (double& b : h->prof_blocks) b = 0.0;
  return GLE_OK;
}

int gle_profile_read(gle_handle* h, int64_t* nlaunch, double* total_ms, double* flops, double* bytes) {
  if (!h) return GLE_ERR_ARG;
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  drain_profile(h);
  HIPCHK(h, hipGetLastError());
  if (nlaunch) *nlaunch = h->prof_n;
  if (total_ms) *total_ms = h->prof_ms;
  if (flops) *flops = h->prof_flops;
  if (bytes) *bytes = h->prof_bytes;
  return GLE_OK;
}

int gle_profile_read_chain(gle_handle* h, int64_t* nlaunch, double* total_ms, double* flops) {
  if (!h) return GLE_ERR_ARG;
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  drain_profile(h);
  HIPCHK(h, hipGetLastError());
  if (nlaunch) *nlaunch = h->prof_ch_n;
  if (total_ms) *total_ms = h->prof_ch_ms;
  if (flops) *flops = h->prof_ch_flops;
  return GLE_OK;
}

int gle_profile_read_device(gle_handle* h, int64_t* nlaunch, double* total_ms) {
  if (!h) return GLE_ERR_ARG;
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  drain_profile(h);
  HIPCHK(h, hipGetLastError());
  if (nlaunch) *nlaunch = h->prof_n_dev;
  if (total_ms) *total_ms = h->prof_ms_dev;
  return GLE_OK;
}

int gle_profile_levels(gle_handle* h, int32_t nmax, int32_t* nlevel, int32_t* P, double* blocks) {
  if (!h || nmax < 0) return GLE_ERR_ARG;
  const int n = (int)h->levels.size();
  if (nlevel) *nlevel = n;
  for (int l = 0; l < n && l < nmax; ++l) {
    if (P) P[l] = h->levels[l].P;
    if (blocks) blocks[l] = h->prof_blocks[l];
  }
  return GLE_OK;
}

// Algorithmic work of one steady-state harmonic step of the plan, all trajectories (SURVEY.md 8d
// conventions: every matrix entry read once, every product counted once, no padding):
//   chain  K0.p_t, K_1.p_t + near lags [2, nn) (S(t+1)), the velocity stage's products (fused:
//          K0.p_half, K0^2.p_half, K0.V, K0.Fpot or (K0 P dyn).q~, dyn.q~; else K0.p_half, K0.p1,
//          dyn.q~) and the bias products;
//   ladder per level (block work) / P: spectral = Gauss GEMMs + segment / inverse transforms
//          (5 N log2 N per complex length-N transform, two real series each), direct = contraction.
// the per-step chain's part of gle_step_work (every launch on the main stream)
static void chain_work(const gle_handle* h, double& fl, double& by) {
  const double B = (double)h->B;
  fl = 0.0;
  by = 0.0;
  double dyn_nnz = 0.0;
  for (double v : h->dyn_h) dyn_nnz += v != 0.0 ? 1.0 : 0.0;
  for (const Bath& b : h->baths) {
    const double nc2 = (double)b.nc * b.nc;
    double kd_nnz = 0.0;  // entries of K0 P dyn in its nonzero 16 x 4 blocks (fused stage)
    for (size_t rt = 0; rt < b.kd_rng.size(); ++rt) {
      int rows = 0;
      for (int r = 0; r < 16 && 16 * (int64_t)rt + r < h->nph; ++r) rows += b.inv[16 * rt + r] >= 0 ? 1 : 0;
      for (const auto& r : b.kd_rng[rt]) kd_nnz += 4.0 * r.second * rows;
    }
    double nprod = 1.0;                              // K0.p_t (stage A)
    if (b.ml > 1) nprod += (double)(b.nn - 1);       // K_1 + near lags [2, nn)
    nprod += h->fuse_bc ? 3.0 : 2.0;                 // K0.p_half, K0^2.p_half / K0.V | K0.p1
    if (b.has_q) nprod += h->fuse_bc ? 3.0 : 2.0;    // Kq.q_t, Kq.q~ (+ K0 Kq.q~)
    fl += 2.0 * nc2 * B * nprod;
    by += 8.0 * nc2 * ((double)b.nn + (h->fuse_bc ? 1.0 : 0.0) + (b.has_q ? 2.0 : 0.0));
    if (h->fuse_bc && !h->bc_fpot) {
      fl += 2.0 * kd_nnz * B;  // (K0 P dyn).q~ on a potential-cache miss (every harmonic step)
      by += 8.0 * kd_nnz;
    }
    if (h->bc_fpot) by += 16.0 * b.nc * B;  // fpot launch: V += Fpot_b (read-modify-write of every bath row)
    by += 8.0 * 12.0 * b.nc * B;  // bath-local vectors: noise rows, S, V, gathers, ring pushes
  }
  fl += 2.0 * dyn_nnz * B;  // dyn.q~ (the potential force at q~; the fpot launch's CSR product under bc_fpot)
  if (h->bc_fpot) by += 4.0 * dyn_nnz + 4.0 * (h->nph + 1) + 8.0 * 3.0 * (double)h->nph * B;  // CSR columns / rows, Qt, Fc, Q0
  by += 8.0 * dyn_nnz + 8.0 * 12.0 * (double)h->nph * B;  // dyn, state vectors (p, q, p_half, q~, F, caches)
  if (h->xstep) {  // composed step: its operators' nonzeros, K0 / K1 / K2, the near lags, dyn (plan_xstep)
    fl = h->x_alg_flops;
    by = h->x_alg_bytes;
  }
}

int gle_chain_work(gle_handle* h, double* flops, double* bytes) {
  if (!h) return GLE_ERR_ARG;
  if (!h->frozen) return fail(h, GLE_ERR_STATE, "no plan yet (call gle_set_state first)");
  double fl = 0.0, by = 0.0;
  chain_work(h, fl, by);
  if (flops) *flops = fl;
  if (bytes) *bytes = by;
  return GLE_OK;
}

int gle_step_work(gle_handle* h, double* flops, double* bytes) {
  if (!h) return GLE_ERR_ARG;
  if (!h->frozen) return fail(h, GLE_ERR_STATE, "no plan yet (call gle_set_state first)");
  const double B = (double)h->B;
  double fl = 0.0, by = 0.0;
  chain_work(h, fl, by);
  for (const Level& lv : h->levels) {
    const double P = (double)lv.P;
    if (lv.spectral) {
      const double N = 2.0 * P;
      double nser = 0.0;  // complex transforms per block (two real series each), per direction
      for (size_t j = 0; j < h->baths.size(); ++j)
        if (lv.lb[j].active) nser += (double)h->baths[j].nc * B / 2.0;
      const double fft = 2.0 * nser * 5.0 * N * std::log2(N);
      double fby = 0.0;
      for (size_t j = 0; j < h->baths.size(); ++j)
        if (lv.lb[j].active) {
          const double ncb = (double)h->baths[j].nc * B;
          fby += 8.0 * ncb * (N + lv.nplanes * (P + 1.0)) + 8.0 * ncb * (3.0 * (P + 1.0) * lv.cg_split + P);
        }
      fl += (lv.cg_flops + fft) / P;
      by += (lv.cg_bytes + fby) / P;
    } else {
      fl += lv.op[0].flops / P;
      by += lv.op[0].bytes / P;
    }
  }
  if (flops) *flops = fl;
  if (bytes) *bytes = by;
  return GLE_OK;
}

int gle_record(gle_handle* h, int32_t flags) {
  if (!h) return GLE_ERR_ARG;
  if (flags & ~(GLE_REC_P | GLE_REC_Q | GLE_REC_F | GLE_REC_HIST)) return fail(h, GLE_ERR_ARG, "bad record flags");
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  h->rec_flags = flags;
  if (!h->frozen) return GLE_OK;  // applied when the plan is built
  return apply_record(h);
}

int gle_record_zero(gle_handle* h, int32_t flags) {
  if (!h) return GLE_ERR_ARG;
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  const size_t n = (size_t)h->nmd * h->nph * h->B * 8;
  if ((flags & GLE_REC_P) && h->d_rec_p) HIPCHK(h, hipMemsetAsync(h->d_rec_p, 0, n, h->stream));
  if ((flags & GLE_REC_Q) && h->d_rec_q) HIPCHK(h, hipMemsetAsync(h->d_rec_q, 0, n, h->stream));
  if ((flags & GLE_REC_HIST) && h->d_rec_hp) {
    const size_t nh = (size_t)h->rec_ml * h->nph * h->B * 8;
    HIPCHK(h, hipMemsetAsync(h->d_rec_hp, 0, nh, h->stream));
    HIPCHK(h, hipMemsetAsync(h->d_rec_hq, 0, nh, h->stream));
  }
  for (size_t j = 0; j < h->baths.size(); ++j)
    if ((flags & GLE_REC_F) && h->d_rec_f[j])
      HIPCHK(h, hipMemsetAsync(h->d_rec_f[j], 0, (size_t)h->nmd * h->baths[j].nc * h->B * 8, h->stream));
  return GLE_OK;
}

int gle_get_record(gle_handle* h, int32_t what, int32_t bath, double* out) {
  if (!h || !out) return GLE_ERR_ARG;
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  const int64_t B = h->B, nmd = h->nmd;
  const double* src = nullptr;
  int64_t rows = 0, cols = 0;
  if (what == GLE_REC_P || what == GLE_REC_Q) {
    src = what == GLE_REC_P ? h->d_rec_p : h->d_rec_q;
    rows = nmd;
    cols = h->nph;
  } else if (what == GLE_REC_F) {
    int rc = check_bath(h, bath);
    if (rc) return rc;
    src = h->d_rec_f[bath];
    rows = nmd;
    cols = h->baths[bath].nc;
  } else {
    return fail(h, GLE_ERR_ARG, "gle_get_record: what must be GLE_REC_P, GLE_REC_Q or GLE_REC_F");
  }
  if (!src) return fail(h, GLE_ERR_STATE, "that quantity was never recorded (gle_record)");
  std::vector<double> buf((size_t)rows * cols * B);
  int rc = download(h, buf.data(), src, buf.size() * 8);
  if (rc) return rc;
  for (int64_t b = 0; b < B; ++b)
    for (int64_t r = 0; r < rows; ++r)
      for (int64_t c = 0; c < cols; ++c) out[((size_t)b * rows + r) * cols + c] = buf[((size_t)r * cols + c) * B + b];
  return GLE_OK;
}

int gle_get_record_history(gle_handle* h, double* phis, double* qhis, int64_t* ml) {
  if (!h) return GLE_ERR_ARG;
  if (ml) *ml = h->rec_ml;
  if (!phis && !qhis) return GLE_OK;
  if (!h->d_rec_hp) return fail(h, GLE_ERR_STATE, "histories were never recorded (gle_record GLE_REC_HIST)");
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  const int64_t B = h->B, n = h->nph, R = h->rec_ml;
  // row i (newest first) = time t-1-i = ring slot (t-1-i) mod R
  for (int k = 0; k < 2; ++k) {
    double* out = k == 0 ? phis : qhis;
    if (!out) continue;
    int rc = hist_to_host(h, k == 0 ? h->d_rec_hp : h->d_rec_hq, B, n * B, (int)R, h->t - 1, (int)R, (int)n, out);
    if (rc) return rc;
  }
  return GLE_OK;
}

int gle_get_full_history(gle_handle* h, int64_t ml, double* phis, double* qhis) {
  if (!h || ml < 0) return GLE_ERR_ARG;
  if (!phis && !qhis) return GLE_OK;
  if (!h->frozen) return fail(h, GLE_ERR_STATE, "no state yet");
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  const int64_t B = h->B, n = h->nph, per = ml * n;
  if (per == 0) return GLE_OK;
  // trajectory chunks through a <= 256 MB device buffer; the copies and the next chunk's kernels
  // are ordered on the handle's stream (one wait at the end)
  const int64_t nbc = std::max<int64_t>(1, std::min<int64_t>(B, (256ll << 20) / (per * 8)));
  double* d_tmp = nullptr;
  HIPCHK(h, tmalloc((void**)&d_tmp, (size_t)(nbc * per * 8)));
  const bool rec = (h->rec_flags & GLE_REC_HIST) && h->d_rec_hp;
  hipError_t e = hipSuccess;
  for (int k = 0; k < 2 && e == hipSuccess; ++k) {
    double* out = k == 0 ? phis : qhis;
    if (!out) continue;
    for (int64_t b0 = 0; b0 < B && e == hipSuccess; b0 += nbc) {
      const int nb = (int)std::min<int64_t>(nbc, B - b0);
      launch_hist_full(rec ? (k == 0 ? h->d_rec_hp : h->d_rec_hq) : nullptr, (int)B, h->rec_ml, h->t - 1, (int)ml,
                       (int)n, (int)b0, nb, d_tmp, h->stream);
      if (k == 0)  // the friction's own rings win on bath DOFs, later baths over earlier ones
        for (const Bath& b : h->baths)
          launch_hist_overlay(b.d_H, b.ldh, (int)B, b.R, h->t - 1, b.d_inv, (int)std::min<int64_t>(ml, b.ml), (int)n,
                              (int)b0, nb, (int)ml, d_tmp, h->stream);
      e = hipMemcpyAsync(out + b0 * per, d_tmp, (size_t)nb * per * 8, hipMemcpyDeviceToHost, h->stream);
    }
  }
  const hipError_t es = hipStreamSynchronize(h->stream);
  tfree(d_tmp);
  if (e == hipSuccess) e = es;
  if (e != hipSuccess) return fail(h, GLE_ERR_HIP, std::string("full history copy: ") + hipGetErrorString(e));
  return GLE_OK;
}

int gle_host_alloc(int64_t bytes, void** p) {
  if (!p || bytes < 0) return GLE_ERR_ARG;
  *p = nullptr;
  const hipError_t e = hipHostMalloc(p, (size_t)std::max<int64_t>(bytes, 8), hipHostMallocDefault);
  if (e != hipSuccess) {
    *p = nullptr;
    return fail(nullptr, GLE_ERR_NOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
  }
  return GLE_OK;
}

int gle_host_free(void* p) {
  if (p && hipHostFree(p) != hipSuccess) return GLE_ERR_HIP;
  return GLE_OK;
}

int gle_set_record(gle_handle* h, int32_t what, int32_t bath, const double* in) {
  if (!h || !in) return GLE_ERR_ARG;
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  const int64_t B = h->B, nmd = h->nmd;
  double* dst = nullptr;
  int64_t cols = 0;
  if (what == GLE_REC_P || what == GLE_REC_Q) {
    dst = what == GLE_REC_P ? h->d_rec_p : h->d_rec_q;
    cols = h->nph;
  } else if (what == GLE_REC_F) {
    int rc = check_bath(h, bath);
    if (rc) return rc;
    dst = h->d_rec_f[bath];
    cols = h->baths[bath].nc;
  } else {
    return fail(h, GLE_ERR_ARG, "gle_set_record: what must be GLE_REC_P, GLE_REC_Q or GLE_REC_F");
  }
  if (!dst) return fail(h, GLE_ERR_STATE, "enable the recording first (gle_record)");
  std::vector<double> buf((size_t)nmd * cols * B);
  for (int64_t b = 0; b < B; ++b)
    for (int64_t r = 0; r < nmd; ++r)
      for (int64_t c = 0; c < cols; ++c) buf[((size_t)r * cols + c) * B + b] = in[((size_t)b * nmd + r) * cols + c];
  return upload(h, dst, buf.data(), buf.size() * 8);
}

int gle_set_record_history(gle_handle* h, const double* phis, const double* qhis) {
  if (!h) return GLE_ERR_ARG;
  if (!h->d_rec_hp) return fail(h, GLE_ERR_STATE, "enable GLE_REC_HIST first (gle_record)");
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  const int64_t B = h->B, n = h->nph, R = h->rec_ml;
  std::vector<double> buf((size_t)R * n * B);
  for (int k = 0; k < 2; ++k) {
    const double* in = k == 0 ? phis : qhis;
    if (!in) continue;
    for (int64_t i = 0; i < R; ++i) {
      const int64_t slot = ((h->t - 1 - i) % R + R) % R;
      for (int64_t b = 0; b < B; ++b)
        for (int64_t d = 0; d < n; ++d) buf[((size_t)slot * n + d) * B + b] = in[((size_t)b * R + i) * n + d];
    }
    int rc = upload(h, k == 0 ? h->d_rec_hp : h->d_rec_hq, buf.data(), buf.size() * 8);
    if (rc) return rc;
  }
  return GLE_OK;
}

int gle_power_spectrum(gle_handle* h, int32_t ngroup, const int64_t* group_len, const int64_t* dofs, double* out) {
  if (!h || ngroup < 1 || !group_len || !dofs || !out) return GLE_ERR_ARG;
  if (!h->d_rec_p) return fail(h, GLE_ERR_STATE, "gle_power_spectrum needs the recorded velocities (gle_record GLE_REC_P)");
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  std::vector<int64_t> off(ngroup + 1, 0);
  for (int g = 0; g < ngroup; ++g) {
    if (group_len[g] < 0) return fail(h, GLE_ERR_ARG, "negative group length");
    off[g + 1] = off[g] + group_len[g];
  }
  for (int64_t i = 0; i < off[ngroup]; ++i)
    if (dofs[i] < 0 || dofs[i] >= h->nph) return fail(h, GLE_ERR_ARG, "power spectrum DOF out of range");
  DevTmp d_off, d_dofs, d_out;
  HIPCHK(h, tmalloc(&d_off.p, off.size() * 8));
  HIPCHK(h, tmalloc(&d_dofs.p, std::max<int64_t>(1, off[ngroup]) * 8));
  const size_t no = (size_t)ngroup * h->B * h->nmd;
  HIPCHK(h, tmalloc(&d_out.p, no * 8));
  HIPCHK(h, hipMemcpyAsync(d_off.p, off.data(), off.size() * 8, hipMemcpyHostToDevice, h->stream));
  if (off[ngroup] > 0)
    HIPCHK(h, hipMemcpyAsync(d_dofs.p, dofs, off[ngroup] * 8, hipMemcpyHostToDevice, h->stream));
  sync_bg(h);
  if (launch_power(h->d_rec_p, h->nph, (int)h->B, h->nmd, ngroup, (const int64_t*)d_off.p, (const int64_t*)d_dofs.p,
                   h->d_tw, (double*)d_out.p, h->stream, off[ngroup]))
    return fail(h, GLE_ERR_HIP, "device power spectrum: transform launch or work buffers failed");
  HIPCHK(h, hipMemcpyAsync(out, d_out.p, no * 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return GLE_OK;
}

int gle_plan_info(gle_handle* h, int64_t* block_len, int64_t* far_items, int64_t* device_bytes,
                  int32_t* far_mode) {
  if (!h) return GLE_ERR_ARG;
  int64_t items = 0;
  for (auto& lv : h->levels) items += (int64_t)(lv.spectral ? lv.cg.size() : lv.op[0].items.size());
  if (block_len) *block_len = h->frozen ? h->P0 : 0;
  if (far_mode) *far_mode = h->frozen ? h->far_mode : h->cfg.far_mode;
  if (far_items) *far_items = items;
  if (device_bytes) *device_bytes = (int64_t)h->dev_bytes;
  return GLE_OK;
}

int gle_set_plan_class(gle_handle* h, int32_t plan_class) {
  if (!h) return GLE_ERR_ARG;
  if (plan_class < GLE_PLAN_AUTO || plan_class > GLE_PLAN_LARGE_BATHS) return fail(h, GLE_ERR_ARG, "bad plan class");
  if (h->frozen) return fail(h, GLE_ERR_STATE, "the plan is already built (set the plan class before gle_set_state)");
  h->plan_class = plan_class;
  return GLE_OK;
}

int gle_plan_detail(gle_handle* h, int32_t* plan_class, int32_t* fused_waves, double* cg_per_cu, int32_t* nlevel,
                    int64_t* dyn_dropped, int32_t* far_fused) {
  if (!h) return GLE_ERR_ARG;
  if (!h->frozen) return fail(h, GLE_ERR_STATE, "no plan yet (gle_set_state builds it)");
  if (plan_class) *plan_class = h->small_baths ? GLE_PLAN_SMALL_BATHS : GLE_PLAN_LARGE_BATHS;
  if (fused_waves) *fused_waves = h->fuse_bc ? h->chBC.nw : 0;
  if (cg_per_cu) *cg_per_cu = h->cg_per_cu;
  if (nlevel) *nlevel = (int32_t)h->levels.size();
  if (dyn_dropped) *dyn_dropped = h->dyn_dropped;
  if (far_fused) *far_fused = h->far_fused ? 1 : 0;
  return GLE_OK;
}

int gle_plan_flags(gle_handle* h, int32_t* flags) {
  if (!h || !flags) return GLE_ERR_ARG;
  if (!h->frozen) return fail(h, GLE_ERR_STATE, "no plan yet (gle_set_state builds it)");
  *flags = (h->fuse_bc ? GLE_PLAN_FUSED_BC : 0) | (h->bc_fpot ? GLE_PLAN_FPOT_LAUNCH : 0) |
           (h->far_fused ? GLE_PLAN_FAR_FUSED : 0) | (h->xstep ? GLE_PLAN_COMPOSED_STEP : 0) |
           (h->xstep && h->x_split ? GLE_PLAN_SPLIT_TILES : 0);
  return GLE_OK;
}

int gle_cache_audit(gle_handle* h, int64_t* counts) {
  if (!h || !counts) return GLE_ERR_ARG;
  counts[0] = counts[1] = 0;
  if (!h->d_guard) return GLE_OK;
  hipSetDevice(h->cfg.device);
  XRESOLVE(h);
  unsigned long long v[2] = {0, 0};
  const int rc = download(h, v, h->d_guard, sizeof(v));
  if (rc) return rc;
  counts[0] = (int64_t)v[0];
  counts[1] = (int64_t)v[1];
  return GLE_OK;
}

// ---- ensemble reduce over RCCL (SURVEY.md 8b gle_reduce_current, 8e) ----------------------
static_assert(GLE_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "RCCL unique-id size");

int gle_comm_unique_id(char* id) {
  if (!id) return fail(nullptr, GLE_ERR_ARG, "null id buffer");
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return fail(nullptr, GLE_ERR_HIP, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return GLE_OK;
}

int gle_comm_init(int32_t nranks, int32_t rank, int32_t device, const char* id, void** comm) {
  if (!id || !comm || nranks < 1 || rank < 0 || rank >= nranks) return fail(nullptr, GLE_ERR_ARG, "bad communicator arguments");
  *comm = nullptr;
  if (hipSetDevice(device) != hipSuccess) return fail(nullptr, GLE_ERR_HIP, "gle_comm_init: no such device");
  ncclUniqueId u;
  memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  const ncclResult_t r = ncclCommInitRank(&c, nranks, u, rank);
  if (r != ncclSuccess) return fail(nullptr, GLE_ERR_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  *comm = (void*)c;
  return GLE_OK;
}

int gle_comm_destroy(void* comm) {
  if (!comm) return GLE_OK;
  const ncclResult_t r = ncclCommDestroy((ncclComm_t)comm);
  if (r != ncclSuccess) return fail(nullptr, GLE_ERR_HIP, std::string("ncclCommDestroy: ") + ncclGetErrorString(r));
  return GLE_OK;
}

int gle_comm_allreduce(gle_handle* h, void* comm, double* buf, int64_t n) {
  if (!h || (!buf && n > 0) || n < 0) return GLE_ERR_ARG;
  if (!comm || n == 0) return GLE_OK;
  hipSetDevice(h->cfg.device);
  double* d = nullptr;
  HIPCHK(h, tmalloc((void**)&d, (size_t)n * 8));
  hipError_t e = hipMemcpyAsync(d, buf, (size_t)n * 8, hipMemcpyHostToDevice, h->stream);
  ncclResult_t r = ncclSuccess;
  if (e == hipSuccess) r = ncclAllReduce(d, d, (size_t)n, ncclDouble, ncclSum, (ncclComm_t)comm, h->stream);
  if (e == hipSuccess && r == ncclSuccess) e = hipMemcpyAsync(buf, d, (size_t)n * 8, hipMemcpyDeviceToHost, h->stream);
  const hipError_t es = hipStreamSynchronize(h->stream);
  tfree(d);
  if (r != ncclSuccess) return fail(h, GLE_ERR_HIP, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
  if (e != hipSuccess || es != hipSuccess)
    return fail(h, GLE_ERR_HIP, std::string("reduce copies: ") + hipGetErrorString(e != hipSuccess ? e : es));
  return GLE_OK;
}

int gle_reduce_current(gle_handle* h, void* comm, double* out) {
  if (!h || !out) return GLE_ERR_ARG;
  const int64_t n = 3 * (int64_t)h->baths.size();
  if (n == 0) return GLE_OK;
  int rc = gle_current_sums(h, out);  // this handle's [sum mean, sum mean^2, ntraj] per bath
  if (rc) return rc;
  return gle_comm_allreduce(h, comm, out, n);
}

}  // extern "C"
