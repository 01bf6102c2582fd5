/*
 * hipgle.h -- C-ABI of the MI355X-native generalized-Langevin (GLE) stepper.
 *
 * This is the drop-in boundary for sclmd's per-step hot path: md.vv + md.force + the bath forces
 * (ebath.bforce / phbath.bforce) + the coloured-noise generator (noise.phnoise / noise.enoise).
 * Plain C types only (no torch, no HIP types).  The Python shim sclmd_amd/ binds it with ctypes;
 * INTEGRATION.md shows the binding a sclmd maintainer would add.
 *
 * Units and array meaning follow the reference exactly (mass-weighted p, q; eV; time unit
 * 0.658211814201041 fs; sclmd/units.py:5-10).
 *
 * Layout conventions of HOST buffers (all row-major, float64, caller-owned, copied in/out):
 *   per-trajectory state  [ntraj][nph]
 *   bath kernel           [ml][nc][nc]          (phbath.kernel / ebath.kernel, baths.py:119,426)
 *   bath noise            [ntraj][nmd][nc]      (bath.noise, baths.py:191,408)
 *   heat current          [nbath][ntraj][nmd]   (bath.cur, md.py:397)
 *   kinetic energy        [ntraj][nmd]          (md.etot, md.py:383)
 *
 * Every entry returns 0 on success and a negative GLE_ERR_* code on failure; gle_last_error()
 * returns a description.  (Deviation from the reference, which prints and calls sys.exit(0) on
 * bad shapes, e.g. baths.py:115-116, md.py:171-176: here errors are reported, never exit.)
 *
 * Threading: a handle is bound to one HIP device and one stream and is not thread-safe.
 * Multi-GPU = one handle per process/device; the ensemble reduce is gle_reduce_current over RCCL.
 */
#ifndef HIPGLE_H
#define HIPGLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GLE_ABI_VERSION 1

#define GLE_OK 0
#define GLE_ERR_ARG (-1)     /* bad argument / shape                      */
#define GLE_ERR_HIP (-2)     /* HIP runtime error (no device, fault, ...) */
#define GLE_ERR_STATE (-3)   /* call out of order (e.g. no noise set)     */
#define GLE_ERR_NOMEM (-4)   /* device allocation failed                  */
#define GLE_ERR_UNSUP (-5)   /* unsupported configuration                 */

#define GLE_BATH_PHONON 0    /* phbath: memory kernel, ml >= 1 (baths.py:258)     */
#define GLE_BATH_ELECTRON 1  /* ebath: time-local, ml == 1, bias terms (baths.py:55) */

typedef struct gle_handle gle_handle;

typedef struct gle_config {
    int64_t nph;        /* system degrees of freedom, md.nph (md.py:86)                      */
    int64_t ntraj;      /* independent trajectories batched on this device (ensemble size)   */
    int64_t nmd;        /* MD steps per run = noise period, md.nmd (md.py:59); even (any even */
                        /* length: powers of two <= 8192 in LDS, others in global memory)    */
    double dt;          /* MD time step, md.dt (md.py:59)                                    */
    int32_t device;     /* HIP device ordinal                                                */
    int32_t block_len;  /* P0: first block length of the memory-sum ladder (near field = lags
                           [1, 2 P0) every step); 0 = auto by the plan class (gle_set_plan_class):
                           8 when every bath has nc <= 512, 4 otherwise                          */
    int32_t far_mode;   /* GLE_FAR_AUTO / GLE_FAR_DIRECT / GLE_FAR_SPECTRAL                      */
    int32_t max_block;  /* largest ladder block length; 0 = auto (256 spectral, direct: L with
                           L * ntraj >= 256, L <= 64)                                           */
} gle_config;

/* memory sum  S(t+1) = sum_{i>=1} K_i p_{t+1-i}   as a ladder:
 *   near field  lags [1, 2 P0) every step;
 *   level l     block P = P0 2^l, lags [2P, 4P) (the last level up to ml): every P steps one block
 *               of P future steps is computed one block ahead, on a background stream that
 *               overlaps the per-step chain.  A level is
 *   DIRECT      one time-blocked MFMA contraction over its kernel slices, or
 *   SPECTRAL    uniformly partitioned overlap-save: kernel partitions of P slices transformed once
 *               (length 2P), one new input segment transformed per block, a per-frequency MFMA
 *               contraction of the spectra (~4(P+1)/P^2 of the direct flops), inverse transform.
 *   AUTO        spectral for power-of-two P >= 8 when ntraj >= 8.  Same result to fp64 rounding. */
#define GLE_FAR_AUTO 0
#define GLE_FAR_DIRECT 1
#define GLE_FAR_SPECTRAL 2

/* Plan class.  AUTO picks by the largest bath: SMALL when every bath has nc <= 512 (the per-step
 * chain is latency-bound: first block length 8, 4-wave fused velocity-stage tiles, far-field GEMM
 * chunks of 1.25 workgroups per CU, a block's ladder pieces spread over its whole window), LARGE
 * otherwise (first block length 4, the
 * potential force at q~ as its own small launch before the fused stage (GLE_PLAN_FPOT_LAUNCH),
 * far-field GEMM chunks of 4 workgroups per CU).  Forcing a class changes only the schedule, never
 * the result beyond fp64
 * rounding; tests use it to run the large-bath plan at small sizes. */
#define GLE_PLAN_AUTO 0
#define GLE_PLAN_SMALL_BATHS 1
#define GLE_PLAN_LARGE_BATHS 2
/* ---- lifetime ------------------------------------------------------------------------- */
int gle_abi_version(void);
/* replaces md.__init__ (md.py:56-130) for the state the hot path needs */
int gle_create(const gle_config* cfg, gle_handle** out);
int gle_destroy(gle_handle* h);
/* last error of h, or of the last failed gle_create when h == NULL */
const char* gle_last_error(const gle_handle* h);
int gle_device_count(int32_t* count);
/* Free and total device memory of HIP device `device` (bytes).  Errors: gle_last_error(NULL). */
int gle_device_mem_info(int32_t device, int64_t* free_bytes, int64_t* total_bytes);

/* ---- system / baths ------------------------------------------------------------------- */
/* md.AddBath (md.py:167-183) + the bath's bforce parameters (baths.py:224-255, 448-458).
 * kind     GLE_BATH_PHONON or GLE_BATH_ELECTRON
 * cids     [nc] DOF indices the bath couples to (bath.cids = cats, baths.py:80,303)
 * kernel   [ml][nc][nc] friction kernel (bath.kernel); the dt factor is applied iff ml > 1
 *          (baths.py:454-457)
 * bias, exim, zeta1, zeta2: electron bath only; exim/zeta2 antisymmetrised, zeta1 symmetrised by
 *          the caller (ebath.CheckEmat, baths.py:100-174).  The bias terms are active only when
 *          all three matrices are non-NULL and nonzero (baths.py:233).  Pass NULL otherwise.
 * bath_id  out: index of this bath (AddBath order) */
int gle_add_bath(gle_handle* h, int32_t kind, const int64_t* cids, int64_t nc, int64_t ml,
                 const double* kernel, double bias, const double* exim, const double* zeta1,
                 const double* zeta2, int32_t* bath_id);
/* phbath.gmem (baths.py:412-445) + md.AddBath on the device: the memory kernel is built in HBM,
 * never crossing PCIe.  gamt (baths.py:19-52) is linear in Gamma through flinterp
 * (functions.py:117-134), so K_i = sum_g W[i][g] gamma[g] with
 *   W      [ml][ngw]      = scale * C(t_i, w) . I(w -> gwl): the cosine (eta = 0) or damped
 *                            (eta != 0) coefficients times the interpolation weights, built by the
 *                            caller (sclmd_amd.baths.gmem_coefficients)
 *   gamma  [ngw][nc][nc]  the friction spectrum on gwl (phbath.gamma before the eta update)
 * Phonon bath, dt factor iff ml > 1 as gle_add_bath. */
int gle_add_bath_gmem(gle_handle* h, const int64_t* cids, int64_t nc, int64_t ml, const double* W,
                      int64_t ngw, const double* gamma, int32_t* bath_id);
/* Copy slices [i0, i0 + n) of a bath's device kernel out: out [n][nc][nc] (bath.kernel). */
int gle_get_kernel(gle_handle* h, int32_t bath, int64_t i0, int64_t n, double* out);
/* Standalone gamt on device `device`: out[i][e] = sum_g W[i][g] G[g][e], out [ml][nel],
 * W [ml][ngw], G [ngw][nel].  Errors: gle_last_error(NULL). */
int gle_gamt(int32_t device, int64_t ml, int64_t ngw, int64_t nel, const double* W, const double* G,
             double* out);
/* md.setDyn (md.py:250-292): harmonic potential force -dyn.q used when no host force is given
 * (md.potforce, md.py:466-467).  dyn [nph][nph] as already processed by setDyn.  setDyn's
 * U diag(w^2) U^T reconstruction leaves roundoff in the entries the matrix does not couple; the
 * device copy drops every pair d_ij, d_ji with max(|d_ij|, |d_ji|) <= 16 * 2^-52 * max(max_k |d_ik|,
 * max_k |d_jk|) (its sparsity pattern then stays the physical, symmetric one; the dropped part is at
 * the dense product's own rounding level; the count is in gle_plan_detail). */
int gle_set_dyn(gle_handle* h, const double* dyn);
/* md.AddConstr (md.py:189) flattened: the DOF indices ApplyConstraint zeroes (md.py:782-794) */
int gle_set_constraint(gle_handle* h, const int64_t* dofs, int64_t n);

/* ---- state ---------------------------------------------------------------------------- */
/* md.p, md.q, md.t (md.py:372, 411).  p, q: [ntraj][nph].  Resets the potential-force cache
 * (md.q0 = [], md.py:105) and re-derives the memory sums from the current history. */
int gle_set_state(gle_handle* h, const double* p, const double* q, int64_t t);
int gle_get_state(gle_handle* h, double* p, double* q, int64_t* t);
/* md.phis restricted to the bath's cids, newest first (md.py:345-346, 386-387).
 * phis: [ntraj][ml][nc] (ml of that bath).  NULL in set = zeros (md.ResetHis, md.py:340-349). */
int gle_set_history(gle_handle* h, int32_t bath, const double* phis);
int gle_get_history(gle_handle* h, int32_t bath, double* phis);
/* last total force md.f (md.py:411): [ntraj][nph] */
int gle_get_force(gle_handle* h, double* f);

/* ---- noise (bath.gnoi, baths.py:176-192, 397-409; noise.py:50-100, 149-206) ----------- */
/* Inject a noise realisation: noise [ntraj][nmd][nc] (bath.noise after gnoi). */
int gle_set_noise(gle_handle* h, int32_t bath, const double* noise);
int gle_get_noise(gle_handle* h, int32_t bath, double* noise);
/* Spectral factors of the noise covariance for the nfreq = nmd/2+1 positive frequencies:
 * m_re/m_im [nfreq][nc][nc] (m_im NULL for a real factor).  The generator computes
 *   a_w = M_w . x_w   for every trajectory, mirrors a into a length-nmd spectrum exactly as
 *   noise.py:87-94 does (Nyquist row -> conj(a_hlen)), applies numpy's forward-FFT convention
 *   times dw/2pi (functions.py:36-53) and keeps the real part (baths.py:191,408).
 * With M = U (eigenvectors) and host draws x = vargau's r (noise.py:297-303) this reproduces the
 * reference draw for draw; with M = U.diag(sqrt(max(lambda,0))) and device Gaussians it is the
 * ensemble generator. */
int gle_noise_factors(gle_handle* h, int32_t bath, int64_t nfreq, const double* m_re,
                      const double* m_im);
/* Generate bath noise on the device.  x_host [ntraj][nfreq][nc] host draws, or NULL to draw
 * N(0,1) on the device with a counter-based Philox stream keyed by (seed, traj_offset + b). */
int gle_noise_generate(gle_handle* h, int32_t bath, const double* x_host, uint64_t seed,
                       uint64_t traj_offset);

/* Streamed generation for baths whose per-frequency factors do not fit on the device beside the
 * spectral kernels (C5: 4097 x 1000^2 doubles per bath): begin allocates the spectrum; each chunk
 * hands over the factors M_w of frequencies [w0, w0 + nw) (row-major [nw][nc][nc], real, or real
 * and imaginary parts), draws N(0,1) on the device with the same Philox keys as
 * gle_noise_generate (so both give the same realisation for the same factors and seed) and forms
 * a_w = M_w x_w; end mirrors, transforms and scales exactly as gle_noise_generate. */
int gle_noise_stream_begin(gle_handle* h, int32_t bath, int32_t is_complex, int64_t max_chunk);
int gle_noise_stream_chunk(gle_handle* h, int32_t bath, int64_t w0, int64_t nw, const double* m_re,
                           const double* m_im, uint64_t seed, uint64_t traj_offset);
/* Frequencies [w0, w0 + nw) whose factor is one shared matrix times a per-frequency scale (a
 * spectrum A_w = s_w H: factor sqrt(s_w) H_+^(1/2), noise.py:73-84 / 171-191 at frequencies where one
 * term is nonzero): m_re / m_im the factor of H (row-major [nc][nc]) handed over once, scale [nw] the
 * sqrt(s_w); the same draws and products as gle_noise_stream_chunk with the scaled matrices. */
int gle_noise_stream_shared(gle_handle* h, int32_t bath, int64_t w0, int64_t nw, const double* scale,
                            const double* m_re, const double* m_im, uint64_t seed, uint64_t traj_offset);
int gle_noise_stream_end(gle_handle* h, int32_t bath);
/* Release a begun stream's scratch without generating (an error between begin and end); the bath's
 * previous noise stays.  gle_destroy releases any stream still open. */
int gle_noise_stream_abort(gle_handle* h, int32_t bath);
/* Keep the factors of the next complete streamed plan of `bath` (every chunk and shared segment
 * from begin to end) in device memory, so that each later run (md.Run draws new noise per run from
 * the same spectrum, md.py:569-570) replays them with new draws instead of handing them over PCIe
 * again (C5: ~11 GB of dense factors per run).  retain = 0 frees them.  A plan that does not fit
 * beside the resident state is streamed as without retention and nothing is kept: retention stops
 * before it would leave less device memory free than every bath's stream scratch plus the history
 * getters' chunk buffer and slack, or exceed the cap of gle_noise_stream_retain_cap. */
int gle_noise_stream_retain(gle_handle* h, int32_t bath, int32_t retain);
/* Cap on the bytes of retained plans over all baths of the handle (max_bytes < 0: no cap, the
 * default; 0: nothing is retained). */
int gle_noise_stream_retain_cap(gle_handle* h, int64_t max_bytes);
/* *bytes = device bytes of the retained complete plan of `bath`, 0 when none is retained. */
int gle_noise_stream_retained(gle_handle* h, int32_t bath, int64_t* bytes);
/* New noise of `bath` from its retained plan: the same result as streaming that plan again with
 * this seed / traj_offset (GLE_ERR_STATE when no plan is retained). */
int gle_noise_stream_replay(gle_handle* h, int32_t bath, uint64_t seed, uint64_t traj_offset);

/* ---- stepping (md.vv, md.py:367-411) -------------------------------------------------- */
/* Phase A of one step: F0 = Fpot(q_t) + sum_b bforce_b(t, id=0), current, half kick, drift.
 * fpot  [ntraj][nph] host force at q_t (driver.force(q), md.py:463-464) or NULL to use the
 *       harmonic -dyn.q with md.potforce's cache rule (sameq, md.py:449-450, 767-779).
 * q_tilde_out [ntraj][nph] receives q_t + p dt + F0 dt^2/2 (the position the host driver must
 *       be evaluated at next), or NULL. */
int gle_step_begin(gle_handle* h, const double* fpot, double* q_tilde_out);
/* Phase B: the two velocity iterations at q~ (md.py:401-404) and the constraints (:407-408).
 * fpot_qt [ntraj][nph] host force at q~ or NULL for the harmonic force. */
int gle_step_end(gle_handle* h, const double* fpot_qt);
/* nsteps full steps with the harmonic force, entirely on the device (no host round trips). */
int gle_run(gle_handle* h, int64_t nsteps);
int gle_sync(gle_handle* h);

/* ---- outputs -------------------------------------------------------------------------- */
/* bath.cur for every bath: [nbath][ntraj][nmd] (md.py:397) */
int gle_get_current(gle_handle* h, double* cur);
/* md.etot: [ntraj][nmd] (md.py:383) */
int gle_get_energy(gle_handle* h, double* etot);
/* Per bath: [sum over trajectories of mean_t cur, sum of (mean_t cur)^2, ntraj] -- the
 * per-run heat-current statistics the ensemble reduce sums (md.py:663, tools.py:193).
 * out: [nbath][3] */
int gle_current_sums(gle_handle* h, double* out);

/* ---- per-step recordings (md.savep / saveq / SaveAll, md.py:374-379, 398, 604-653) ---------- */
#define GLE_REC_P 1     /* md.ps: p_t of every step of the run, slot t mod nmd            */
#define GLE_REC_Q 2     /* md.qs: q_t likewise                                              */
#define GLE_REC_F 4     /* md.fhis[i]: bath i's id0 force of every step (bath rows)        */
#define GLE_REC_HIST 8  /* md.phis / md.qhis on every DOF: rings of the last ml p_t / q_t  */
/* Record the selected quantities from the next step on, on the device (stage A of each step writes
 * them; nothing crosses PCIe per step); 0 stops recording.  Buffers start zeroed. */
int gle_record(gle_handle* h, int32_t flags);
/* Zero the selected recordings (md.ResetSavepq at a new run, md.py:571-574). */
int gle_record_zero(gle_handle* h, int32_t flags);
/* what = GLE_REC_P / GLE_REC_Q: out [ntraj][nmd][nph] (md.ps / md.qs); GLE_REC_F: out
 * [ntraj][nmd][nc] of bath `bath` (md.fhis restricted to the bath's cids, md.py:398). */
int gle_get_record(gle_handle* h, int32_t what, int32_t bath, double* out);
/* md.phis / md.qhis on every DOF, newest first: [ntraj][ml][nph] (rows of times before the
 * recording started read as zeros); *ml = the ring length (max over baths of ml). */
int gle_get_record_history(gle_handle* h, double* phis, double* qhis, int64_t* ml);
/* md.phis / md.qhis as MD{j}.nc stores them (md.py:346-349, 717-731): [ntraj][ml][nph] each, newest
 * first.  p and q rows come from the full-DOF recording (GLE_REC_HIST; rows past its length, and
 * every row when it is not recording, read zero); the p rows i < ml_b of each bath's DOFs come from
 * that bath's own history ring, the friction's operand (baths in order: a later bath's ring wins on
 * shared DOFs).  Either output may be NULL.  The transposes run on the device; page-locked outputs
 * (gle_host_alloc) are written at the link's rate. */
int gle_get_full_history(gle_handle* h, int64_t ml, double* phis, double* qhis);
/* Page-locked host memory (hipHostMalloc) for large device reads such as a checkpoint's histories;
 * errors: gle_last_error(NULL). */
int gle_host_alloc(int64_t bytes, void** p);
int gle_host_free(void* p);
/* Restore recordings (a resumed run, md.py:513-534): in has gle_get_record's / _history's layout. */
int gle_set_record(gle_handle* h, int32_t what, int32_t bath, const double* in);
int gle_set_record_history(gle_handle* h, const double* phis, const double* qhis);
/* Velocity power spectra of the recorded ps (functions.powerspecp, functions.py:221-236, and
 * md.GetPower's per-section spectra, md.py:351-360) for ngroup DOF groups (group g = the next
 * group_len[g] entries of dofs): out [ngroup][ntraj][nmd] = sum_{k in group} |DFT_t ps[:, k]|^2
 * per frequency index; the reference's power is dt / nmd times this. */
int gle_power_spectrum(gle_handle* h, int32_t ngroup, const int64_t* group_len, const int64_t* dofs,
                       double* out);

/* ---- ensemble reduce ------------------------------------------------ */
/* The per-run heat-current statistics of the whole ensemble: out [nbath][3] = the sum over every
 * rank's gle_current_sums, by one RCCL all-reduce (sum, fp64) over xGMI on the handle's stream.
 * comm: an RCCL communicator (ncclComm_t, e.g. from gle_comm_init) with one rank per handle, or
 * NULL for this handle's trajectories alone.  Collective: every rank of comm must call it. */
int gle_reduce_current(gle_handle* h, void* comm, double* out);
/* Sum n doubles (host buffer, in place) over the ranks of comm on the handle's stream, fp64 (the
 * ensemble power spectra of md.Run, md.py:604-653).  comm NULL: no-op.  Collective. */
int gle_comm_allreduce(gle_handle* h, void* comm, double* buf, int64_t n);
/* RCCL communicator helpers for C callers without their own RCCL setup: rank 0 makes the id
 * (GLE_COMM_ID_BYTES opaque bytes), the caller distributes it (MPI, sockets, torch.distributed),
 * every rank then calls gle_comm_init with its own rank and HIP device. */
#define GLE_COMM_ID_BYTES 128
int gle_comm_unique_id(char* id);
int gle_comm_init(int32_t nranks, int32_t rank, int32_t device, const char* id, void** comm);
int gle_comm_destroy(void* comm);

/* ---- measurement ---------------------------------------------------------------------- */
/* enable = GLE_PROFILE_EVENTS | GLE_PROFILE_COUNT: HIP events around every launch of the dominant
 * far-field kernel, on the stream it is launched on (gle_profile_read), and the ladder's per-level
 * block counts (gle_profile_levels).  GLE_PROFILE_COUNT alone counts without events (the events
 * add launch-queue packets); 0 switches both off and resets the counters either way. */
#define GLE_PROFILE_EVENTS 1
#define GLE_PROFILE_COUNT 2
#define GLE_PROFILE_CHAIN 4 /* per-workgroup start / end stamps of the chain launches (gle_profile_read_chain) */
int gle_profile(gle_handle* h, int32_t enable);
/* launches, total milliseconds, algorithmic flops and bytes of the profiled contraction
 * launches since profiling was enabled (flops/bytes per SURVEY.md section 8d). */
int gle_profile_read(gle_handle* h, int64_t* nlaunch, double* total_ms, double* flops,
                     double* bytes);
/* The same launches timed on the device: first workgroup start to last workgroup end of each
 * launch (s_memrealtime, 100 MHz), i.e. the kernel duration a kernel trace reports; the HIP events
 * of gle_profile_read also include each launch's wait for free compute units. */
int gle_profile_read_device(gle_handle* h, int64_t* nlaunch, double* total_ms);
/* The per-step chain's launches (md.vv stages: A and the fused velocity stage, or A / B / C) since
 * profiling was enabled with GLE_PROFILE_CHAIN, timed like gle_profile_read_device (first
 * workgroup start to last end), with the algorithmic flops of their products. */
int gle_profile_read_chain(gle_handle* h, int64_t* nlaunch, double* total_ms, double* flops);
/* Planner summary of the current configuration: block length L, far-field work items, bytes of
 * device memory in use, far-field mode actually chosen. */
int gle_plan_info(gle_handle* h, int64_t* block_len, int64_t* far_items, int64_t* device_bytes,
                  int32_t* far_mode);
/* Force the plan class (GLE_PLAN_*) before the plan is built (the first gle_set_state). */
int gle_set_plan_class(gle_handle* h, int32_t plan_class);
/* The plan actually built: its class (GLE_PLAN_SMALL_BATHS / _LARGE_BATHS), the waves per
 * workgroup of the fused velocity stage (0 when the stages are not fused), the far-field GEMM
 * workgroups per CU per chunk (background schedule), the number of ladder levels, the dyn entries
 * gle_set_dyn dropped as reconstruction roundoff, and whether the spectral levels' GEMM items ride
 * in the per-step chain launches (1, the fused schedule) or run on background streams (0).
 * Requires a plan.  Any pointer may be NULL. */
int gle_plan_detail(gle_handle* h, int32_t* plan_class, int32_t* fused_waves, double* cg_per_cu,
                    int32_t* nlevel, int64_t* dyn_dropped, int32_t* far_fused);
/* Plan flags of the built plan: GLE_PLAN_FUSED_BC (the velocity stages B + C run as one launch),
 * GLE_PLAN_FPOT_LAUNCH (md.potforce at q~ runs as a small launch before the fused stage, which
 * then needs no K0 P dyn product; the large-bath plan), GLE_PLAN_FAR_FUSED.  Requires a plan. */
#define GLE_PLAN_FUSED_BC 1
#define GLE_PLAN_FPOT_LAUNCH 2
#define GLE_PLAN_FAR_FUSED 4
/* GLE_PLAN_COMPOSED_STEP: gle_run steps with one chain launch per step (small-bath harmonic plans
 * without a biased electron bath): md.vv is linear in (p_t, q_t) and the bath vectors, so p_{t+1}
 * is one product of composed operators (precomputed at plan time) and q_{t+1} = q~ follows from the
 * step's own K0.p_t and dyn.q_t (same result to fp64 rounding; steps with a host force, gle_step_begin
 * / gle_step_end, keep the two-launch path).  The potential force is evaluated fresh, which is
 * md.potforce's result unless its cache rule (sameq, md.py:449-450, 767-779) reuses the force of q0 at
 * a point within 1e-9 of q0 but not equal to it.  Each launch audits the previous step for that
 * case; a run that meets it stops storing at once and the library replays it from the step it
 * tripped at on the two-launch path, which applies the rule, before any call reads the state (the
 * replay runs in gle_sync or the next call on the handle).  See gle_cache_audit. */
#define GLE_PLAN_COMPOSED_STEP 8
/* GLE_PLAN_SPLIT_TILES: composed-step plans with few DOF tiles (small B, e.g. one trajectory) split
 * each tile's products over up to 8 workgroups by k-steps; the last to finish adds the partial sums
 * in a fixed order and runs the tile's md.vv epilogue (same result to fp64 rounding). */
#define GLE_PLAN_SPLIT_TILES 16
int gle_plan_flags(gle_handle* h, int32_t* flags);
/* Trajectories found by the composed step's audit (GLE_PLAN_COMPOSED_STEP) at which md.potforce's
 * cache rule (sameq, md.py:767-779) reuses a force at a point within 1e-9 of, but not equal to, the
 * point it was evaluated at: counts[0] at q~ (0 < max|q~ - q_t| < 1e-9), counts[1] at q_{t+1} after
 * a constraint (0 < max|q_{t+1} - q~_t| < 1e-9).  Each such finding stopped a composed run, which
 * was replayed on the two-launch path from that step.  Cumulative. */
int gle_cache_audit(gle_handle* h, int64_t* counts);
/* Memory-sum ladder levels: *nlevel = number of levels; for the first nmax levels the block length
 * P[l] and the blocks of that level issued since profiling was enabled (a block issued in pieces
 * counts its pieces' share).  Over a window of K steps a level in steady state issues K / P. */
int gle_profile_levels(gle_handle* h, int32_t nmax, int32_t* nlevel, int32_t* P, double* blocks);
/* Algorithmic work of one steady-state harmonic step of the plan, all trajectories on this device:
 * flops and bytes (every matrix entry read once, every product counted once, no padding; ladder
 * blocks averaged over their period).  Requires a plan (after gle_set_state). */
int gle_step_work(gle_handle* h, double* flops, double* bytes);
/* The per-step chain's part of gle_step_work (the md.vv launches on the main stream: for the
 * composed step its operators' nonzeros, K0 / K1 / K2, the near lags and dyn, every entry once). */
int gle_chain_work(gle_handle* h, double* flops, double* bytes);

#ifdef __cplusplus
}
#endif
#endif /* HIPGLE_H */
