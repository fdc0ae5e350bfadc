/*
 * rvk.h -- C-ABI of the MI355X RV log-likelihood engine (librvk.so).
 *
 * The drop-in boundary for ravest's per-walker log-probability hot path.
 * Plain pointers and sizes only; no C++ exceptions cross it; every entry point
 * returns 0 on success or a negative RVK_E* code, and rvk_last_error() gives
 * the thread's last message.  Non-finite results follow ravest's mask
 * semantics exactly: an invalid walker yields -INFINITY, never NaN.
 *
 * Reference interfaces replaced (ross-dobson/ravest v0.4.0, src/ravest/):
 *   rvk_create            LogLikelihood.__init__ precompute       fit.py:3535-3598
 *   rvk_loglike           LogLikelihood.__call__ (batched over W) fit.py:3600-3660
 *                          incl. Planet(...) conversion/validation model.py:259-275,
 *                          param.py:88-105,198-234, Planet.radial_velocity
 *                          model.py:329-354, _compute_rv/_njit_kepler_rv/
 *                          _solve_kepler model.py:23-243, Trend model.py:483-509
 *   rvk_loglike_device    same, device-resident in/out, stream-ordered
 *   rvk_solve_kepler      _solve_kepler                            model.py:23-70
 *   rvk_predict           Planet/Trend radial_velocity summed per sample
 *                          (posterior predictive, fit.py:2690-2939)
 *
 * theta row layout ("full parameter order"), row-major [W][P_full] fp64:
 *   for each planet p < n_planets, in parameterisation order:
 *        [P, K, e | secosw, w | sesinw, Tp | Tc]          (5 values)
 *   then g[n_inst], jit[n_inst], gd, gdd                  (2*n_inst + 2 values)
 *   P_full = 5*n_planets + 2*n_inst + 2 (a larger row stride is allowed).
 * Instrument index i refers to ravest's np.unique (sorted) instrument order
 * (fit.py:113, 3585-3586).
 *
 * Threading.  The blocking host-buffer entry points (rvk_loglike, rvk_predict,
 * rvk_logpost, rvk_gp_loglike, rvk_gp_predict, rvk_gp_logpost) may be called from
 * several threads on one handle, or on posteriors / GP objects built on one handle:
 * they share the handle's stream and host staging, so a per-handle mutex serialises
 * them (ravest hands log_probability to emcee's map or pool, fit.py:1068-1075; a
 * thread pool works, calls on one handle just take turns -- create one handle per
 * thread for concurrency).  The stream-ordered *_device entry points, the samplers'
 * rvk_*stretch* calls, rvk_*reserve and rvk_set_option are NOT serialised: each
 * object's device workspace is single-owner, so order such calls on one object
 * yourself (one thread, or one stream with the caller's own lock).  rvk_destroy
 * must not race any call on the handle or the objects built on it.
 */
#ifndef RVK_H
#define RVK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* parameterisation codes (param.py:5-10; ecosw/esinw are disabled upstream) */
#define RVK_PAR_PKEWTP            0   /* "P K e w Tp" */
#define RVK_PAR_PKEWTC            1   /* "P K e w Tc" */
#define RVK_PAR_PKSECOSWSESINWTP  2   /* "P K secosw sesinw Tp" */
#define RVK_PAR_PKSECOSWSESINWTC  3   /* "P K secosw sesinw Tc" */

/* Limits of one handle.  Up to 8 planets run kernels specialised on the planet count; 9 to
 * RVK_MAX_PLANETS run one generic kernel (planet constants in LDS).  Instruments are a runtime
 * loop. */
#define RVK_MAX_PLANETS 32
#define RVK_MAX_INST    64

/* error codes */
#define RVK_OK          0
#define RVK_E_ARG      -1   /* bad argument / shape */
#define RVK_E_HIP      -2   /* HIP runtime error */
#define RVK_E_NODEV    -3   /* no usable gfx950 device */
#define RVK_E_NOMEM    -4

/* rvk_predict component mask */
#define RVK_PRED_PLANETS  0x00FFu  /* bit p: include planet p (p < 8) */
#define RVK_PRED_TREND    0x0100u  /* include gd*(t-t0) + gdd*(t-t0)^2 */
#define RVK_PRED_GAMMA    0x0200u  /* include g[inst] (needs inst per time) */
#define RVK_PRED_ALL_PLANETS 0x0400u  /* include every planet (any count) */
#define RVK_PRED_PLANET(p) (0x0800u | ((uint32_t)(p) << 16))   /* include planet p (any p) */

typedef struct rvk_handle rvk_handle;

/* Create a handle bound to HIP device `device` (ordinal; -1 = current device).
 * Copies the data arrays to the device once (LogLikelihood precompute).
 * inst_idx may be NULL when n_inst == 1.  n_epochs == 0 (NULL arrays) makes a
 * model-only handle for rvk_predict*.  Returns NULL on error. */
rvk_handle *rvk_create(const double *time, const double *vel, const double *velerr,
                       const int32_t *inst_idx, int32_t n_epochs, int32_t n_inst,
                       int32_t n_planets, int32_t parameterisation, double t0,
                       int32_t device);

void rvk_destroy(rvk_handle *h);

/* Blocking, host buffers: out[w] = log-likelihood of walker w (−inf if a planet
 * is invalid, exactly where ravest's Planet() raises ValueError). */
int rvk_loglike(rvk_handle *h, const double *theta, int64_t n_walkers, int64_t row_stride,
                double *out);

/* Asynchronous, device buffers, stream-ordered on `stream` (a hipStream_t on
 * the handle's device, used as given: NULL is HIP's default stream; see
 * rvk_stream() for the handle's own).  Inputs must be resident on that device. */
int rvk_loglike_device(rvk_handle *h, const double *d_theta, int64_t n_walkers,
                       int64_t row_stride, double *d_out, void *stream);

/* Pre-size any device workspace for up to max_walkers per call, so that
 * rvk_loglike_device never allocates inside a captured HIP graph.  (The current
 * kernels need none: this returns RVK_OK; call it anyway before capture.) */
int rvk_reserve(rvk_handle *h, int64_t max_walkers);

/* Posterior predictive: out[s][j] = sum of the selected components for sample
 * s (theta row s) at time t[j]; inst (len n_t) only needed with RVK_PRED_GAMMA.
 * Invalid planets give NaN rows. Host buffers, blocking. */
int rvk_predict(rvk_handle *h, const double *theta, int64_t n_samples, int64_t row_stride,
                const double *t, const int32_t *inst, int64_t n_t, uint32_t what, double *out);

/* rvk_predict on device buffers, stream-ordered (d_inst may be NULL unless
 * RVK_PRED_GAMMA with n_inst > 1).  d_out is [n_samples][n_t]. */
int rvk_predict_device(rvk_handle *h, const double *d_theta, int64_t n_samples, int64_t row_stride,
                       const double *d_t, const int32_t *d_inst, int64_t n_t, uint32_t what,
                       double *d_out, void *stream);

/* Kepler solve on the device for arrays (host buffers): cos E, sin E of
 * E - e sin E = M.  solver 0: production solver (fp32 seed + fp64 Halley
 * polish, converged to ~1 ulp); solver 1: ravest's Halley iteration restated
 * (E0 = M, |dE| < 1.48e-8, <= 50 iterations) in a 2*pi-reduced frame. */
int rvk_solve_kepler(const double *M, const double *e, int64_t n, double *cosE, double *sinE,
                     int32_t device, int32_t solver);

/* Options. RVK_OPT_SOLVER: 0 = production solver (default), 1 = reference Halley.
 * RVK_OPT_GRAPH: 0 (default) = rvk_stretch_run issues plain stream launches;
 * 1 = it replays a cached HIP graph of each draw block (up to 256 steps, a multiple
 * of 8; same kernels; measured equal on MI355X at 4096 walkers, kept for
 * launch-bound hosts). */
#define RVK_OPT_SOLVER 1
#define RVK_OPT_GRAPH  2
/* RVK_OPT_LPW: lanes of a wave per walker for the log-likelihood kernel: 0 (default)
 * = chosen per launch from (walkers, epochs); 64, 32 or 16 = forced.  Fewer lanes per
 * walker share a wave's fixed costs between 2 or 4 walkers when epochs are few. */
#define RVK_OPT_LPW    3
/* RVK_OPT_HOSTIO: how the blocking host-buffer calls (rvk_loglike, rvk_logpost,
 * rvk_gp_loglike, rvk_gp_logpost on this handle and the posteriors built on it) move
 * their arrays.  Results are identical in every mode; only the latency differs.
 *   RVK_HOSTIO_AUTO (default)  zero-copy up to 1 MB of input, pinned DMA above;
 *   RVK_HOSTIO_PAGEABLE        async copies from / to the caller's own buffers;
 *   RVK_HOSTIO_PINNED          one memcpy into pinned staging, one DMA each way;
 *   RVK_HOSTIO_ZEROCOPY        memcpy into pinned staging; the kernels read their
 *                              inputs and write their output there over PCIe. */
#define RVK_OPT_HOSTIO 4
#define RVK_HOSTIO_AUTO      0
#define RVK_HOSTIO_PAGEABLE  1
#define RVK_HOSTIO_PINNED    2
#define RVK_HOSTIO_ZEROCOPY  3
/* RVK_OPT_LDS_POISON (tests only; default 0): every kernel LAUNCHED FOR A HANDLE (likelihood,
 * log-posterior, sampler, predictive, GP) that stages the sin/cos table in LDS first writes
 * each entry as NaN and the real value ~10 us later, before the barrier
 * that publishes the table.  A read of the table that is not ordered after that barrier
 * then sees NaN and the results are NaN: the GPU parity tests run with it on to catch a
 * publish-order race (round 4 found one that green tests had missed).  Same results when
 * the kernels are race-free; slower.  rvk_solve_kepler (no handle) does not take it.
 * Value 2 (the tests' positive control): the real value is never stored, every table read
 * is NaN, so the results of every kernel the option reaches are NaN. */
#define RVK_OPT_LDS_POISON 5
int rvk_set_option(rvk_handle *h, int32_t key, int32_t value);

/* Stream the handle uses (hipStream_t as void*). */
void *rvk_stream(rvk_handle *h);
int rvk_sync(rvk_handle *h);

int rvk_device_count(void);
const char *rvk_last_error(void);
/* 100*major + minor.  101: rvk_stretch_run / rvk_gp_stretch_run take an int32 flags
 * argument after step0 and rvk_stretch_half is gone (a caller built against 100 must
 * not call them); RVK_OPT_HOSTIO added.  102: RVK_OPT_LDS_POISON; the blocking calls
 * are serialised per handle (Threading, above).  103: RVK_OPT_LDS_POISON value 2 (the
 * tests' positive control). */
int rvk_version(void);

#ifdef __cplusplus
}
#endif
#endif /* RVK_H */
