/*
 * rvk_gp.h -- batched GP log-likelihood (quasi-periodic kernel) on MI355X (librvk.so).
 *
 * SURVEY.md §8(f) row 2 / BASELINE config 5: ravest's GPLogLikelihood
 * (src/ravest/fit.py:7942-8105) with the kernel of GPKernel("Quasiperiodic")
 * (src/ravest/gp.py:126-156), evaluated for a whole walker block:
 *   mean   = sum of planets + trend + gamma[inst]            fit.py:7995-8047
 *   r      = vel - mean
 *   K_ij   = amp^2 exp(-gamma sin^2(pi |t_i - t_j| / P_gp)) exp(-(t_i - t_j)^2 / (2 lambda_e^2)),
 *            gamma = 1 / (2 lambda_p^2)                       gp.py:126-156
 *   C      = K + diag(velerr^2 + jit[inst]^2)                fit.py:8090-8105
 *   ll     = -1/2 r^T C^-1 r - sum log diag(L) - N/2 log(2 pi),  C = L L^T
 *            (tinygp 0.3 GaussianProcess(kernel, X=t, diag=...).log_probability(r),
 *             DirectSolver: Cholesky; tinygp is not in this image -- its published
 *             algorithm is restated, see DESIGN.md "GP").
 * Mean model and the final sums in fp64; the factorisation in the handle's
 * precision mode (rvk_gp_set_precision):
 *   RVK_GP_FP32                fp32 blocked Cholesky on MFMA (BASELINE config 5 is
 *                              fp32); a covariance that is not positive definite in
 *                              fp32 gives NaN;
 *   RVK_GP_FP32_FP64_FALLBACK  as RVK_GP_FP32, then every walker the fp32
 *                              factorisation rejected (NaN) is re-evaluated in fp64 in
 *                              the same stream-ordered call -- no host round trip;
 *   RVK_GP_FP64                (default) fp64 throughout (the reference's precision: ravest runs
 *                              tinygp with jax_enable_x64, fit.py:39); NaN only where
 *                              the covariance is not positive definite in fp64.
 * An invalid planet gives -inf (the reference's mean-model fail-fast).
 * Epochs: 1 <= n_epochs <= RVK_GP_MAX_EPOCHS (4096; the fp32 modes run the fp64 factorisation above 1024).  Calls on one rvk_gp share its workspaces: keep
 * them on one stream (or serialise them).
 *
 * hyper row layout [W][hyper_stride] fp64: gp_amp, gp_lambda_e, gp_lambda_p,
 * gp_period (GPKernel.expected_hyperparams order, gp.py:37).
 */
#ifndef RVK_GP_H
#define RVK_GP_H

#include <stdint.h>

#include "rvk.h"
#include "rvk_post.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RVK_GP_QUASIPERIODIC 0
#define RVK_GP_NHYPER        4
#define RVK_GP_MAX_EPOCHS    4096   /* fp32 factorisation up to 1024 epochs; above, the fp64 one in every mode */

#define RVK_GP_FP32                 0
#define RVK_GP_FP32_FP64_FALLBACK   1
#define RVK_GP_FP64                 2

typedef struct rvk_gp rvk_gp;
typedef struct rvk_gp_post rvk_gp_post;

/* GP likelihood over the handle's dataset, planets and parameterisation.  The
 * handle must outlive it. */
rvk_gp *rvk_gp_create(rvk_handle *h, int32_t kernel_type);
void rvk_gp_destroy(rvk_gp *g);

/* out[w] = GP log-likelihood of theta row w (rvk.h layout) with hyper row w.
 * Device buffers, stream-ordered. */
int rvk_gp_loglike_device(rvk_gp *g, const double *d_theta, const double *d_hyper, int64_t n_walkers,
                          int64_t row_stride, int64_t hyper_stride, double *d_out, void *stream);
/* Host buffers, blocking. */
int rvk_gp_loglike(rvk_gp *g, const double *theta, const double *hyper, int64_t n_walkers,
                   int64_t row_stride, int64_t hyper_stride, double *out);

/* Precision mode of the factorisation (RVK_GP_FP32 / _FP32_FP64_FALLBACK / _FP64). */
int rvk_gp_set_precision(rvk_gp *g, int32_t mode);

/* GP-conditioned posterior predictive (GPFitter.calculate_rv_gp_custom, fit.py:7494-7554,
 * and calculate_rv_gp_from_samples, fit.py:7342-7386), fp64: for every sample s (a theta
 * row and a hyper row), the GP conditioned on the residuals r = vel - mean(t_data) with
 * the diagonal velerr^2 + jit^2, evaluated at the query times:
 *   out[s][q] = K(t_q, t_data) (K(t_data, t_data) + diag)^-1 r
 * (tinygp GaussianProcess.condition(y, X_test).mean, zero mean function).  A sample
 * with an invalid planet gives a row of NaN (the reference's Planet() raises). */
int rvk_gp_predict_device(rvk_gp *g, const double *d_theta, const double *d_hyper, int64_t n_samples,
                          int64_t row_stride, int64_t hyper_stride, const double *d_tq, int64_t n_times,
                          double *d_out, void *stream);
int rvk_gp_predict(rvk_gp *g, const double *theta, const double *hyper, int64_t n_samples,
                   int64_t row_stride, int64_t hyper_stride, const double *tq, int64_t n_times,
                   double *out);

/* GP log-posterior (GPLogPosterior, fit.py:7596-7939), batched over walkers.
 * The walker's combined row is [theta_full (rvk.h layout) | gp_amp, gp_lambda_e,
 * gp_lambda_p, gp_period] (P_full + 4 columns); free_idx[n_free] gives the combined-row
 * column of each free coordinate, in emcee's order (free_params_names then
 * free_hyperparams_names, fit.py:4982); template_row[P_full + 4] holds the fixed values.
 * Prior slots (include/rvk_post.h kinds and sources; sources index the combined row)
 * [0, n_param_prior) are the LogPrior over the parameters and [n_param_prior, n_prior)
 * the hyperpriors, each summed in the given (the reference's dict) order.
 * out = (((ll + lp) + lhp) + log_jacobian) + log_renorm; -inf for a negative jitter,
 * invalid hyperparameters (non-finite or <= 0, gp.py:73-82), a prior-side conversion
 * error, a non-finite log-prior or log-hyperprior, or an invalid planet -- the
 * reference's order of checks (fit.py:7849-7901).  The GP handle must outlive it. */
rvk_gp_post *rvk_gp_post_create(rvk_gp *g, int32_t n_free, const int32_t *free_idx, const double *template_row,
                                int32_t n_prior, int32_t n_param_prior, const int32_t *prior_kind,
                                const int32_t *prior_src, const double *prior_par, double log_jacobian,
                                double log_renorm, int32_t flags);
void rvk_gp_post_destroy(rvk_gp_post *p);
int rvk_gp_post_reserve(rvk_gp_post *p, int64_t max_walkers);
int rvk_gp_logpost_device(rvk_gp_post *p, const double *d_free, int64_t n_walkers, int64_t row_stride,
                          double *d_out, void *stream);
int rvk_gp_logpost(rvk_gp_post *p, const double *free, int64_t n_walkers, int64_t row_stride, double *out);

/* Device-resident stretch move over the GP log-posterior (GPFitter.run_mcmc's emcee
 * EnsembleSampler with the default StretchMove(a=2), fit.py:4982-4990): the same contract,
 * draws and chain layout as rvk_stretch_run (include/rvk_post.h) -- per half-step the
 * proposals, rvk_gp_logpost_device on them, and the accept / reject, all stream-ordered. */
int rvk_gp_stretch_run(rvk_gp_post *p, double *d_x, double *d_lp, int64_t n_walkers, int32_t n_steps, double a,
                       uint64_t seed, uint64_t step0, int32_t flags, const int32_t *d_set, const double *d_zu,
                       const int32_t *d_rint, const double *d_au, double *d_chain, double *d_lnp,
                       int64_t *d_naccepted, int32_t *d_status, void *stream);

/* The multi-GPU form of rvk_gp_stretch_run (GPFitter.run_mcmc's pool.map over walkers,
 * fit.py:4983-4990), with rvk_stretch_draws / _propose / _update's contract (include/rvk_post.h):
 * every rank holds the whole ensemble and the same draws; per half-step rank r evaluates the
 * GP log-posterior of its slice [j0, j0 + count) of the W/2 proposals (rvk_gp_stretch_propose),
 * the W/2 log-posteriors are all-gathered (8 bytes each) and every rank applies the accept /
 * reject to the whole half (rvk_gp_stretch_update).  The chain equals rvk_gp_stretch_run's
 * with the same seed bit for bit. */
int rvk_gp_stretch_draws(rvk_gp_post *p, int64_t n_walkers, int32_t n_steps, double a, uint64_t seed, uint64_t step0,
                         int32_t flags, void *stream);
int rvk_gp_stretch_propose(rvk_gp_post *p, const double *d_x, int64_t n_walkers, int32_t s, int32_t half, int64_t j0,
                           int64_t count, double *d_out, void *stream);
int rvk_gp_stretch_update(rvk_gp_post *p, double *d_x, double *d_lp, int64_t n_walkers, int32_t s, int32_t half,
                          const double *d_nlp, double *d_chain_step, double *d_lnp_step, const int64_t *d_nacc_in,
                          int64_t *d_nacc_out, int32_t *d_status, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* RVK_GP_H */
