/*
 * rvk_post.h -- device log-posterior and device-resident stretch move (librvk.so).
 *
 * SURVEY.md §8(f) rows 3 and 4, on top of the log-likelihood of rvk.h:
 *   rvk_post_create     LogPosterior.__init__: priors, fixed/free split,
 *                       correction constants                     fit.py:3228-3397
 *   rvk_logpost[_device] LogPosterior.log_probability batched over walkers:
 *                       free -> full scatter (build_params_dict fit.py:1390-1430),
 *                       jitter < 0 check, prior-side conversion
 *                       (_convert_params_for_prior_evaluation fit.py:3399-3446),
 *                       built-in priors (prior.py:9-511), log-likelihood,
 *                       + Jacobian / renormalisation corrections fit.py:3448-3495
 *   rvk_stretch_run     emcee's EnsembleSampler.run_mcmc with the default
 *                       StretchMove(a=2) / RedBlueMove(nsplits=2) as ravest's
 *                       Fitter.run_mcmc drives it                fit.py:1021-1111
 *                       -- every sub-step on the device, chain written in
 *                       emcee's (steps, walkers, ndim) layout (get_chain,
 *                       fit.py:1168-1228).
 *
 * Same conventions as rvk.h: 0 / negative RVK_E* codes, rvk_last_error().
 */
#ifndef RVK_POST_H
#define RVK_POST_H

#include <stdint.h>

#include "rvk.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Built-in prior kinds.  Each slot carries p[RVK_PRIOR_NPAR] doubles; the host
 * fills the constants listed (so the device repeats the reference's arithmetic
 * with the reference's own constants). */
#define RVK_PRIOR_NPAR          8
#define RVK_PRIOR_UNIFORM       0  /* lower, upper, -log(upper-lower)              prior.py:9-68    */
#define RVK_PRIOR_ECC_UNIFORM   1  /* upper, -log(upper)                            prior.py:71-125  */
#define RVK_PRIOR_NORMAL        2  /* mean, std, 0.5*log(std^2*2*pi)                prior.py:128-175 */
#define RVK_PRIOR_TRUNCNORM     3  /* mean, std, lower, upper, log(sqrt(2 pi)),
                                      log_gauss_mass(a, b), log(std)                prior.py:178-249 */
#define RVK_PRIOR_HALFNORMAL    4  /* std, log(std), 0.5*log(2/pi)                  prior.py:252-306 */
#define RVK_PRIOR_RAYLEIGH      5  /* scale, log(scale)                             prior.py:309-362 */
#define RVK_PRIOR_VANEYLEN19    6  /* sigma_n, log sigma_n, sigma_r, log sigma_r,
                                      1-f, f, 0.5*log(2/pi)                         prior.py:365-443 */
#define RVK_PRIOR_BETA          7  /* a, b, log B(a, b)                             prior.py:446-511 */

/* Source of a prior slot's value: src >= 0 is a column of the full theta row
 * (rvk.h layout); src < 0 is -(1 + 5*p + j): default parameter j (0..4 = P, K,
 * e, w, Tp) of planet p converted from the handle's parameterisation (ravest's
 * Case 3, fit.py:3418-3446; a conversion ValueError rejects the walker). */
#define RVK_PRIOR_SRC_DEFAULT(p, j) (-(1 + 5 * (p) + (j)))

typedef struct rvk_post rvk_post;

/* Convert every planet to the default parameterisation before the priors and
 * reject the walker where that raises -- ravest does this whenever the prior
 * keys differ from the free parameters (fit.py:3418-3446), even if no prior
 * reads a converted value. */
#define RVK_POST_CONVERT 1

/* free_idx[n_free]: full-row column of each free parameter, in emcee's
 * coordinate order (free_params_names); full_template[P_full]: fixed values
 * (free columns are ignored).  Slots (prior_kind/prior_src[n_prior],
 * prior_par[n_prior][RVK_PRIOR_NPAR]) are summed in the given order (the
 * reference's dict order).  log_jacobian and log_renorm are the constant
 * corrections of fit.py:3306-3397.  The handle must outlive the posterior. */
rvk_post *rvk_post_create(rvk_handle *h, int32_t n_free, const int32_t *free_idx,
                          const double *full_template, int32_t n_prior,
                          const int32_t *prior_kind, const int32_t *prior_src,
                          const double *prior_par, double log_jacobian, double log_renorm,
                          int32_t flags);
void rvk_post_destroy(rvk_post *p);

/* Pre-size the workspace for up to max_walkers per call (no allocation inside
 * a captured HIP graph afterwards). */
int rvk_post_reserve(rvk_post *p, int64_t max_walkers);

/* out[w] = log-posterior of free row w ([W][row_stride], n_free used): -inf
 * exactly where the reference returns -inf, NaN where it returns NaN. */
int rvk_logpost_device(rvk_post *p, const double *d_free, int64_t n_walkers, int64_t row_stride,
                       double *d_out, void *stream);
int rvk_logpost(rvk_post *p, const double *free, int64_t n_walkers, int64_t row_stride, double *out);

/* RedBlueMove(randomize_split=False): the halves are the even / odd walkers (emcee 3.1's
 * unshuffled `arange(W) % 2`).  Default (0): emcee's StretchMove, randomize_split=True. */
#define RVK_STRETCH_FIXED_SPLIT 1

/* Device-resident stretch move: n_steps emcee steps over the W-walker state
 * d_x[W][n_free] / d_lp[W] (updated in place; d_lp must hold the state's
 * log-posterior).  Per step, both halves in turn: proposals
 * q = c - (c - s) z, z = ((a-1) u + 1)^2 / a, log-posterior of q, accept when
 * (n_free-1) log z + lp(q) - lp(s) > log(u').
 *
 * Random numbers:
 *   d_set == NULL: counter-based Philox4x32-10 keyed by `seed`, counters = (global
 *     step step0 + step, walker / proposal index).  The split is emcee 3's
 *     randomize_split=True: per step a uniformly random balanced split of the W
 *     walkers into two halves (each half's walkers ascending, as emcee's boolean
 *     mask orders them); with RVK_STRETCH_FIXED_SPLIT the even / odd halves.  A
 *     draw depends only on (seed, global step, half, proposal), so a run split
 *     into several calls (step0 = steps done) is the same chain as one call.
 *   otherwise host-supplied draws for steps [0, n_steps), H = W/2, laid out
 *     [step][half][H]: d_set (walker indices of each half, ascending: emcee's
 *     shuffled `inds % 2` split), d_zu (u for z), d_rint (complement index in
 *     [0, H)), d_au (u' for the acceptance).  Drawn in emcee's call order these
 *     reproduce emcee's chain for the same seed (flags ignored).
 * d_chain[n_steps][W][n_free] and d_lnp[n_steps][W] (either may be NULL) get
 * every step's state; d_naccepted[W] (int64, may be NULL) counts acceptances;
 * *d_status |= 1 if a NaN log-posterior was met (emcee raises ValueError).
 * Stream-ordered on `stream`. */
int rvk_stretch_run(rvk_post *p, double *d_x, double *d_lp, int64_t n_walkers, int32_t n_steps,
                    double a, uint64_t seed, uint64_t step0, int32_t flags, const int32_t *d_set,
                    const double *d_zu, const int32_t *d_rint, const double *d_au,
                    double *d_chain, double *d_lnp, int64_t *d_naccepted, int32_t *d_status,
                    void *stream);

/* The same stretch move split for several GPUs (ravest_amd.distributed.ShardedDeviceSampler;
 * ravest's pool.map over walkers, fit.py:1068-1075).  Every rank holds the whole state; per
 * half-step each rank evaluates only a slice of the proposals, the H per-proposal
 * log-posteriors are all-gathered (the one exchange: H doubles), and every rank applies the
 * accept / reject to the whole half itself.  The chain equals rvk_stretch_run's bit for bit.
 *
 *   rvk_stretch_draws    the Philox draws of steps [step0, step0 + n_steps) into the
 *                        posterior's draw table (same draws as rvk_stretch_run's);
 *   rvk_stretch_propose  d_out[count] = log-posterior of proposals [j0, j0 + count) of
 *                        (table step s, half) -- q = c - (c - s) z from the state d_x;
 *   rvk_stretch_update   accept / reject of all W/2 proposals of (s, half) given their
 *                        log-posteriors d_nlp[W/2]; updates d_x, d_lp; writes the half's
 *                        walkers into d_chain_step[W][n_free] / d_lnp_step[W] (the step's
 *                        chain rows; either may be NULL) and their acceptance counts
 *                        d_nacc_out[w] = d_nacc_in[w] + accepted (equal pointers: a running
 *                        count; separate ones: per-step counts; both may be NULL);
 *                        *d_status |= 1 on NaN.
 * Stream-ordered; rvk_stretch_run overwrites the draw table. */
int rvk_stretch_draws(rvk_post *p, int64_t n_walkers, int32_t n_steps, double a, uint64_t seed, uint64_t step0,
                      int32_t flags, void *stream);
int rvk_stretch_propose(rvk_post *p, const double *d_x, int64_t n_walkers, int32_t s, int32_t half, int64_t j0,
                        int64_t count, double *d_out, void *stream);
/* Copy `bytes` (a multiple of 16, 16-byte aligned) from device memory to pinned host memory
 * with `workgroups` workgroups (1..1024), stream-ordered: how the samplers stream each finished
 * chunk of the chain out over PCIe beside the running chunk without a full-grid copy kernel. */
int rvk_copy_to_host(const void *d_src, void *h_dst, int64_t bytes, int32_t workgroups, void *stream);

/* Diagnostics: the drawn table's (walker, complement, z) of the W/2 proposals of (s, half), into
 * host buffers (blocking; synchronises the device). */
int rvk_stretch_table_read(rvk_post *p, int32_t s, int32_t half, int64_t *walker, int64_t *complement, double *z);
int rvk_stretch_update(rvk_post *p, double *d_x, double *d_lp, int64_t n_walkers, int32_t s, int32_t half,
                       const double *d_nlp, double *d_chain_step, double *d_lnp_step, const int64_t *d_nacc_in,
                       int64_t *d_nacc_out, int32_t *d_status, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* RVK_POST_H */
