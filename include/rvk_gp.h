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
 * Factorisation in fp32 (BASELINE config 5 is fp32), mean model and the
 * final sums in fp64.  An invalid planet gives -inf (the reference's mean-model
 * fail-fast); a covariance that is not positive definite in fp32 gives NaN.
 * Epochs: 1 <= n_epochs <= 1024.
 *
 * hyper row layout [W][hyper_stride] fp64: gp_amp, gp_lambda_e, gp_lambda_p,
 * gp_period (GPKernel.expected_hyperparams order, gp.py:37).
 */
#ifndef RVK_GP_H
#define RVK_GP_H

#include <stdint.h>

#include "rvk.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RVK_GP_QUASIPERIODIC 0
#define RVK_GP_NHYPER        4
#define RVK_GP_MAX_EPOCHS    1024

typedef struct rvk_gp rvk_gp;

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

#ifdef __cplusplus
}
#endif
#endif /* RVK_GP_H */
