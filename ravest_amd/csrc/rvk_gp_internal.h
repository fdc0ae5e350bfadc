// rvk_gp_internal.h -- declarations shared by the GP translation units of librvk.so
// (rvk_gp.hip: fp32 factorisation, C-ABI; rvk_gp64.hip: fp64 factorisation,
// conditioning).  Not part of the C-ABI.
#pragma once

#include "rvk_internal.h"

namespace rvk {

// The fp32 factorisation keeps a column panel of the walker's factor in LDS: up to this many
// epochs (the fp64 factorisation, its panels in the workspace, goes to RVK_GP_MAX_EPOCHS).
constexpr int kGpF32MaxEpochs = 1024;

// Optional GP log-posterior epilogue (GPLogPosterior.log_probability, fit.py:7836-7901):
// lp == nullptr: out = GP log-likelihood.  Otherwise lp[w] / lhp[w] are the walker's
// log-prior and log-hyperprior (lp[w] = -inf: rejected before the likelihood -- negative
// jitter, invalid hyperparameters, a prior-side conversion error, a non-finite prior or
// hyperprior), and out = (((ll + lp) + lhp) + jac) + renorm in the reference's order.
struct GpPost {
    const double *lp;
    const double *lhp;
    double jac, renorm;
};

// Arguments of one fp64 launch (rvk_gp64.hip).
struct Gp64Args {
    EpochData d;
    int n, ni, np;
    const double *theta, *hyper;
    long long W, stride, hstride;
    double *work;             // per-workgroup workspace: tiles of L (fragment layout)
    long long work_stride;    // doubles per workgroup
    double *out;              // [W] log-likelihood / log-posterior (LOGLIKE mode)
    const double *gate;       // if set: only walkers with isnan(gate[w]) are evaluated (fp32 fallback)
    GpPost post;
    // CONDITION mode (tinygp GaussianProcess.condition(y, X_test).mean, fit.py:7494-7554)
    const double *tq;         // [T] query times
    long long T;
    double *pred;             // [W][T] conditional mean of the GP at tq
};

typedef void (*gp64_launch_t)(hipStream_t, unsigned grid, size_t lds, const Gp64Args &);

struct Gp64Shape {
    int nw, maxr;
    bool grouped;   // more tile rows per wave than maxr (rows accumulated in groups)
};
Gp64Shape gp64_shape(int n);
size_t gp64_lds_bytes(int n, int np, int nw);
long long gp64_work_doubles(int n);        // per workgroup
// nullptr if unsupported (np outside 1..8)
gp64_launch_t pick_gp64(int np, bool multi, bool tp, bool condition, Gp64Shape sh);

}  // namespace rvk
