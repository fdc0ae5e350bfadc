// rvk_post.hip -- device log-posterior and device-resident stretch move
// (include/rvk_post.h).
//
// One thread per walker builds the full theta row (fixed template + free
// coordinates), checks the jitters, converts to the default parameterisation
// where the priors need it, sums the built-in priors and writes the row plus
// its log-prior.  The log-likelihood kernel (rvk.hip) then runs on those rows
// with its posterior epilogue (a rejected walker skips its epoch loop; the
// others get ((ll + lp) + jac) + renorm).  The sampler adds the stretch-move
// proposal in front of that (same thread) and an accept kernel behind it;
// all state stays in HBM between steps.
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/rvk_post.h"
#include "rvk_internal.h"

using namespace rvk;

namespace {

struct PriorSlot {
    int32_t kind, src;
    double p[RVK_PRIOR_NPAR];
};

struct PostDev {
    int n_free, p_full, n_prior, n_planets, n_inst, par;
    bool convert;                // convert every planet to P K e w Tp first (RVK_POST_CONVERT or a src < 0)
    const int32_t *colmap;       // [p_full]: free position of a column, or -1 (fixed)
    const double *tmpl;          // [p_full]
    const PriorSlot *slots;      // [n_prior]
};

// scipy.stats halfnorm / rayleigh logpdf as scipy evaluates them (x >= 0):
// _logpdf(x / scale) - log(scale)
__device__ __forceinline__ double halfnorm_lp(double x, double scale, double log_scale, double c) {
    const double y = x / scale;
    return (c - y * y / 2.0) - log_scale;                  // 0.5*log(2/pi) - x*x/2.0
}
__device__ __forceinline__ double rayleigh_lp(double x, double scale, double log_scale) {
    const double y = x / scale;
    return (log(y) - 0.5 * y * y) - log_scale;             // log(r) - 0.5 * r * r
}

// One prior term, the reference's formula and bounds (prior.py).
__device__ double prior_lp(const PriorSlot &s, double x) {
    const double *p = s.p;
    switch (s.kind) {
        case RVK_PRIOR_UNIFORM:
            return (x < p[0] || x > p[1]) ? -INFINITY : p[2];
        case RVK_PRIOR_ECC_UNIFORM:
            return (x < 0.0 || x >= p[0]) ? -INFINITY : p[1];
        case RVK_PRIOR_NORMAL: {
            const double y = (x - p[0]) / p[1];
            return -0.5 * (y * y) - p[2];
        }
        case RVK_PRIOR_TRUNCNORM: {                      // scipy truncnorm.logpdf inside the bounds
            if (x < p[2] || x > p[3]) return -INFINITY;
            const double y = (x - p[0]) / p[1];
            return ((-(y * y) / 2.0 - p[4]) - p[5]) - p[6];
        }
        case RVK_PRIOR_HALFNORMAL:
            if (x < 0.0) return -INFINITY;
            return halfnorm_lp(x, p[0], p[1], p[2]);
        case RVK_PRIOR_RAYLEIGH:
            if (x < 0.0) return -INFINITY;
            return rayleigh_lp(x, p[0], p[1]);
        case RVK_PRIOR_VANEYLEN19: {                     // scipy 1.15 logsumexp([hn, ry], b=[1-f, f])
            if (x < 0.0) return -INFINITY;
            const double b0 = p[4], b1 = p[5];
            double a0 = halfnorm_lp(x, p[0], p[1], p[6]), a1 = rayleigh_lp(x, p[2], p[3]);
            if (b0 == 0.0) a0 = -INFINITY;
            if (b1 == 0.0) a1 = -INFINITY;
            const double amax = (isnan(a0) || isnan(a1)) ? NAN : fmax(a0, a1);
            const bool m0 = a0 == amax, m1 = a1 == amax;
            const double m = b0 * (m0 ? 1.0 : 0.0) + b1 * (m1 ? 1.0 : 0.0);
            const double shift = isfinite(amax) ? amax : 0.0;
            double sum = b0 * exp((m0 ? -INFINITY : a0) - shift) + b1 * exp((m1 ? -INFINITY : a1) - shift);
            sum = (sum == 0.0) ? sum : sum / m;
            return (log1p(sum) + log(m)) + amax;
        }
        case RVK_PRIOR_BETA: {                           // xlogy(a-1, x) + xlog1py(b-1, -x) - log B
            if (x < 0.0 || x > 1.0) return -INFINITY;
            const double am1 = p[0] - 1.0, bm1 = p[1] - 1.0;
            const double t1 = (am1 == 0.0 && !isnan(x)) ? 0.0 : am1 * log(x);
            const double t2 = (bm1 == 0.0 && !isnan(x)) ? 0.0 : bm1 * log1p(-x);
            return (t1 + t2) - p[2];
        }
        default:
            return NAN;
    }
}

// ---- Philox4x32-10 (counter-based; Salmon et al. 2011) -------------------------------
__device__ __forceinline__ uint4 philox(uint4 c, uint2 k) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
        c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
        k.x += 0x9E3779B9u;
        k.y += 0xBB67AE85u;
    }
    return c;
}
// 53-bit uniform in [0, 1) from two words (numpy's construction)
__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

// Draws of one (step, half, walker-in-half).
struct Draw {
    long long s, c;     // active walker, complementary walker
    double zu, au;
};

struct RngArgs {
    const int32_t *set;   // [steps][2][H] or nullptr (Philox)
    const double *zu;
    const int32_t *rint;
    const double *au;
    uint64_t seed, step0;
};

__device__ __forceinline__ Draw draw(const RngArgs &r, int step, int half, long long j, long long H) {
    Draw d;
    if (r.set) {
        const long long o = ((long long)step * 2 + half) * H + j;
        const long long ob = ((long long)step * 2 + (1 - half)) * H;
        d.s = r.set[o];
        d.c = r.set[ob + r.rint[o]];
        d.zu = r.zu[o];
        d.au = r.au[o];
    } else {
        const uint64_t st = r.step0 + (uint64_t)step;
        const uint2 key = make_uint2((uint32_t)r.seed, (uint32_t)(r.seed >> 32));
        const uint4 a = philox(make_uint4((uint32_t)j, (uint32_t)half, (uint32_t)st, (uint32_t)(st >> 32)), key);
        const uint4 b = philox(make_uint4((uint32_t)j, (uint32_t)half | 2u, (uint32_t)st, (uint32_t)(st >> 32)), key);
        d.s = (long long)half * H + j;
        // complement index in [0, H): multiply-shift (bias <= H / 2^32)
        d.c = (long long)(1 - half) * H + (long long)(((uint64_t)b.x * (uint64_t)H) >> 32);
        d.zu = u53(a.x, a.y);
        d.au = u53(a.z, a.w);
    }
    return d;
}

// Per-walker prologue: x (n_free coordinates) -> full row + log-prior.
__device__ void post_row(const PostDev &pd, const double *x, double *full, double *lp_out) {
    for (int c = 0; c < pd.p_full; ++c) {
        const int f = pd.colmap[c];
        full[c] = f >= 0 ? x[f] : pd.tmpl[c];
    }
    bool dead = false;
    const int jit0 = 5 * pd.n_planets + pd.n_inst;
    for (int k = 0; k < pd.n_inst; ++k) dead |= full[jit0 + k] < 0.0;   // fit.py:3465-3468
    double def[RVK_MAX_PLANETS][5];
    if (pd.convert) {                                                   // fit.py:3426-3444
        for (int p = 0; p < pd.n_planets; ++p) {
            const bool ok = to_default_t<-1>(full + 5 * p, def[p][0], def[p][1], def[p][2], def[p][3], def[p][4],
                                             pd.par);
            dead |= !ok;                                                // ValueError -> -inf
        }
    }
    double lp = 0.0;                                                    // fit.py:3684-3691
    for (int k = 0; k < pd.n_prior; ++k) {
        const PriorSlot &s = pd.slots[k];
        double v;
        if (s.src >= 0) {
            v = full[s.src];
        } else {
            const int q = -s.src - 1;
            v = def[q / 5][q % 5];
        }
        lp += prior_lp(s, v);
    }
    if (!isfinite(lp)) dead = true;                                     // fit.py:3481-3482
    *lp_out = dead ? -INFINITY : lp;
}

__global__ __launch_bounds__(256) void logprior_kernel(PostDev pd, const double *__restrict__ xf, long long W,
                                                       long long stride, double *__restrict__ full,
                                                       double *__restrict__ lp) {
    const long long w = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    post_row(pd, xf + w * stride, full + w * pd.p_full, lp + w);
}

// Stretch-move proposal for the walkers of one half (emcee StretchMove.get_proposal):
// q = c - (c - s) * z, z = ((a - 1) u + 1)^2 / a, factor = (ndim - 1) log z.
__global__ __launch_bounds__(256) void propose_kernel(PostDev pd, RngArgs rng, int step, int half, long long H,
                                                      double a, const double *__restrict__ x,
                                                      double *__restrict__ q, double *__restrict__ full,
                                                      double *__restrict__ lp, double *__restrict__ fac) {
    const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= H) return;
    const Draw d = draw(rng, step, half, j, H);
    const double zt = (a - 1.0) * d.zu + 1.0;
    const double z = zt * zt / a;
    const int D = pd.n_free;
    const double *xs = x + d.s * D, *xc = x + d.c * D;
    double *qj = q + j * D;
    for (int k = 0; k < D; ++k) qj[k] = xc[k] - (xc[k] - xs[k]) * z;
    fac[j] = ((double)D - 1.0) * log(z);
    post_row(pd, qj, full + j * pd.p_full, lp + j);
}

// Accept / reject (RedBlueMove.propose + update) and the chain write of the half.
__global__ __launch_bounds__(256) void accept_kernel(RngArgs rng, int step, int half, long long H, int D,
                                                     const double *__restrict__ q, const double *__restrict__ fac,
                                                     const double *__restrict__ nlp_all, double *__restrict__ x,
                                                     double *__restrict__ lp, long long *__restrict__ nacc,
                                                     double *__restrict__ chain, double *__restrict__ lnpc,
                                                     int *__restrict__ status) {
    const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= H) return;
    const Draw d = draw(rng, step, half, j, H);
    const double nlp = nlp_all[j];
    if (isnan(nlp)) atomicOr(status, 1);
    const double lnpdiff = fac[j] + nlp - lp[d.s];
    double *xs = x + d.s * D;
    if (lnpdiff > log(d.au)) {
        for (int k = 0; k < D; ++k) xs[k] = q[j * D + k];
        lp[d.s] = nlp;
        if (nacc) nacc[d.s] += 1;
    }
    if (chain)
        for (int k = 0; k < D; ++k) chain[d.s * D + k] = xs[k];
    if (lnpc) lnpc[d.s] = lp[d.s];
}

unsigned blocks_for(long long n) { return (unsigned)((n + 255) / 256); }

}  // namespace

struct rvk_post {
    rvk_handle *h = nullptr;
    int n_free = 0, n_prior = 0;
    bool convert = false;
    double jac = 0.0, renorm = 0.0;
    int32_t *d_colmap = nullptr;
    double *d_tmpl = nullptr;
    PriorSlot *d_slots = nullptr;
    // workspace, sized for cap walkers
    long long cap = 0;
    double *d_full = nullptr, *d_lp = nullptr, *d_q = nullptr, *d_fac = nullptr, *d_nlp = nullptr;

    PostDev dev() const {
        return PostDev{n_free, h->p_full(), n_prior, h->n_planets, h->n_inst, h->par, convert, d_colmap, d_tmpl,
                       d_slots};
    }
};

static void free_post(rvk_post *p) {
    if (!p) return;
    if (p->h) (void)hipSetDevice(p->h->device);
    (void)hipFree(p->d_colmap);
    (void)hipFree(p->d_tmpl);
    (void)hipFree(p->d_slots);
    (void)hipFree(p->d_full);
    (void)hipFree(p->d_lp);
    (void)hipFree(p->d_q);
    (void)hipFree(p->d_fac);
    (void)hipFree(p->d_nlp);
    delete p;
}

static int reserve_impl(rvk_post *p, long long W) {
    if (W <= p->cap) return RVK_OK;
    HIPCHK(hipSetDevice(p->h->device));
    (void)hipFree(p->d_full);
    (void)hipFree(p->d_lp);
    (void)hipFree(p->d_q);
    (void)hipFree(p->d_fac);
    (void)hipFree(p->d_nlp);
    p->d_full = p->d_lp = p->d_q = p->d_fac = p->d_nlp = nullptr;
    p->cap = 0;
    const size_t w = (size_t)W;
    HIPCHK(hipMalloc(&p->d_full, sizeof(double) * w * (size_t)p->h->p_full()));
    HIPCHK(hipMalloc(&p->d_lp, sizeof(double) * w));
    HIPCHK(hipMalloc(&p->d_q, sizeof(double) * w * (size_t)(p->n_free > 0 ? p->n_free : 1)));
    HIPCHK(hipMalloc(&p->d_fac, sizeof(double) * w));
    HIPCHK(hipMalloc(&p->d_nlp, sizeof(double) * w));
    p->cap = W;
    return RVK_OK;
}

static int create_post(rvk_post *p, rvk_handle *h, int32_t n_free, const int32_t *free_idx, const double *tmpl,
                       int32_t n_prior, const int32_t *kind, const int32_t *src, const double *par, double jac,
                       double renorm, int32_t flags) {
    if (!h) return fail(RVK_E_ARG, "NULL handle");
    if (h->n < 1) return fail(RVK_E_ARG, "model-only handle (n_epochs = 0) cannot evaluate a posterior");
    const int pf = h->p_full();
    if (n_free < 1 || n_free > pf || !free_idx || !tmpl) return fail(RVK_E_ARG, "bad free-parameter layout");
    if (n_prior < 0 || (n_prior > 0 && (!kind || !src || !par))) return fail(RVK_E_ARG, "bad prior arrays");
    std::vector<int32_t> colmap(pf, -1);
    for (int i = 0; i < n_free; ++i) {
        if (free_idx[i] < 0 || free_idx[i] >= pf) return fail(RVK_E_ARG, "free_idx out of range");
        if (colmap[free_idx[i]] >= 0) return fail(RVK_E_ARG, "free_idx has a duplicate column");
        colmap[free_idx[i]] = i;
    }
    std::vector<PriorSlot> slots(n_prior);
    if (flags & ~RVK_POST_CONVERT) return fail(RVK_E_ARG, "unknown flags");
    bool convert = (flags & RVK_POST_CONVERT) != 0;
    for (int k = 0; k < n_prior; ++k) {
        if (kind[k] < RVK_PRIOR_UNIFORM || kind[k] > RVK_PRIOR_BETA) return fail(RVK_E_ARG, "unknown prior kind");
        if (src[k] >= pf) return fail(RVK_E_ARG, "prior source column out of range");
        if (src[k] < 0 && -src[k] - 1 >= 5 * h->n_planets) return fail(RVK_E_ARG, "prior source planet out of range");
        convert |= src[k] < 0;
        slots[k].kind = kind[k];
        slots[k].src = src[k];
        std::memcpy(slots[k].p, par + (size_t)k * RVK_PRIOR_NPAR, sizeof(double) * RVK_PRIOR_NPAR);
    }
    p->h = h;
    p->n_free = n_free;
    p->n_prior = n_prior;
    p->convert = convert;
    p->jac = jac;
    p->renorm = renorm;
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipMalloc(&p->d_colmap, sizeof(int32_t) * pf));
    HIPCHK(hipMalloc(&p->d_tmpl, sizeof(double) * pf));
    HIPCHK(hipMalloc(&p->d_slots, sizeof(PriorSlot) * (n_prior > 0 ? n_prior : 1)));
    HIPCHK(hipMemcpy(p->d_colmap, colmap.data(), sizeof(int32_t) * pf, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(p->d_tmpl, tmpl, sizeof(double) * pf, hipMemcpyHostToDevice));
    if (n_prior > 0)
        HIPCHK(hipMemcpy(p->d_slots, slots.data(), sizeof(PriorSlot) * n_prior, hipMemcpyHostToDevice));
    return RVK_OK;
}

extern "C" {

rvk_post *rvk_post_create(rvk_handle *h, int32_t n_free, const int32_t *free_idx, const double *full_template,
                          int32_t n_prior, const int32_t *prior_kind, const int32_t *prior_src,
                          const double *prior_par, double log_jacobian, double log_renorm, int32_t flags) {
    rvk_post *p = new (std::nothrow) rvk_post();
    if (!p) {
        fail(RVK_E_NOMEM, "out of host memory");
        return nullptr;
    }
    if (create_post(p, h, n_free, free_idx, full_template, n_prior, prior_kind, prior_src, prior_par, log_jacobian,
                    log_renorm, flags)) {
        free_post(p);
        return nullptr;
    }
    return p;
}

void rvk_post_destroy(rvk_post *p) { free_post(p); }

int rvk_post_reserve(rvk_post *p, int64_t max_walkers) {
    if (!p || max_walkers < 0) return fail(RVK_E_ARG, "bad arguments");
    return reserve_impl(p, max_walkers);
}

int rvk_logpost_device(rvk_post *p, const double *d_free, int64_t W, int64_t stride, double *d_out, void *stream) {
    if (!p) return fail(RVK_E_ARG, "NULL posterior");
    if (W < 0 || stride < p->n_free) return fail(RVK_E_ARG, "bad walker block shape");
    if (W == 0) return RVK_OK;
    if (!d_free || !d_out) return fail(RVK_E_ARG, "NULL device buffer");
    int rc = reserve_impl(p, W);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    rvk_handle *h = p->h;
    HIPCHK(hipSetDevice(h->device));
    hipLaunchKernelGGL(logprior_kernel, dim3(blocks_for(W)), dim3(256), 0, st, p->dev(), d_free, (long long)W,
                       (long long)stride, p->d_full, p->d_lp);
    h->launch(st, h->epochs(), h->n, h->n_inst, p->d_full, W, h->p_full(), d_out, PostArgs{p->d_lp, p->jac, p->renorm});
    HIPCHK(hipGetLastError());
    return RVK_OK;
}

int rvk_logpost(rvk_post *p, const double *xf, int64_t W, int64_t stride, double *out) {
    if (!p) return fail(RVK_E_ARG, "NULL posterior");
    if (W < 0 || stride < p->n_free) return fail(RVK_E_ARG, "bad walker block shape");
    if (W == 0) return RVK_OK;
    if (!xf || !out) return fail(RVK_E_ARG, "NULL host buffer");
    rvk_handle *h = p->h;
    HIPCHK(hipSetDevice(h->device));
    double *d_x = nullptr, *d_o = nullptr;
    HIPCHK(hipMalloc(&d_x, sizeof(double) * (size_t)W * (size_t)stride));
    if (hipMalloc(&d_o, sizeof(double) * (size_t)W) != hipSuccess) {
        (void)hipFree(d_x);
        return fail(RVK_E_HIP, "hipMalloc failed");
    }
    int rc = RVK_OK;
    if (hipMemcpyAsync(d_x, xf, sizeof(double) * (size_t)W * (size_t)stride, hipMemcpyHostToDevice, h->stream) !=
        hipSuccess)
        rc = fail(RVK_E_HIP, "hipMemcpyAsync H2D failed");
    if (rc == RVK_OK) rc = rvk_logpost_device(p, d_x, W, stride, d_o, h->stream);
    if (rc == RVK_OK &&
        hipMemcpyAsync(out, d_o, sizeof(double) * (size_t)W, hipMemcpyDeviceToHost, h->stream) != hipSuccess)
        rc = fail(RVK_E_HIP, "hipMemcpyAsync D2H failed");
    if (hipStreamSynchronize(h->stream) != hipSuccess && rc == RVK_OK) rc = fail(RVK_E_HIP, "stream sync failed");
    (void)hipFree(d_x);
    (void)hipFree(d_o);
    return rc;
}

int rvk_stretch_run(rvk_post *p, double *d_x, double *d_lp, int64_t W, int32_t n_steps, double a, uint64_t seed,
                    uint64_t step0, const int32_t *d_set, const double *d_zu, const int32_t *d_rint,
                    const double *d_au, double *d_chain, double *d_lnp, int64_t *d_naccepted, int32_t *d_status,
                    void *stream) {
    if (!p) return fail(RVK_E_ARG, "NULL posterior");
    if (W < 4 || (W & 1)) return fail(RVK_E_ARG, "n_walkers must be even and >= 4");
    if (n_steps < 0) return fail(RVK_E_ARG, "n_steps < 0");
    if (!(a > 1.0)) return fail(RVK_E_ARG, "stretch scale a must be > 1");
    if (!d_x || !d_lp || !d_status) return fail(RVK_E_ARG, "NULL device buffer");
    if (d_set && (!d_zu || !d_rint || !d_au)) return fail(RVK_E_ARG, "host draws need set, zu, rint and au");
    if (n_steps == 0) return RVK_OK;
    const long long H = W / 2;
    int rc = reserve_impl(p, H);
    if (rc) return rc;
    rvk_handle *h = p->h;
    hipStream_t st = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    const RngArgs rng{d_set, d_zu, d_rint, d_au, seed, step0};
    const PostDev pd = p->dev();
    const int D = p->n_free;
    for (int s = 0; s < n_steps; ++s) {
        double *ch = d_chain ? d_chain + (size_t)s * (size_t)W * (size_t)D : nullptr;
        double *lc = d_lnp ? d_lnp + (size_t)s * (size_t)W : nullptr;
        for (int half = 0; half < 2; ++half) {
            hipLaunchKernelGGL(propose_kernel, dim3(blocks_for(H)), dim3(256), 0, st, pd, rng, s, half, H, a, d_x,
                               p->d_q, p->d_full, p->d_lp, p->d_fac);
            h->launch(st, h->epochs(), h->n, h->n_inst, p->d_full, H, h->p_full(), p->d_nlp,
                      PostArgs{p->d_lp, p->jac, p->renorm});
            hipLaunchKernelGGL(accept_kernel, dim3(blocks_for(H)), dim3(256), 0, st, rng, s, half, H, D, p->d_q,
                               p->d_fac, p->d_nlp, d_x, d_lp, (long long *)d_naccepted, ch, lc, (int *)d_status);
        }
    }
    HIPCHK(hipGetLastError());
    return RVK_OK;
}

}  // extern "C"
