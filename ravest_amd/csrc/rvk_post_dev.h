// rvk_post_dev.h -- device pieces of the log-posterior and the stretch move, shared by
// the stand-alone posterior kernels (rvk_post.hip) and the fused sampler mode of the
// log-likelihood kernel (rvk.hip).  Not part of the C-ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../include/rvk_post.h"
#include "rvk_math.h"

namespace rvk {

constexpr int kMaxPFull = 5 * RVK_MAX_PLANETS + 2 * RVK_MAX_INST + 2;   // 74
constexpr int kMaxPFullPad = 80;

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

// The prior kinds whose log-density needs no transcendental function (Uniform,
// EccentricityUniform, Normal, TruncatedNormal, HalfNormal: their logs are host constants);
// the fused sampler (loglike_kernel SAMPLE == 2) evaluates these inline.
constexpr int kMaxBasicPriorKind = RVK_PRIOR_HALFNORMAL;
__device__ __forceinline__ double prior_lp_basic(int kind, const double *p, double x) {
    switch (kind) {
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
        default:
            return NAN;
    }
}

// One prior term, the reference's formula and bounds (prior.py).
inline __device__ double prior_lp(const PriorSlot &s, double x) {
    const double *p = s.p;
    if (s.kind <= kMaxBasicPriorKind) return prior_lp_basic(s.kind, p, x);
    switch (s.kind) {
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

// Per-call arguments of rvk_stretch_run, kept in device memory (written by a one-thread
// kernel at the start of each chunk of steps) so that the kernels of a chunk have
// call-invariant arguments and can be replayed from a cached HIP graph.
struct RunArgs {
    double *x;            // [W][D] walker state (in/out)
    double *lp;           // [W]
    long long *nacc;      // [W] or nullptr
    int *status;
    double *chain;        // this chunk's first step [W][D] or nullptr
    double *lnpc;         // this chunk's first step [W] or nullptr
    const int32_t *set;   // host draws for this chunk's steps [step][2][H], or nullptr (Philox)
    const double *zu;
    const int32_t *rint;
    const double *au;
    uint64_t seed, step0; // Philox key, global step of the chunk's first step
    double a;
};

__device__ __forceinline__ Draw draw(const RunArgs &r, int step, int half, long long j, long long H) {
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

// One proposal's draws as the fused half-step uses them, precomputed for a chunk of steps by
// set_run_draws_kernel: the walker and its complement, z, (D - 1) log z and log u'.  The same
// expressions as the fused kernel's in-kernel path (make_pre), so either gives the same bits.
struct PreDraw {
    double z, fac, lau;
    long long s, c;
};

__device__ __forceinline__ PreDraw make_pre(const RunArgs &r, int step, int half, long long j, long long H, int D) {
    const Draw dr = draw(r, step, half, j, H);
    const double zt = (r.a - 1.0) * dr.zu + 1.0;
    PreDraw p;
    p.z = zt * zt / r.a;
    p.fac = ((double)D - 1.0) * log(p.z);
    p.lau = log(dr.au);
    p.s = dr.s;
    p.c = dr.c;
    return p;
}

// Per-walker prologue, one wave per walker: x (n_free coordinates, in LDS `lx`)
// -> full row (LDS `lf` and global `full`) and the log-prior, which is returned
// in every lane.  Lanes work over columns, planets and prior slots; the slot
// terms are then summed by one lane in the reference's key order (fit.py:3684-3691).
struct PostWaveLds {
    double x[kMaxPFullPad];
    double f[kMaxPFullPad];
    double def[5 * RVK_MAX_PLANETS];
    double term[kMaxPFullPad];
};

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The posterior's per-lane constants for one row (column c = lane: its free position and
// fixed value; prior slot k = lane), when p_full <= 64 and n_prior <= 64: loaded once per
// kernel by row_pre() so their latency is off each proposal's dependent chain.
struct RowPre {
    bool on;
    int f;
    double t;
    PriorSlot s;
};

inline __device__ RowPre row_pre(const PostDev &pd) {
    const int lane = threadIdx.x & 63;
    RowPre r{};
    r.on = pd.p_full <= 64 && pd.n_prior <= 64;
    r.f = -1;
    if (r.on) {
        if (lane < pd.p_full) {
            r.f = pd.colmap[lane];
            r.t = pd.tmpl[lane];
        }
        if (lane < pd.n_prior) r.s = pd.slots[lane];
    }
    return r;
}

inline __device__ double post_row_wave(const PostDev &pd, PostWaveLds &L, double *__restrict__ full,
                                       const RowPre &pre = RowPre{}) {
    const int lane = threadIdx.x & 63;
    if (pre.on) {
        if (lane < pd.p_full) {
            const double v = pre.f >= 0 ? L.x[pre.f] : pre.t;
            L.f[lane] = v;
            full[lane] = v;
        }
    } else {
        for (int c = lane; c < pd.p_full; c += 64) {
            const int f = pd.colmap[c];
            const double v = f >= 0 ? L.x[f] : pd.tmpl[c];
            L.f[c] = v;
            full[c] = v;
        }
    }
    wave_lds_sync();
    const int jit0 = 5 * pd.n_planets + pd.n_inst;
    bool dead = false;
    if (lane < pd.n_inst) dead = L.f[jit0 + lane] < 0.0;                         // fit.py:3465-3468
    if (pd.convert && lane < pd.n_planets) {                                       // fit.py:3426-3444
        double *dp = L.def + 5 * lane;
        const bool ok = to_default_t<-1>(L.f + 5 * lane, dp[0], dp[1], dp[2], dp[3], dp[4], pd.par);
        dead |= !ok;                                                                // ValueError -> -inf
    }
    wave_lds_sync();
    if (pre.on) {
        if (lane < pd.n_prior) {
            const double v = pre.s.src >= 0 ? L.f[pre.s.src] : L.def[-pre.s.src - 1];
            L.term[lane] = prior_lp(pre.s, v);
        }
    } else {
        for (int k = lane; k < pd.n_prior; k += 64) {
            const PriorSlot &s = pd.slots[k];
            const double v = s.src >= 0 ? L.f[s.src] : L.def[-s.src - 1];
            L.term[k] = prior_lp(s, v);
        }
    }
    wave_lds_sync();
    dead = __builtin_amdgcn_ballot_w64(dead) != 0;
    double lp = 0.0;
    for (int k = 0; k < pd.n_prior; ++k) lp += L.term[k];                          // same order, every lane
    if (!isfinite(lp)) dead = true;                                                 // fit.py:3481-3482
    return dead ? -INFINITY : lp;
}

// The accept / reject of one stretch-move half-step, fused into the epilogue of the
// log-likelihood kernel (include/rvk_post.h rvk_stretch_run).  The kernel's walker w
// is the w-th proposal of the active half (rows, log-priors from propose_kernel).
struct SampleArgs {
    int D;                      // n_free
    const double *q;            // [H][D] proposals
    const double *fac;          // [H] (ndim - 1) log z
    const double *au;           // [H] acceptance uniforms
    const long long *sidx;      // [H] walker index of proposal w
    const RunArgs *run;         // state, chain and status pointers
    int step;                   // step within the chunk
    int half;                   // active half (fused proposals, SAMPLE == 2)
    PostDev pd;                 // the posterior (fused proposals, SAMPLE == 2)
    long long j0;               // the launch's proposals are j0 .. j0 + count - 1 of the half
    long long hfull;            // walkers per half (the complement's range; chain row stride / 2)
    const PreDraw *pre;         // [steps][2][hfull] this chunk's draws, or nullptr (drawn in the kernel)
};

// Limits of the fused proposal path (loglike_kernel SAMPLE == 2): the proposal, its full row
// and the old state are staged in LDS per walker of a pass; priors basic kinds only, no
// prior-side conversion.
constexpr int kFuseMaxD = 16;
constexpr int kFuseMaxPFull = 32;
constexpr int kFuseMaxPrior = 32;

// Accept / reject (RedBlueMove.propose + update) and the chain write of the half, for the
// unfused path (reference solver) and the GP sampler: one thread per proposal.
static __global__ __launch_bounds__(256) void stretch_accept_kernel(const RunArgs *__restrict__ runp, int step, long long H, int D,
                                                     const double *__restrict__ q, const double *__restrict__ fac,
                                                     const double *__restrict__ au,
                                                     const long long *__restrict__ sidx,
                                                     const double *__restrict__ nlp_all) {
    const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= H) return;
    const RunArgs &run = *runp;
    const long long s = sidx[j];
    const double nlp = nlp_all[j];
    if (isnan(nlp)) atomicOr(run.status, 1);
    const double lnpdiff = fac[j] + nlp - run.lp[s];
    double *xs = run.x + s * D;
    if (lnpdiff > log(au[j])) {
        for (int k = 0; k < D; ++k) xs[k] = q[j * D + k];
        run.lp[s] = nlp;
        if (run.nacc) run.nacc[s] += 1;
    }
    if (run.chain)
        for (int k = 0; k < D; ++k) run.chain[((long long)step * 2 * H + s) * D + k] = xs[k];
    if (run.lnpc) run.lnpc[(long long)step * 2 * H + s] = run.lp[s];
}

static __global__ void set_run_kernel(RunArgs *dst, RunArgs v) { *dst = v; }

// The chunk's arguments plus, for the fused half-step, every proposal's draws of its n steps
// (one thread per proposal): the fused kernel then reads one PreDraw (a wave-uniform address)
// instead of running two Philox blocks on its critical path.
static __global__ __launch_bounds__(256) void set_run_draws_kernel(RunArgs *dst, RunArgs v, PreDraw *pre, int n,
                                                                   long long H, int D) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) *dst = v;
    if (i >= (long long)n * 2 * H) return;
    const long long sh = i / H;
    pre[i] = make_pre(v, (int)(sh >> 1), (int)(sh & 1), i - sh * H, H, D);
}


}  // namespace rvk
