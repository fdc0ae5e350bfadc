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

constexpr int kMaxPFull = 5 * RVK_MAX_PLANETS + 2 * RVK_MAX_INST + 2;   // 290
constexpr int kMaxPFullPad = (kMaxPFull + 7) / 8 * 8;

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

// The prior kinds with a transcendental function (Rayleigh, VanEylen19Mixture, Beta).
__device__ __forceinline__ double prior_lp_trans(int kind, const double *p, double x) {
    switch (kind) {
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

// One prior term, the reference's formula and bounds (prior.py).
inline __device__ double prior_lp(const PriorSlot &s, double x) {
    if (s.kind <= kMaxBasicPriorKind) return prior_lp_basic(s.kind, s.p, x);
    return prior_lp_trans(s.kind, s.p, x);
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

// Per-call arguments of rvk_stretch_run, kept in device memory (written by a small kernel at
// the start of each chunk of steps) so that the kernels of a chunk have call-invariant
// arguments and can be replayed from a cached HIP graph.
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

// One proposal's draws, as every sampler kernel consumes them: the walker and its complement,
// z, (D - 1) log z and log u'.  Made by split_draws_kernel (device Philox) or from host draws
// (emcee's RandomState stream) by chunk_args_kernel -- the same expressions either way.
struct PreDraw {
    double z, fac, lau;
    long long s, c;
};

// StretchMove.get_proposal: z = ((a - 1) u + 1)^2 / a (emcee 3.1, moves/stretch.py)
__device__ __forceinline__ PreDraw pre_from(double zu, double au, long long s, long long c, double a, int D) {
    const double zt = (a - 1.0) * zu + 1.0;
    PreDraw p;
    p.z = zt * zt / a;
    p.fac = ((double)D - 1.0) * log(p.z);
    p.lau = log(au);
    p.s = s;
    p.c = c;
    return p;
}

// q = c - (c - s) z as one fused multiply-add (every sampler path: the proposal has the same
// bits wherever it is formed -- the fused half-step, propose_kernel, the sharded update).
__device__ __forceinline__ double stretch_q(double xc, double xs, double z) { return __builtin_fma(xs - xc, z, xc); }

// RedBlueMove.propose: accept when (ndim - 1) log z + lp(q) - lp(s) > log u'
__device__ __forceinline__ bool stretch_accept(double fac, double nlp, double lp_old, double lau) {
    return fac + nlp - lp_old > lau;
}

// Host-supplied draws (emcee's call order, sampler.emcee_step_draws) of (step, half, j).
__device__ __forceinline__ PreDraw make_pre_host(const RunArgs &r, int step, int half, long long j, long long H,
                                                 int D) {
    const long long o = ((long long)step * 2 + half) * H + j;
    const long long ob = ((long long)step * 2 + (1 - half)) * H;
    return pre_from(r.zu[o], r.au[o], r.set[o], r.set[ob + r.rint[o]], r.a, D);
}

// Flags of the device draws (include/rvk_post.h RVK_STRETCH_*).
constexpr int kSplitThreads = 1024;

// Block-wide exclusive prefix sum of one int per thread (blockDim.x <= 1024); `total` gets the sum.
__device__ __forceinline__ long long block_excl_scan(long long v, long long *wtot, long long &total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    long long x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const long long y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wtot[wv] = x;
    __syncthreads();
    long long before = 0;
    total = 0;
    for (int k = 0; k < nw; ++k) {
        const long long w = wtot[k];
        if (k < wv) before += w;
        total += w;
    }
    __syncthreads();   // wtot is reused by the next scan
    return before + x - v;
}

// Every draw of n steps of the stretch move, one workgroup of kSplitThreads per step (grid n):
//   * the split (emcee 3.1 RedBlueMove, randomize_split=True: inds = arange(W) % 2 shuffled,
//     half h = the walkers with inds == h, ascending): each walker gets a 32-bit Philox key and
//     half 0 is the H walkers with the smallest (key, index) -- a uniformly random balanced
//     split, found by an 8-bit radix select of the H-th smallest key and two block scans; with
//     RVK_STRETCH_FIXED_SPLIT the halves are the even / odd walkers (randomize_split=False);
//   * per proposal j of each half: u (for z), u' (acceptance) and the complement index
//     r in [0, H) (multiply-shift, bias <= H / 2^32), keyed by (j, half, global step) -- so a
//     draw does not depend on how proposals are shared out between launches or GPUs.
// table[s][half][j] = PreDraw; keys / sets are scratch [n][W].
static __global__ __launch_bounds__(kSplitThreads) void split_draws_kernel(PreDraw *__restrict__ table,
                                                                           uint32_t *__restrict__ keys_g,
                                                                           int32_t *__restrict__ sets_g, long long H,
                                                                           int D, uint64_t seed, uint64_t step0,
                                                                           double a, int fixed) {
    __shared__ int hist[256];
    __shared__ long long wtot[kSplitThreads / 64];
    __shared__ unsigned sh_prefix;
    __shared__ long long sh_k;
    const int s = blockIdx.x;
    const uint64_t st = step0 + (uint64_t)s;
    const long long W = 2 * H;
    const int t = threadIdx.x, nt = blockDim.x;
    const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
    int32_t *set = sets_g + (size_t)s * (size_t)W;                      // [0, H): half 0, [H, 2H): half 1
    if (fixed) {
        for (long long i = t; i < W; i += nt) set[(i & 1) * H + (i >> 1)] = (int32_t)i;
    } else {
        uint32_t *kk = keys_g + (size_t)s * (size_t)W;
        const long long C = (W + nt - 1) / nt;                           // contiguous walkers per thread
        const long long i0 = (long long)t * C, i1 = (i0 + C < W) ? i0 + C : W;
        for (long long i = i0; i < i1; ++i)
            kk[i] = philox(make_uint4((uint32_t)i, 4u, (uint32_t)st, (uint32_t)(st >> 32)), key).x;
        unsigned prefix = 0, pmask = 0;
        long long k = H;                                                 // rank (1-based) of the threshold
        for (int pass = 0; pass < 4; ++pass) {
            const int shift = 24 - 8 * pass;
            for (int b = t; b < 256; b += nt) hist[b] = 0;
            __syncthreads();
            for (long long i = i0; i < i1; ++i) {
                const uint32_t u = kk[i];
                if ((u & pmask) == prefix) atomicAdd(&hist[(u >> shift) & 255u], 1);
            }
            __syncthreads();
            if (t < 64) {                                                // lane l: bins 4l .. 4l + 3
                const int c0 = hist[4 * t], c1 = hist[4 * t + 1], c2 = hist[4 * t + 2], c3 = hist[4 * t + 3];
                long long x = (long long)c0 + c1 + c2 + c3;
                const long long own = x;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const long long y = __shfl_up(x, d, 64);
                    if (t >= d) x += y;
                }
                long long ex = x - own;                                  // keys in bins below 4l
                if (ex < k && k <= x) {                                  // exactly one lane
                    int dig = 4 * t;
                    const int cs[4] = {c0, c1, c2, c3};
                    for (int q = 0; q < 4; ++q) {
                        if (k <= ex + cs[q]) {
                            dig = 4 * t + q;
                            break;
                        }
                        ex += cs[q];
                    }
                    sh_prefix = prefix | ((unsigned)dig << shift);
                    sh_k = k - ex;
                }
            }
            __syncthreads();
            prefix = sh_prefix;
            k = sh_k;
            pmask |= 255u << shift;
            __syncthreads();
        }
        // half 0 = keys < T, plus the first k (by index) of the keys == T
        const uint32_t T = prefix;
        long long neq = 0;
        for (long long i = i0; i < i1; ++i) neq += kk[i] == T;
        long long tot;
        const long long eq0 = block_excl_scan(neq, wtot, tot);
        long long nin = 0, r = eq0;
        for (long long i = i0; i < i1; ++i) {
            const uint32_t u = kk[i];
            if (u < T) ++nin;
            else if (u == T) nin += (r++ < k);
        }
        long long m = block_excl_scan(nin, wtot, tot);                  // walkers of half 0 before i0
        r = eq0;
        for (long long i = i0; i < i1; ++i) {
            const uint32_t u = kk[i];
            const bool in0 = u < T || (u == T && r++ < k);
            if (in0) set[m++] = (int32_t)i;
            else set[H + (i - m)] = (int32_t)i;                          // i - m = half-1 walkers before i
        }
    }
    __syncthreads();                                                     // the block's set writes
    for (long long q = t; q < W; q += nt) {
        const int half = q >= H;
        const long long j = q - (half ? H : 0);
        const uint4 ra = philox(make_uint4((uint32_t)j, (uint32_t)half, (uint32_t)st, (uint32_t)(st >> 32)), key);
        const uint4 rb = philox(make_uint4((uint32_t)j, (uint32_t)half | 2u, (uint32_t)st, (uint32_t)(st >> 32)), key);
        const long long rr = (long long)(((uint64_t)rb.x * (uint64_t)H) >> 32);
        table[((long long)s * 2 + half) * H + j] =
            pre_from(u53(ra.x, ra.y), u53(ra.z, ra.w), set[half * H + j], set[(1 - half) * H + rr], a, D);
    }
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
    const double *lau;          // [H] log of the acceptance uniforms
    const long long *sidx;      // [H] walker index of proposal w
    const RunArgs *run;         // state, chain and status pointers
    int step;                   // step within the chunk
    int half;                   // active half (fused proposals, SAMPLE >= 2)
    PostDev pd;                 // the posterior (fused proposals, SAMPLE >= 2)
    long long j0;               // the launch's proposals are j0 .. j0 + count - 1 of the half
    long long hfull;            // walkers per half (the complement's range; chain row stride / 2)
    const PreDraw *pre;         // [steps][2][hfull] the draws, indexed by (step, half, j0 + w)
    double *out;                // SAMPLE == 3: out[w] = the proposal's log-posterior (no accept / reject)
    long long qstride;          // SAMPLE & 16 (DIRECT): row stride of q, the given free coordinates
    const PreDraw *pre_next;    // the next half-step's draw row [hfull] (prefetched into L2), or nullptr
};

// Limits of the fused proposal path (loglike_kernel SAMPLE >= 2): lane c of the walker's wave
// holds coordinate c, column c of the full row and prior slot c, so each is at most a wave;
// every built-in prior kind and the prior-side conversion (Case 3) are evaluated in the prep.
constexpr int kFuseMaxD = 64;
constexpr int kFuseMaxPFull = 64;
constexpr int kFuseMaxPrior = 64;

// Out of line (atan/tan/atan2 for the Tc and secosw/sesinw forms): the prior-side conversion
// of one planet (fit.py:3418-3446) costs registers only while it runs.
__device__ __attribute__((noinline)) bool to_default_call(int par, const double *p5, double *d5) {
    return to_default_t<-1>(p5, d5[0], d5[1], d5[2], d5[3], d5[4], par);
}

// Accept / reject (RedBlueMove.propose + update) and the chain write of the half, for the
// unfused path (reference solver) and the GP sampler: one thread per proposal.
static __global__ __launch_bounds__(256) void stretch_accept_kernel(const RunArgs *__restrict__ runp, int step, long long H, int D,
                                                     const double *__restrict__ q, const double *__restrict__ fac,
                                                     const double *__restrict__ lau,
                                                     const long long *__restrict__ sidx,
                                                     const double *__restrict__ nlp_all) {
    const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= H) return;
    const RunArgs &run = *runp;
    const long long s = sidx[j];
    const double nlp = nlp_all[j];
    if (isnan(nlp)) atomicOr(run.status, 1);
    double *xs = run.x + s * D;
    if (stretch_accept(fac[j], nlp, run.lp[s], lau[j])) {
        for (int k = 0; k < D; ++k) xs[k] = q[j * D + k];
        run.lp[s] = nlp;
        if (run.nacc) run.nacc[s] += 1;
    }
    if (run.chain)
        for (int k = 0; k < D; ++k) run.chain[((long long)step * 2 * H + s) * D + k] = xs[k];
    if (run.lnpc) run.lnpc[(long long)step * 2 * H + s] = run.lp[s];
}

// The multi-GPU half-step's second part (rvk_stretch_update): every rank holds the log-posteriors
// of ALL H proposals of the half (all-gathered) and applies the accept / reject to the whole half
// itself, re-forming each proposal from the draws and the (replicated) state exactly as the
// fused half-step forms it.  One thread per proposal.
static __global__ __launch_bounds__(256) void stretch_update_kernel(const PreDraw *__restrict__ pre, long long H, int D,
                                                                    double *__restrict__ x, double *__restrict__ lp,
                                                                    const double *__restrict__ nlp_all,
                                                                    const long long *nacc_in, long long *nacc_out,
                                                                    int *__restrict__ status, double *__restrict__ chain,
                                                                    double *__restrict__ lnpc) {
    const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= H) return;
    const PreDraw p = pre[j];
    const double nlp = nlp_all[j];
    if (isnan(nlp)) atomicOr(status, 1);
    double *xs = x + p.s * D;
    const double *xc = x + p.c * D;
    const bool acc = stretch_accept(p.fac, nlp, lp[p.s], p.lau);
    for (int k = 0; k < D; ++k) {
        const double v = acc ? stretch_q(xc[k], xs[k], p.z) : xs[k];
        if (acc) xs[k] = v;
        if (chain) chain[p.s * D + k] = v;
    }
    if (acc) lp[p.s] = nlp;
    if (nacc_out) nacc_out[p.s] = nacc_in[p.s] + (acc ? 1 : 0);   // in == out: a running count
    if (lnpc) lnpc[p.s] = lp[p.s];
}

static __global__ void set_run_kernel(RunArgs *dst, RunArgs v) { *dst = v; }

// Host-supplied draws (emcee's RandomState stream, RunArgs v.set / zu / rint / au for the block's
// n steps) into the draw table the sampler kernels read: one thread per proposal.
static __global__ __launch_bounds__(256) void host_draws_kernel(PreDraw *__restrict__ tab, RunArgs v, int n,
                                                                long long H, int D) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)n * 2 * H) return;
    const long long sh = i / H;
    tab[i] = make_pre_host(v, (int)(sh >> 1), (int)(sh & 1), i - sh * H, H, D);
}


}  // namespace rvk
