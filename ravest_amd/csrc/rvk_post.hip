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
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/rvk_post.h"
#include "rvk_internal.h"
#include "rvk_post_dev.h"

using namespace rvk;

namespace {

// Log-prior + full rows of a walker block (rvk_logpost_device): one wave per walker.
__global__ __launch_bounds__(256) void logprior_kernel(PostDev pd, const double *__restrict__ xf, long long W,
                                                       long long stride, double *__restrict__ full,
                                                       double *__restrict__ lp) {
    __shared__ PostWaveLds lds[kWavesPerBlock];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    PostWaveLds &L = lds[wv];
    for (long long w = (long long)blockIdx.x * kWavesPerBlock + wv; w < W; w += (long long)gridDim.x * kWavesPerBlock) {
        for (int c = lane; c < pd.n_free; c += 64) L.x[c] = xf[w * stride + c];
        wave_lds_sync();
        const double v = post_row_wave(pd, L, full + w * pd.p_full);
        if (lane == 0) lp[w] = v;
        wave_lds_sync();
    }
}

// Stretch-move proposals of one half (emcee StretchMove.get_proposal), one wave per
// proposal: q = c - (c - s) z with the draws of (step, half, j0 + j) from `pre`; then its full
// row and log-prior.  The accept / reject runs in the epilogue of the log-likelihood kernel
// (SAMPLE mode) or in stretch_accept_kernel.
__global__ __launch_bounds__(256) void propose_kernel(PostDev pd, const RunArgs *__restrict__ runp,
                                                      const PreDraw *__restrict__ pre, int step, int half, long long H,
                                                      long long j0, long long hfull, double *__restrict__ q,
                                                      double *__restrict__ full, double *__restrict__ lp,
                                                      double *__restrict__ fac, double *__restrict__ lau,
                                                      long long *__restrict__ sidx) {
    __shared__ PostWaveLds lds[kWavesPerBlock];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    PostWaveLds &L = lds[wv];
    const int D = pd.n_free;
    const double *x = runp->x;
    const RowPre rp = row_pre(pd);
    for (long long j = (long long)blockIdx.x * kWavesPerBlock + wv; j < H; j += (long long)gridDim.x * kWavesPerBlock) {
        const PreDraw d = pre[((long long)step * 2 + half) * hfull + j0 + j];   // proposal j0 + j of the half
        const double *xs = x + d.s * D, *xc = x + d.c * D;
        for (int c = lane; c < D; c += 64) {
            const double v = stretch_q(xc[c], xs[c], d.z);
            L.x[c] = v;
            q[j * D + c] = v;
        }
        wave_lds_sync();
        const double v = post_row_wave(pd, L, full + j * pd.p_full, rp);
        if (lane == 0) {
            lp[j] = v;
            fac[j] = d.fac;
            lau[j] = d.lau;
            sidx[j] = d.s;
        }
        wave_lds_sync();
    }
}

// Device -> pinned host memory with a few workgroups (rvk_copy_to_host): a sampler chunk's chain
// streams out over PCIe on a handful of CUs beside the sampler's kernels, instead of a full-grid
// blit kernel competing with them for every CU.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void egress_kernel(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst,
                                                     long long n16) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long long)gridDim.x * 256)
        dst[i] = __builtin_nontemporal_load(src + i);
}

unsigned blocks_for(long long n) { return (unsigned)((n + 255) / 256); }

// one wave per item, at most 2^16 blocks (grid-stride beyond)
unsigned wave_blocks(long long n) {
    long long b = (n + kWavesPerBlock - 1) / kWavesPerBlock;
    return (unsigned)(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

}  // namespace

struct rvk_post {
    rvk_handle *h = nullptr;
    int device = -1;                       // the handle's, kept so destruction never dereferences h
    int n_free = 0, n_prior = 0;
    bool convert = false;
    bool fusable = false;                  // proposals can be made inside the likelihood kernel
    bool two_kernel = false;               // rvk_logpost_device: logprior_kernel + likelihood (RVK_LOGPOST_FUSE=0)
    int ext = 0;                           // ... 1: with a transcendental prior kind, 2: + the conversion
    double jac = 0.0, renorm = 0.0;
    int32_t *d_colmap = nullptr;
    double *d_tmpl = nullptr;
    PriorSlot *d_slots = nullptr;
    // workspace, sized for cap walkers
    long long capw = 0;
    double *d_full = nullptr, *d_lp = nullptr, *d_q = nullptr, *d_fac = nullptr, *d_nlp = nullptr, *d_lau = nullptr;
    long long *d_sidx = nullptr;
    RunArgs *d_run = nullptr;              // rvk_stretch_run's per-chunk arguments
    DrawTable tab;                         // the draws of a block of steps (split_draws_kernel / host draws)
    HostIO io;                             // rvk_logpost's host-buffer transport (RVK_OPT_HOSTIO)
    hipStream_t cap = nullptr;             // capture stream
    hipGraphExec_t graph = nullptr;        // cached block of steps (draws_block_steps(H) steps)
    long long graph_H = 0;
    const PreDraw *graph_tab = nullptr;    // the draw table the graph reads
    int graph_solver = -1;

    PostDev dev() const {
        return PostDev{n_free, h->p_full(), n_prior, h->n_planets, h->n_inst, h->par, convert, d_colmap, d_tmpl,
                       d_slots};
    }
};

// Kernels of one half-step over proposals [j0, j0 + count) of a half of hfull walkers, reading
// this chunk's RunArgs (p->d_run) and draws `pre` ([steps][2][hfull]): the proposals made and
// accepted inside the likelihood kernel (fused path), or propose_kernel + the likelihood with
// the accept / reject fused in (production solver), or + stretch_accept_kernel (reference solver).
static void enqueue_half(rvk_post *p, hipStream_t st, int s, int half, long long j0, long long count,
                         long long hfull, const PreDraw *pre, const PreDraw *pre_next = nullptr) {
    rvk_handle *h = p->h;
    const PostDev pd = p->dev();
    const PostArgs post{p->d_lp, p->jac, p->renorm};
    const bool fused = p->fusable && h->solver == 0 && h->sample_fused[p->ext];
    const long long H = count;
    if (fused) {
        const SampleArgs sa{p->n_free, nullptr, nullptr, nullptr, nullptr, p->d_run, s, half, pd, j0, hfull, pre,
                            nullptr, 0, pre_next};
        h->sample_fused[p->ext](st, h->epochs(), h->n, h->n_inst, nullptr, H, h->p_full(), post, sa);
        return;
    }
    hipLaunchKernelGGL(propose_kernel, dim3(wave_blocks(H)), dim3(256), 0, st, pd, p->d_run, pre, s, half, H, j0, hfull,
                       p->d_q, p->d_full, p->d_lp, p->d_fac, p->d_lau, p->d_sidx);
    if (h->solver == 0 && h->sample) {
        const SampleArgs sa{p->n_free, p->d_q, p->d_fac, p->d_lau, p->d_sidx, p->d_run, s, half, pd, j0, hfull, pre,
                            nullptr};
        h->sample(st, h->epochs(), h->n, h->n_inst, p->d_full, H, h->p_full(), post, sa);
    } else {
        h->launch(st, h->epochs(), h->n, h->n_inst, p->d_full, H, h->p_full(), p->d_nlp, post);
        hipLaunchKernelGGL(stretch_accept_kernel, dim3(blocks_for(H)), dim3(256), 0, st, p->d_run, s, H, p->n_free,
                           p->d_q, p->d_fac, p->d_lau, p->d_sidx, p->d_nlp);
    }
}

#ifndef RVK_PREFETCH_DRAWS
#define RVK_PREFETCH_DRAWS 0   // 1: each fused half-step touches the next half-step's draw row into L2 (measured +-0)
#endif
// Kernels of n steps (both halves, all proposals) reading the block's RunArgs and draw table.
static void enqueue_steps(rvk_post *p, hipStream_t st, long long H, int n) {
    for (int s = 0; s < n; ++s)
        for (int half = 0; half < 2; ++half) {
            // the next half-step's draws, within this block's n steps (never past the table)
            const PreDraw *next = (half == 0 || s + 1 < n) ? p->tab.block + ((long long)s * 2 + half + 1) * H : nullptr;
            enqueue_half(p, st, s, half, 0, H, H, p->tab.block, RVK_PREFETCH_DRAWS ? next : nullptr);
        }
}

// A whole block of steps (2 x draws_block_steps(H) half-step kernels) as one HIP graph, captured
// once per (H, solver, draw table) and replayed: its kernel arguments never change (everything
// per call is in d_run and the draw table), so a block is one launch.
static int ensure_graph(rvk_post *p, long long H, int steps) {
    if (p->graph && p->graph_H == H && p->graph_solver == p->h->solver && p->graph_tab == p->tab.block) return RVK_OK;
    if (p->graph) (void)hipGraphExecDestroy(p->graph);
    p->graph = nullptr;
    if (!p->cap) HIPCHK(hipStreamCreateWithFlags(&p->cap, hipStreamNonBlocking));
    hipGraph_t g = nullptr;
    HIPCHK(hipStreamBeginCapture(p->cap, hipStreamCaptureModeRelaxed));
    enqueue_steps(p, p->cap, H, steps);
    HIPCHK(hipStreamEndCapture(p->cap, &g));
    const hipError_t e = hipGraphInstantiate(&p->graph, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) {
        p->graph = nullptr;
        return fail(RVK_E_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
    }
    p->graph_H = H;
    p->graph_solver = p->h->solver;
    p->graph_tab = p->tab.block;
    return RVK_OK;
}

static void free_post(rvk_post *p) {
    if (!p) return;
    if (p->device >= 0) (void)hipSetDevice(p->device);   // never through p->h: it may be gone already
    (void)hipFree(p->d_colmap);
    (void)hipFree(p->d_tmpl);
    (void)hipFree(p->d_slots);
    (void)hipFree(p->d_full);
    (void)hipFree(p->d_lp);
    (void)hipFree(p->d_q);
    (void)hipFree(p->d_fac);
    (void)hipFree(p->d_nlp);
    (void)hipFree(p->d_lau);
    (void)hipFree(p->d_sidx);
    (void)hipFree(p->d_run);
    p->tab.release();
    p->io.release();
    if (p->graph) (void)hipGraphExecDestroy(p->graph);
    if (p->cap) (void)hipStreamDestroy(p->cap);
    delete p;
}

static int reserve_impl(rvk_post *p, long long W) {
    if (W <= p->capw) return RVK_OK;
    if (p->graph) (void)hipGraphExecDestroy(p->graph);   // it holds the old workspace pointers
    p->graph = nullptr;
    HIPCHK(hipSetDevice(p->h->device));
    (void)hipFree(p->d_full);
    (void)hipFree(p->d_lp);
    (void)hipFree(p->d_q);
    (void)hipFree(p->d_fac);
    (void)hipFree(p->d_nlp);
    (void)hipFree(p->d_lau);
    (void)hipFree(p->d_sidx);
    p->d_full = p->d_lp = p->d_q = p->d_fac = p->d_nlp = p->d_lau = nullptr;
    p->d_sidx = nullptr;
    p->capw = 0;
    const size_t w = (size_t)W;
    HIPCHK(hipMalloc(&p->d_full, sizeof(double) * w * (size_t)p->h->p_full()));
    HIPCHK(hipMalloc(&p->d_lp, sizeof(double) * w));
    HIPCHK(hipMalloc(&p->d_q, sizeof(double) * w * (size_t)(p->n_free > 0 ? p->n_free : 1)));
    HIPCHK(hipMalloc(&p->d_fac, sizeof(double) * w));
    HIPCHK(hipMalloc(&p->d_nlp, sizeof(double) * w));
    HIPCHK(hipMalloc(&p->d_lau, sizeof(double) * w));
    HIPCHK(hipMalloc(&p->d_sidx, sizeof(long long) * w));
    p->capw = W;
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
    p->device = h->device;
    p->n_free = n_free;
    p->n_prior = n_prior;
    p->convert = convert;
    // The fused sampler path (loglike_kernel SAMPLE >= 2) makes a walker's proposal, full row,
    // conversion and priors lane-parallel in the walker's wave; RVK_SAMPLER_FUSE=0 (experiment
    // hook) keeps the two-kernel path.
    const char *fe = getenv("RVK_SAMPLER_FUSE");
    p->fusable = n_free <= kFuseMaxD && pf <= kFuseMaxPFull && n_prior <= kFuseMaxPrior && !(fe && atoi(fe) == 0);
    const char *le = getenv("RVK_LOGPOST_FUSE");        // experiment / test hook: the two-kernel form
    p->two_kernel = le && atoi(le) == 0;
    bool basic = true;
    for (int k = 0; k < n_prior; ++k) basic &= kind[k] <= kMaxBasicPriorKind;
    p->ext = convert ? 2 : basic ? 0 : 1;
    p->jac = jac;
    p->renorm = renorm;
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipMalloc(&p->d_colmap, sizeof(int32_t) * pf));
    HIPCHK(hipMalloc(&p->d_tmpl, sizeof(double) * pf));
    HIPCHK(hipMalloc(&p->d_slots, sizeof(PriorSlot) * (n_prior > 0 ? n_prior : 1)));
    HIPCHK(hipMalloc(&p->d_run, sizeof(RunArgs)));
    HIPCHK(hipMemcpy(p->d_colmap, colmap.data(), sizeof(int32_t) * pf, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(p->d_tmpl, tmpl, sizeof(double) * pf, hipMemcpyHostToDevice));
    if (n_prior > 0)
        HIPCHK(hipMemcpy(p->d_slots, slots.data(), sizeof(PriorSlot) * n_prior, hipMemcpyHostToDevice));
    return RVK_OK;
}

void rvk::DrawTable::release() {
    (void)hipFree(block);
    (void)hipFree(keys);
    (void)hipFree(sets);
    block = nullptr;
    keys = nullptr;
    sets = nullptr;
    cap_block = cap_keys = cap_sets = 0;
    H = 0;
    steps = 0;
}

int rvk::draws_block_steps(long long H) {
    const long long per = 2 * H * (long long)(sizeof(PreDraw) + 8);      // table + scratch per step
    long long n = (256LL << 20) / (per > 0 ? per : 1);
    if (n > 256) n = 256;
    n -= n % kStepsPerGraph;
    return (int)(n < kStepsPerGraph ? kStepsPerGraph : n);
}

// Room for a block of draws: at least draws_block_steps(H) steps, so the table (and a graph reading
// it) keeps its address from one block to the next.
static int draws_reserve(DrawTable &t, long long H, int n_steps) {
    const int blk = draws_block_steps(H);
    const size_t n = (size_t)(n_steps > blk ? n_steps : blk);
    return grow_dev((void **)&t.block, &t.cap_block, sizeof(PreDraw) * 2 * (size_t)H * n);
}

int rvk::draws_fill_host(DrawTable &t, hipStream_t st, long long H, int n_steps, int D, const RunArgs &run) {
    int rc = draws_reserve(t, H, n_steps);
    if (rc) return rc;
    const long long np = (long long)n_steps * 2 * H;
    hipLaunchKernelGGL(host_draws_kernel, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, st, t.block, run, n_steps,
                       H, D);
    HIPCHK(hipGetLastError());
    t.H = H;
    t.steps = n_steps;
    return RVK_OK;
}

int rvk::draws_fill(DrawTable &t, hipStream_t st, long long H, int n_steps, int D, uint64_t seed, uint64_t step0,
                    double a, int flags) {
    const size_t W = 2 * (size_t)H, n = (size_t)n_steps;
    int rc;
    if ((rc = draws_reserve(t, H, n_steps)) ||
        (rc = grow_dev((void **)&t.keys, &t.cap_keys, sizeof(uint32_t) * W * n)) ||
        (rc = grow_dev((void **)&t.sets, &t.cap_sets, sizeof(int32_t) * W * n)))
        return rc;
    hipLaunchKernelGGL(split_draws_kernel, dim3((unsigned)n_steps), dim3(kSplitThreads), 0, st, t.block, t.keys, t.sets,
                       H, D, seed, step0, a, (flags & RVK_STRETCH_FIXED_SPLIT) ? 1 : 0);
    HIPCHK(hipGetLastError());
    t.H = H;
    t.steps = n_steps;
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
    if (p->fusable && h->solver == 0 && h->sample_direct[p->ext] && !p->two_kernel) {
        // one kernel: each wave builds its walker's row, jitter check, conversion and priors
        // lane-parallel (the fused sampler's prep on the given coordinates), then the epoch loop
        SampleArgs sa{};
        sa.D = p->n_free;
        sa.q = d_free;
        sa.qstride = stride;
        sa.pd = p->dev();
        sa.out = d_out;
        h->sample_direct[p->ext](st, h->epochs(), h->n, h->n_inst, nullptr, W, h->p_full(),
                                 PostArgs{nullptr, p->jac, p->renorm}, sa);
        HIPCHK(hipGetLastError());
        return RVK_OK;
    }
    hipLaunchKernelGGL(logprior_kernel, dim3(wave_blocks(W)), dim3(256), 0, st, p->dev(), d_free, (long long)W,
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
    std::lock_guard<std::mutex> lock(h->mu);   // one blocking call per handle at a time (rvk.h, threading)
    HIPCHK(hipSetDevice(h->device));
    int rc = reserve_impl(p, W);       // before staging: a failed allocation leaves nothing in flight
    if (rc) return rc;
    const size_t bx = sizeof(double) * (size_t)W * (size_t)stride, bo = sizeof(double) * (size_t)W;
    const void *src = xf, *d_x = nullptr;
    void *d_out = nullptr;
    if ((rc = p->io.begin(h->hostio, h->stream, 1, &src, &bx, bo, &d_x, &d_out))) return rc;
    if ((rc = rvk_logpost_device(p, (const double *)d_x, W, stride, (double *)d_out, h->stream))) {
        (void)hipStreamSynchronize(h->stream);
        return rc;
    }
    return p->io.end(h->stream, out, bo);
}

int rvk_stretch_run(rvk_post *p, double *d_x, double *d_lp, int64_t W, int32_t n_steps, double a, uint64_t seed,
                    uint64_t step0, int32_t flags, const int32_t *d_set, const double *d_zu, const int32_t *d_rint,
                    const double *d_au, double *d_chain, double *d_lnp, int64_t *d_naccepted, int32_t *d_status,
                    void *stream) {
    if (!p) return fail(RVK_E_ARG, "NULL posterior");
    if (W < 4 || (W & 1)) return fail(RVK_E_ARG, "n_walkers must be even and >= 4");
    if (n_steps < 0) return fail(RVK_E_ARG, "n_steps < 0");
    if (!(a > 1.0)) return fail(RVK_E_ARG, "stretch scale a must be > 1");
    if (flags & ~RVK_STRETCH_FIXED_SPLIT) return fail(RVK_E_ARG, "unknown flags");
    if (!d_x || !d_lp || !d_status) return fail(RVK_E_ARG, "NULL device buffer");
    if (d_set && (!d_zu || !d_rint || !d_au)) return fail(RVK_E_ARG, "host draws need set, zu, rint and au");
    if (n_steps == 0) return RVK_OK;
    const long long H = W / 2;
    int rc = reserve_impl(p, H);
    if (rc) return rc;
    rvk_handle *h = p->h;
    hipStream_t st = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIPCHK(hipStreamIsCapturing(st, &cs));
    const bool use_graph = h->graph && cs == hipStreamCaptureStatusNone;   // a caller's capture records the launches
    const size_t wd = (size_t)W * (size_t)p->n_free, hh = 2 * (size_t)H;
    const int blk = draws_block_steps(H);                                 // steps per draw block (and graph)
    for (int b0 = 0; b0 < n_steps; b0 += blk) {
        const int nb = (n_steps - b0) < blk ? (n_steps - b0) : blk;
        const RunArgs run{d_x,
                          d_lp,
                          (long long *)d_naccepted,
                          (int *)d_status,
                          d_chain ? d_chain + (size_t)b0 * wd : nullptr,
                          d_lnp ? d_lnp + (size_t)b0 * (size_t)W : nullptr,
                          d_set ? d_set + (size_t)b0 * hh : nullptr,
                          d_set ? d_zu + (size_t)b0 * hh : nullptr,
                          d_set ? d_rint + (size_t)b0 * hh : nullptr,
                          d_set ? d_au + (size_t)b0 * hh : nullptr,
                          seed,
                          step0 + (uint64_t)b0,
                          a};
        rc = d_set ? draws_fill_host(p->tab, st, H, nb, p->n_free, run)
                   : draws_fill(p->tab, st, H, nb, p->n_free, seed, step0 + (uint64_t)b0, a, flags);
        if (rc) return rc;
        hipLaunchKernelGGL(set_run_kernel, dim3(1), dim3(1), 0, st, p->d_run, run);
        if (use_graph && nb == blk) {
            if ((rc = ensure_graph(p, H, blk))) return rc;
            HIPCHK(hipGraphLaunch(p->graph, st));
        } else {
            enqueue_steps(p, st, H, nb);
        }
    }
    HIPCHK(hipGetLastError());
    return RVK_OK;
}

int rvk_stretch_draws(rvk_post *p, int64_t W, int32_t n_steps, double a, uint64_t seed, uint64_t step0, int32_t flags,
                      void *stream) {
    if (!p) return fail(RVK_E_ARG, "NULL posterior");
    if (W < 4 || (W & 1)) return fail(RVK_E_ARG, "n_walkers must be even and >= 4");
    if (n_steps < 1) return fail(RVK_E_ARG, "n_steps must be >= 1");
    if (!(a > 1.0)) return fail(RVK_E_ARG, "stretch scale a must be > 1");
    if (flags & ~RVK_STRETCH_FIXED_SPLIT) return fail(RVK_E_ARG, "unknown flags");
    HIPCHK(hipSetDevice(p->h->device));
    return draws_fill(p->tab, (hipStream_t)stream, W / 2, n_steps, p->n_free, seed, step0, a, flags);
}

int rvk_stretch_propose(rvk_post *p, const double *d_x, int64_t W, int32_t s, int32_t half, int64_t j0, int64_t count,
                        double *d_out, void *stream) {
    if (!p) return fail(RVK_E_ARG, "NULL posterior");
    const long long H = W / 2;
    if (W < 4 || (W & 1) || H != p->tab.H) return fail(RVK_E_ARG, "n_walkers differs from the drawn table's");
    if (s < 0 || s >= p->tab.steps) return fail(RVK_E_ARG, "step outside the drawn table");
    if (half != 0 && half != 1) return fail(RVK_E_ARG, "half must be 0 or 1");
    if (j0 < 0 || count < 0 || j0 + count > H) return fail(RVK_E_ARG, "proposal slice outside the half");
    if (!d_x || !d_out) return fail(RVK_E_ARG, "NULL device buffer");
    if (count == 0) return RVK_OK;
    int rc = reserve_impl(p, count);
    if (rc) return rc;
    rvk_handle *h = p->h;
    hipStream_t st = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    const RunArgs run{const_cast<double *>(d_x), nullptr, nullptr, nullptr, nullptr, nullptr,
                      nullptr, nullptr, nullptr, nullptr, 0, 0, 2.0};
    hipLaunchKernelGGL(set_run_kernel, dim3(1), dim3(1), 0, st, p->d_run, run);
    const PostDev pd = p->dev();
    const PostArgs post{p->d_lp, p->jac, p->renorm};
    if (p->fusable && h->solver == 0 && h->sample_eval[p->ext]) {
        const SampleArgs sa{p->n_free, nullptr, nullptr, nullptr, nullptr, p->d_run, s, half, pd, j0, H, p->tab.block,
                            d_out};
        h->sample_eval[p->ext](st, h->epochs(), h->n, h->n_inst, nullptr, count, h->p_full(), post, sa);
    } else {
        hipLaunchKernelGGL(propose_kernel, dim3(wave_blocks(count)), dim3(256), 0, st, pd, p->d_run, p->tab.block, s,
                           half, count, j0, H, p->d_q, p->d_full, p->d_lp, p->d_fac, p->d_lau, p->d_sidx);
        h->launch(st, h->epochs(), h->n, h->n_inst, p->d_full, count, h->p_full(), d_out, post);
    }
    HIPCHK(hipGetLastError());
    return RVK_OK;
}

int rvk_copy_to_host(const void *d_src, void *h_dst, int64_t bytes, int32_t workgroups, void *stream) {
    if (bytes < 0 || (bytes > 0 && (!d_src || !h_dst))) return fail(RVK_E_ARG, "bad copy arguments");
    if (bytes == 0) return RVK_OK;
    if (((uintptr_t)d_src | (uintptr_t)h_dst | (uintptr_t)bytes) & 15u)
        return fail(RVK_E_ARG, "rvk_copy_to_host needs 16-byte aligned pointers and size");
    if (workgroups < 1) workgroups = 1;
    if (workgroups > 1024) workgroups = 1024;
    hipLaunchKernelGGL(egress_kernel, dim3((unsigned)workgroups), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4 *)d_src, (u32x4 *)h_dst, (long long)(bytes / 16));
    HIPCHK(hipGetLastError());
    return RVK_OK;
}

int rvk_stretch_table_read(rvk_post *p, int32_t s, int32_t half, int64_t *walker, int64_t *complement, double *z) {
    if (!p) return fail(RVK_E_ARG, "NULL posterior");
    if (s < 0 || s >= p->tab.steps || (half != 0 && half != 1)) return fail(RVK_E_ARG, "step / half outside the table");
    if (!walker || !complement || !z) return fail(RVK_E_ARG, "NULL host buffer");
    const long long H = p->tab.H;
    std::vector<PreDraw> v((size_t)H);
    HIPCHK(hipSetDevice(p->h->device));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(v.data(), p->tab.block + ((size_t)s * 2 + (size_t)half) * (size_t)H, sizeof(PreDraw) * (size_t)H,
                     hipMemcpyDeviceToHost));
    for (long long j = 0; j < H; ++j) {
        walker[j] = v[(size_t)j].s;
        complement[j] = v[(size_t)j].c;
        z[j] = v[(size_t)j].z;
    }
    return RVK_OK;
}

int rvk_stretch_update(rvk_post *p, double *d_x, double *d_lp, int64_t W, int32_t s, int32_t half,
                       const double *d_nlp, double *d_chain_step, double *d_lnp_step, const int64_t *d_nacc_in,
                       int64_t *d_nacc_out, int32_t *d_status, void *stream) {
    if (!p) return fail(RVK_E_ARG, "NULL posterior");
    const long long H = W / 2;
    if (W < 4 || (W & 1) || H != p->tab.H) return fail(RVK_E_ARG, "n_walkers differs from the drawn table's");
    if (s < 0 || s >= p->tab.steps) return fail(RVK_E_ARG, "step outside the drawn table");
    if (half != 0 && half != 1) return fail(RVK_E_ARG, "half must be 0 or 1");
    if (!d_x || !d_lp || !d_nlp || !d_status) return fail(RVK_E_ARG, "NULL device buffer");
    if (d_nacc_out && !d_nacc_in) return fail(RVK_E_ARG, "d_nacc_out needs d_nacc_in");
    HIPCHK(hipSetDevice(p->h->device));
    hipLaunchKernelGGL(stretch_update_kernel, dim3(blocks_for(H)), dim3(256), 0, (hipStream_t)stream,
                       p->tab.block + ((size_t)s * 2 + (size_t)half) * (size_t)H, H, p->n_free, d_x, d_lp, d_nlp,
                       (const long long *)d_nacc_in, (long long *)d_nacc_out, (int *)d_status, d_chain_step,
                       d_lnp_step);
    HIPCHK(hipGetLastError());
    return RVK_OK;
}

}  // extern "C"
