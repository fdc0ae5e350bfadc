// rvk_gp.hip -- batched quasi-periodic GP log-likelihood (include/rvk_gp.h;
// SURVEY.md §8(f) row 2, BASELINE config 5).
//
// One workgroup (4 waves) per walker, grid-stride over walkers.  Per walker:
//   1. planet constants (lanes over planets) and the mean model in fp64 (the
//      log-likelihood kernel's Kepler solver, threads over epochs) -> residuals
//      r and the diagonal velerr^2 + jit^2 in LDS (fp32);
//   2. left-looking blocked Cholesky over 32-column steps kb with the right-hand
//      side carried along (no triangular solve afterwards).  The covariance is
//      never stored: each tile (bi, kb) is generated in registers when its step
//      comes, and only the finished L tiles below the diagonal go to the
//      walker's workspace (packed 32x32 tiles, fp32), read back by later steps:
//        a. all waves: pre = C_(bi,kb) - sum_j L_(bi,j) L_(kb,j)^T with
//           v_mfma_f32_32x32x2_f32 (wave 0 the diagonal tile and its rhs);
//        b. wave 0 factors the diagonal tile in registers (v_readlane broadcasts),
//           its rhs and inverse, log det and r^T C^-1 r in fp64;
//        c. all waves: L_(bi,kb) = pre L_kk^-T with MFMA, stored.
//   ll = -1/2 r^T C^-1 r - sum log L_ii - N/2 log(2 pi).
// Padding rows/columns up to a multiple of 32 are identity rows with r = 0.
#include <cmath>
#include <vector>

#include "../../include/rvk_gp.h"
#include "rvk_internal.h"

using namespace rvk;

namespace {

#ifndef RVK_GP_ABLATE
#define RVK_GP_ABLATE 0   // timing experiments only (wrong results): 1 no off-diagonal accumulation, 2 no solve
#endif
#ifndef RVK_GP_WGPCU
#define RVK_GP_WGPCU 2    // concurrent workgroups per CU (each its own workspace), LDS permitting
#endif
constexpr int TB = 32;              // tile edge
constexpr int PS = TB + 1;          // LDS row stride of the panel / diagonal tile (bank spread)

using f32x16 = __attribute__((ext_vector_type(16))) float;

__device__ __forceinline__ float rlf(float v, int lane) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}

__device__ __forceinline__ long long tile_index(int bi, int bj) { return (long long)bi * (bi + 1) / 2 + bj; }

// MFMA 32x32 C/D map (cdna_hip_programming.md): register r of lane l holds
// (row = (r & 3) + 8 (r >> 2) + 4 (l >> 5), col = l & 31).
__device__ __forceinline__ int cd_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

struct GpLds {
    // carved from dynamic shared memory
    float *pan;      // [(npad - TB)][TB]  the step's tiles below the diagonal, before the solve
    float *li;       // [TB][PS]           inverse of the step's diagonal tile
    float *r;        // [npad]             rhs (residuals), solved in place
    float *dia;      // [npad]             velerr^2 + jit^2
    SC *tab;         // [kTabN]
    PlanetK *pk;     // [NP]
    int *ok;         // [NP]
};

template <int NP, bool MULTI, bool TP>
__global__ __launch_bounds__(kBlock, 2) void gp_loglike_kernel(EpochData d, int n, int ni,
                                                           const double *__restrict__ theta,
                                                           const double *__restrict__ hyper, long long W,
                                                           long long stride, long long hstride,
                                                           float *__restrict__ work, long long work_stride,
                                                           double *__restrict__ out) {
    extern __shared__ double smem_d[];
    const int nt = (n + TB - 1) / TB, npad = nt * TB;
    GpLds L;
    {
        float *f = reinterpret_cast<float *>(smem_d);
        L.pan = f;
        f += (npad - TB) * TB;
        L.li = f;
        f += TB * PS;
        L.r = f;
        f += npad;
        L.dia = f;
        f += npad;
        L.tab = reinterpret_cast<SC *>(reinterpret_cast<uintptr_t>(f + 3) & ~uintptr_t(15));
        L.pk = reinterpret_cast<PlanetK *>(L.tab + kTabN);
        L.ok = reinterpret_cast<int *>(L.pk + NP);
    }
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < kTabN; i += kBlock) L.tab[i] = d.tab[i];
    float *A = work + (long long)blockIdx.x * work_stride;

    for (long long w = blockIdx.x; w < W; w += gridDim.x) {
        const double *row = theta + w * stride;
        const double *hp = hyper + w * hstride;
        // ---- 1. planets, mean model, residuals -------------------------------------------
        if (tid < NP) {
            PlanetK pk;
            const bool ok = TP ? planet_consts_t<0, true>(row + 5 * tid, pk, 0, L.tab)
                               : planet_consts(d.par, row + 5 * tid, pk);
            L.pk[tid] = pk;
            L.ok[tid] = ok;
        }
        __syncthreads();   // (the table fill of the first trip lands here too)
        bool alive = true;
#pragma unroll
        for (int p = 0; p < NP; ++p) alive &= L.ok[p] != 0;
        if (!alive) {                                   // fit.py:8083-8085: mean model failed
            if (tid == 0) out[w] = -INFINITY;
            __syncthreads();
            continue;
        }
        const double *g = row + 5 * NP, *jit = g + ni;
        const double gd = jit[ni], gdd = jit[ni + 1];
        for (int i = tid; i < npad; i += kBlock) {
            float ri = 0.0f, di = 1.0f;
            if (i < n) {
                const double t = d.t[i];
                const int ii = MULTI ? d.inst[i] : 0;
                double rv = 0.0;
#pragma unroll
                for (int p = 0; p < NP; ++p) rv = planet_rv<0>(L.pk[p], t, L.tab, rv);
                const double dt = t - d.t0;
                rv += __builtin_fma(gd, dt, gdd * (dt * dt));      // Trend (fit.py:8031-8035)
                rv += g[ii];                                       // gamma (fit.py:8041-8045)
                ri = (float)(d.vel[i] - rv);
                di = (float)(d.s2[i] + jit[ii] * jit[ii]);         // fit.py:8096-8098
            }
            L.r[i] = ri;
            L.dia[i] = di;
        }
        __syncthreads();
        // ---- 2. left-looking blocked Cholesky, covariance generated on the fly ------------
        const double amp = hp[0], lam_e = hp[1], lam_p = hp[2], per = hp[3];
        const float amp2 = (float)(amp * amp);
        const float gam = (float)(1.0 / (2.0 * lam_p * lam_p));   // gp.py:150
        const double inv_per = 1.0 / per, inv_le = 1.0 / lam_e;
        // C_ij (gp.py:126-156 + fit.py:8090-8105); padding is identity
        auto cov = [&](int i, int j) -> float {
            if (i >= n || j >= n) return (i == j) ? 1.0f : 0.0f;
            const double tau = d.t[i] - d.t[j];
            // sin^2(pi tau / P) from the phase reduced in fp64, then fp32
            const double ph = tau * inv_per;
            const float fr = (float)(ph - __builtin_rint(ph));
            const float s = __builtin_amdgcn_sinf(0.5f * fr);     // v_sin_f32 takes revolutions
            const float x = (float)(tau * inv_le);
            float v = amp2 * __expf(-(gam * (s * s) + 0.5f * (x * x)));
            if (i == j) v += L.dia[i];
            return v;
        };
        double logdet = 0.0, quad = 0.0;    // meaningful in wave 0
        for (int kb = 0; kb < nt; ++kb) {
            // lane-derived addresses are recomputed per step, not hoisted and held for the kernel
            int ln = lane;
            asm volatile("" : "+v"(ln));
            const int h = ln >> 5, c = ln & 31;
            const int m = nt - kb - 1;               // tiles below the diagonal
            // a. Every tile (bi, kb), bi >= kb, is accumulated as its transpose in MFMA C/D
            //    layout,  pre^T = C_(bi,kb)^T - sum_j L_(kb,j) L_(bi,j)^T  (16 MFMAs per j; both
            //    operands are rows of finished L tiles, lane l reading row l & 31 at columns
            //    16 (l >> 5) + ks).  Lane l then holds row (l & 31) of pre at the columns
            //    cd_row(r, l): the A operand of the solve below, with K permuted the same way.
            //    Wave 0 takes the diagonal tile, its rhs and its factorisation; waves 1..3 the
            //    tiles below, parked in LDS for the solve.
            auto accumulate = [&](int bi, f32x16 &acc, float &srhs, bool rhs) {
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = cov(bi * TB + c, kb * TB + cd_row(r, ln));
                for (int j = 0; j < kb; ++j) {
                    const float4 *pk4 = reinterpret_cast<const float4 *>(A + tile_index(kb, j) * (TB * TB) + c * TB + 16 * h);
                    const float4 *pb4 = reinterpret_cast<const float4 *>(A + tile_index(bi, j) * (TB * TB) + c * TB + 16 * h);
                    float ka[16], kbv[16];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float4 u = pk4[q], v = pb4[q];
                        ka[4 * q] = u.x; ka[4 * q + 1] = u.y; ka[4 * q + 2] = u.z; ka[4 * q + 3] = u.w;
                        kbv[4 * q] = v.x; kbv[4 * q + 1] = v.y; kbv[4 * q + 2] = v.z; kbv[4 * q + 3] = v.w;
                    }
#pragma unroll
                    for (int ks = 0; ks < 16; ++ks) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(-ka[ks], kbv[ks], acc, 0, 0, 0);
                    if (rhs) {
                        const float *yj = L.r + j * TB + 16 * h;
#pragma unroll
                        for (int ks = 0; ks < 16; ++ks) srhs = __builtin_fmaf(ka[ks], yj[ks], srhs);
                    }
                }
            };
            if (wv == 0) {
                f32x16 acc;
                float srhs = 0.0f;
                accumulate(kb, acc, srhs, true);
                // b. factor the diagonal tile in registers: lane i (< 32) gathers row i (the
                //    other half of its columns from lane i + 32; pre is symmetric), then
                //    left-looking, one column per step r: row r of L (lane r's finished entries
                //    L[r][k], k < r) is broadcast with v_readlane and shared by the column update
                //    a_i[r] -= sum_k a_i[k] L[r][k], the rhs y_r and the inverse's row
                //    X[r][j] = (delta_rj - sum_k L[r][k] X[k][j]) / L[r][r] (lane j = column j).
                const int i = c;
                float a[TB];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    a[cd_row(r, 0)] = acc[r];
                    a[cd_row(r, 32)] = __shfl_xor(acc[r], 32);
                }
                srhs += __shfl_xor(srhs, 32);
                const float rb = L.r[kb * TB + i] - srhs;
                float xinv[TB], y[TB];
                double dprod = 1.0;                   // log det via products of 8 pivots
                float yown = 0.0f;                    // y[i]
#pragma unroll
                for (int r = 0; r < TB; ++r) {
                    float col = a[r], xs = (r == i) ? 1.0f : 0.0f, ys = rlf(rb, r);
#pragma unroll
                    for (int k = 0; k < r; ++k) {
                        const float lrk = rlf(a[k], r);
                        col = __builtin_fmaf(-a[k], lrk, col);
                        xs = __builtin_fmaf(-lrk, xinv[k], xs);
                        ys = __builtin_fmaf(-lrk, y[k], ys);
                    }
                    const float dc = __builtin_sqrtf(rlf(col, r));    // not positive definite -> NaN
                    const float inv = 1.0f / dc;
                    a[r] = col * inv;                                 // rows i < r: upper part, unused
                    xinv[r] = xs * inv;
                    y[r] = ys * inv;
                    yown = (i == r) ? y[r] : yown;
                    asm volatile("" : "+v"(xinv[r]), "+v"(y[r]), "+v"(a[r]), "+v"(yown));   // finish step r here
                    const bool live = kb * TB + r < n;
                    dprod *= live ? (double)dc : 1.0;
                    quad += live ? (double)y[r] * (double)y[r] : 0.0;
                    if ((r & 7) == 7) { logdet += log(dprod); dprod = 1.0; }
                }
                if (ln < TB) {
                    L.r[kb * TB + i] = yown;
#pragma unroll
                    for (int r = 0; r < TB; ++r) L.li[r * PS + i] = xinv[r];   // L_kk^-1, row-major
                }
            } else {
                for (int q = wv; q <= ((RVK_GP_ABLATE & 1) ? 0 : m); q += kWavesPerBlock - 1) {
                    f32x16 acc;
                    float unused = 0.0f;
                    accumulate(kb + q, acc, unused, false);
                    float *pre = L.pan + (q - 1) * (TB * TB);
#pragma unroll
                    for (int r = 0; r < 16; ++r) pre[r * 64 + ln] = acc[r];
                }
            }
            __syncthreads();
            if (m == 0) break;
            // c. L_(bi,kb) = pre L_kk^-T (16 MFMAs per tile): A = pre's rows as parked, B[k][j] =
            //    L_kk^-1[j][k] at the permuted k; the C/D result is stored row-major.
            for (int q = 1 + wv; q <= ((RVK_GP_ABLATE & 2) ? 0 : m); q += kWavesPerBlock) {
                const float *pre = L.pan + (q - 1) * (TB * TB);
                f32x16 acc = {};
#pragma unroll
                for (int ks = 0; ks < 16; ++ks)
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(pre[ks * 64 + ln], L.li[c * PS + cd_row(ks, ln)], acc, 0, 0, 0);
                float *T = A + tile_index(kb + q, kb) * (TB * TB);
#pragma unroll
                for (int r = 0; r < 16; ++r) T[cd_row(r, ln) * TB + c] = acc[r];
            }
            __syncthreads();
        }
        if (tid == 0) out[w] = -0.5 * quad - logdet - 0.5 * (double)n * kLog2Pi;
        __syncthreads();
    }
}

size_t gp_lds_bytes(int n, int np) {
    const int npad = ((n + TB - 1) / TB) * TB;
    size_t b = sizeof(float) * ((size_t)(npad - TB) * TB + TB * PS + 2 * (size_t)npad) + 16;
    b += sizeof(SC) * kTabN + (sizeof(PlanetK) + sizeof(int)) * (size_t)np + 16;
    return b;
}

typedef void (*gp_launch_t)(hipStream_t, unsigned, size_t, EpochData, int, int, const double *, const double *,
                            long long, long long, long long, float *, long long, double *);

template <int NP, bool MULTI, bool TP>
void launch_gp(hipStream_t st, unsigned grid, size_t lds, EpochData d, int n, int ni, const double *th,
               const double *hy, long long W, long long stride, long long hs, float *work, long long wstride,
               double *out) {
    static size_t allowed = 0;   // dynamic LDS beyond the default needs the attribute
    if (lds > allowed) {
        (void)hipFuncSetAttribute((const void *)gp_loglike_kernel<NP, MULTI, TP>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        allowed = lds;
    }
    hipLaunchKernelGGL((gp_loglike_kernel<NP, MULTI, TP>), dim3(grid), dim3(kBlock), lds, st, d, n, ni, th, hy, W,
                       stride, hs, work, wstride, out);
}

template <bool MULTI, bool TP>
gp_launch_t pick_gp_s(int np) {
    switch (np) {
        case 1: return launch_gp<1, MULTI, TP>;
        case 2: return launch_gp<2, MULTI, TP>;
        case 3: return launch_gp<3, MULTI, TP>;
        case 4: return launch_gp<4, MULTI, TP>;
        case 5: return launch_gp<5, MULTI, TP>;
        case 6: return launch_gp<6, MULTI, TP>;
        case 7: return launch_gp<7, MULTI, TP>;
        case 8: return launch_gp<8, MULTI, TP>;
        default: return nullptr;
    }
}

gp_launch_t pick_gp(int np, bool multi, bool tp) {
    if (multi) return tp ? pick_gp_s<true, true>(np) : pick_gp_s<true, false>(np);
    return tp ? pick_gp_s<false, true>(np) : pick_gp_s<false, false>(np);
}

}  // namespace

struct rvk_gp {
    rvk_handle *h = nullptr;
    gp_launch_t launch = nullptr;
    unsigned grid = 0;           // concurrent walkers (one workgroup each)
    size_t lds = 0;
    long long wstride = 0;       // floats per workgroup workspace
    float *d_work = nullptr;
};

static void free_gp(rvk_gp *g) {
    if (!g) return;
    if (g->h) (void)hipSetDevice(g->h->device);
    (void)hipFree(g->d_work);
    delete g;
}

static int create_gp(rvk_gp *g, rvk_handle *h, int32_t kernel) {
    if (!h) return fail(RVK_E_ARG, "NULL handle");
    if (kernel != RVK_GP_QUASIPERIODIC) return fail(RVK_E_ARG, "unknown GP kernel type");
    if (h->n < 1 || h->n > RVK_GP_MAX_EPOCHS) return fail(RVK_E_ARG, "GP needs 1 <= n_epochs <= 1024");
    g->h = h;
    g->launch = pick_gp(h->n_planets, h->n_inst > 1, h->par == RVK_PAR_PKEWTP);
    g->lds = gp_lds_bytes(h->n, h->n_planets);
    HIPCHK(hipSetDevice(h->device));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, h->device));
    // workgroups that fit at once (LDS-limited), each with its own workspace
    const size_t per_cu = (size_t)160 * 1024 / g->lds;
    g->grid = (unsigned)(prop.multiProcessorCount * (per_cu < 1 ? 1 : (per_cu > RVK_GP_WGPCU ? RVK_GP_WGPCU : per_cu)));
    const int nt = (h->n + TB - 1) / TB;
    g->wstride = (long long)nt * (nt + 1) / 2 * TB * TB;
    HIPCHK(hipMalloc(&g->d_work, sizeof(float) * (size_t)g->wstride * g->grid));
    return RVK_OK;
}

extern "C" {

rvk_gp *rvk_gp_create(rvk_handle *h, int32_t kernel_type) {
    rvk_gp *g = new (std::nothrow) rvk_gp();
    if (!g) {
        fail(RVK_E_NOMEM, "out of host memory");
        return nullptr;
    }
    if (create_gp(g, h, kernel_type)) {
        free_gp(g);
        return nullptr;
    }
    return g;
}

void rvk_gp_destroy(rvk_gp *g) { free_gp(g); }

int rvk_gp_loglike_device(rvk_gp *g, const double *d_theta, const double *d_hyper, int64_t W, int64_t stride,
                          int64_t hstride, double *d_out, void *stream) {
    if (!g) return fail(RVK_E_ARG, "NULL GP handle");
    rvk_handle *h = g->h;
    if (W < 0 || stride < h->p_full() || hstride < RVK_GP_NHYPER) return fail(RVK_E_ARG, "bad walker block shape");
    if (W == 0) return RVK_OK;
    if (!d_theta || !d_hyper || !d_out) return fail(RVK_E_ARG, "NULL device buffer");
    HIPCHK(hipSetDevice(h->device));
    const unsigned grid = (unsigned)((long long)g->grid < W ? g->grid : W);
    g->launch((hipStream_t)stream, grid, g->lds, h->epochs(), h->n, h->n_inst, d_theta, d_hyper, W, stride, hstride,
              g->d_work, g->wstride, d_out);
    HIPCHK(hipGetLastError());
    return RVK_OK;
}

int rvk_gp_loglike(rvk_gp *g, const double *theta, const double *hyper, int64_t W, int64_t stride, int64_t hstride,
                   double *out) {
    if (!g) return fail(RVK_E_ARG, "NULL GP handle");
    if (W == 0) return RVK_OK;
    if (!theta || !hyper || !out || W < 0) return fail(RVK_E_ARG, "bad host buffers");
    rvk_handle *h = g->h;
    HIPCHK(hipSetDevice(h->device));
    double *dt = nullptr, *dh = nullptr, *dout = nullptr;
    const size_t bt = sizeof(double) * (size_t)W * (size_t)stride, bh = sizeof(double) * (size_t)W * (size_t)hstride;
    int rc = RVK_OK;
    if (hipMalloc(&dt, bt) != hipSuccess || hipMalloc(&dh, bh) != hipSuccess ||
        hipMalloc(&dout, sizeof(double) * (size_t)W) != hipSuccess)
        rc = fail(RVK_E_HIP, "hipMalloc failed");
    if (rc == RVK_OK && (hipMemcpyAsync(dt, theta, bt, hipMemcpyHostToDevice, h->stream) != hipSuccess ||
                         hipMemcpyAsync(dh, hyper, bh, hipMemcpyHostToDevice, h->stream) != hipSuccess))
        rc = fail(RVK_E_HIP, "hipMemcpyAsync H2D failed");
    if (rc == RVK_OK) rc = rvk_gp_loglike_device(g, dt, dh, W, stride, hstride, dout, h->stream);
    if (rc == RVK_OK &&
        hipMemcpyAsync(out, dout, sizeof(double) * (size_t)W, hipMemcpyDeviceToHost, h->stream) != hipSuccess)
        rc = fail(RVK_E_HIP, "hipMemcpyAsync D2H failed");
    if (hipStreamSynchronize(h->stream) != hipSuccess && rc == RVK_OK) rc = fail(RVK_E_HIP, "stream sync failed");
    (void)hipFree(dt);
    (void)hipFree(dh);
    (void)hipFree(dout);
    return rc;
}

}  // extern "C"
