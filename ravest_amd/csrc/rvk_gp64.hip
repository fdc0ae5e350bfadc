// rvk_gp64.hip -- fp64 factorisation of the batched quasi-periodic GP (include/rvk_gp.h):
// the reference's precision (ravest runs tinygp with jax_enable_x64, fit.py:39), used
//   * as the RVK_GP_FP64 precision mode of rvk_gp_loglike[_device],
//   * as the fallback of the fp32 path for walkers whose covariance is not positive
//     definite in fp32 (gate = the fp32 output: only NaN walkers are re-evaluated),
//   * for the GP-conditioned posterior predictive (CONDITION mode: tinygp
//     GaussianProcess.condition(y, X_test).mean, fit.py:7494-7554).
//
// One workgroup of NW = 8 waves per walker (one per CU: 2 waves per SIMD, 256 VGPRs each),
// grid-stride over walkers.  Per walker:
//   1. planet constants and the fp64 mean model (the log-likelihood kernel's solver) ->
//      times, residuals r and the diagonal velerr^2 + jit^2 in LDS (fp64);
//   2. blocked left-looking Cholesky over 32-wide tile columns with the right-hand side
//      carried along (y = L^-1 r) and a one-column lookahead -- the schedule of the fp32
//      kernel (rvk_gp.hip), with fp64 tiles as 2 x 2 blocks of v_mfma_f64_16x16x4_f64:
//        P(k)  the owner of tile row k factors the diagonal tile (one wave: lanes 0-31
//              the rows of L_kk, lanes 32-63 the columns of X = L_kk^-1, from the same
//              LDS row broadcasts) and y_k = X r_k; every wave accumulates the next
//              column's tiles, acc(bi, k+1) = C(bi, k+1) - sum_{j<k} L(bi, j) L(k+1, j)^T;
//        S1(k) L(bi, k) = acc(bi, k) X^T (MFMA), stored; r_bi -= L(bi, k) y_k;
//        S2(k) acc(bi, k+1) -= L(bi, k) L(k+1, k)^T, parked in the workspace slot of
//              tile (bi, k+1) (the diagonal one stays in its owner's registers).
//      A wave holds MAXR accumulator rows in registers; when it owns more rows (large n) it
//      accumulates them MAXR at a time and parks each group in the rows' workspace tiles
//      (bi, k+1) at once, and S2 reads them back: n is bounded by the LDS vectors, not by
//      registers (RVK_GP_MAX_EPOCHS).
//      Accumulators hold the NEGATED transposed tiles in MFMA C/D layout (every MFMA
//      adds; the C/D layout of a transposed tile is the operand layout of the next
//      product, so tiles are never reshuffled).  Finished tiles are kept in the
//      walker's workspace in "fragment layout": frag(s, kk)[lane] = T[16 s + (lane & 15)]
//      [4 kk + (lane >> 4)], which is the A and the B operand layout of the f64 MFMA,
//      stored as lane-contiguous 16-byte pairs (kk, kk + 1).
//   3. LOGLIKE: ll = -1/2 y.y - 1/2 sum log L_ii^2 - n/2 log 2 pi (tinygp DirectSolver);
//      CONDITION: alpha = L^-T y (blocked back substitution over the stored tiles and
//      diagonal inverses), mean(t_q) = sum_i k(t_q - t_i) alpha_i.
// The covariance is generated in fp64 from tau = t_i - t_j, as the reference does:
// A^2 exp(-gamma sin^2(pi |tau| / P) - tau^2 / (2 lambda_e^2))   (gp.py:126-156).
#include <cmath>
#include <type_traits>

#include "../../include/rvk_gp.h"
#include "rvk_gp_internal.h"

using namespace rvk;

namespace {

#ifndef RVK_GP64_ABLATE
#define RVK_GP64_ABLATE 0 // timing experiments only (wrong results): 1 A tiles, 2 B tiles of the accumulation from tile j = 0,
                          // 4 no diagonal factor, 8 no accumulation MFMAs (loads kept), 16 no covariance
                          // function (tau / 2 instead of the QP kernel)
#endif
#ifndef RVK_GP64_TRACE
#define RVK_GP64_TRACE 0  // timing experiments only: s_memtime per phase, first walker of block 0
#endif
#if RVK_GP64_TRACE
__device__ unsigned long long g_gp64_trace[8][32][8];
#define G64_MARK(k, slot)                                                                             \
    do {                                                                                              \
        if (blockIdx.x == 0 && w == 0 && lane == 0 && (k) < 32) g_gp64_trace[wr][k][slot] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define G64_MARK(k, slot) do {} while (0)
#endif

constexpr int TB = 32;            // tile edge
constexpr int TILE = TB * TB;     // doubles per tile
constexpr int FS = 34;            // row stride (doubles) of the factor's row buffer: 16-byte aligned rows
using f64x4 = __attribute__((ext_vector_type(4))) double;

// Transposed 32 x 32 tile in MFMA f64 C/D layout (cdna_hip_programming.md: 16x16x4 f64 C/D
// col = lane & 15, row = (lane >> 4) + 4 reg): c[p][q][i] at lane l is element
// [16 p + (l >> 4) + 4 i][16 q + (l & 15)] of the transposed tile.
struct Acc {
    f64x4 c[2][2];
};

__device__ __forceinline__ f64x4 mfma64(double a, double b, f64x4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
// tile (bi, j), bi >= j, of a walker's workspace (lower triangle incl. the diagonal)
__device__ __forceinline__ long long tix(int bi, int j) { return (long long)bi * (bi + 1) / 2 + j; }
// double offset of fragment pair (s, kk2) of `lane` in a fragment-layout tile
__device__ __forceinline__ int fpair(int s, int kk2, int lane) { return ((s * 4 + kk2) * 64 + lane) * 2; }
// double offset of element (row, col) in a fragment-layout tile
__device__ __forceinline__ int felem(int row, int col) {
    const int kk = col >> 2;
    return fpair(row >> 4, kk >> 1, (col & 3) * 16 + (row & 15)) + (kk & 1);
}

// park / unpark / load_frags take a global or an LDS (address_space(3)) tile pointer.
using lds_d = __attribute__((address_space(3))) double;
using v2d = __attribute__((ext_vector_type(2))) double;     // 16-byte pair, any address space
using lds_v2d = __attribute__((address_space(3))) v2d;
__device__ __forceinline__ v2d *d2p(double *p) { return reinterpret_cast<v2d *>(p); }
__device__ __forceinline__ const v2d *d2p(const double *p) { return reinterpret_cast<const v2d *>(p); }
__device__ __forceinline__ lds_v2d *d2p(lds_d *p) { return (lds_v2d *)p; }
__device__ __forceinline__ const lds_v2d *d2p(const lds_d *p) { return (const lds_v2d *)p; }
template <class P>
__device__ __forceinline__ void park(P tile, const Acc &a, int lane) {
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int ih = 0; ih < 2; ++ih) {
                const int o = (((p * 2 + q) * 2 + ih) * 64 + lane) * 2;
                *d2p(tile + o) = v2d{a.c[p][q][2 * ih], a.c[p][q][2 * ih + 1]};
            }
}
template <class P>
__device__ __forceinline__ void unpark(P tile, Acc &a, int lane) {
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int ih = 0; ih < 2; ++ih) {
                const v2d v = *d2p(tile + (((p * 2 + q) * 2 + ih) * 64 + lane) * 2);
                a.c[p][q][2 * ih] = v.x;
                a.c[p][q][2 * ih + 1] = v.y;
            }
}
// all 16 fragments of a fragment-layout tile: f[s][kk]
template <class P>
__device__ __forceinline__ void load_frags(P tile, double (&f)[2][8], int lane) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int kk2 = 0; kk2 < 4; ++kk2) {
            const v2d v = *d2p(tile + ((s * 4 + kk2) * 64 + lane) * 2);
            f[s][2 * kk2] = v.x;
            f[s][2 * kk2 + 1] = v.y;
        }
}

// The same from an LDS slot written by S1 in slot order: fragment pair (s, kk2) of L lives at
// pair index (kk2 / 2, s, kk2 % 2) -- where S1 read the matching half of the parked accumulator.
#ifndef RVK_GP64_S1HALF
#define RVK_GP64_S1HALF 1
#endif
__device__ __forceinline__ void load_slot_frags(const lds_d *tile, double (&f)[2][8], int lane) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int kk2 = 0; kk2 < 4; ++kk2) {
            const v2d v = *d2p(tile + ((((kk2 >> 1) * 2 + s) * 2 + (kk2 & 1)) * 64 + lane) * 2);
            f[s][2 * kk2] = v.x;
            f[s][2 * kk2 + 1] = v.y;
        }
}

// Quasi-periodic covariance of two epochs tau apart (gp.py:126-156; tinygp ExpSineSquared x
// ExpSquared, scaled by amp^2), fp64.
struct QP {
    double amp2, gam, inv_per, inv_le;
};
#ifndef RVK_GP64_FASTCOV
#define RVK_GP64_FASTCOV 1   // lean sin(pi u) and exp (below); 0: the device library's sinpi / exp
#endif
// sin(pi u)^2 for any finite u: u - rint(u) is exact and |r| <= 1/2, sin(pi u) = +-sin(pi r);
// sin(pi r) = pi r + r^3 Q(r^2) (least-squares fit, <= 2.7 ulp measured on [0, 1/2]) with pi
// split hi + lo so the leading term rounds once.  NaN / inf propagate as NaN.
__device__ __forceinline__ double sinpi_sq(double u) {
    const double r = u - __builtin_rint(u);
    const double r2 = r * r;
    double q = fma_s(r2, 7.696389727699914e-07, -2.1903364526655565e-05);
    q = fma_s(r2, q, 0.0004662997683854282);
    q = fma_s(r2, q, -0.007370430497584462);
    q = fma_s(r2, q, 0.0821458865724345);
    q = fma_s(r2, q, -0.5992645293189337);
    q = fma_s(r2, q, 2.550164039877302);
    q = fma_s(r2, q, -5.167712780049969);
    const double s = __builtin_fma(r, 3.141592653589793, r * fma_s(r2, q, 1.2246467991473532e-16));
    return s * s;
}
// exp(x) for x <= 0 (the covariance's exponent): k = rint(x / ln 2), r = x - k ln 2 in two parts
// (|r| <= ln2 / 2), exp(r) = 1 + r (1 + r P(r)) (least-squares fit, <= 1.3 ulp measured), 2^k by
// ldexp (0 below the subnormal range).  ocml's exp adds range and special-value checks the
// covariance never needs.
__device__ __forceinline__ double exp_nonpos(double x) {
    x = x < -800.0 ? -800.0 : x;                        // -inf -> 0 like exp (NaN passes: compare false)
    const double k = __builtin_rint(x * 1.4426950408889634);
    double r = __builtin_fma(k, -0.6931471805599453, x);
    r = __builtin_fma(k, -2.3190468138462996e-17, r);
    double p = fma_s(r, 2.50246452096493e-08, 2.7631125446226205e-07);
    p = fma_s(r, p, 2.755750728541229e-06);
    p = fma_s(r, p, 2.480149034623507e-05);
    p = fma_s(r, p, 0.00019841269597118904);
    p = fma_s(r, p, 0.0013888888946678828);
    p = fma_s(r, p, 0.008333333333451433);
    p = fma_s(r, p, 0.04166666666651632);
    p = fma_s(r, p, 0.16666666666666483);
    p = fma_s(r, p, 0.5000000000000012);
    p = __builtin_fma(r, __builtin_fma(r, p, 1.0), 1.0);
    int ki;
    asm("v_cvt_i32_f64 %0, %1" : "=v"(ki) : "v"(k));   // saturating (k <= 0 here)
    return __builtin_ldexp(p, ki);
}
// RVK_GP64_SINADD: sin(pi tau / P) = sin(a_i - a_j) = s_i c_j - c_i s_j with a_i = pi (t_i - t_0) / P
// reduced exactly (r = u - rint(u)), s_i = sin(pi r_i), c_i = cos(pi r_i) once per epoch: the squared
// value drops the (-1)^k signs of the reduction.  Same absolute error as the direct form (t_i - t_0
// is exact for dates of one magnitude; host check on config 5: 1.7e-14 vs 1.4e-14 max abs error
// in sin^2 against 40-digit values), 10 fewer fp64 instructions per covariance element.
#ifndef RVK_GP64_KILLACC
#define RVK_GP64_KILLACC 1   // zero the accumulator slots at each step start (ends their live ranges)
#endif
#ifndef RVK_GP64_COVSB
#define RVK_GP64_COVSB 0     // scheduling barrier after each covariance element (measured 6.43 vs 6.54 ms without)
#endif
#ifndef RVK_GP64_SINADD
#define RVK_GP64_SINADD 1
#endif
__device__ __forceinline__ double sinpi_red(double r) {    // sin(pi r), |r| <= 1/2 (sinpi_sq's fit)
    const double r2 = r * r;
    double q = fma_s(r2, 7.696389727699914e-07, -2.1903364526655565e-05);
    q = fma_s(r2, q, 0.0004662997683854282);
    q = fma_s(r2, q, -0.007370430497584462);
    q = fma_s(r2, q, 0.0821458865724345);
    q = fma_s(r2, q, -0.5992645293189337);
    q = fma_s(r2, q, 2.550164039877302);
    q = fma_s(r2, q, -5.167712780049969);
    return __builtin_fma(r, 3.141592653589793, r * fma_s(r2, q, 1.2246467991473532e-16));
}
__device__ __forceinline__ double cospi_red(double r) {    // cos(pi r), |r| <= 1/2: Taylor to r^20 (< 2e-17)
    const double z = r * r;
    double c = fma_s(z, 3.604730797462501e-09, -1.3878952462213771e-07);
    c = fma_s(z, c, 4.303069587032947e-06);
    c = fma_s(z, c, -0.0001046381049248457);
    c = fma_s(z, c, 0.0019295743094039231);
    c = fma_s(z, c, -0.02580689139001406);
    c = fma_s(z, c, 0.2353306303588932);
    c = fma_s(z, c, -1.3352627688545895);
    c = fma_s(z, c, 4.0587121264167685);
    c = fma_s(z, c, -4.934802200544679);
    return __builtin_fma(z, c, 1.0);
}
__device__ __forceinline__ double qp_cov_sn(const QP &h, double sn, double tau) {   // sn = sin(pi tau / P)
    const double x = tau * h.inv_le;
    return h.amp2 * exp_nonpos(-(h.gam * (sn * sn) + 0.5 * (x * x)));
}
__device__ __forceinline__ double qp_cov(const QP &h, double tau) {
#if RVK_GP64_FASTCOV
    const double sn2 = sinpi_sq(fabs(tau) * h.inv_per);
    const double x = tau * h.inv_le;
    return h.amp2 * exp_nonpos(-(h.gam * sn2 + 0.5 * (x * x)));
#else
    const double sn = sinpi(fabs(tau) * h.inv_per);
    const double x = tau * h.inv_le;
    return h.amp2 * exp(-(h.gam * (sn * sn) + 0.5 * (x * x)));
#endif
}

// The diagonal factor of one step, one wave (its own register allocation: a 32-double row or
// inverse column per lane never shares the register file with the accumulators).  fb holds
// acc(k, k) row-major on entry (its rows are then reused for the columns of L); li gets
// -X = -L_kk^-1 in fragment layout (and xdiag, if set); r_k = Lr[0..31] is replaced by y_k = X r_k.
// Right-looking: lane i < 32 holds row i of the symmetric acc(k, k) and applies every column m
// of L to it as soon as the column exists (a[i][t] -= L[i][m] L[t][m], t > m; the whole row, so
// the rows stay symmetric and the update is the same instruction for every lane); lane 32 + j
// turns column j of the identity into column j of X by the same update (b[t] -= L[t][m] x[m]).
// Column m reaches the other lanes through one LDS row (broadcast reads), except L[m+1][m],
// which the next pivot needs first: that one is read from lane m + 1 directly, so the pivot
// chain is readlane -> rsq -> scale -> readlane -> one FMA with the other 30 - m updates
// beside it.  Round 5 (sessions r5rlf / r5rlf3 / r5bal, 3 interleaved reps each, config 5
// fp64): 5.76-5.88 vs 5.90-5.97 ms for the left-looking form (row r of L read back through LDS
// before every pivot: 17.4 k cycles per factor vs 15.0 k, tools/gp64_trace.py); every column
// as scalars (v_readlane, no LDS) 18.3 k; the LDS form without its fence 17.0 k.
struct FactorAcc {
    double quad, dpr;
    int pexp;
};
__device__ __attribute__((noinline)) FactorAcc factor_diag(lds_d *fb, lds_d *li, lds_d *Lr, double *xdiag,
                                                           FactorAcc fa) {
    const int lane = threadIdx.x & 63;
    double quad = fa.quad, dpr = fa.dpr;
    int pexp = fa.pexp;
    double av[TB];
    const int lr = lane < 32 ? lane : 0;
#pragma unroll
    for (int m = 0; m < TB; ++m) {
        const double x = fb[lr * FS + m];
        av[m] = lane < 32 ? x : (m == lane - 32 ? 1.0 : 0.0);
    }
    wave_lds_sync();   // acc(k, k) is in registers: fb's rows now carry the columns of L
#pragma unroll
    for (int m = 0; m < TB; ++m) {
        const double piv = readlane_d(av[m], m);         // a[m][m] after columns < m: L[m][m]^2
        double y = __builtin_amdgcn_rsq(piv);            // 1 / L[m][m] (two Newton steps: ~1 ulp)
        y = y * __builtin_fma(-0.5 * piv, y * y, 1.5);
        y = y * __builtin_fma(-0.5 * piv, y * y, 1.5);
        const double c = lane == m ? piv * y : av[m] * y;   // L[i][m] (lane i < 32) or x[m] (lane >= 32)
        av[m] = c;
        dpr *= piv;
        if ((m & 7) == 7) {
            int e;
            dpr = __builtin_frexp(dpr, &e);
            pexp += e;
        }
        if (m + 1 < TB) {
            if (lane < 32) fb[m * FS + lane] = c;        // column m of L, as row m of fb
            av[m + 1] = __builtin_fma(-c, readlane_d(c, m + 1), av[m + 1]);
            if (m + 2 < TB) {
                wave_lds_sync();
#pragma unroll
                for (int t2 = (m + 2) & ~1; t2 < TB; t2 += 2) {
                    const v2d v = *d2p(fb + m * FS + t2);    // L[t2][m], L[t2 + 1][m] (broadcast)
                    if (t2 >= m + 2) av[t2] = __builtin_fma(-c, v.x, av[t2]);
                    av[t2 + 1] = __builtin_fma(-c, v.y, av[t2 + 1]);
                }
            }
        }
    }
    wave_lds_sync();
    if (lane >= 32) {                               // -X, fragment layout
        const int j = lane - 32, kk = j >> 2;
#pragma unroll
        for (int r = 0; r < TB; ++r) {
            const int o = fpair(r >> 4, kk >> 1, (j & 3) * 16 + (r & 15)) + (kk & 1);
            li[o] = -av[r];
            if (xdiag) xdiag[o] = -av[r];   // kept for the back substitution
        }
    }
    wave_lds_sync();
    if (lane < 32) {                                // y_k = X r_k, in place of r_k
        double y = 0.0;
#pragma unroll
        for (int j = 0; j < TB; ++j) y = __builtin_fma(-li[felem(lane, j)], Lr[j], y);
        quad += y * y;
        Lr[lane] = y;
    }
    return FactorAcc{quad, dpr, pexp};
}

// ---- the accumulation of one step (row owners), software-pipelined -------------------------
// acc(bi, k+1) -= sum_{j<k} L(bi, j) L(k+1, j)^T for the wave's live rows bi = wr + NA r, r = A..B
// (at most 3 at a time: the B operands of every live row share one load of the A operand
// L(k+1, j)).  The operands stream in quarter tiles (2 of the 8 k-steps of a 32 x 32 x 32
// product: one 16-byte load per lane per fragment row) through a ring of D register sets:
// D - 1 quarters are always in flight while one is consumed, and scheduling barriers keep the
// compiler from sinking the loads next to their MFMAs (which left every quarter's load latency
// exposed: the accumulation ran at ~40 % of the matrix pipe, profiles/round2/gp64_phase_trace.txt).
#ifndef RVK_GP64_RING
#define RVK_GP64_RING 2   // operand register sets (round 4: 6.24-6.34 ms vs 6.40-6.46 with 3, after the other changes)
#endif
template <int R>
struct Ops64 {
    double2 a[2];
    double2 b[R][2];
};

// The tile rows a row-owning wave owns, ascending (so the rows still live at a step are a suffix).
// Default: wr, wr + NA, wr + 2 NA, ...  RVK_GP64_BAL (nt == 16, 7 row waves, MAXR 3): a table that
// evens out each SIMD's matrix-pipe work per step (waves w and w + 4 share SIMD w mod 4; wave 7
// factors): summed over the 16 steps, the busiest SIMD's accumulation + S1 + S2 MFMAs drop from
// 9312 to 8192 (of 6400 per SIMD if perfectly even).
#ifndef RVK_GP64_BAL
#define RVK_GP64_BAL 1
#endif
template <int MAXR>
struct RowMap {
    int bi[MAXR];
    int nown;
};
template <int MAXR, int NA>
__device__ __forceinline__ RowMap<MAXR> row_map(int wr, int nt) {
    RowMap<MAXR> m;
    m.nown = 0;
#pragma unroll
    for (int q = 0; q < MAXR; ++q) m.bi[q] = wr + NA * q;
    m.nown = wr < nt ? (nt - wr + NA - 1) / NA : 0;
    if constexpr (RVK_GP64_BAL && RVK_GP64_RING > 1 && MAXR == 3 && NA == 7) {
        if (nt == 16) {
            constexpr int tab[7][3] = {{2, 10, 99}, {3, 11, 99}, {0, 1, 8}, {5, 9, 12}, {4, 13, 99}, {7, 14, 99}, {6, 15, 99}};
            constexpr int cnt[7] = {2, 2, 3, 3, 2, 2, 2};
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                int v = 99;
#pragma unroll
                for (int w = 0; w < 7; ++w) v = wr == w ? tab[w][q] : v;
                m.bi[q] = v;
            }
            int c = 0;
#pragma unroll
            for (int w = 0; w < 7; ++w) c = wr == w ? cnt[w] : c;
            m.nown = c;
        }
    }
    return m;
}

// HALFDIAG: a diagonal tile's block above the diagonal (rows 0-15, columns 16-31: C/D block
// c[1][0]) is never formed -- no covariance, no accumulation MFMAs, no S2 MFMAs: the
// right-looking factor reads only lane i's a[i][j <= i] (values above the diagonal stay above it),
// so that block is don't-care; it is left 0.  1/4 of every diagonal tile's MFMAs (the diagonal
// row is the first live row of its owner's first span): config 5 fp64 5.73-5.79 vs 5.79-5.87 ms
// (sessions r5hd / r5hd2, 3 + 4 interleaved reps, profiles/round5/ab_gp_round5b.json).
#ifndef RVK_GP64_HALFDIAG
#define RVK_GP64_HALFDIAG 1
#endif
// S1TRI: S1's A operand -X = -L_kk^-1 is lower triangular, so its block of rows 0-15 and columns
// 16-31 is exactly zero (the factor's inverse lanes never leave 0 above the diagonal for a positive
// definite tile): the 8 MFMAs of each S1 product that only multiply that block are skipped (the
// sums they would add are +-0: the same bits, checked with tools/gp_dump.py on the log-likelihood
// and the conditioned mean): config 5 fp64 5.61-5.74 vs 5.73-5.79 ms (session r5s1, 4 interleaved reps).
#ifndef RVK_GP64_S1TRI
#define RVK_GP64_S1TRI 1
#endif
template <int MAXR, int NA, int A, int B, int D>
__device__ __forceinline__ void accum_span(Acc (&acc)[MAXR], const double *__restrict__ wk, int k, const RowMap<MAXR> &rm,
                                           int lane) {
    constexpr int R = B - A + 1;
    const bool dg = RVK_GP64_HALFDIAG && rm.bi[A] == k + 1;   // wave-uniform
    const int NQ = 4 * k;                           // quarters (j, part), j < k
    const double2 *rowa = reinterpret_cast<const double2 *>(wk + tix(k + 1, 0) * TILE) + lane;
    const double2 *rowb[R];
#pragma unroll
    for (int r = 0; r < R; ++r) rowb[r] = reinterpret_cast<const double2 *>(wk + tix(rm.bi[A + r], 0) * TILE) + lane;
    Ops64<R> ops[D];
    auto issue = [&](Ops64<R> &o, int hx) {         // unconditional (clamped past the end): the
        hx = hx < NQ ? hx : NQ - 1;                 // wait counts stay exact on every path
        const int j = hx >> 2, part = hx & 3;
        const int off = j * (TILE / 2) + part * 64;  // double2 units: tiles of row bi are contiguous in j
        const int offa = (RVK_GP64_ABLATE & 1) ? part * 64 : off, offb = (RVK_GP64_ABLATE & 2) ? part * 64 : off;
        o.a[0] = rowa[offa];
        o.a[1] = rowa[offa + 256];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            o.b[r][0] = rowb[r][offb];
            o.b[r][1] = rowb[r][offb + 256];
        }
    };
    auto consume = [&](const Ops64<R> &o) {
#pragma unroll
        for (int cmp = 0; cmp < 2; ++cmp)
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int p = 0; p < 2; ++p)
#pragma unroll
                    for (int q = 0; q < 2; ++q) {
                        if (RVK_GP64_HALFDIAG && r == 0 && p == 1 && q == 0 && dg) continue;
                        acc[A + r].c[p][q] = mfma64(cmp ? o.a[p].y : o.a[p].x, cmp ? o.b[r][q].y : o.b[r][q].x,
                                                    acc[A + r].c[p][q]);
                    }
    };
#pragma unroll
    for (int d = 0; d < D - 1; ++d) issue(ops[d], d);
    for (int hx = 0; hx < NQ; hx += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            issue(ops[(d + D - 1) % D], hx + d + D - 1);
            __builtin_amdgcn_sched_barrier(0);
            if (hx + d < NQ) consume(ops[d]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// The live rows A0 .. B0 of a wave (a suffix of its rows: rows finish in order), in spans of <= 3.
template <int MAXR, int NA, int D>
__device__ __forceinline__ void accum_rows(Acc (&acc)[MAXR], const double *__restrict__ wk, int k, const RowMap<MAXR> &rm,
                                           int lane, int a0, int b0) {
    for (int a = a0; a <= b0; a += 3) {
        const int b = a + 2 < b0 ? a + 2 : b0;
#define RVK_SPAN(X, Y)                                                                   \
    if constexpr (Y < MAXR) {                                                            \
        if (a == X && b == Y) accum_span<MAXR, NA, X, Y, D>(acc, wk, k, rm, lane);       \
    }
        RVK_SPAN(0, 0) RVK_SPAN(0, 1) RVK_SPAN(0, 2) RVK_SPAN(1, 1) RVK_SPAN(1, 2) RVK_SPAN(1, 3)
        RVK_SPAN(2, 2) RVK_SPAN(2, 3) RVK_SPAN(2, 4) RVK_SPAN(3, 3) RVK_SPAN(3, 4) RVK_SPAN(4, 4)
#undef RVK_SPAN
    }
}

#ifndef RVK_GP64_LDSPARK
#define RVK_GP64_LDSPARK 1   // parked accumulators and S1's new tiles in LDS slots (nt <= 16)
#endif
template <int MAXR, bool GROUPED>
constexpr bool gp64_ldsp() { return RVK_GP64_LDSPARK && MAXR == 3 && !GROUPED; }

// MAXR tile rows per row-owning wave; GROUPED: the rows go through the workspace in
// groups of MAXR (a separate instantiation: the common shape keeps its register allocation)
template <int NW, int MAXR, bool COND, bool GROUPED>
__global__ __launch_bounds__(64 * NW, 1) void gp64_kernel(const Gp64Args a) {
    constexpr int NT = 64 * NW;
    extern __shared__ double smem64[];
    const int n = a.n, ni = a.ni, np = a.np;
    const int nt = (n + TB - 1) / TB, npad = nt * TB;
    // LDSP (nt <= 16): every tile row bi >= 1 has an LDS slot that holds, in turn, its parked
    // accumulator acc(bi, k) (S2(k-1) -> S1(k)) and its new factor tile L(bi, k) (S1(k) -> S2(k)),
    // so S1 and S2 read their operands from LDS instead of the workspace (15 x 8 KB at n = 512)
    constexpr bool LDSP = gp64_ldsp<MAXR, GROUPED>();
    double *slots = smem64;           // [nt - 1][TILE] (LDSP)
    auto pslot = [&](int bi) { return (lds_d *)(slots + (bi - 1) * TILE); };
    double *Lt = smem64 + (LDSP ? (nt - 1) * TILE : 0);   // [npad] epochs (padding: t[n-1])
    double *Lr = Lt + npad;           // [npad] rhs r, reduced in place; segment k becomes y_k (then alpha_k)
    // [npad] velerr^2 + jit^2 (padding: 1); SINADD: [npad] s_i, [npad] c_i instead (the diagonal
    // tiles read velerr^2 + jit^2 from global memory)
    double *Ldia = Lr + npad;
    double *Ls = Lr + npad, *Lc = Ls + npad;
    double *fb = Lr + (RVK_GP64_SINADD ? 3 : 2) * npad;   // [TB][FS] the factor's row buffer; back substitution partial sums
    double *li = fb + TB * FS;        // [TILE] -X = -L_kk^-1 of the step, fragment layout
    double *red = li + TILE;          // [2 NW]
    SC *tab = reinterpret_cast<SC *>(red + 2 * NW);
    PlanetK *pks = reinterpret_cast<PlanetK *>(tab + kTabN);
    int *oks = reinterpret_cast<int *>(pks + np);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wr = __builtin_amdgcn_readfirstlane(tid >> 6);   // this wave owns tile rows wr, wr + NW, ...
    const EpochData &d = a.d;
    const bool multi = ni > 1, tp = d.par == RVK_PAR_PKEWTP;
    for (int i = tid; i < kTabN; i += NT) tab_put(tab, i, d.tab[i], d.poison);
    __syncthreads();   // the table is read by the planet prep below (threads < np), before any other barrier
    double *wk = a.work + (long long)blockIdx.x * a.work_stride;

    for (long long w = blockIdx.x; w < a.W; w += gridDim.x) {
        if (a.gate && !__builtin_isnan(a.gate[w])) continue;          // fallback: only the fp32 NaN walkers
        if (!COND && a.post.lp && a.post.lp[w] == -INFINITY) {           // rejected before the likelihood
            if (tid == 0) a.out[w] = -INFINITY;
            continue;
        }
        const double *row = a.theta + w * a.stride;
        const double *hp = a.hyper + w * a.hstride;
        // ---- 1. planets, mean model, residuals -----------------------------------------------
        if (tid < np) {
            PlanetK pk;
            const bool ok = tp ? planet_consts_t<0, true>(row + 5 * tid, pk, 0, tab) : planet_consts(d.par, row + 5 * tid, pk);
            pks[tid] = pk;
            oks[tid] = ok;
        }
        __syncthreads();   // (the table fill of the first trip lands here too)
        bool alive = true;
        for (int p = 0; p < np; ++p) alive &= oks[p] != 0;
        if (!alive) {                                      // fit.py:8083-8085 / Planet() raises
            if (COND) {
                for (long long q = tid; q < a.T; q += NT) a.pred[w * a.T + q] = NAN;
            } else if (tid == 0) {
                a.out[w] = -INFINITY;
            }
            __syncthreads();
            continue;
        }
        const double *g = row + 5 * np, *jit = g + ni;
        const double gd = jit[ni], gdd = jit[ni + 1];
        const QP h{hp[0] * hp[0], 1.0 / (2.0 * hp[2] * hp[2]), 1.0 / hp[3], 1.0 / hp[1]};
        for (int i = tid; i < npad; i += NT) {
            const double t = d.t[i < n ? i : n - 1];
            Lt[i] = t;
            double ri = 0.0, di = 1.0;
            if (i < n) {
                const int ii = multi ? d.inst[i] : 0;
                double rv = 0.0;
                for (int p = 0; p < np; ++p) rv = planet_rv<0>(pks[p], t, tab, rv);
                const double dt = t - d.t0;
                rv += __builtin_fma(gd, dt, gdd * (dt * dt));      // Trend (fit.py:8031-8035)
                rv += g[ii];                                       // gamma (fit.py:8041-8045)
                ri = d.vel[i] - rv;
                di = d.s2[i] + jit[ii] * jit[ii];                  // fit.py:8096-8098
            }
            Lr[i] = ri;
            if constexpr (RVK_GP64_SINADD) {
                const double u = (t - d.t[0]) * h.inv_per;
                const double r = u - __builtin_rint(u);
                Ls[i] = sinpi_red(r);
                Lc[i] = cospi_red(r);
                (void)di;
            } else {
                Ldia[i] = di;
            }
        }
        __syncthreads();
        // ---- 2. pipelined blocked Cholesky -----------------------------------------------------
        // -C(bi, bj)^T in C/D layout; padding rows/columns are identity
        // k(t_i - t_j) for this lane's row value (ti, and s_i, c_i under SINADD) and column gj
        auto kval = [&](double ti, double si, double ci, int gj) -> double {
            const double tj = Lt[gj];
            if (RVK_GP64_ABLATE & 16) return 0.5 * (ti - tj);
            if constexpr (RVK_GP64_SINADD) return qp_cov_sn(h, __builtin_fma(si, Lc[gj], -(ci * Ls[gj])), ti - tj);
            else return qp_cov(h, ti - tj);
        };
        auto cov_tile = [&](int bi, int bj, Acc &A) {
            if (bi != bj && (bi + 1) * TB <= n) {          // off-diagonal tile inside the data (bj < bi)
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int gi = bi * TB + 16 * q + (lane & 15);
                    const double ti = Lt[gi];
                    const double si = RVK_GP64_SINADD ? Ls[gi] : 0.0, ci = RVK_GP64_SINADD ? Lc[gi] : 0.0;
#pragma unroll
                    for (int p = 0; p < 2; ++p)
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            A.c[p][q][i] = -kval(ti, si, ci, bj * TB + 16 * p + (lane >> 4) + 4 * i);
                            if (RVK_GP64_COVSB) __builtin_amdgcn_sched_barrier(0);   // one element at a time
                        }
                }
                return;
            }
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int gi = bi * TB + 16 * q + (lane & 15);
                const double ti = Lt[gi];
                const double si = RVK_GP64_SINADD ? Ls[gi] : 0.0, ci = RVK_GP64_SINADD ? Lc[gi] : 0.0;
                double di = 1.0;
                if constexpr (RVK_GP64_SINADD) {                   // (as phase 1 forms it)
                    if (bi == bj && gi < n) {
                        const int ii = multi ? d.inst[gi] : 0;
                        di = d.s2[gi] + jit[ii] * jit[ii];
                    }
                } else {
                    di = Ldia[gi];
                }
#pragma unroll
                for (int p = 0; p < 2; ++p)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        if (RVK_GP64_HALFDIAG && p == 1 && q == 0 && bi == bj) {   // above the diagonal
                            A.c[p][q][i] = 0.0;
                            continue;
                        }
                        const int gj = bj * TB + 16 * p + (lane >> 4) + 4 * i;
                        const double kv = kval(ti, si, ci, gj);
                        const bool in = gi < n && gj < n, dg = gi == gj;
                        const double v = in ? (dg ? kv + di : kv) : (dg ? 1.0 : 0.0);
                        A.c[p][q][i] = -v;
                    }
            }
        };
        double quad = 0.0;          // sum of y^2 (the factor wave's lanes)
        double dpr = 1.0;           // product of the pivots L_ii^2, renormalised (x 2^pexp; factor wave)
        int pexp = 0;
        // Waves 0 .. NA-1 own the tile rows (wr, wr + NA, ...) and do the MFMA work; wave NA
        // factors every diagonal tile.  The roles run separate loops with the same barriers,
        // so the factor's registers (a 32-double row per lane) never coexist with the
        // accumulators.  acc(k, k) travels to the factor wave through fb.
        constexpr int NA = NW - 1;
        auto put_diag = [&](const Acc &A) {          // fb[row][col] = acc(k, k) (from -acc^T, C/D layout)
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int q = 0; q < 2; ++q)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        fb[(16 * q + (lane & 15)) * FS + 16 * p + (lane >> 4) + 4 * i] = -A.c[p][q][i];
        };
        const RowMap<MAXR> rm = row_map<MAXR, NA>(wr, nt);   // the non-grouped shapes' row ownership
        auto col0 = [&](int bi) {
            Acc t;
            cov_tile(bi, 0, t);
            if (bi == 0) put_diag(t);
            else if constexpr (LDSP) park(pslot(bi), t, lane);
            else park(wk + tix(bi, 0) * TILE, t, lane);
        };
        if (wr < NA) {
            if constexpr (GROUPED) {
                for (int bi = wr; bi < nt; bi += NA) col0(bi);   // every owned row (also past MAXR)
            } else {
#pragma unroll
                for (int q = 0; q < MAXR; ++q)
                    if (q < rm.nown) col0(rm.bi[q]);
            }
        }
        __syncthreads();
        if (wr == NA) {
            // ---- the factor wave: P(k) for every k, then the step's barriers ----------------------
            for (int k = 0; k < nt; ++k) {
                G64_MARK(k, 0);
                __builtin_amdgcn_s_setprio(1);    // the step's critical path goes first on its SIMD
                if (!(RVK_GP64_ABLATE & 4)) {
                    const FactorAcc fa = factor_diag((lds_d *)fb, (lds_d *)li, (lds_d *)(Lr + k * TB),
                                                     COND ? wk + tix(k, k) * TILE : nullptr, FactorAcc{quad, dpr, pexp});
                    quad = fa.quad;
                    dpr = fa.dpr;
                    pexp = fa.pexp;
                }
                __builtin_amdgcn_s_setprio(0);
                G64_MARK(k, 1);
                G64_MARK(k, 2);
                __syncthreads();                            // B1: -X and y_k published
                G64_MARK(k, 3);
                if (k + 1 == nt) break;
                G64_MARK(k, 4);
                __syncthreads();                            // B2 (S1 runs on the other waves)
                G64_MARK(k, 5);
                __syncthreads();                            // B3: acc(k+1, k+1) in fb
                G64_MARK(k, 6);
            }
        } else {
            // ---- the row owners: the next column's accumulation, S1, S2 --------------------------
            Acc nacc[MAXR];
            const int nown = GROUPED ? (nt - wr + NA - 1) / NA : rm.nown;   // rows this wave owns
            constexpr bool grouped = GROUPED;               // more rows than accumulator registers
            for (int k = 0; k < nt; ++k) {
                G64_MARK(k, 0);
                G64_MARK(k, 1);
                if (RVK_GP64_KILLACC) {
                    // every live slot is re-formed from the covariance below and the previous step's
                    // values were parked by S2: ending their live ranges here keeps the compiler from
                    // carrying all MAXR accumulators (and spilling them) across the whole step
#pragma unroll
                    for (int q = 0; q < MAXR; ++q)
#pragma unroll
                        for (int p = 0; p < 2; ++p)
#pragma unroll
                            for (int qq = 0; qq < 2; ++qq) nacc[q].c[p][qq] = f64x4{0.0, 0.0, 0.0, 0.0};
                }
                for (int qo = 0; qo < (grouped ? nown : 1) && k + 1 < nt; qo += MAXR) {   // one trip unless grouped
                    if (grouped && wr + NA * (qo + MAXR - 1) < k + 1) continue;    // the group's rows are finished
#pragma unroll
                    for (int q = 0; q < MAXR; ++q) {
                        const int bi = grouped ? wr + NA * (qo + q) : rm.bi[q];
                        if (bi >= k + 1 && bi < nt && (grouped || q < nown)) cov_tile(bi, k + 1, nacc[q]);
                    }
                    // operands: the A tile L(k+1, j) and the B tiles L(bi, j) of two owned rows at a time,
                    // a quarter tile (2 of the 8 k-steps) per register set; sets X / Y alternate so the
                    // next quarter's loads are in flight during this quarter's MFMAs.  The trip past the
                    // end re-reads the last quarter (unconditional loads, exact waits).
                    auto pass = [&](auto q0c) {
                        constexpr int Q0 = decltype(q0c)::value;
                        constexpr int R = (MAXR - Q0) < 2 ? (MAXR - Q0) : 2;
                        bool any = false;
#pragma unroll
                        for (int q = Q0; q < Q0 + R; ++q) any |= (wr + NA * (qo + q) >= k + 1) && (wr + NA * (qo + q) < nt);
                        if (!any || k == 0) return;
                        constexpr int KP = 1, NSET = 4 / KP;   // fragment pairs per register set, sets per tile
                        struct Ops {
                            double2 a[2][KP], b[R][2][KP];
                        };
                        auto issue = [&](Ops &o, int hx) {
                            const int hh = hx < NSET * k ? hx : NSET * k - 1;
                            const int j = hh / NSET, part = hh % NSET;
                            const double2 *ta = reinterpret_cast<const double2 *>(
                                wk + tix(k + 1, (RVK_GP64_ABLATE & 1) ? 0 : j) * TILE);
#pragma unroll
                            for (int s = 0; s < 2; ++s)
#pragma unroll
                                for (int u = 0; u < KP; ++u) o.a[s][u] = ta[(s * 4 + KP * part + u) * 64 + lane];
#pragma unroll
                            for (int r = 0; r < R; ++r) {
                                const int bi = wr + NA * (qo + Q0 + r);
                                const bool live = bi >= k + 1 && bi < nt;
                                const double2 *tb = reinterpret_cast<const double2 *>(
                                    wk + tix(live ? bi : k + 1, (RVK_GP64_ABLATE & 2) ? 0 : j) * TILE);
#pragma unroll
                                for (int s = 0; s < 2; ++s)
#pragma unroll
                                    for (int u = 0; u < KP; ++u) o.b[r][s][u] = tb[(s * 4 + KP * part + u) * 64 + lane];
                            }
                        };
                        auto consume = [&](const Ops &o) {
#pragma unroll
                            for (int r = 0; r < R; ++r) {
                                const int bi = wr + NA * (qo + Q0 + r);
                                if (bi >= k + 1 && bi < nt) {
                                    Acc &acc = nacc[Q0 + r];
#pragma unroll
                                    for (int u = 0; u < KP; ++u)
#pragma unroll
                                        for (int cmp = 0; cmp < 2; ++cmp)
#pragma unroll
                                            for (int p = 0; p < 2; ++p)
#pragma unroll
                                                for (int q = 0; q < 2; ++q)
                                                    acc.c[p][q] = mfma64(cmp ? o.a[p][u].y : o.a[p][u].x,
                                                                         cmp ? o.b[r][q][u].y : o.b[r][q][u].x, acc.c[p][q]);
                                }
                            }
                        };
                        Ops X, Y;
                        issue(X, 0);
                        for (int hx = 0; hx < NSET * k; hx += 2) {
                            issue(Y, hx + 1);
                            if (!(RVK_GP64_ABLATE & 8)) consume(X);
                            issue(X, hx + 2);
                            if (!(RVK_GP64_ABLATE & 8)) consume(Y);
                        }
                    };
                    if constexpr (!grouped && RVK_GP64_RING > 1) {
                        // the live rows (a suffix of the owned ones), software-pipelined
                        int r0 = nown;                          // the first live row
#pragma unroll
                        for (int q = MAXR - 1; q >= 0; --q)
                            if (q < nown && rm.bi[q] >= k + 1) r0 = q;
                        if (k > 0 && r0 < nown && !(RVK_GP64_ABLATE & 8))
                            accum_rows<MAXR, NA, RVK_GP64_RING>(nacc, wk, k, rm, lane, r0, nown - 1);
                    } else {
                        pass(std::integral_constant<int, 0>{});
                        if constexpr (MAXR > 2) pass(std::integral_constant<int, 2>{});
                        if constexpr (MAXR > 4) pass(std::integral_constant<int, 4>{});
                        if constexpr (MAXR > 6) pass(std::integral_constant<int, 6>{});
                    }
                    if constexpr (grouped) {                // park the group: S2 reads it back
#pragma unroll
                        for (int q = 0; q < MAXR; ++q) {
                            const int bi = wr + NA * (qo + q);
                            if (bi >= k + 1 && bi < nt) park(wk + tix(bi, k + 1) * TILE, nacc[q], lane);
                        }
                    }
                }
                G64_MARK(k, 2);
                __syncthreads();                            // B1: -X and y_k published
                G64_MARK(k, 3);
                if (k + 1 == nt) break;
                // ---- S1(k): L(bi, k) = acc(bi, k) X^T, stored; rhs update ----------------------
            {
                double xa[2][8];
                {
                    const double2 *X2 = reinterpret_cast<const double2 *>(li);
#pragma unroll
                    for (int s = 0; s < 2; ++s)
#pragma unroll
                        for (int kk2 = 0; kk2 < 4; ++kk2) {
                            const double2 v = X2[(s * 4 + kk2) * 64 + lane];
                            xa[s][2 * kk2] = v.x;
                            xa[s][2 * kk2 + 1] = v.y;
                        }
                }
                double yv[2][4];
#pragma unroll
                for (int p = 0; p < 2; ++p)
#pragma unroll
                    for (int i = 0; i < 4; ++i) yv[p][i] = Lr[k * TB + 16 * p + (lane >> 4) + 4 * i];
#pragma unroll
                for (int q = 0; q < (grouped ? nown : MAXR); ++q) {
                    const int bi = grouped ? wr + NA * q : rm.bi[q];
                    if (bi > k && bi < nt && q < nown) {
                        double *T = wk + tix(bi, k) * TILE;
                        if constexpr (LDSP && RVK_GP64_S1HALF) {
                            // by output column half qq: the half of the parked acc it reads (slot pairs
                            // (x, qq, ih)) is the half its L columns overwrite, in the slot's own order
                            // (load_slot_frags), so a wave holds half of cur and half of L at a time
                            const lds_d *sl = pslot(bi);
#pragma unroll
                            for (int qq = 0; qq < 2; ++qq) {
                                f64x4 cu[2];
#pragma unroll
                                for (int x = 0; x < 2; ++x)
#pragma unroll
                                    for (int ih = 0; ih < 2; ++ih) {
                                        const v2d v = *d2p(sl + (((x * 2 + qq) * 2 + ih) * 64 + lane) * 2);
                                        cu[x][2 * ih] = v.x;
                                        cu[x][2 * ih + 1] = v.y;
                                    }
                                f64x4 o[2] = {f64x4{0.0, 0.0, 0.0, 0.0}, f64x4{0.0, 0.0, 0.0, 0.0}};
#pragma unroll
                                for (int kk = 0; kk < 8; ++kk)
#pragma unroll
                                    for (int p = 0; p < 2; ++p) {
                                        if (RVK_GP64_S1TRI && p == 0 && kk >= 4) continue;   // X rows 0-15, cols 16-31: 0
                                        o[p] = mfma64(xa[p][kk], cu[kk >> 2][kk & 3], o[p]);
                                    }
                                double s = 0.0;
#pragma unroll
                                for (int p = 0; p < 2; ++p) {
#pragma unroll
                                    for (int ih = 0; ih < 2; ++ih) {
                                        const v2d v = {o[p][2 * ih], o[p][2 * ih + 1]};
                                        d2p(T)[(qq * 4 + 2 * p + ih) * 64 + lane] = v;
                                        d2p(pslot(bi))[((p * 2 + qq) * 2 + ih) * 64 + lane] = v;   // slot order
                                    }
#pragma unroll
                                    for (int i = 0; i < 4; ++i) s = __builtin_fma(o[p][i], yv[p][i], s);
                                }
                                s += __shfl_xor(s, 16);
                                s += __shfl_xor(s, 32);
                                if (lane < 16) Lr[bi * TB + 16 * qq + lane] -= s;
                            }
                            continue;
                        }
                        Acc cur;
                        if constexpr (LDSP) unpark(pslot(bi), cur, lane);
                        else unpark(T, cur, lane);
                        Acc o;
#pragma unroll
                        for (int p = 0; p < 2; ++p)
#pragma unroll
                            for (int qq = 0; qq < 2; ++qq) o.c[p][qq] = f64x4{0.0, 0.0, 0.0, 0.0};
                        // L(bi, k)^T = (-X) (-acc)^T: A = -X fragments, B = the parked C/D registers
#pragma unroll
                        for (int kk = 0; kk < 8; ++kk)
#pragma unroll
                            for (int p = 0; p < 2; ++p)
#pragma unroll
                                for (int qq = 0; qq < 2; ++qq) {
                                    if (RVK_GP64_S1TRI && p == 0 && kk >= 4) continue;   // X rows 0-15, cols 16-31: 0
                                    o.c[p][qq] = mfma64(xa[p][kk], cur.c[kk >> 2][qq][kk & 3], o.c[p][qq]);
                                }
                        // o.c[p][qq][i] at lane l = L(bi, k)[16 qq + (l & 15)][16 p + (l >> 4) + 4 i]
                        //                         = frag(qq, 4 p + i)[l]
#pragma unroll
                        for (int qq = 0; qq < 2; ++qq) {
                            double s = 0.0;
#pragma unroll
                            for (int p = 0; p < 2; ++p) {
#pragma unroll
                                for (int ih = 0; ih < 2; ++ih) {
                                    const v2d v = {o.c[p][qq][2 * ih], o.c[p][qq][2 * ih + 1]};
                                    d2p(T)[(qq * 4 + 2 * p + ih) * 64 + lane] = v;
                                    if constexpr (LDSP) d2p(pslot(bi))[(qq * 4 + 2 * p + ih) * 64 + lane] = v;   // for S2
                                }
#pragma unroll
                                for (int i = 0; i < 4; ++i) s = __builtin_fma(o.c[p][qq][i], yv[p][i], s);
                            }
                            s += __shfl_xor(s, 16);
                            s += __shfl_xor(s, 32);
                            if (lane < 16) Lr[bi * TB + 16 * qq + lane] -= s;
                        }
                    }
                }
            }
                G64_MARK(k, 4);
                __syncthreads();                            // B2: L(k+1, k) published
                G64_MARK(k, 5);
                // ---- S2(k): the j = k term; park for S1(k+1), the diagonal tile to fb -----------
            {
                double af[2][8];
                if constexpr (LDSP && RVK_GP64_S1HALF) load_slot_frags(pslot(k + 1), af, lane);
                else if constexpr (LDSP) load_frags(pslot(k + 1), af, lane);
                else load_frags(wk + tix(k + 1, k) * TILE, af, lane);
                auto s2 = [&](Acc &acc, int bi) {
                    double bf[2][8];
                    if constexpr (LDSP && RVK_GP64_S1HALF) load_slot_frags(pslot(bi), bf, lane);
                    else if constexpr (LDSP) load_frags(pslot(bi), bf, lane);
                    else load_frags(wk + tix(bi, k) * TILE, bf, lane);
#pragma unroll
                    for (int kk = 0; kk < 8; ++kk)
#pragma unroll
                        for (int p = 0; p < 2; ++p)
#pragma unroll
                            for (int qq = 0; qq < 2; ++qq) {
                                if (RVK_GP64_HALFDIAG && p == 1 && qq == 0 && bi == k + 1) continue;
                                acc.c[p][qq] = mfma64(af[p][kk], bf[qq][kk], acc.c[p][qq]);
                            }
                    if (bi == k + 1) put_diag(acc);
                    else if constexpr (LDSP) park(pslot(bi), acc, lane);
                    else park(wk + tix(bi, k + 1) * TILE, acc, lane);
                };
                if constexpr (!grouped) {
#pragma unroll
                    for (int q = 0; q < MAXR; ++q) {
                        const int bi = rm.bi[q];
                        if (bi > k && bi < nt && q < nown) s2(nacc[q], bi);
                    }
                } else {
                    for (int q = 0; q < nown; ++q) {
                        const int bi = wr + NA * q;
                        if (bi > k && bi < nt) {
                            Acc acc;
                            unpark(wk + tix(bi, k + 1) * TILE, acc, lane);
                            s2(acc, bi);
                        }
                    }
                }
            }
                __syncthreads();                            // B3: acc(k+1, k+1) in fb
                G64_MARK(k, 6);
            }
        }
        if (!COND) {
            // ---- 3. ll = -1/2 y.y - 1/2 sum log L_ii^2 - n/2 log 2 pi ---------------------------
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) quad += __shfl_xor(quad, o);
            if (lane == 0) {
                red[2 * wr] = quad;
                red[2 * wr + 1] = log(dpr) + (double)pexp * kLn2;
            }
            __syncthreads();
            if (tid == 0) {
                double qs = 0.0, ls = 0.0;
                for (int u = 0; u < NW; ++u) {
                    qs += red[2 * u];
                    ls += red[2 * u + 1];
                }
                double ll = -0.5 * qs - 0.5 * ls - 0.5 * (double)n * kLog2Pi;
                if (!__builtin_isfinite(ll)) ll = NAN;             // not positive definite
                if (a.post.lp) ll = (((ll + a.post.lp[w]) + a.post.lhp[w]) + a.post.jac) + a.post.renorm;
                a.out[w] = ll;
            }
            __syncthreads();
        } else {
            // ---- 3'. alpha = L^-T y: alpha_k = X_kk^T (y_k - sum_{bi > k} L(bi, k)^T alpha_bi) -----
            constexpr int G = NT / TB;
            const int c = tid & (TB - 1), gq = tid / TB;
            for (int k = nt - 1; k >= 0; --k) {
                double part = 0.0;
                for (int bi = k + 1 + gq; bi < nt; bi += G) {
                    const double *T = wk + tix(bi, k) * TILE;
#pragma unroll 8
                    for (int r = 0; r < TB; ++r) part = __builtin_fma(T[felem(r, c)], Lr[bi * TB + r], part);
                }
                fb[gq * TB + c] = part;
                __syncthreads();
                if (tid < TB) {
                    double z = Lr[k * TB + c];
                    for (int u = 0; u < G; ++u) z -= fb[u * TB + c];
                    fb[G * TB + c] = z;
                }
                __syncthreads();
                if (tid < TB) {
                    const double *X = wk + tix(k, k) * TILE;    // -X, fragment layout
                    double al = 0.0;
#pragma unroll 8
                    for (int i = 0; i < TB; ++i) al = __builtin_fma(-X[felem(i, c)], fb[G * TB + i], al);
                    Lr[k * TB + c] = al;
                }
                __syncthreads();
            }
            // mean(t_q) = sum_i k(t_q - t_i) alpha_i   (K(X_test, X) alpha; no diagonal term)
            for (long long q = tid; q < a.T; q += NT) {
                const double tq = a.tq[q];
                double acc = 0.0;
                for (int i = 0; i < n; ++i) acc = __builtin_fma(qp_cov(h, tq - Lt[i]), Lr[i], acc);
                a.pred[w * a.T + q] = acc;
            }
            __syncthreads();
        }
    }
}

template <int NW, int MAXR, bool COND, bool GROUPED>
void launch_gp64(hipStream_t st, unsigned grid, size_t lds, const Gp64Args &a) {
    static size_t allowed = 0;   // dynamic LDS beyond the default needs the attribute
    if (lds > allowed) {
        (void)hipFuncSetAttribute((const void *)gp64_kernel<NW, MAXR, COND, GROUPED>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        allowed = lds;
    }
    hipLaunchKernelGGL((gp64_kernel<NW, MAXR, COND, GROUPED>), dim3(grid), dim3(64 * NW), lds, st, a);
}

}  // namespace

namespace rvk {

Gp64Shape gp64_shape(int n) {
    const int nt = (n + TB - 1) / TB;
    // 7 row-owning waves + the factor wave.  nt <= 16: three accumulator rows per wave, parked in LDS
    // slots; 17..35: the rows go through the workspace in groups of three; beyond: groups of five.
    // (Round 6, fp64, 4096 walkers: the grouped 3-row kernel -- 0 VGPRs spilled, 96 B of scratch --
    // against the ungrouped 5-row kernel it replaces for 17..35 -- 253 VGPRs spilled, 944 B --
    // n = 700 16.6 vs 20.4 ms, n = 1024 48.2 vs 52.1; at n = 2048 the 5-row groups stay ahead, 373.9
    // vs 377.9; at n = 512 the LDS-slot kernel stays ahead of any grouped form, 5.65 vs 7.2 ms;
    // profiles/round6/gp64/ab_shapes.json.  The ungrouped 5-row kernel was also the one whose
    // register allocation faulted twice at n = 700 under semantically neutral changes: DESIGN §3.)
    return nt <= 16 ? Gp64Shape{8, 3, false} : nt <= 35 ? Gp64Shape{8, 3, true} : Gp64Shape{8, 5, true};
}

size_t gp64_lds_bytes(int n, int np, int nw) {
    const int nt = (n + TB - 1) / TB;
    size_t b = sizeof(double) * ((RVK_GP64_SINADD ? 4 : 3) * (size_t)nt * TB + TB * FS + TILE + 2 * (size_t)nw);
    const Gp64Shape sh = gp64_shape(n);
    if (sh.maxr == 3 && !sh.grouped && gp64_ldsp<3, false>()) b += sizeof(double) * (size_t)(nt - 1) * TILE;   // LDS slots
    b += sizeof(SC) * kTabN + (sizeof(PlanetK) + sizeof(int)) * (size_t)np + 16;
    return b;
}

long long gp64_work_doubles(int n) {
    const long long nt = (n + TB - 1) / TB;
    return nt * (nt + 1) / 2 * TILE;
}

gp64_launch_t pick_gp64(int np, bool multi, bool tp, bool condition, Gp64Shape sh) {
    (void)multi;
    (void)tp;
    if (np < 1 || np > RVK_MAX_PLANETS) return nullptr;
    if (sh.maxr == 3 && !sh.grouped) return condition ? launch_gp64<8, 3, true, false> : launch_gp64<8, 3, false, false>;
    if (sh.maxr == 3) return condition ? launch_gp64<8, 3, true, true> : launch_gp64<8, 3, false, true>;
    return condition ? launch_gp64<8, 5, true, true> : launch_gp64<8, 5, false, true>;
}

}  // namespace rvk

#if RVK_GP64_TRACE
extern "C" int rvk_gp64_trace_dump(unsigned long long *host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gp64_trace), sizeof(g_gp64_trace)) == hipSuccess ? 0 : -1;
}
#endif
