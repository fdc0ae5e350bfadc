// rvk_gp.hip -- batched quasi-periodic GP log-likelihood (include/rvk_gp.h;
// SURVEY.md §8(f) row 2, BASELINE config 5).
//
// One workgroup of NW waves per walker (NW = 4 for n <= 512, 8 for n <= 1024),
// grid-stride over walkers.  Per walker:
//   1. planet constants (lanes over planets) and the mean model in fp64 (the
//      log-likelihood kernel's Kepler solver, threads over epochs) -> residuals
//      r and the diagonal velerr^2 + jit^2 in LDS (fp32);
//   2. blocked fp32 Cholesky over 32-wide tile columns k with the right-hand
//      side carried along, pipelined one column ahead.  Tile row bi belongs to
//      wave bi % NW for the whole factorisation; covariance tiles are generated
//      in registers when first needed (never stored); finished L tiles go to
//      the walker's workspace (packed 32x32 row-major tiles), the tiles of
//      the column in flight are parked in LDS.  Step k:
//        P(k)  wave k % NW factors the diagonal tile (registers; half the wave
//              builds the rows of L_kk, the other half the columns of its
//              inverse from the same v_readlane broadcasts), y_k = L_kk^-1 r_k;
//              meanwhile every wave accumulates the NEXT column's tiles
//              acc(bi, k+1) = C(bi, k+1) - sum_{j<k} L(bi, j) L(k+1, j)^T
//              (v_mfma_f32_32x32x2_f32, in registers) -- the j = k term is
//              the only part that waits for this step's factor;
//        S1(k) every wave: L(bi, k) = acc(bi, k) L_kk^-T (MFMA), stored;
//              r_bi -= L(bi, k) y_k;
//        S2(k) every wave: acc(bi, k+1) -= L(bi, k) L(k+1, k)^T, parked for
//              S1(k+1) (the diagonal tile stays in its owner's registers).
//      Tiles are held transposed in MFMA C/D layout (lane l: row l & 31 of the
//      tile at columns cd_row(r, l)), which is also the operand layout of the
//      next product, so no tile is ever reshuffled.
//   ll = -1/2 r^T C^-1 r - sum log L_ii - N/2 log(2 pi)  (fp64 sums).
// Padding rows/columns up to a multiple of 32 are identity rows with r = 0.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "../../include/rvk_gp.h"
#include "rvk_gp_internal.h"

using namespace rvk;

namespace {

#ifndef RVK_GP_WGPCU
#define RVK_GP_WGPCU 2    // concurrent workgroups per CU (each its own workspace), LDS permitting
#endif
#ifndef RVK_GP_ABLATE
#define RVK_GP_ABLATE 0   // timing experiments only (wrong results): 1 part1 operands from LDS, 2 no factor,
                          // 4 no covariance function, 8 no accumulation MFMAs
#endif
#ifndef RVK_GP_PRIO
#define RVK_GP_PRIO 1     // s_setprio of the factoring wave (1 and 3 measured equal, 0 within noise)
#endif
#ifndef RVK_GP_AGPR
#define RVK_GP_AGPR 0     // accumulators in AGPRs (MFMA C/D off the VGPR file)
#endif
#ifndef RVK_GP_FACTOR_LDS
#define RVK_GP_FACTOR_LDS 1   // diagonal factor: row broadcasts through LDS (1) or v_readlane (0); with the balanced schedule 1 is 2 % faster
#endif
#ifndef RVK_GP_TRACE
#define RVK_GP_TRACE 0    // timing experiments only: s_memtime per phase for the first walker of block 0
#endif
#ifndef RVK_GP_TWOCOL
#define RVK_GP_TWOCOL 0   // each workspace tile read in P(k) serves columns k+1 and k+2 (see P(k))
#endif
#ifndef RVK_GP_HALF
#define RVK_GP_HALF 1     // one-column P(k): operand tiles streamed in halves (no spills: 3.43 -> 3.21 ms)
#endif
#ifndef RVK_GP_QU
#define RVK_GP_QU (RVK_GP_HALF ? 2 : 4)   // float4 per operand tile and register set (4 = whole tiles)
#endif
#ifndef RVK_GP_RPASS
#define RVK_GP_RPASS 2    // rows per accumulation pass (the A tiles are re-read once per pass)
#endif
#ifndef RVK_GP_SCHEDB
#define RVK_GP_SCHEDB 1   // scheduling barriers around each ring set's loads and MFMAs (measured 3.21-3.26 vs 3.28-3.29 ms without; fp64: see rvk_gp64.hip)
#endif
#ifndef RVK_GP_NBUF
#define RVK_GP_NBUF 2     // operand register sets in the ring (NBUF - 1 in flight)
#endif
#ifndef RVK_GP_BAL
#define RVK_GP_BAL 1      // P(k)/S2(k) rows go to the waves that do not factor in step k (see prow)
#endif
#ifndef RVK_GP_SPLIT
#define RVK_GP_SPLIT 0    // mid steps: (row, j) units split evenly over the row waves (see plan; measured = base)
#endif
#ifndef RVK_GP_FU
#define RVK_GP_FU 6       // RVK_GP_BAL == 2: the factor's cost in (row, j) accumulation units
#endif
#if RVK_GP_TRACE
__device__ unsigned long long g_gp_trace[8][32][8];
#define GP_HWID() (__builtin_amdgcn_s_getreg((31 << 11) | 4))   // HW_REG_HW_ID: wave, SIMD, CU ids
#define GP_MARK(k, slot)                                                                          \
    do {                                                                                          \
        if (blockIdx.x == 0 && w == 0 && lane == 0) g_gp_trace[wv][k][slot] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define GP_MARK(k, slot) do {} while (0)
#endif
constexpr int TB = 32;              // tile edge
constexpr int TILE = TB * TB;
constexpr int PS = TB + 1;          // LDS row stride of the diagonal inverse (bank spread)
constexpr int RS = TB + 4;          // row stride of the factor's row buffer (b128-aligned rows), same LDS
using f32x2 = __attribute__((ext_vector_type(2))) float;

using f32x16 = __attribute__((ext_vector_type(16))) float;

__device__ __forceinline__ float rlf(float v, int lane) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}


// MFMA 32x32 C/D map (cdna_hip_programming.md): register r of lane l holds
// (row = (r & 3) + 8 (r >> 2) + 4 (l >> 5), col = l & 31).
__device__ __forceinline__ int cd_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

struct GpLds {
    // carved from dynamic shared memory
    float *uph;      // [npad]          per walker: fract(t_i / P_gp) (fp64 reduction, then fp32)
    float *tsc;      // [npad]          per walker: (t_i - t_0) / lambda_e (padding: t[n-1]'s)
    float *pan;      // [nt - 1][TILE]  tile rows 1.. of the column in flight (C/D register order);
                     //                 after S1(k) slot k holds L(k+1, k), read by every wave in S2(k)
    float *li;       // [TB][RS]        inverse of the step's diagonal tile, row-major (stride PS);
                     //                 the factor's row buffer (stride RS) while it runs
    float *r;        // [npad]          rhs (residuals), reduced in place
    float *dia;      // [npad]          velerr^2 + jit^2
    float *yk;       // [TB]            y_k = L_kk^-1 r_k
    double *red;     // [3 NW]          per-wave partial sums
    SC *tab;         // [kTabN]
    PlanetK *pk;     // [NP]
    int *ok;         // [NP]
    short *slot;     // [nt][nt]        workspace slot of tile (bi, j) (build_slots)
};

template <int NW>
__device__ __forceinline__ GpLds carve(void *smem, int nt, int np) {
    GpLds L;
    float *f = reinterpret_cast<float *>(smem);
    L.uph = f;
    f += nt * TB;
    L.tsc = f;
    f += nt * TB;
    L.pan = f;
    f += (nt - 1) * TILE;
    L.li = f;
    f += TB * RS;
    L.r = f;
    f += nt * TB;
    L.dia = f;
    f += nt * TB;
    L.yk = f;
    f += TB;
    // every offset so far is a multiple of 16 bytes; plain pointer arithmetic on the shared
    // base (no integer casts) keeps these LDS pointers: integer casts would turn every access
    // into a flat one, which waits on vmcnt as well
    L.red = reinterpret_cast<double *>(f);
    static_assert((3 * NW * sizeof(double)) % 16 == 0, "table alignment");
    L.tab = reinterpret_cast<SC *>(L.red + 3 * NW);
    L.pk = reinterpret_cast<PlanetK *>(L.tab + kTabN);
    L.ok = reinterpret_cast<int *>(L.pk + np);
    L.slot = reinterpret_cast<short *>(L.ok + ((np + 3) & ~3));
    return L;
}

template <bool MULTI, bool TP, int NW, int MAXR>   // MAXR tile rows per wave: nt <= MAXR * NW
__global__ __launch_bounds__(64 * NW, (MAXR == 2 ? 4 : 2)) void gp_loglike_kernel(EpochData d, int n, int ni, int np,
                                                                             const double *__restrict__ theta,
                                                                             const double *__restrict__ hyper,
                                                                             long long W, long long stride,
                                                                             long long hstride,
                                                                             const short *__restrict__ slots,
                                                                             float *__restrict__ work,
                                                                             long long work_stride,
                                                                             double *__restrict__ out, GpPost post) {
    constexpr int NT = 64 * NW;
    extern __shared__ double smem_d[];
    const int nt = (n + TB - 1) / TB, npad = nt * TB;
    const GpLds L = carve<NW>(smem_d, nt, np);
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, c = lane & 31;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    // Tile rows are owned round-robin by waves, rotated per workgroup: in the last steps only one
    // or two rows are left, and workgroups sharing a CU then keep different SIMDs busy.
#ifndef RVK_GP_ROT
#define RVK_GP_ROT 1
#endif
    const int rot = RVK_GP_ROT ? (int)((blockIdx.x * 7u + (blockIdx.x >> 8)) % NW) : 0;
    const int wr = (wv - rot + NW) % NW;    // this wave owns tile rows wr, wr + NW, ...
#if RVK_GP_AGPR
    {   // an AGPR operand anywhere makes the compiler select the AGPR form of every MFMA
        float z = 0.0f;
        asm volatile("; agpr hint %0" : "+a"(z));
    }
#endif
    for (int i = tid; i < kTabN; i += NT) tab_put(L.tab, i, d.tab[i], d.poison);
    for (int i = tid; i < nt * nt; i += NT) L.slot[i] = slots[i];
    __syncthreads();   // the table is read by the planet prep below (threads < np), before any other barrier
    float *A = work + (long long)blockIdx.x * work_stride;

    for (long long w = blockIdx.x; w < W; w += gridDim.x) {
        if (post.lp && post.lp[w] == -INFINITY) {        // rejected before the likelihood (uniform)
            if (tid == 0) out[w] = -INFINITY;
            continue;
        }
        const double *row = theta + w * stride;
        const double *hp = hyper + w * hstride;
        // ---- 1. planets, mean model, residuals -------------------------------------------
        if (tid < np) {
            PlanetK pk;
            const bool ok = TP ? planet_consts_t<0, true>(row + 5 * tid, pk, 0, L.tab)
                               : planet_consts(d.par, row + 5 * tid, pk);
            L.pk[tid] = pk;
            L.ok[tid] = ok;
        }
        __syncthreads();   // (the table fill of the first trip lands here too)
        bool alive = true;
        for (int p = 0; p < np; ++p) alive &= L.ok[p] != 0;
        if (!alive) {                                   // fit.py:8083-8085: mean model failed
            if (tid == 0) out[w] = -INFINITY;
            __syncthreads();
            continue;
        }
        const double *g = row + 5 * np, *jit = g + ni;
        const double gd = jit[ni], gdd = jit[ni + 1];
        const double amp = hp[0], lam_e = hp[1], lam_p = hp[2], per = hp[3];
        const double inv_per = 1.0 / per, inv_le = 1.0 / lam_e, tref = d.t[0];
        for (int i = tid; i < npad; i += NT) {
            // covariance inputs: sin^2(pi (t_i - t_j) / P) needs only the phase fractions (their
            // difference is exact to fp32 rounding), exp(-(t_i - t_j)^2 / 2 lambda_e^2) the scaled
            // times relative to t_0 (bounded by the span of the data, not by BJD magnitudes)
            const double ti = d.t[i < n ? i : n - 1];
            L.uph[i] = (float)__builtin_amdgcn_fract(ti * inv_per);
            L.tsc[i] = (float)((ti - tref) * inv_le);
            float ri = 0.0f, di = 1.0f;
            if (i < n) {
                const double t = d.t[i];
                const int ii = MULTI ? d.inst[i] : 0;
                double rv = 0.0;
                for (int p = 0; p < np; ++p) rv = planet_rv<0>(L.pk[p], t, L.tab, rv);
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
        // ---- 2. pipelined blocked Cholesky ---------------------------------------------------
        const float namp2 = -(float)(amp * amp);
        const float gam = (float)(1.0 / (2.0 * lam_p * lam_p));   // gp.py:150
        // -C(bi, bj)^T in C/D layout: lane l, register r = -C[bi*32 + (l & 31)][bj*32 + cd_row(r, l)]
        // (gp.py:126-156 + fit.py:8090-8105); padding rows/columns are identity.  Accumulators hold
        // the NEGATED trailing tiles, -acc = -C + sum L L^T, so every MFMA adds (no sign flips).
        auto cov_tile = [&](int bi, int bj, f32x16 &t) {
            const float ui = L.uph[bi * TB + c], si = L.tsc[bi * TB + c];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const float4 uj = *reinterpret_cast<const float4 *>(L.uph + bj * TB + 8 * u + 4 * h);
                const float4 sj = *reinterpret_cast<const float4 *>(L.tsc + bj * TB + 8 * u + 4 * h);
                const float ujv[4] = {uj.x, uj.y, uj.z, uj.w}, sjv[4] = {sj.x, sj.y, sj.z, sj.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float sn = __builtin_amdgcn_sinf(0.5f * (ui - ujv[e]));   // v_sin_f32: revolutions
                    const float x = si - sjv[e];
                    t[4 * u + e] = (RVK_GP_ABLATE & 4) ? 0.5f * x : namp2 * __expf(-(gam * (sn * sn) + 0.5f * (x * x)));
                }
            }
            if (bi == bj || (bi + 1) * TB > n || (bj + 1) * TB > n) {
                const int i = bi * TB + c;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int j = bj * TB + cd_row(r, lane);
                    float v = (i < n && j < n) ? t[r] : 0.0f;
                    v -= (i == j) ? L.dia[i] : 0.0f;                 // dia = 1 on padding
                    t[r] = v;
                }
            }
        };
        // Tile row held in accumulator slot q during P(k) and S2(k).  The factor of step k is the
        // step's serial critical path, so (RVK_GP_BAL) its wave f = k % NW takes no rows while the
        // other NW - 1 waves can hold them: rows k+1, k+2, ... go round-robin over waves f+1, f+2,
        // ..., so row k+1 (whose S2 result is the next diagonal tile, kept in registers as dacc)
        // lands on wave (k+1) % NW, the factor wave of step k+1; rows past the others' MAXR slots
        // (only in the first steps, where the row work is small) fall to wave f.  The accumulators
        // are re-formed every step and parked in LDS between S2(k) and S1(k+1), so the assignment
        // may change from step to step.  Otherwise: fixed round-robin ownership.
        auto prow = [&](int k, int q) -> int {
#if RVK_GP_BAL == 2 && !RVK_GP_TWOCOL
            // the factor wave also takes the last rf rows when that shortens the step: in units
            // of one (row, j) accumulation, the factor costs about RVK_GP_FU and a row k
            const int m = nt - 1 - k;
            int rf = m - (NW - 1) * MAXR > 0 ? m - (NW - 1) * MAXR : 0, best = 1 << 30;
            for (int r = rf; r < MAXR && r <= m; ++r) {
                const int tf = RVK_GP_FU + r * k, to = (m - r + NW - 2) / (NW - 1) * k;
                const int tm = tf > to ? tf : to;
                if (tm < best) {
                    best = tm;
                    rf = r;
                }
            }
            const int no = m - rf, t = (wr - k % NW + NW) % NW;
            if (!t) return k + 1 + no + q;
            const int i = t - 1 + (NW - 1) * q;
            return i < no ? k + 1 + i : nt;
#elif RVK_GP_BAL && !RVK_GP_TWOCOL
            const int t = (wr - k % NW + NW) % NW;
            return t ? k + t + (NW - 1) * q : k + 1 + (NW - 1) * MAXR + q;
#else
            (void)k;
            return wr + NW * q;
#endif
        };
        // The step's accumulation plan: slot q holds row bi[q] over j in [lo[q], hi[q]).  Whole
        // rows (prow) in the first and last steps; in the middle steps (RVK_GP_SPLIT) the m k
        // (row, j) units are split evenly over the NW - 1 row waves in row-major order, so
        // the waves' shares differ by at most one unit instead of one row.  A row cut at a
        // wave boundary is started (C and its first j's) by the lower wave, which finishes it
        // in S2; the upper wave accumulates its tail from zero and parks that partial in a
        // free panel slot (rows <= k-1 are finished), alternating between two slot sets by
        // the parity of k so the next step's parking never meets this step's S2 read.
        struct Plan {
            int bi[MAXR], lo[MAXR], hi[MAXR];
            int sec_slot;     // >= 0: slot 0 is a row tail; park its partial at pan[sec_slot]
            int add_q;        // >= 0: the next wave parks the tail of row bi[add_q] at pan[add_slot]
            int add_slot;
        };
        auto plan = [&](int k) -> Plan {
            Plan P;
            P.sec_slot = -1;
            P.add_q = -1;
            P.add_slot = 0;
#pragma unroll
            for (int q = 0; q < MAXR; ++q) {
                P.bi[q] = prow(k, q);
                P.lo[q] = 0;
                P.hi[q] = k;
            }
#if RVK_GP_SPLIT && RVK_GP_BAL == 1 && !RVK_GP_TWOCOL
            constexpr int NA = NW - 1;
            const int m = nt - 1 - k, ut = m * k;
            bool split = NA > 1 && k >= 2 * NA - 1 && m >= NA && m <= NA * MAXR;
            for (int t = 1; t <= NA && split; ++t) {      // every wave's rows must fit its slots
                const int s0 = (t - 1) * ut / NA, e0 = t * ut / NA;
                split = e0 > s0 && (e0 - 1) / k - s0 / k < MAXR;
            }
            if (split) {
                const int t = (wr - k % NW + NW) % NW;
#pragma unroll
                for (int q = 0; q < MAXR; ++q) P.bi[q] = nt;
                if (t) {
                    const int s0 = (t - 1) * ut / NA, e0 = t * ut / NA;
                    const int rs = s0 / k, re = (e0 - 1) / k;
#pragma unroll
                    for (int q = 0; q < MAXR; ++q) {
                        const int ri = rs + q;
                        if (ri <= re) {
                            P.bi[q] = k + 1 + ri;
                            P.lo[q] = ri == rs ? s0 - rs * k : 0;
                            P.hi[q] = ri == re ? e0 - re * k : k;
                        }
                    }
                    if (s0 > rs * k) P.sec_slot = (t - 2) + (NA - 1) * (k & 1);
                    if (e0 - re * k < k) {
                        P.add_q = re - rs;
                        P.add_slot = (t - 1) + (NA - 1) * (k & 1);
                    }
                }
            }
#endif
            return P;
        };
        double quad = 0.0;          // sum of y^2 over this wave's lanes
        double dp = 1.0;            // product of this wave's pivots L_ii^2, renormalised (x 2^pexp)
        int pexp = 0;
        f32x16 nacc[MAXR], dacc;
#if RVK_GP_TWOCOL
        f32x16 nacc2[MAXR];      // column k+2's partial sum, carried into step k+1 as nacc
#endif
        // acc(bi, 0) = C(bi, 0): the diagonal tile in wave 0's registers, the rest parked
#pragma unroll
        for (int q = 0; q < MAXR; ++q) {
            const int bi = wr + NW * q;
            if (bi < nt) {
                f32x16 t;
                cov_tile(bi, 0, t);
                if (bi == 0) {
                    dacc = t;
                } else {
#pragma unroll
                    for (int r = 0; r < 16; ++r) L.pan[(bi - 1) * TILE + r * 64 + lane] = t[r];
                }
            }
#if RVK_GP_TWOCOL
            if (bi >= 1 && bi < nt) cov_tile(bi, 1, nacc2[q]);   // column 1 has no j < 0 terms
#endif
        }
        __syncthreads();
#if RVK_GP_TRACE
        if (blockIdx.x == 0 && w == 0 && lane == 0) g_gp_trace[wv][31][7] = GP_HWID();
#endif
        for (int k = 0; k < nt; ++k) {
            GP_MARK(k, 0);
            // ---- P(k): factor the diagonal tile (wave k % NW) --------------------------------
#pragma unroll
            for (int q = 0; q < MAXR; ++q) {
#if RVK_GP_TWOCOL
                nacc[q] = nacc2[q];                   // column k+1: C and the j in S(k-1) terms
#else
                nacc[q] = f32x16{};                   // (ends the previous step's live ranges)
#endif
            }
            if (wr == k % NW && !(RVK_GP_ABLATE & 2)) {
                // the factor is the step's critical path: its VALU chain goes ahead of the
                // co-resident waves' instructions (MI355X_MICROARCH.md, two waves per SIMD)
                __builtin_amdgcn_s_setprio(RVK_GP_PRIO);
                // lane i < 32: row i of acc(k,k) (half its columns from lane i + 32);
                // lane 32 + j: column j of the identity, turned into column j of L_kk^-1
                float a[TB];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float o = __shfl_xor(dacc[r], 32);
                    const int x0 = cd_row(r, 0), x1 = cd_row(r, 32);
                    a[x0] = h ? (x0 == c ? 1.0f : 0.0f) : -dacc[r];
                    a[x1] = h ? (x1 == c ? 1.0f : 0.0f) : -o;
                }
                // left-looking, one column per step r: L[r][k'] (lane r's finished a[k'])
                // broadcast by v_readlane serves both halves:
                //   rows:    a_i[r]  -= sum_k' a_i[k'] L[r][k'],   L[i][r] = a_i[r] / L[r][r]
                //   inverse: X[r][j] = (delta_rj - sum_k' L[r][k'] X[k'][j]) / L[r][r]
#if RVK_GP_FACTOR_LDS
                // Row r of L (L[r][0..r-1]) reaches every lane through LDS instead of r
                // v_readlane: each finished column is written once (lane i: L[i][c'] at
                // rb[i][c'], row stride RS), row r is read back as uniform-address b128
                // broadcasts, and pairs of terms go through v_pk_fma_f32.  li is free here
                // (S1 of the previous step is behind the last barrier) and is rewritten
                // with the inverse afterwards.
                float *rb = L.li;
#endif
#pragma unroll
                for (int r = 0; r < TB; ++r) {
                    int rr = r;                                      // opaque: this column's
                    asm volatile("" : "+s"(rr));                     // broadcasts are not hoisted
#if RVK_GP_FACTOR_LDS
                    if (r > 0 && !h) rb[c * RS + (r - 1)] = a[r - 1];   // publish column r - 1
                    __builtin_amdgcn_wave_barrier();
                    asm volatile("" ::: "memory");
                    float lr[TB];
#pragma unroll
                    for (int m = 0; m < (r + 3) / 4; ++m) {
                        const float4 x = *reinterpret_cast<const float4 *>(rb + rr * RS + 4 * m);
                        lr[4 * m] = x.x; lr[4 * m + 1] = x.y; lr[4 * m + 2] = x.z; lr[4 * m + 3] = x.w;
                    }
                    f32x2 acc2 = {a[r], 0.0f};
#pragma unroll
                    for (int kk = 0; kk + 1 < r; kk += 2) {
                        const f32x2 av = {a[kk], a[kk + 1]}, lv = {lr[kk], lr[kk + 1]};
                        acc2 = acc2 - av * lv;
                    }
                    if (r & 1) acc2.x = __builtin_fmaf(-a[r - 1], lr[r - 1], acc2.x);
                    const float v = acc2.x + acc2.y;
#else
                    float v0 = a[r], v1 = 0.0f;
#pragma unroll
                    for (int kk = 0; kk < r; ++kk) {
                        const float lrk = rlf(a[kk], rr);
                        if (kk & 1) v1 = __builtin_fmaf(-a[kk], lrk, v1);
                        else v0 = __builtin_fmaf(-a[kk], lrk, v0);
                    }
                    const float v = v0 + v1;
#endif
                    const float p = rlf(v, rr);                      // L[r][r]^2 (<= 0 or NaN: NaN/inf
                    a[r] = v * __builtin_amdgcn_rsqf(p);             //  propagate to y and the log)
                    dp *= (double)p;
                    asm volatile("" : "+v"(a[r]), "+v"(dp));        // column r finished here
                    if ((r & 7) == 7) {
                        int e;
                        dp = __builtin_frexp(dp, &e);
                        pexp += e;
                    }
                }
#if RVK_GP_FACTOR_LDS
                __builtin_amdgcn_wave_barrier();
                asm volatile("" ::: "memory");
#endif
                if (h) {
#pragma unroll
                    for (int r = 0; r < TB; ++r) L.li[r * PS + c] = -a[r];    // -X[r][c]
                }
                __builtin_amdgcn_wave_barrier();
                asm volatile("" ::: "memory");
                if (!h) {                                   // y_c = sum_j X[c][j] r_k[j]
                    float y = 0.0f;
                    const float *rk = L.r + k * TB;
#pragma unroll
                    for (int j = 0; j < TB; ++j) y = __builtin_fmaf(L.li[c * PS + j], rk[j], y);
                    y = -y;
                    L.yk[c] = y;
                    quad += (double)y * (double)y;
                }
                __builtin_amdgcn_s_setprio(0);
            }
            GP_MARK(k, 1);
            // ---- P(k): the next column's tiles, all but the j = k term ------------------------
#if RVK_GP_TWOCOL
            // Two columns per workspace read.  Column c's sum over j < c - 1 is split between
            // steps c - 2 and c - 1 by the parity of j: step k reads only the tiles of
            // S(k) = {j < k : j = k + 1 (mod 2)} and applies each to column k+1 (completing it:
            // S(k-1) and S(k) partition [0, k)) and to column k+2 (which step k+1 completes
            // with S(k+1), the rest of [0, k+1)).  Every B tile is read once for two columns
            // (half the left-looking re-reads) and each step does the same MFMA work as a
            // one-column step.  The A tiles L(k+1, j), L(k+2, j) and the B tiles of two owned
            // rows are streamed in half tiles (8 k-steps), double buffered.
            if (k + 1 < nt) {
                const bool two = k + 2 < nt;
#pragma unroll
                for (int q = 0; q < MAXR; ++q) {
                    const int bi = wr + NW * q;
                    if (two && bi >= k + 2 && bi < nt) cov_tile(bi, k + 2, nacc2[q]);
                }
                const long long lane_off = c * TB + 16 * h;
                const int j0 = (k + 1) & 1;
                auto pass = [&](auto q0c) {
                    constexpr int Q0 = decltype(q0c)::value;
                    constexpr int R = (MAXR - Q0) < 2 ? (MAXR - Q0) : 2;
                    bool any = false;
#pragma unroll
                    for (int q = Q0; q < Q0 + R; ++q) any |= (wr + NW * q >= k + 1) && (wr + NW * q < nt);
                    if (!any || k == 0) return;
                    struct Ops {
                        float4 a1[2], a2[2], b[R][2];
                    };
                    // half hf of the tiles of j (the trip past the end re-reads j0's: L1 hits, so
                    // every load is unconditional and vmcnt waits are exact)
                    auto issue = [&](Ops &o, int j, int hf) {
                        const int jj = j < k ? j : j0;
                        const int s1 = L.slot[(k + 1) * nt + jj];
                        const int s2 = two ? L.slot[(k + 2) * nt + jj] : s1;
                        const float4 *pa1 = reinterpret_cast<const float4 *>(A + s1 * TILE + lane_off) + 2 * hf;
                        const float4 *pa2 = reinterpret_cast<const float4 *>(A + s2 * TILE + lane_off) + 2 * hf;
                        o.a1[0] = pa1[0];
                        o.a1[1] = pa1[1];
                        o.a2[0] = pa2[0];
                        o.a2[1] = pa2[1];
#pragma unroll
                        for (int q = 0; q < R; ++q) {
                            const int bi = wr + NW * (Q0 + q);
                            const bool live = bi >= k + 1 && bi < nt;
                            const float4 *pb = reinterpret_cast<const float4 *>(
                                                   A + L.slot[(live ? bi : k + 1) * nt + jj] * TILE + lane_off) + 2 * hf;
                            o.b[q][0] = pb[0];
                            o.b[q][1] = pb[1];
                        }
                    };
                    auto consume = [&](const Ops &o) {
#pragma unroll
                        for (int q = 0; q < R; ++q) {
                            const int bi = wr + NW * (Q0 + q);
                            if (bi >= k + 1 && bi < nt) {
                                f32x16 &acc = nacc[Q0 + q];
#pragma unroll
                                for (int u = 0; u < 2; ++u) {
                                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(o.a1[u].x, o.b[q][u].x, acc, 0, 0, 0);
                                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(o.a1[u].y, o.b[q][u].y, acc, 0, 0, 0);
                                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(o.a1[u].z, o.b[q][u].z, acc, 0, 0, 0);
                                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(o.a1[u].w, o.b[q][u].w, acc, 0, 0, 0);
                                }
                            }
                            if (two && bi >= k + 2 && bi < nt) {
                                f32x16 &acc = nacc2[Q0 + q];
#pragma unroll
                                for (int u = 0; u < 2; ++u) {
                                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(o.a2[u].x, o.b[q][u].x, acc, 0, 0, 0);
                                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(o.a2[u].y, o.b[q][u].y, acc, 0, 0, 0);
                                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(o.a2[u].z, o.b[q][u].z, acc, 0, 0, 0);
                                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(o.a2[u].w, o.b[q][u].w, acc, 0, 0, 0);
                                }
                            }
                        }
                    };
                    Ops X, Y;
                    issue(X, j0, 0);
                    for (int j = j0; j < k; j += 2) {
                        issue(Y, j, 1);
                        consume(X);
                        issue(X, j + 2, 0);
                        consume(Y);
                    }
                };
                pass(std::integral_constant<int, 0>{});
                if constexpr (MAXR > 2) pass(std::integral_constant<int, 2>{});
            }
#else
            const Plan P = plan(k);
            if (k + 1 < nt) {
#pragma unroll
                for (int q = 0; q < MAXR; ++q) {
                    const int bi = P.bi[q];
                    if (bi >= k + 1 && bi < nt) {
                        if (P.lo[q] == 0) cov_tile(bi, k + 1, nacc[q]);
                        else nacc[q] = f32x16{};              // a row's tail: its partial sum only
                    }
                }
                // Operand tiles: the A tile L(k+1, j) and the B tiles L(bi, j) of two of the
                // step's rows at a time (slots q0, q0 + 1; a second pass takes slots 2, 3 and
                // re-reads the A tiles from L2), streamed in QU-float4 sets through a ring of NB
                // register sets, so NB - 1 sets are in flight during a set's MFMAs.  The pass runs
                // over the union of its rows' j ranges; a row outside its range (or finished, or
                // the trip past the end) re-reads the A tile, an L1 hit, so every load is
                // unconditional and every path leaves the same loads outstanding (exact vmcnt).
                const long long lane_off = c * TB + 16 * h;
                auto pass = [&](auto q0c) {
                    constexpr int Q0 = decltype(q0c)::value;
                    constexpr int R = (MAXR - Q0) < RVK_GP_RPASS ? (MAXR - Q0) : RVK_GP_RPASS;
                    constexpr int QU = RVK_GP_QU, NSET = 4 / QU, NB = RVK_GP_NBUF;
                    bool any = false;
                    int jmin = k, jmax = 0;
#pragma unroll
                    for (int q = Q0; q < Q0 + R; ++q) {
                        if (P.bi[q] >= k + 1 && P.bi[q] < nt) {
                            any = true;
                            jmin = P.lo[q] < jmin ? P.lo[q] : jmin;
                            jmax = P.hi[q] > jmax ? P.hi[q] : jmax;
                        }
                    }
                    if (!any || k == 0) return;
                    struct Ops {
                        float4 a[QU], b[R][QU];
                    };
                    const int H0 = NSET * jmin, H1 = NSET * jmax;
                    auto in_range = [&](int q, int jj) {
                        return P.bi[Q0 + q] >= k + 1 && P.bi[Q0 + q] < nt && jj >= P.lo[Q0 + q] && jj < P.hi[Q0 + q];
                    };
                    auto issue = [&](Ops &o, int hx) {
                        const int hh = hx < H1 ? hx : H1 - 1;
                        const int jj = hh / NSET, part = hh % NSET;
                        const float4 *pa = reinterpret_cast<const float4 *>(A + L.slot[(k + 1) * nt + jj] * TILE + lane_off) + QU * part;
#pragma unroll
                        for (int u = 0; u < QU; ++u) o.a[u] = pa[u];
#pragma unroll
                        for (int q = 0; q < R; ++q) {
                            const float4 *pb = reinterpret_cast<const float4 *>(
                                A + L.slot[(in_range(q, jj) ? P.bi[Q0 + q] : k + 1) * nt + jj] * TILE + lane_off) + QU * part;
#pragma unroll
                            for (int u = 0; u < QU; ++u) o.b[q][u] = pb[u];
                        }
                    };
                    auto consume = [&](const Ops &o, int hx) {
                        const int jj = hx / NSET;
#pragma unroll
                        for (int q = 0; q < R; ++q) {
                            if (in_range(q, jj)) {
                                f32x16 &acc = nacc[Q0 + q];
#pragma unroll
                                for (int u = 0; u < QU; ++u) {
                                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(o.a[u].x, o.b[q][u].x, acc, 0, 0, 0);
                                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(o.a[u].y, o.b[q][u].y, acc, 0, 0, 0);
                                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(o.a[u].z, o.b[q][u].z, acc, 0, 0, 0);
                                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(o.a[u].w, o.b[q][u].w, acc, 0, 0, 0);
                                }
                            }
                        }
                    };
                    Ops ring[NB];
#pragma unroll
                    for (int b = 0; b + 1 < NB; ++b) issue(ring[b], H0 + b);
                    for (int hx = H0; hx < H1; hx += NB) {
#pragma unroll
                        for (int b = 0; b < NB; ++b) {
                            issue(ring[(b + NB - 1) % NB], hx + b + NB - 1);
                            if (RVK_GP_SCHEDB) __builtin_amdgcn_sched_barrier(0);   // keep the loads ahead
                            if ((b == 0 || hx + b < H1) && !(RVK_GP_ABLATE & 8)) consume(ring[b], hx + b);
                            if (RVK_GP_SCHEDB) __builtin_amdgcn_sched_barrier(0);
                        }
                    }
                };
                pass(std::integral_constant<int, 0>{});
                if constexpr (MAXR > RVK_GP_RPASS) pass(std::integral_constant<int, RVK_GP_RPASS>{});
                if constexpr (MAXR > 2 * RVK_GP_RPASS) pass(std::integral_constant<int, 2 * RVK_GP_RPASS>{});
                if constexpr (MAXR > 3 * RVK_GP_RPASS) pass(std::integral_constant<int, 3 * RVK_GP_RPASS>{});
                if (P.sec_slot >= 0) {                      // a row's tail: park the partial sum
#pragma unroll
                    for (int r = 0; r < 16; ++r) L.pan[P.sec_slot * TILE + r * 64 + lane] = nacc[0][r];
                }
            }
#endif
            GP_MARK(k, 2);
            __syncthreads();                                // B1: L_kk^-1 and y_k published
            GP_MARK(k, 3);
            if (k + 1 == nt) break;
            // ---- S1(k): L(bi, k) = acc(bi, k) L_kk^-T, stored; rhs update ---------------------
            {
                float ykv[16], la[16];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const float4 x = *reinterpret_cast<const float4 *>(L.yk + 8 * u + 4 * h);
                    ykv[4 * u] = x.x; ykv[4 * u + 1] = x.y; ykv[4 * u + 2] = x.z; ykv[4 * u + 3] = x.w;
                }
#pragma unroll
                for (int ks = 0; ks < 16; ++ks) la[ks] = L.li[c * PS + cd_row(ks, lane)];
#pragma unroll
                for (int q = 0; q < MAXR; ++q) {
                    const int bi = wr + NW * q;
                    if (bi > k && bi < nt) {
                        float *slot = L.pan + (bi - 1) * TILE;
                        float sb[16];
#pragma unroll
                        for (int ks = 0; ks < 16; ++ks) sb[ks] = slot[ks * 64 + lane];
                        f32x16 lt = {};
#pragma unroll
                        for (int ks = 0; ks < 16; ++ks) lt = __builtin_amdgcn_mfma_f32_32x32x2f32(la[ks], sb[ks], lt, 0, 0, 0);
                        // lane l: row c of L(bi, k) at columns cd_row(r, l) -> row-major tile
                        // (L(k+1, k) is only ever read from LDS, in S2: not stored)
                        float4 *T = reinterpret_cast<float4 *>(A + L.slot[bi * nt + k] * TILE + c * TB + 4 * h);
                        float s = 0.0f;
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            if (bi > k + 1) T[2 * u] = make_float4(lt[4 * u], lt[4 * u + 1], lt[4 * u + 2], lt[4 * u + 3]);
#pragma unroll
                            for (int e = 0; e < 4; ++e) s = __builtin_fmaf(lt[4 * u + e], ykv[4 * u + e], s);
                        }
                        s += __shfl_xor(s, 32);
                        if (!h) L.r[bi * TB + c] -= s;
#pragma unroll
                        for (int r = 0; r < 16; ++r) slot[r * 64 + lane] = lt[r];   // L(k+1, k): read by all in S2
                    }
                }
            }
            GP_MARK(k, 4);
            __syncthreads();                                // B2: L(k+1, k) published
            GP_MARK(k, 5);
            // ---- S2(k): the j = k term; park for S1(k+1) ---------------------------------------
            float lk[16];
#pragma unroll
            for (int ks = 0; ks < 16; ++ks) lk[ks] = L.pan[k * TILE + ks * 64 + lane];
#pragma unroll
            for (int q = 0; q < MAXR; ++q) {
#if RVK_GP_TWOCOL
                const int bi = prow(k, q);
                if (bi > k && bi < nt) {
#else
                const int bi = P.bi[q];
                if (bi > k && bi < nt && !(q == 0 && P.sec_slot >= 0)) {   // (a tail: the lower wave's row)
                    if (q == P.add_q) {                     // the upper wave's partial of this row
#pragma unroll
                        for (int r = 0; r < 16; ++r) nacc[q][r] += L.pan[P.add_slot * TILE + r * 64 + lane];
                    }
#endif
                    const float *src = L.pan + (bi - 1) * TILE;
                    float sb[16];
#pragma unroll
                    for (int ks = 0; ks < 16; ++ks) sb[ks] = src[ks * 64 + lane];
#pragma unroll
                    for (int ks = 0; ks < 16; ++ks) nacc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(lk[ks], sb[ks], nacc[q], 0, 0, 0);
                    if (bi == k + 1) {
                        dacc = nacc[q];
                    } else {
#pragma unroll
                        for (int r = 0; r < 16; ++r) L.pan[(bi - 1) * TILE + r * 64 + lane] = nacc[q][r];
                    }
                }
            }
            GP_MARK(k, 6);
        }
        // ---- 3. ll = -1/2 r^T C^-1 r - 1/2 sum log L_ii^2 - n/2 log 2 pi ------------------------
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) quad += __shfl_xor(quad, o);
        if (lane == 0) {
            L.red[3 * wv] = quad;
            L.red[3 * wv + 1] = log(dp) + (double)pexp * 0.69314718055994530942;
        }
        __syncthreads();
        if (tid == 0) {
            double qs = 0.0, ls = 0.0;
            for (int u = 0; u < NW; ++u) {
                qs += L.red[3 * u];
                ls += L.red[3 * u + 1];
            }
            double ll = -0.5 * qs - 0.5 * ls - 0.5 * (double)n * kLog2Pi;
            if (!__builtin_isfinite(ll)) ll = NAN;          // not positive definite in fp32: NaN
            if (post.lp) ll = (((ll + post.lp[w]) + post.lhp[w]) + post.jac) + post.renorm;
            out[w] = ll;
        }
        __syncthreads();
    }
}

size_t gp_lds_bytes(int n, int np, int nw) {
    const int nt = (n + TB - 1) / TB;
    size_t b = sizeof(float) * 2 * (size_t)nt * TB;
    b += sizeof(float) * ((size_t)(nt - 1) * TILE + TB * RS + 2 * (size_t)nt * TB + TB) + 16;
    b += sizeof(double) * 3 * nw;
    b += sizeof(SC) * kTabN + sizeof(PlanetK) * (size_t)np + sizeof(int) * (size_t)((np + 3) & ~3) + 16;
    b += sizeof(short) * (size_t)nt * nt;
    return b;
}

// Workspace slots.  Tile (bi, j), bi >= j + 2, is written in S1(j) and read in the P phases of
// steps j + 1 .. bi - 1 (L(j + 1, j) never leaves LDS); a P-phase read precedes the same
// step's S1 writes, so lifetimes [2j + 1, 2(bi - 1)] that do not overlap can share a slot.
// Greedy interval colouring in order of first write: max_k (nt-1-k) k slots (56 at nt = 16)
// instead of nt (nt - 1) / 2 (120), so concurrent walkers' workspaces stay in the Infinity Cache.
int build_slots(int nt, std::vector<short> &slot) {
    slot.assign((size_t)nt * nt, 0);
    std::vector<int> free_at;            // per slot: the phase time after which it is free
    for (int j = 0; j < nt; ++j)
        for (int bi = j + 2; bi < nt; ++bi) {
            const int start = 2 * j + 1, end = 2 * (bi - 1);
            int s = -1;
            for (size_t u = 0; u < free_at.size(); ++u)
                if (free_at[u] < start) {
                    s = (int)u;
                    break;
                }
            if (s < 0) {
                s = (int)free_at.size();
                free_at.push_back(0);
            }
            free_at[s] = end;
            slot[(size_t)bi * nt + j] = (short)s;
        }
    return (int)free_at.size();
}

// launch shapes: waves per walker x tile rows per wave (nt <= NW * MAXR)
struct GpShape {
    int nw, maxr;
};
GpShape gp_shape(int n, int prefer_nw) {
    const int nt = (n + TB - 1) / TB;
    if (nt > 16) return {8, 4};
    return prefer_nw == 8 ? GpShape{8, 2} : GpShape{4, 4};
}

typedef void (*gp_launch_t)(hipStream_t, unsigned, size_t, EpochData, int, int, int, const double *,
                            const double *, long long, long long, long long, const short *, float *, long long,
                            double *, GpPost);

template <bool MULTI, bool TP, int NW, int MAXR>
void launch_gp(hipStream_t st, unsigned grid, size_t lds, EpochData d, int n, int ni, int np, const double *th,
               const double *hy, long long W, long long stride, long long hs, const short *slots, float *work,
               long long wstride, double *out, GpPost post) {
    static size_t allowed = 0;   // dynamic LDS beyond the default needs the attribute
    if (lds > allowed) {
        (void)hipFuncSetAttribute((const void *)gp_loglike_kernel<MULTI, TP, NW, MAXR>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        allowed = lds;
    }
    hipLaunchKernelGGL((gp_loglike_kernel<MULTI, TP, NW, MAXR>), dim3(grid), dim3(64 * NW), lds, st, d, n, ni, np,
                       th, hy, W, stride, hs, slots, work, wstride, out, post);
}

template <int NW, int MAXR>
gp_launch_t pick_gp_w(bool multi, bool tp) {
    if (multi) return tp ? launch_gp<true, true, NW, MAXR> : launch_gp<true, false, NW, MAXR>;
    return tp ? launch_gp<false, true, NW, MAXR> : launch_gp<false, false, NW, MAXR>;
}

gp_launch_t pick_gp(int np, bool multi, bool tp, GpShape sh) {
    if (np < 1 || np > RVK_MAX_PLANETS) return nullptr;
    if (sh.nw == 4) return pick_gp_w<4, 4>(multi, tp);
    return sh.maxr == 2 ? pick_gp_w<8, 2>(multi, tp) : pick_gp_w<8, 4>(multi, tp);
}

// GP log-prior of a walker block (GPLogPosterior.log_probability up to the likelihood,
// fit.py:7851-7885), one wave per walker: the combined row [theta_full | hyper] from the
// fixed template and the free coordinates, the jitter check, the hyperparameter validity
// (GPKernel._validate_hyperparams_values: finite and > 0, gp.py:73-82), the prior-side
// conversion, the prior terms; priors (slots [0, n_lp)) and hyperpriors (the rest) are
// summed separately, each in the reference's key order.  lp = -inf rejects the walker.
__global__ __launch_bounds__(256) void gp_logprior_kernel(PostDev pd, int n_lp, const double *__restrict__ xf,
                                                          long long W, long long stride, double *__restrict__ full,
                                                          double *__restrict__ lp, double *__restrict__ lhp) {
    __shared__ PostWaveLds lds[kWavesPerBlock];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    PostWaveLds &L = lds[wv];
    const int hy0 = pd.p_full - RVK_GP_NHYPER;            // first hyperparameter column
    for (long long w = (long long)blockIdx.x * kWavesPerBlock + wv; w < W; w += (long long)gridDim.x * kWavesPerBlock) {
        for (int c = lane; c < pd.n_free; c += 64) L.x[c] = xf[w * stride + c];
        wave_lds_sync();
        double *frow = full + w * pd.p_full;
        for (int c = lane; c < pd.p_full; c += 64) {
            const int f = pd.colmap[c];
            const double v = f >= 0 ? L.x[f] : pd.tmpl[c];
            L.f[c] = v;
            frow[c] = v;
        }
        wave_lds_sync();
        const int jit0 = 5 * pd.n_planets + pd.n_inst;
        bool dead = false;
        if (lane < pd.n_inst) dead = L.f[jit0 + lane] < 0.0;                          // fit.py:7853-7856
        if (lane < RVK_GP_NHYPER) {                                                     // fit.py:7860-7867
            const double v = L.f[hy0 + lane];
            dead |= !(__builtin_isfinite(v) && v > 0.0);
        }
        if (pd.convert && lane < pd.n_planets) {                                        // fit.py:7787-7834
            double *dp = L.def + 5 * lane;
            dead |= !to_default_t<-1>(L.f + 5 * lane, dp[0], dp[1], dp[2], dp[3], dp[4], pd.par);
        }
        wave_lds_sync();
        for (int k = lane; k < pd.n_prior; k += 64) {
            const PriorSlot &sl = pd.slots[k];
            const double v = sl.src >= 0 ? L.f[sl.src] : L.def[-sl.src - 1];
            L.term[k] = prior_lp(sl, v);
        }
        wave_lds_sync();
        dead = __builtin_amdgcn_ballot_w64(dead) != 0;
        double a = 0.0, b = 0.0;
        for (int k = 0; k < n_lp; ++k) a += L.term[k];                                  // LogPrior, dict order
        for (int k = n_lp; k < pd.n_prior; ++k) b += L.term[k];                         // hyperpriors
        if (!__builtin_isfinite(a) || !__builtin_isfinite(b)) dead = true;              // fit.py:7878-7885
        if (lane == 0) {
            lp[w] = dead ? -INFINITY : a;
            lhp[w] = b;
        }
        wave_lds_sync();
    }
}

// Stretch-move proposals of one half for the GP sampler (emcee StretchMove.get_proposal), one
// thread per proposal: q = c - (c - s) z with the draws of (step, half, j) from `pre`; the
// log-posterior of the block of proposals is then rvk_gp_logpost_device, the accept / reject
// stretch_accept_kernel.
// Proposals [j0, j0 + H) of a half of hfull (the whole half on one GPU; a rank's slice when sharded).
__global__ __launch_bounds__(256) void gp_propose_kernel(const RunArgs *__restrict__ runp, const PreDraw *__restrict__ pre,
                                                         int D, int step, int half, long long H, long long j0,
                                                         long long hfull, double *__restrict__ q,
                                                         double *__restrict__ fac, double *__restrict__ lau,
                                                         long long *__restrict__ sidx) {
    const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= H) return;
    const RunArgs &run = *runp;
    const PreDraw d = pre[((long long)step * 2 + half) * hfull + j0 + j];
    const double *xs = run.x + d.s * D, *xc = run.x + d.c * D;
    for (int c = 0; c < D; ++c) q[j * D + c] = stretch_q(xc[c], xs[c], d.z);
    fac[j] = d.fac;
    lau[j] = d.lau;
    sidx[j] = d.s;
}

unsigned gp_wave_blocks(long long n) {
    long long b = (n + kWavesPerBlock - 1) / kWavesPerBlock;
    return (unsigned)(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

}  // namespace

struct rvk_gp {
    rvk_handle *h = nullptr;
    int device = -1;                         // the handle's, kept so destruction never dereferences h
    int mode = RVK_GP_FP64;                  // the reference's precision (fit.py:39)
    gp_launch_t launch = nullptr;
    unsigned grid = 0;           // concurrent walkers (one workgroup each)
    size_t lds = 0;
    long long wstride = 0;       // floats per workgroup workspace
    float *d_work = nullptr;
    short *d_slots = nullptr;    // [nt][nt] tile -> workspace slot
    // fp64 factorisation / conditioning (rvk_gp64.hip)
    gp64_launch_t launch64 = nullptr, cond64 = nullptr;
    unsigned grid64 = 0;
    size_t lds64 = 0;
    long long w64stride = 0;     // doubles per workgroup workspace
    double *d_work64 = nullptr;
    // host-buffer paths: rvk_gp_loglike's transport (RVK_OPT_HOSTIO); rvk_gp_predict's device
    // copies kept across calls, grown on demand
    HostIO io;
    double *d_theta = nullptr, *d_hyper = nullptr, *d_out = nullptr, *d_tq = nullptr;
    size_t cap_theta = 0, cap_hyper = 0, cap_out = 0, cap_tq = 0;
};

static int gp_grow(double **p, size_t *cap, size_t need) { return grow_dev((void **)p, cap, need); }

static void free_gp(rvk_gp *g) {
    if (!g) return;
    if (g->device >= 0) (void)hipSetDevice(g->device);   // never through g->h: it may be gone already
    (void)hipFree(g->d_work);
    (void)hipFree(g->d_slots);
    (void)hipFree(g->d_work64);
    (void)hipFree(g->d_theta);
    (void)hipFree(g->d_hyper);
    (void)hipFree(g->d_out);
    (void)hipFree(g->d_tq);
    g->io.release();
    delete g;
}

// LDS per CU on this device (gfx950: 160 KB; the runtime reports it as the per-CU or the
// per-block figure, whichever it fills in): the fp32 occupancy estimate only.
static size_t lds_per_cu(const hipDeviceProp_t &prop) {
    const size_t a = prop.maxSharedMemoryPerMultiProcessor, b = prop.sharedMemPerBlock;
    return a > b ? a : b;
}

// LDS ONE workgroup may allocate (the launch limit): the per-block figure, the per-CU one only
// when the runtime leaves the per-block figure at 0.
static size_t lds_per_block(const hipDeviceProp_t &prop) {
    return prop.sharedMemPerBlock ? (size_t)prop.sharedMemPerBlock : (size_t)prop.maxSharedMemoryPerMultiProcessor;
}

// The fp32 factorisation's launch shape and workspace (n <= kGpF32MaxEpochs: its column panel
// lives in LDS).
static int create_gp32(rvk_gp *g, rvk_handle *h, const hipDeviceProp_t &prop) {
    // experiment hooks (tools/gp_ab.sh), never set in production: waves per walker, workgroups per CU
    int wgpcu = RVK_GP_WGPCU, prefer_nw = 4;
    if (const char *e = getenv("RVK_GP_NW")) prefer_nw = atoi(e);
    if (const char *e = getenv("RVK_GP_WGPCU")) wgpcu = atoi(e) > 1 ? atoi(e) : 1;
    const GpShape sh = gp_shape(h->n, prefer_nw);
    g->launch = pick_gp(h->n_planets, h->n_inst > 1, h->par == RVK_PAR_PKEWTP, sh);
    if (!g->launch) return fail(RVK_E_ARG, "GP supports 1..32 planets");
    g->lds = gp_lds_bytes(h->n, h->n_planets, sh.nw);
    // workgroups that fit at once (LDS-limited), each with its own workspace
    const size_t per_cu = lds_per_cu(prop) / g->lds;
    g->grid = (unsigned)(prop.multiProcessorCount * (per_cu < 1 ? 1 : (per_cu > (size_t)wgpcu ? (size_t)wgpcu : per_cu)));
    const int nt = (h->n + TB - 1) / TB;
    std::vector<short> slots;
    const int nslots = build_slots(nt, slots);
    g->wstride = (long long)(nslots > 0 ? nslots : 1) * TILE;
    HIPCHK(hipMalloc(&g->d_work, sizeof(float) * (size_t)g->wstride * g->grid));
    HIPCHK(hipMalloc(&g->d_slots, sizeof(short) * slots.size()));
    HIPCHK(hipMemcpy(g->d_slots, slots.data(), sizeof(short) * slots.size(), hipMemcpyHostToDevice));
    return RVK_OK;
}

static int create_gp(rvk_gp *g, rvk_handle *h, int32_t kernel) {
    if (!h) return fail(RVK_E_ARG, "NULL handle");
    if (kernel != RVK_GP_QUASIPERIODIC) return fail(RVK_E_ARG, "unknown GP kernel type");
    if (h->n < 1 || h->n > RVK_GP_MAX_EPOCHS) return fail(RVK_E_ARG, "GP needs 1 <= n_epochs <= 4096");
    g->h = h;
    g->device = h->device;
    HIPCHK(hipSetDevice(h->device));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, h->device));
    int rc;
    if (h->n <= kGpF32MaxEpochs && (rc = create_gp32(g, h, prop))) return rc;
    // fp64 path: one 4-wave-per-SIMD workgroup per CU, the whole lower triangle of L per workgroup
    const Gp64Shape s64 = gp64_shape(h->n);
    g->launch64 = pick_gp64(h->n_planets, h->n_inst > 1, h->par == RVK_PAR_PKEWTP, false, s64);
    g->cond64 = pick_gp64(h->n_planets, h->n_inst > 1, h->par == RVK_PAR_PKEWTP, true, s64);
    if (!g->launch64 || !g->cond64) return fail(RVK_E_ARG, "GP supports 1..32 planets");
    g->lds64 = gp64_lds_bytes(h->n, h->n_planets, s64.nw);
    if (g->lds64 > lds_per_block(prop))
        return fail(RVK_E_ARG, "GP fp64 kernel: LDS need (" + std::to_string(g->lds64) + " B) exceeds the device's " +
                                   std::to_string(lds_per_block(prop)) + " B per workgroup");
    g->grid64 = (unsigned)prop.multiProcessorCount;
    g->w64stride = gp64_work_doubles(h->n);
    HIPCHK(hipMalloc(&g->d_work64, sizeof(double) * (size_t)g->w64stride * g->grid64));
    return RVK_OK;
}

static Gp64Args args64(rvk_gp *g, const double *th, const double *hy, long long W, long long stride, long long hs) {
    rvk_handle *h = g->h;
    Gp64Args a{};
    a.d = h->epochs();
    a.n = h->n;
    a.ni = h->n_inst;
    a.np = h->n_planets;
    a.theta = th;
    a.hyper = hy;
    a.W = W;
    a.stride = stride;
    a.hstride = hs;
    a.work = g->d_work64;
    a.work_stride = g->w64stride;
    return a;
}

// The GP log-likelihood (or log-posterior, post.lp set) of a device walker block, in the
// handle's precision mode; stream-ordered.
static int gp_run(rvk_gp *g, const double *th, const double *hy, long long W, long long stride, long long hs,
                  double *out, GpPost post, hipStream_t st) {
    rvk_handle *h = g->h;
    const bool f32 = g->mode != RVK_GP_FP64 && g->launch;   // (n > kGpF32MaxEpochs: fp64 in every mode)
    if (f32) {
        const unsigned grid = (unsigned)((long long)g->grid < W ? g->grid : W);
        g->launch(st, grid, g->lds, h->epochs(), h->n, h->n_inst, h->n_planets, th, hy, W, stride, hs, g->d_slots,
                  g->d_work, g->wstride, out, post);
        HIPCHK(hipGetLastError());
    }
    if (g->mode != RVK_GP_FP32 || !f32) {
        Gp64Args a = args64(g, th, hy, W, stride, hs);
        a.out = out;
        a.post = post;
        a.gate = f32 ? out : nullptr;                      // fallback: the fp32 NaN walkers only
        const unsigned grid = (unsigned)((long long)g->grid64 < W ? g->grid64 : W);
        g->launch64(st, grid, g->lds64, a);
        HIPCHK(hipGetLastError());
    }
    return RVK_OK;
}

extern "C" {

#if RVK_GP_TRACE
int rvk_gp_trace_dump(unsigned long long *host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gp_trace), sizeof(g_gp_trace)) == hipSuccess ? 0 : -1;
}
#endif

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

int rvk_gp_set_precision(rvk_gp *g, int32_t mode) {
    if (!g) return fail(RVK_E_ARG, "NULL GP handle");
    if (mode != RVK_GP_FP32 && mode != RVK_GP_FP32_FP64_FALLBACK && mode != RVK_GP_FP64)
        return fail(RVK_E_ARG, "unknown GP precision mode");
    g->mode = mode;
    return RVK_OK;
}

int rvk_gp_loglike_device(rvk_gp *g, const double *d_theta, const double *d_hyper, int64_t W, int64_t stride,
                          int64_t hstride, double *d_out, void *stream) {
    if (!g) return fail(RVK_E_ARG, "NULL GP handle");
    rvk_handle *h = g->h;
    if (W < 0 || stride < h->p_full() || hstride < RVK_GP_NHYPER) return fail(RVK_E_ARG, "bad walker block shape");
    if (W == 0) return RVK_OK;
    if (!d_theta || !d_hyper || !d_out) return fail(RVK_E_ARG, "NULL device buffer");
    HIPCHK(hipSetDevice(h->device));
    return gp_run(g, d_theta, d_hyper, W, stride, hstride, d_out, GpPost{nullptr, nullptr, 0.0, 0.0},
                  (hipStream_t)stream);
}

int rvk_gp_loglike(rvk_gp *g, const double *theta, const double *hyper, int64_t W, int64_t stride, int64_t hstride,
                   double *out) {
    if (!g) return fail(RVK_E_ARG, "NULL GP handle");
    if (W == 0) return RVK_OK;
    if (!theta || !hyper || !out || W < 0) return fail(RVK_E_ARG, "bad host buffers");
    rvk_handle *h = g->h;
    if (stride < h->p_full() || hstride < RVK_GP_NHYPER) return fail(RVK_E_ARG, "bad walker block shape");
    std::lock_guard<std::mutex> lock(h->mu);   // one blocking call per handle at a time (rvk.h, threading)
    HIPCHK(hipSetDevice(h->device));
    const size_t b[2] = {sizeof(double) * (size_t)W * (size_t)stride, sizeof(double) * (size_t)W * (size_t)hstride};
    const size_t bo = sizeof(double) * (size_t)W;
    const void *src[2] = {theta, hyper}, *d_in[2] = {nullptr, nullptr};
    void *d_out = nullptr;
    int rc;
    if ((rc = g->io.begin(h->hostio, h->stream, 2, src, b, bo, d_in, &d_out))) return rc;
    if ((rc = rvk_gp_loglike_device(g, (const double *)d_in[0], (const double *)d_in[1], W, stride, hstride,
                                     (double *)d_out, h->stream))) {
        (void)hipStreamSynchronize(h->stream);
        return rc;
    }
    return g->io.end(h->stream, out, bo);
}

int rvk_gp_predict_device(rvk_gp *g, const double *d_theta, const double *d_hyper, int64_t S, int64_t stride,
                          int64_t hstride, const double *d_tq, int64_t T, double *d_out, void *stream) {
    if (!g) return fail(RVK_E_ARG, "NULL GP handle");
    rvk_handle *h = g->h;
    if (S < 0 || T < 0 || stride < h->p_full() || hstride < RVK_GP_NHYPER) return fail(RVK_E_ARG, "bad sample block shape");
    if (S == 0 || T == 0) return RVK_OK;
    if (!d_theta || !d_hyper || !d_tq || !d_out) return fail(RVK_E_ARG, "NULL device buffer");
    HIPCHK(hipSetDevice(h->device));
    Gp64Args a = args64(g, d_theta, d_hyper, S, stride, hstride);
    a.tq = d_tq;
    a.T = T;
    a.pred = d_out;
    const unsigned grid = (unsigned)((long long)g->grid64 < S ? g->grid64 : S);
    g->cond64((hipStream_t)stream, grid, g->lds64, a);
    HIPCHK(hipGetLastError());
    return RVK_OK;
}

int rvk_gp_predict(rvk_gp *g, const double *theta, const double *hyper, int64_t S, int64_t stride, int64_t hstride,
                   const double *tq, int64_t T, double *out) {
    if (!g) return fail(RVK_E_ARG, "NULL GP handle");
    if (S == 0 || T == 0) return RVK_OK;
    if (!theta || !hyper || !tq || !out || S < 0 || T < 0) return fail(RVK_E_ARG, "bad host buffers");
    rvk_handle *h = g->h;
    if (stride < h->p_full() || hstride < RVK_GP_NHYPER) return fail(RVK_E_ARG, "bad sample block shape");
    std::lock_guard<std::mutex> lock(h->mu);   // one blocking call per handle at a time (rvk.h, threading)
    HIPCHK(hipSetDevice(h->device));
    const size_t bt = sizeof(double) * (size_t)S * (size_t)stride, bh = sizeof(double) * (size_t)S * (size_t)hstride;
    const size_t bq = sizeof(double) * (size_t)T, bo = sizeof(double) * (size_t)S * (size_t)T;
    int rc;
    if ((rc = gp_grow(&g->d_theta, &g->cap_theta, bt)) || (rc = gp_grow(&g->d_hyper, &g->cap_hyper, bh)) ||
        (rc = gp_grow(&g->d_tq, &g->cap_tq, bq)) || (rc = gp_grow(&g->d_out, &g->cap_out, bo)))
        return rc;
    HIPCHK_SYNC(h->stream, hipMemcpyAsync(g->d_theta, theta, bt, hipMemcpyHostToDevice, h->stream));
    HIPCHK_SYNC(h->stream, hipMemcpyAsync(g->d_hyper, hyper, bh, hipMemcpyHostToDevice, h->stream));
    HIPCHK_SYNC(h->stream, hipMemcpyAsync(g->d_tq, tq, bq, hipMemcpyHostToDevice, h->stream));
    if ((rc = rvk_gp_predict_device(g, g->d_theta, g->d_hyper, S, stride, hstride, g->d_tq, T, g->d_out, h->stream))) {
        (void)hipStreamSynchronize(h->stream);
        return rc;
    }
    HIPCHK_SYNC(h->stream, hipMemcpyAsync(out, g->d_out, bo, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return RVK_OK;
}

}  // extern "C"

// ---- GP log-posterior ---------------------------------------------------------------------

struct rvk_gp_post {
    rvk_gp *g = nullptr;
    int device = -1;               // the GP handle's, kept so destruction never dereferences g
    int n_free = 0, n_prior = 0, n_lp = 0, p_comb = 0;
    bool convert = false;
    double jac = 0.0, renorm = 0.0;
    int32_t *d_colmap = nullptr;
    double *d_tmpl = nullptr;
    PriorSlot *d_slots = nullptr;
    long long capw = 0;
    double *d_full = nullptr, *d_lp = nullptr, *d_lhp = nullptr;   // workspace for capw walkers
    // rvk_gp_stretch_run: proposals of a half, their log-posteriors, per-chunk arguments
    long long caph = 0;
    double *d_q = nullptr, *d_fac = nullptr, *d_lau = nullptr, *d_nlp = nullptr;
    long long *d_sidx = nullptr;
    RunArgs *d_run = nullptr;
    DrawTable tab;                 // the draws of a block of steps
    HostIO io;                     // rvk_gp_logpost's host-buffer transport (RVK_OPT_HOSTIO)

    PostDev dev() const {
        const rvk_handle *h = g->h;
        return PostDev{n_free, p_comb, n_prior, h->n_planets, h->n_inst, h->par, convert, d_colmap, d_tmpl, d_slots};
    }
};

static void free_gp_post(rvk_gp_post *p) {
    if (!p) return;
    if (p->device >= 0) (void)hipSetDevice(p->device);   // never through p->g: it may be gone already
    (void)hipFree(p->d_colmap);
    (void)hipFree(p->d_tmpl);
    (void)hipFree(p->d_slots);
    (void)hipFree(p->d_full);
    (void)hipFree(p->d_lp);
    (void)hipFree(p->d_lhp);
    p->io.release();
    (void)hipFree(p->d_q);
    (void)hipFree(p->d_fac);
    (void)hipFree(p->d_lau);
    (void)hipFree(p->d_nlp);
    (void)hipFree(p->d_sidx);
    (void)hipFree(p->d_run);
    p->tab.release();
    delete p;
}

static int gp_post_reserve_half(rvk_gp_post *p, long long H) {
    if (H <= p->caph) return RVK_OK;
    HIPCHK(hipSetDevice(p->g->h->device));
    (void)hipFree(p->d_q);
    (void)hipFree(p->d_fac);
    (void)hipFree(p->d_lau);
    (void)hipFree(p->d_nlp);
    (void)hipFree(p->d_sidx);
    p->d_q = p->d_fac = p->d_lau = p->d_nlp = nullptr;
    p->d_sidx = nullptr;
    p->caph = 0;
    HIPCHK(hipMalloc(&p->d_q, sizeof(double) * (size_t)H * (size_t)p->n_free));
    HIPCHK(hipMalloc(&p->d_fac, sizeof(double) * (size_t)H));
    HIPCHK(hipMalloc(&p->d_lau, sizeof(double) * (size_t)H));
    HIPCHK(hipMalloc(&p->d_nlp, sizeof(double) * (size_t)H));
    HIPCHK(hipMalloc(&p->d_sidx, sizeof(long long) * (size_t)H));
    if (!p->d_run) HIPCHK(hipMalloc(&p->d_run, sizeof(RunArgs)));
    p->caph = H;
    return RVK_OK;
}

static int gp_post_reserve(rvk_gp_post *p, long long W) {
    if (W <= p->capw) return RVK_OK;
    HIPCHK(hipSetDevice(p->g->h->device));
    (void)hipFree(p->d_full);
    (void)hipFree(p->d_lp);
    (void)hipFree(p->d_lhp);
    p->d_full = p->d_lp = p->d_lhp = nullptr;
    p->capw = 0;
    HIPCHK(hipMalloc(&p->d_full, sizeof(double) * (size_t)W * (size_t)p->p_comb));
    HIPCHK(hipMalloc(&p->d_lp, sizeof(double) * (size_t)W));
    HIPCHK(hipMalloc(&p->d_lhp, sizeof(double) * (size_t)W));
    p->capw = W;
    return RVK_OK;
}

static int create_gp_post(rvk_gp_post *p, rvk_gp *g, int32_t n_free, const int32_t *free_idx, const double *tmpl,
                          int32_t n_prior, int32_t n_param_prior, const int32_t *kind, const int32_t *src,
                          const double *par, double jac, double renorm, int32_t flags) {
    if (!g) return fail(RVK_E_ARG, "NULL GP handle");
    rvk_handle *h = g->h;
    const int pc = h->p_full() + RVK_GP_NHYPER;
    if (n_free < 1 || n_free > pc || !free_idx || !tmpl) return fail(RVK_E_ARG, "bad free-parameter layout");
    if (n_prior < 0 || n_param_prior < 0 || n_param_prior > n_prior || (n_prior > 0 && (!kind || !src || !par)))
        return fail(RVK_E_ARG, "bad prior arrays");
    if (flags & ~RVK_POST_CONVERT) return fail(RVK_E_ARG, "unknown flags");
    std::vector<int32_t> colmap(pc, -1);
    for (int i = 0; i < n_free; ++i) {
        if (free_idx[i] < 0 || free_idx[i] >= pc) return fail(RVK_E_ARG, "free_idx out of range");
        if (colmap[free_idx[i]] >= 0) return fail(RVK_E_ARG, "free_idx has a duplicate column");
        colmap[free_idx[i]] = i;
    }
    std::vector<PriorSlot> slots(n_prior);
    bool convert = (flags & RVK_POST_CONVERT) != 0;
    for (int k = 0; k < n_prior; ++k) {
        if (kind[k] < RVK_PRIOR_UNIFORM || kind[k] > RVK_PRIOR_BETA) return fail(RVK_E_ARG, "unknown prior kind");
        if (src[k] >= pc) return fail(RVK_E_ARG, "prior source column out of range");
        if (src[k] < 0 && -src[k] - 1 >= 5 * h->n_planets) return fail(RVK_E_ARG, "prior source planet out of range");
        convert |= src[k] < 0;
        slots[k].kind = kind[k];
        slots[k].src = src[k];
        std::memcpy(slots[k].p, par + (size_t)k * RVK_PRIOR_NPAR, sizeof(double) * RVK_PRIOR_NPAR);
    }
    p->g = g;
    p->device = g->h->device;
    p->n_free = n_free;
    p->n_prior = n_prior;
    p->n_lp = n_param_prior;
    p->p_comb = pc;
    p->convert = convert;
    p->jac = jac;
    p->renorm = renorm;
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipMalloc(&p->d_colmap, sizeof(int32_t) * pc));
    HIPCHK(hipMalloc(&p->d_tmpl, sizeof(double) * pc));
    HIPCHK(hipMalloc(&p->d_slots, sizeof(PriorSlot) * (n_prior > 0 ? n_prior : 1)));
    HIPCHK(hipMemcpy(p->d_colmap, colmap.data(), sizeof(int32_t) * pc, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(p->d_tmpl, tmpl, sizeof(double) * pc, hipMemcpyHostToDevice));
    if (n_prior > 0)
        HIPCHK(hipMemcpy(p->d_slots, slots.data(), sizeof(PriorSlot) * n_prior, hipMemcpyHostToDevice));
    return RVK_OK;
}

extern "C" {

rvk_gp_post *rvk_gp_post_create(rvk_gp *g, int32_t n_free, const int32_t *free_idx, const double *template_row,
                                int32_t n_prior, int32_t n_param_prior, const int32_t *prior_kind,
                                const int32_t *prior_src, const double *prior_par, double log_jacobian,
                                double log_renorm, int32_t flags) {
    rvk_gp_post *p = new (std::nothrow) rvk_gp_post();
    if (!p) {
        fail(RVK_E_NOMEM, "out of host memory");
        return nullptr;
    }
    if (create_gp_post(p, g, n_free, free_idx, template_row, n_prior, n_param_prior, prior_kind, prior_src, prior_par,
                       log_jacobian, log_renorm, flags)) {
        free_gp_post(p);
        return nullptr;
    }
    return p;
}

void rvk_gp_post_destroy(rvk_gp_post *p) { free_gp_post(p); }

int rvk_gp_post_reserve(rvk_gp_post *p, int64_t max_walkers) {
    if (!p || max_walkers < 0) return fail(RVK_E_ARG, "bad arguments");
    return gp_post_reserve(p, max_walkers);
}

int rvk_gp_logpost_device(rvk_gp_post *p, const double *d_free, int64_t W, int64_t stride, double *d_out,
                          void *stream) {
    if (!p) return fail(RVK_E_ARG, "NULL GP posterior");
    if (W < 0 || stride < p->n_free) return fail(RVK_E_ARG, "bad walker block shape");
    if (W == 0) return RVK_OK;
    if (!d_free || !d_out) return fail(RVK_E_ARG, "NULL device buffer");
    int rc = gp_post_reserve(p, W);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    rvk_handle *h = p->g->h;
    HIPCHK(hipSetDevice(h->device));
    hipLaunchKernelGGL(gp_logprior_kernel, dim3(gp_wave_blocks(W)), dim3(256), 0, st, p->dev(), p->n_lp, d_free,
                       (long long)W, (long long)stride, p->d_full, p->d_lp, p->d_lhp);
    HIPCHK(hipGetLastError());
    return gp_run(p->g, p->d_full, p->d_full + h->p_full(), W, p->p_comb, p->p_comb, d_out,
                  GpPost{p->d_lp, p->d_lhp, p->jac, p->renorm}, st);
}

int rvk_gp_logpost(rvk_gp_post *p, const double *xf, int64_t W, int64_t stride, double *out) {
    if (!p) return fail(RVK_E_ARG, "NULL GP posterior");
    if (W < 0 || stride < p->n_free) return fail(RVK_E_ARG, "bad walker block shape");
    if (W == 0) return RVK_OK;
    if (!xf || !out) return fail(RVK_E_ARG, "NULL host buffer");
    rvk_handle *h = p->g->h;
    std::lock_guard<std::mutex> lock(h->mu);   // one blocking call per handle at a time (rvk.h, threading)
    HIPCHK(hipSetDevice(h->device));
    const size_t bx = sizeof(double) * (size_t)W * (size_t)stride, bo = sizeof(double) * (size_t)W;
    const void *src = xf, *d_x = nullptr;
    void *d_out = nullptr;
    int rc;
    if ((rc = p->io.begin(h->hostio, h->stream, 1, &src, &bx, bo, &d_x, &d_out))) return rc;
    if ((rc = rvk_gp_logpost_device(p, (const double *)d_x, W, stride, (double *)d_out, h->stream))) {
        (void)hipStreamSynchronize(h->stream);
        return rc;
    }
    return p->io.end(h->stream, out, bo);
}

int rvk_gp_stretch_run(rvk_gp_post *p, double *d_x, double *d_lp, int64_t W, int32_t n_steps, double a, uint64_t seed,
                       uint64_t step0, int32_t flags, const int32_t *d_set, const double *d_zu, const int32_t *d_rint,
                       const double *d_au, double *d_chain, double *d_lnp, int64_t *d_naccepted, int32_t *d_status,
                       void *stream) {
    if (!p) return fail(RVK_E_ARG, "NULL GP posterior");
    if (W < 4 || (W & 1)) return fail(RVK_E_ARG, "n_walkers must be even and >= 4");
    if (n_steps < 0) return fail(RVK_E_ARG, "n_steps < 0");
    if (!(a > 1.0)) return fail(RVK_E_ARG, "stretch scale a must be > 1");
    if (flags & ~RVK_STRETCH_FIXED_SPLIT) return fail(RVK_E_ARG, "unknown flags");
    if (!d_x || !d_lp || !d_status) return fail(RVK_E_ARG, "NULL device buffer");
    if (d_set && (!d_zu || !d_rint || !d_au)) return fail(RVK_E_ARG, "host draws need set, zu, rint and au");
    if (n_steps == 0) return RVK_OK;
    const long long H = W / 2;
    int rc;
    if ((rc = gp_post_reserve_half(p, H)) || (rc = gp_post_reserve(p, H))) return rc;
    hipStream_t st = (hipStream_t)stream;
    HIPCHK(hipSetDevice(p->g->h->device));
    const int D = p->n_free;
    const size_t wd = (size_t)W * (size_t)D, hh = 2 * (size_t)H;
    const unsigned blocks = (unsigned)((H + 255) / 256);
    const int blk = draws_block_steps(H);
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
        rc = d_set ? draws_fill_host(p->tab, st, H, nb, D, run)
                   : draws_fill(p->tab, st, H, nb, D, seed, step0 + (uint64_t)b0, a, flags);
        if (rc) return rc;
        hipLaunchKernelGGL(set_run_kernel, dim3(1), dim3(1), 0, st, p->d_run, run);
        for (int s = 0; s < nb; ++s)
            for (int half = 0; half < 2; ++half) {
                hipLaunchKernelGGL(gp_propose_kernel, dim3(blocks), dim3(256), 0, st, p->d_run, p->tab.block, D, s,
                                   half, H, 0LL, H, p->d_q, p->d_fac, p->d_lau, p->d_sidx);
                if ((rc = rvk_gp_logpost_device(p, p->d_q, H, D, p->d_nlp, st))) return rc;
                hipLaunchKernelGGL(stretch_accept_kernel, dim3(blocks), dim3(256), 0, st, p->d_run, s, H, D, p->d_q,
                                   p->d_fac, p->d_lau, p->d_sidx, p->d_nlp);
            }
    }
    HIPCHK(hipGetLastError());
    return RVK_OK;
}

int rvk_gp_stretch_draws(rvk_gp_post *p, int64_t W, int32_t n_steps, double a, uint64_t seed, uint64_t step0,
                         int32_t flags, void *stream) {
    if (!p) return fail(RVK_E_ARG, "NULL GP posterior");
    if (W < 4 || (W & 1)) return fail(RVK_E_ARG, "n_walkers must be even and >= 4");
    if (n_steps < 1) return fail(RVK_E_ARG, "n_steps must be >= 1");
    if (!(a > 1.0)) return fail(RVK_E_ARG, "stretch scale a must be > 1");
    if (flags & ~RVK_STRETCH_FIXED_SPLIT) return fail(RVK_E_ARG, "unknown flags");
    HIPCHK(hipSetDevice(p->g->h->device));
    return draws_fill(p->tab, (hipStream_t)stream, W / 2, n_steps, p->n_free, seed, step0, a, flags);
}

int rvk_gp_stretch_propose(rvk_gp_post *p, const double *d_x, int64_t W, int32_t s, int32_t half, int64_t j0,
                           int64_t count, double *d_out, void *stream) {
    if (!p) return fail(RVK_E_ARG, "NULL GP posterior");
    const long long H = W / 2;
    if (W < 4 || (W & 1) || H != p->tab.H) return fail(RVK_E_ARG, "n_walkers differs from the drawn table's");
    if (s < 0 || s >= p->tab.steps) return fail(RVK_E_ARG, "step outside the drawn table");
    if (half != 0 && half != 1) return fail(RVK_E_ARG, "half must be 0 or 1");
    if (j0 < 0 || count < 0 || j0 + count > H) return fail(RVK_E_ARG, "proposal slice outside the half");
    if (!d_x || !d_out) return fail(RVK_E_ARG, "NULL device buffer");
    if (count == 0) return RVK_OK;
    int rc;
    if ((rc = gp_post_reserve_half(p, count)) || (rc = gp_post_reserve(p, count))) return rc;
    hipStream_t st = (hipStream_t)stream;
    HIPCHK(hipSetDevice(p->g->h->device));
    const RunArgs run{const_cast<double *>(d_x), nullptr, nullptr, nullptr, nullptr, nullptr,
                      nullptr, nullptr, nullptr, nullptr, 0, 0, 2.0};
    hipLaunchKernelGGL(set_run_kernel, dim3(1), dim3(1), 0, st, p->d_run, run);
    hipLaunchKernelGGL(gp_propose_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st, p->d_run,
                       p->tab.block, p->n_free, s, half, (long long)count, (long long)j0, H, p->d_q, p->d_fac, p->d_lau,
                       p->d_sidx);
    HIPCHK(hipGetLastError());
    return rvk_gp_logpost_device(p, p->d_q, count, p->n_free, d_out, st);
}

int rvk_gp_stretch_update(rvk_gp_post *p, double *d_x, double *d_lp, int64_t W, int32_t s, int32_t half,
                          const double *d_nlp, double *d_chain_step, double *d_lnp_step, const int64_t *d_nacc_in,
                          int64_t *d_nacc_out, int32_t *d_status, void *stream) {
    if (!p) return fail(RVK_E_ARG, "NULL GP posterior");
    const long long H = W / 2;
    if (W < 4 || (W & 1) || H != p->tab.H) return fail(RVK_E_ARG, "n_walkers differs from the drawn table's");
    if (s < 0 || s >= p->tab.steps) return fail(RVK_E_ARG, "step outside the drawn table");
    if (half != 0 && half != 1) return fail(RVK_E_ARG, "half must be 0 or 1");
    if (!d_x || !d_lp || !d_nlp || !d_status) return fail(RVK_E_ARG, "NULL device buffer");
    if (d_nacc_out && !d_nacc_in) return fail(RVK_E_ARG, "d_nacc_out needs d_nacc_in");
    HIPCHK(hipSetDevice(p->g->h->device));
    hipLaunchKernelGGL(stretch_update_kernel, dim3((unsigned)((H + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       p->tab.block + ((size_t)s * 2 + (size_t)half) * (size_t)H, H, p->n_free, d_x, d_lp, d_nlp,
                       (const long long *)d_nacc_in, (long long *)d_nacc_out, (int *)d_status, d_chain_step,
                       d_lnp_step);
    HIPCHK(hipGetLastError());
    return RVK_OK;
}

}  // extern "C"
