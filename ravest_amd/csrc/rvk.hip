// rvk.hip -- MI355X (gfx950) kernels and the C-ABI of include/rvk.h.
//
// Hot path: ravest's LogLikelihood.__call__ (src/ravest/fit.py:3600-3660)
// batched over walkers.  Mapping (see DESIGN.md "Kernels"):
//   * one wave64 per walker (grid-stride over walkers); the walker index is
//     wave-uniform (readfirstlane), so its theta row is fetched with scalar
//     loads and the per-planet prologue (conversion + validity, param.py) is
//     computed once per wave;
//   * lanes stride the epochs: lane l handles epochs l, l+64, ... -- the
//     time / velocity / velerr^2 / instrument arrays are read coalesced;
//   * per (walker, epoch): sum over planets of the Kepler RV (Halley in a
//     2*pi-reduced frame), + trend + gamma[inst]; s^2 = velerr^2 + jit[inst]^2;
//     chi^2 accumulates in a register and sum(log s^2) as a renormalised
//     running product (frexp), so the epoch loop has no log;
//   * a wave64 butterfly reduction gives 1 fp64 per walker; -inf for
//     invalid walkers (mask semantics of fit.py:3622-3627).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "rvk_internal.h"
#include "rvk_post_dev.h"

#ifndef RVK_TU_SAMPLE
#define RVK_TU_SAMPLE 0   // 1 / 2: rvk_sample.hip / rvk_sample1.hip's builds of this file (the fused half-steps)
#endif

using namespace rvk;

namespace {

#ifndef RVK_CHI_NR2
#define RVK_CHI_NR2 0
#endif
#ifndef RVK_TAB_LDS
#define RVK_TAB_LDS 1                 // sin/cos table staged in LDS (1) or read through L1 (0)
#endif
#ifndef RVK_UNROLL2
#define RVK_UNROLL2 0                 // epoch loop: two epochs per trip, ping-pong prefetch registers (1)
#endif
#ifndef RVK_PREP_TAB
#define RVK_PREP_TAB 1                // prep's sin/cos(w) from the LDS table (1) or fdlibm (0)
#endif
#ifndef RVK_TP_INLINE
#define RVK_TP_INLINE 1               // "P K e w Tp": inline conversion in the prep (1) or the out-of-line one (0)
#endif
#ifndef RVK_SEG_LB3
#define RVK_SEG_LB3 4                 // min blocks per CU of the segmented kernel for NP >= 3 (4: <= 128 VGPRs)
#endif
#ifndef RVK_FUSE_PROLOGUE
#define RVK_FUSE_PROLOGUE 1           // fused kernel prologue: loads first, LDS stores after (see loglike_kernel)
#endif
#ifndef RVK_FUSE_SLOTREG
#define RVK_FUSE_SLOTREG 1            // fused prep: the lane's prior slot copied to registers before the prior formula
#endif
#ifndef RVK_FUSE_COMPOSE
#define RVK_FUSE_COMPOSE 0            // fused prep: operands straight from q by the composed column map (1): measured 18.4 vs 17.9 us per step, off
#endif
#ifndef RVK_PREP_GTAB
#define RVK_PREP_GTAB 1               // prep's sin/cos(w) from the global (L2) table (1), or from the LDS copy behind an
                                      // extra block barrier (0): measured 7.4 vs 7.7 us on config 2
#endif
#ifndef RVK_EPOCH_OFF32
#define RVK_EPOCH_OFF32 1             // epoch loads through one 32-bit byte offset (global_load saddr form)
#endif
#ifndef RVK_EPOCH_UNI
// epoch loop with a wave-uniform trip count over the padded epoch block (1); the fused half-step
// units keep the per-lane loop (sessions sa1/sa2, tools/sampler_ab.sh: 16.5-16.7 vs 17.0 us per
// config-2 sampler step; the plain likelihood kernels take the uniform loop)
#define RVK_EPOCH_UNI (RVK_TU_SAMPLE == 0)
#endif
#ifndef RVK_SOLVE_UNI
#define RVK_SOLVE_UNI 1               // loglike_kernel (one walker per wave): e-dependent solver choices as scalar branches
#endif
#ifndef RVK_PAIR_RENORM
#define RVK_PAIR_RENORM 1             // epoch pairs share one renormalisation of the s^2 product when safe (same bits)
#endif
#ifndef RVK_PK_SGPR
#define RVK_PK_SGPR 2                 // NP >= this: planet constants moved to SGPRs, else left in VGPRs
                                      // (NP = 1 in VGPRs: 34 -> 7 SGPR spills, -2.5 % config 2;
                                      //  NP = 3 in VGPRs: +3.6 %)
#endif
#ifndef RVK_SAMPLE_BLOCK
#define RVK_SAMPLE_BLOCK 512          // threads per fused half-step block: one block per CU at H = 2048 (256: 18.8, 512: 18.2, 768: 20.9 us per step)
#endif
#ifndef RVK_LL_BLOCK
#define RVK_LL_BLOCK 1024             // threads per loglike_kernel block for NP = 1 and W >= 256 blocks' worth
                                      // (one wave preps 16 walkers: -7 % "P K e w Tc", +-0 "P K e w Tp")
#endif
#ifndef RVK_FUSE_LB
#define RVK_FUSE_LB 8                 // fused half-step kernels, NP > 1: min waves per SIMD x BLK / kBlock (8: 4 waves, <= 128 VGPRs,
                                      // two 512-thread blocks per CU; session lb: config 3 257 -> 227-237 us, config 4
                                      // 347 -> 292-296 us per sampler step, against 130-140 VGPRs at 1 block per CU)
#endif
#ifndef RVK_LB_WAVES
#define RVK_LB_WAVES 1                // min waves/SIMD for loglike_kernel, NP > 1 (NP == 1: 4, <= 128 VGPRs)
#endif

// base[off / sizeof(T)] for a byte offset below 4 GiB: the 64-bit base stays in SGPRs and the
// 32-bit offset is the load's VGPR operand (global_load's saddr form), so a lane advancing
// through the epochs keeps one 32-bit induction variable instead of a 64-bit address per array.
template <class T>
__device__ __forceinline__ T ld_off(const T *base, unsigned off) {
    return *reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) + off);
}

// RVK_OPT_LDS_POISON for the kernels whose first parameter is the EpochData: the flag re-read
// from the kernel-argument segment where the table is stored (a volatile scalar load, K$-resident),
// so it holds no SGPR across the prologue (a live flag there cost SGPR spills, ~8 VALU
// instructions per wave on config 2).
__device__ __forceinline__ int poison_arg() {
    using kp = const __attribute__((address_space(4))) char *;
    const kp p = (kp)__builtin_amdgcn_kernarg_segment_ptr();
    return *(volatile const __attribute__((address_space(4))) int *)(p + offsetof(EpochData, poison));
}

// Copy the sin/cos table into LDS (whole block; one barrier, before any
// per-wave work so no wave can skip it).
__device__ __forceinline__ void load_tab(SC *lds, const SC *__restrict__ g, int poison = 0) {
    for (int i = threadIdx.x; i < kTabN; i += blockDim.x) tab_put(lds, i, g[i], poison);
    __syncthreads();
}

#ifndef RVK_LL_TRACE
#define RVK_LL_TRACE 0    // timing experiments only: s_memtime per phase for 4 sampled blocks
#endif
#if RVK_LL_TRACE
__device__ unsigned long long g_ll_trace[16][8];
#define LL_MARK(slot)                                                                                   \
    do {                                                                                                \
        const int tb_ = (blockIdx.x == 0) ? 0 : (blockIdx.x == 100) ? 1 : (blockIdx.x == 500) ? 2 :      \
                        (blockIdx.x == 1000) ? 3 : -1;                                                  \
        if (tb_ >= 0 && (threadIdx.x & 63) == 0) g_ll_trace[tb_ * 4 + (threadIdx.x >> 6)][slot] =        \
            (slot == 0 || slot == 7) ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define LL_MARK(slot) do {} while (0)
#endif

// One walker's epoch loop (fit.py:3632-3658 over model.py:173-213 per planet), one wave, lanes
// striding the epochs (l, l + 64, ...): gamma[inst] + sum over planets (+ trend, the loop
// versioned on the wave-uniform gd / gdd), s^2 = sigma^2 + jit^2, chi^2 += r^2 rcp(s^2), sum
// log s^2 as a frexp-renormalised running product, then one log per lane and the fixed-order
// wave sum.  Returns chi^2 + sum log s^2 of the walker in every lane.  g / jit point at the
// walker's gamma[] and jit[] (then gd, gdd); pk holds NP > 0 planets' constants (registers or
// SGPRs), pks the generic kernel's np planets (LDS).  (t_1, v_1, s_1, i_1): the lane's first
// epoch, loaded by the caller at kernel start.
template <int NP, bool MULTI, int SOLVER>
__device__ __forceinline__ double epoch_sum(const EpochData &d, int n_epochs, int n_inst, const double *g,
                                            const double *jit, const PlanetK *pk, const PlanetK *pks, int np,
                                            const SC *tab, double t_1, double v_1, double s_1, int i_1, int lane) {
    const double gd = jit[n_inst], gdd = jit[n_inst + 1];
    const double g0 = g[0], j0 = jit[0] * jit[0];
    double chi2 = 0.0, prod = 0.5;   // prod * 2^expo = running product of s^2
    int expo = 1;
    KFlags kf[NP > 0 ? NP : 1];      // the solver's per-planet choices, wave-uniform (one walker per wave)
    if constexpr (RVK_SOLVE_UNI && NP > 0) {
#pragma unroll
        for (int p = 0; p < NP; ++p) kf[p] = kflags_uniform(pk[p].e);
    }
    // The epoch loop, versioned on the (wave-uniform) trend so the trend-free
    // common case carries no trend arithmetic at all.
    auto epochs = [&](auto trend_c) {
        constexpr bool TREND = decltype(trend_c)::value;
        // one epoch: gamma + planets (+ trend), chi^2 term, s^2 into the running product.
        // PAIR: the first epoch of a pair on the walker-safe path (below): no renormalisation
        // after it, and no fmin in 1/s^2 (s^2 is finite and normal there, where the fmin is a
        // no-op): the same bits, since frexp only scales by a power of two.
        auto one = [&](double t, double vel, double s2b, int ii, auto pair_c) {
            constexpr int PM = decltype(pair_c)::value;   // 0 single, 1 first of a pair, 2 second
            constexpr bool PAIR = PM != 0;
            double gam = g0, jj = j0;
            if (MULTI) {
                for (int k = 1; k < n_inst; ++k) {
                    if (ii == k) { gam = g[k]; jj = jit[k] * jit[k]; }
                }
            }
            double rv = gam - vel;   // the residual itself: each planet's K * (...) lands in one FMA
            if constexpr (NP > 0) {
#pragma unroll
                for (int p = 0; p < NP; ++p) rv = planet_rv<SOLVER, RVK_SOLVE_UNI>(pk[p], t, tab, rv, kf[p]);
            } else {
                for (int p = 0; p < np; ++p) rv = planet_rv<SOLVER>(pks[p], t, tab, rv);
            }
            if (TREND) {
                const double dt = t - d.t0;
                rv += __builtin_fma(gd, dt, gdd * (dt * dt));
            }
            const double s2 = s2b + jj;
            const double r = rv;
#if RVK_CHI_NR2
            chi2 = __builtin_fma(r * r, rcp_nr(s2), chi2);
#else
            if constexpr (PAIR) chi2 = __builtin_fma(r * r, rcp_nr1_finite(s2), chi2);
            else chi2 = __builtin_fma(r * r, rcp_nr1(s2), chi2);   // <= 2.2e-15 relative per term
#endif
            prod *= s2;
            if constexpr (PM != 1) {
                int ex;
                prod = __builtin_frexp(prod, &ex);
                expo += ex;
            }
        };
        const auto single = std::integral_constant<int, 0>{};
        const auto first = std::integral_constant<int, 1>{};
        const auto second = std::integral_constant<int, 2>{};
        // pairs of epochs may share one renormalisation when every s^2 of this walker lies in
        // [2^-500, 2^501]: then prod in [0.5, 1) times two of them stays a normal number
        // (no overflow, underflow or denormal), so skipping the power-of-two scaling in
        // between changes no bit.  Wave-uniform (the data's flag and the walker's jitter).
        const bool pairsafe = !MULTI && RVK_PAIR_RENORM && d.s2ok && (j0 <= 0x1p500);
        // Lane epochs i, i+64, ...  RVK_UNROLL2: two per trip with ping-pong registers
        // (A, B), no register shuffling between trips; invariant: A holds epoch i.
#if RVK_UNROLL2
        double tA = t_1, vA = v_1, sA = s_1, tB = 0.0, vB = 0.0, sB = 1.0;
        int iA = i_1, iB = 0;
        int i = lane;
        for (; i + 64 < n_epochs; i += 128) {
            tB = d.t[i + 64]; vB = d.vel[i + 64]; sB = d.s2[i + 64];
            if (MULTI) iB = d.inst[i + 64];
            one(tA, vA, sA, iA, single);
            if (i + 128 < n_epochs) {
                tA = d.t[i + 128]; vA = d.vel[i + 128]; sA = d.s2[i + 128];
                if (MULTI) iA = d.inst[i + 128];
            }
            one(tB, vB, sB, iB, single);
        }
        if (i < n_epochs) one(tA, vA, sA, iA, single);
#elif RVK_EPOCH_UNI
        // Every lane runs `full` = n / 64 trips whose epoch exists, then lanes < n % 64 one more:
        // the trip count is wave-uniform, so the loop runs on a scalar counter -- no per-lane
        // compare, exec-mask update or address increment per epoch.  The prefetch of epoch i + 64
        // is unconditional: the epoch arrays are one padded block (rvk_create: t | vel | s2 | inst,
        // kEpochPad entries after each), so it reads padding past the end, never out of bounds.
        // All four arrays are read through ONE buffer descriptor based at t: the lane's offset
        // (8 lane, 4 lane) is the VGPR operand, the array and the trip are the scalar offset, so
        // addressing costs no VALU.  One planet: two epochs per trip with ping-pong registers (A
        // holds the trip's first epoch: no register copies between trips).  Same epochs in the
        // same order per lane as the other forms: bitwise the same results.
        const int full = n_epochs >> 6;
        const bool tail = lane < (n_epochs & 63);
        const char *b0 = reinterpret_cast<const char *>(d.t);
        const int ov = (int)(reinterpret_cast<const char *>(d.vel) - b0);
        const int os = (int)(reinterpret_cast<const char *>(d.s2) - b0);
        const int oi = (int)(reinterpret_cast<const char *>(d.inst) - b0);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(b0), 0, oi + 4 * (n_epochs + kEpochPad), 0x00020000);
        const int lo = 8 * lane, li = 4 * lane;
        auto ldd = [&](int voff, int soff) -> double {
            return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0));
        };
        auto ldi = [&](int soff) -> int { return (int)__builtin_amdgcn_raw_buffer_load_b32(rs, li, soff, 0); };
        double tA = t_1, vA = v_1, sA = s_1, tB, vB, sB;
        int iA = i_1, iB = 0;
        int k = 0;
        if constexpr (NP == 1) {
            auto pairs = [&](auto m1, auto m2) {
                for (; k + 2 <= full; k += 2) {
                    const int e1 = 512 * (k + 1), e2 = 512 * (k + 2);   // byte offsets of epochs k+1, k+2
                    tB = ldd(lo, e1); vB = ldd(lo, ov + e1); sB = ldd(lo, os + e1);
                    if (MULTI) iB = ldi(oi + (e1 >> 1));
                    one(tA, vA, sA, iA, m1);
                    tA = ldd(lo, e2); vA = ldd(lo, ov + e2); sA = ldd(lo, os + e2);
                    if (MULTI) iA = ldi(oi + (e2 >> 1));
                    one(tB, vB, sB, iB, m2);
                }
            };
            if (pairsafe) pairs(first, second);
            else pairs(single, single);
        }
        for (; k < full; ++k) {            // one trip (NP != 1), or the odd last full trip (NP == 1)
            const int e1 = 512 * (k + 1);
            tB = ldd(lo, e1); vB = ldd(lo, ov + e1); sB = ldd(lo, os + e1);
            if (MULTI) iB = ldi(oi + (e1 >> 1));
            one(tA, vA, sA, iA, single);
            tA = tB; vA = vB; sA = sB; iA = iB;
        }
        if (tail) one(tA, vA, sA, iA, single);
#elif RVK_EPOCH_OFF32
        // one epoch per trip; the next epoch's loads are issued before this one's solve.
        // off = 8 (i + 64), the next epoch's byte offset, is the only induction variable:
        // epoch i is live while off < 8 n + 512, epoch i + 64 exists while off < 8 n.
        double tn = t_1, vn = v_1, sn = s_1;
        int in_ = i_1;
        const unsigned lim = 8u * (unsigned)n_epochs;
        for (unsigned off = 8u * (unsigned)(lane + 64); off < lim + 512u; off += 512u) {
            const double t = tn, vel = vn, s2b = sn;
            const int ii = in_;
            if (off < lim) {
                tn = ld_off(d.t, off); vn = ld_off(d.vel, off); sn = ld_off(d.s2, off);
                if (MULTI) in_ = ld_off(d.inst, off >> 1);
            }
            one(t, vel, s2b, ii, single);
        }
#else
        // one epoch per trip; the next epoch's loads are issued before this one's solve
        double tn = t_1, vn = v_1, sn = s_1;
        int in_ = i_1;
        for (int i = lane; i < n_epochs; i += 64) {
            const double t = tn, vel = vn, s2b = sn;
            const int ii = in_;
            if (i + 64 < n_epochs) {
                tn = d.t[i + 64]; vn = d.vel[i + 64]; sn = d.s2[i + 64];
                if (MULTI) in_ = d.inst[i + 64];
            }
            one(t, vel, s2b, ii, single);
        }
#endif
    };
    if ((gd != 0.0) | (gdd != 0.0)) epochs(std::true_type{});
    else epochs(std::false_type{});
    LL_MARK(4);
    // prod is a frexp mantissa in [0.5, 1) unless the product hit 0 (some s^2 = 0), inf or NaN,
    // whose log is -inf, inf, NaN whatever the exponent
    double lsum = log_frexp(prod, expo);
    if (!(prod >= 0.5 && prod < 1.0)) lsum = prod == 0.0 ? -INFINITY : prod;
    return wave_sum(chi2 + lsum);
}

// Block-level structure.  A block (4 waves) owns passes of up to WB walkers
// (contiguous).  Each pass:
//   1. prep, lane-parallel over (walker, planet): thread k builds PlanetK for
//      walker k/NP, planet k%NP into LDS -- one conversion latency per pass
//      instead of one per walker, and no planet state lives in registers.  The
//      conversion (param.py:198-234, 299-362) is an out-of-line call with
//      register-light atan/atan2/tan (rvk_math.h), so it does not set the
//      epoch loop's VGPR budget;
//   2. __syncthreads (the first pass also covers the sin/cos table fill);
//   3. wave wv evaluates walkers wv, wv+4, ... of the pass: lanes stride the
//      epochs, planet constants are re-read from LDS with a wave-uniform
//      address (broadcast), a wave64 butterfly gives the walker's sum.
//
// SAMPLE (rvk_stretch_run): the rows are the proposals of the active half
// (propose_kernel), lp their log-priors; after the reduction the wave accepts
// or rejects its proposal and writes the walker's state and chain row.
//
// SAMPLE == 2 (fused proposals): each wave makes the stretch-move proposal of its walker
// itself, lanes over coordinates, columns, prior slots and planets -- draws, q = c - (c - s) z,
// the full row, the jitter check, the basic-kind priors (fit.py:3461-3482) and the planet
// constants -- into its LDS slots, then runs the epoch loop: a half-step is one kernel instead
// of propose_kernel + this one, and no block barrier separates a walker's prep from its loop.
// Same arithmetic and order as propose_kernel / post_row_wave (rvk_post.hip,
// rvk_post_dev.h), so the chain is the same bit for bit.
// NP = 0: the generic kernel, planet count d.np (9 .. RVK_MAX_PLANETS), one walker per wave per pass
// and its planet constants read from LDS in the epoch loop.
template <int NP>
struct PassCfg {
    static constexpr int WB = NP == 0 ? kWavesPerBlock : (NP <= 4) ? 64 : 32;   // walkers per pass (LDS: WB*NP*64 B)
    static constexpr int NPA = NP > 0 ? NP : RVK_MAX_PLANETS;                   // planet slots per walker
};

template <int NP, bool MULTI, int SOLVER, bool TP, int SAMPLE, int BLK = kBlock>
__global__ __launch_bounds__(BLK, ((NP == 1 || (SAMPLE & 3) >= 2) ? (NP == 1 ? 4 : RVK_FUSE_LB) : RVK_LB_WAVES) * kBlock / BLK) void loglike_kernel(EpochData d, int n_epochs, int n_inst,
                                                         const double *__restrict__ theta, long long n_walkers,
                                                         long long stride, int wb, double *__restrict__ out,
                                                         PostArgs post, SampleArgs sa) {
    constexpr int WB = PassCfg<NP>::WB, NPA = PassCfg<NP>::NPA;
    const int np = NP > 0 ? NP : d.np;
    // SAMPLE & 3: 1 accept / reject of propose_kernel's proposals; 2 proposals made in this kernel
    // + accept / reject; 3 proposals made here, log-posterior out (rvk_stretch_propose).
    // SAMPLE & 4 (ALLP): every prior kind in the fused prep (else the basic kinds only);
    // SAMPLE & 8 (CONV): + the prior-side conversion (Case 3; an out-of-line call, whose frame
    // only this variant pays).
    // SAMPLE & 16 (DIRECT, with MODE 3): the walker's free coordinates are given (sa.q, row stride
    // sa.qstride) instead of proposed -- the device log-posterior in one kernel (rvk_logpost[_device]).
    constexpr int MODE = SAMPLE & 3;
    constexpr bool DIRECT = (SAMPLE & 16) != 0;
    constexpr bool FUSE = MODE >= 2;
    constexpr bool ACCEPT = MODE == 1 || MODE == 2;
    constexpr bool CONV = (SAMPLE & 8) != 0;
    constexpr bool EXT = CONV || (SAMPLE & 4) != 0;
    constexpr int WF = FUSE ? BLK / 64 : 1;   // fused: one walker per wave per pass (launch_sample_fused)
    __shared__ PlanetK pks[WB][NPA];
    __shared__ int okp[WB][NPA];
    __shared__ double fq[WF][kFuseMaxD], fx[WF][kFuseMaxD], ff[WF][kFuseMaxPFull];
    constexpr int FP = FUSE ? kFuseMaxPFull : 1, FS = FUSE ? kFuseMaxPrior : 1;
    __shared__ int fcol[FP];
    __shared__ double ftm[FP];
    __shared__ PriorSlot fsl[FS];
    const int lane = threadIdx.x & 63;
    // Epoch data does not depend on the walker: this lane's first epoch is loaded once,
    // before anything else, so its latency hides under the table fill and the prep.
    double t_1 = 0.0, v_1 = 0.0, s_1 = 1.0;
    int i_1 = 0;
    if (lane < n_epochs) {
        t_1 = d.t[lane]; v_1 = d.vel[lane]; s_1 = d.s2[lane];
        if (MULTI) i_1 = d.inst[lane];
    }
    // FUSE (RVK_FUSE_PROLOGUE): the table fill and the posterior constants are loaded into
    // registers first and stored to LDS only after the walker's draw / row loads are issued, so
    // the prologue is three memory round trips (constants and draws || rows || barrier), not a
    // chain of a wait per kind of load
    // (the plain likelihood likewise when its prep reads the global table: the LDS copy is
    // stored after the prep's row loads and conversion, before the pass barrier)
    constexpr bool TDEF = RVK_FUSE_PROLOGUE && RVK_TAB_LDS && BLK >= kTabN && (FUSE || !TP || RVK_PREP_GTAB);
#if RVK_TAB_LDS
    __shared__ SC tab[kTabN];
    double tab_s = 0.0, tab_c = 0.0;   // (scalars: a struct here is promoted to a per-thread LDS copy)
    if constexpr (TDEF) {
        if (threadIdx.x < kTabN) {
            tab_s = d.tab[threadIdx.x].s;
            tab_c = d.tab[threadIdx.x].c;
        }
    } else {
        for (int i = threadIdx.x; i < kTabN; i += BLK) tab_put(tab, i, d.tab[i], poison_arg());
    }
#else
    const SC *__restrict__ tab = d.tab;   // L1/L2-resident gather, no LDS fill
#endif
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // FUSE: a wave's proposal draws and reads of the walker rows (emcee's StretchMove), issued
    // for the wave's first walker before the barrier so their latency hides under the table
    // fill; the posterior's constants are staged in LDS (each is read in a loop with a runtime
    // trip count: from global memory every iteration would wait on a load).
    struct Fetch {
        long long s, c;    // the walker and its complement
        double z, a, b, lpo;
        double fac, lau;   // (D - 1) log z and log u': the draws' logs, off the prep's chain
        long long nacc;    // the walker's acceptance count (read here, written +1 at the tail)
    };
    auto fetch = [&](long long w) {
        Fetch f;
        const int D = sa.pd.n_free;
        if constexpr (DIRECT) {
            f.s = w;
            f.c = 0;
            f.z = f.fac = f.lau = f.lpo = f.b = 0.0;
            f.nacc = 0;
            f.a = lane < D ? sa.q[w * sa.qstride + lane] : 0.0;
            return f;
        }
        const long long j = sa.j0 + w;   // global proposal index within the half
        const PreDraw *pp = sa.pre + ((long long)sa.step * 2 + sa.half) * sa.hfull + j;
        using gdp = const __attribute__((address_space(1))) double *;   // global loads (a flat one holds lgkmcnt)
        // every scalar load of the fetch (the draw, the state pointers) issued before any is used:
        // one wait for all of them instead of a wait per load
        const long long ps = pp->s, pc = pp->c;
        const double pz = pp->z, pfac = pp->fac, plau = pp->lau;
        const gdp rx = (gdp)sa.run->x;
        const gdp rlp = (gdp)sa.run->lp;
        const __attribute__((address_space(1))) long long *const rnacc =
            (const __attribute__((address_space(1))) long long *)sa.run->nacc;
        if (RVK_FUSE_PROLOGUE) __builtin_amdgcn_sched_barrier(0);
        f.s = ps;
        f.c = pc;
        f.z = pz;
        f.fac = pfac;
        f.lau = plau;
        // the rows first, then the walker's log-prob and count: all four loads in flight together
        f.a = f.b = 0.0;
        if (lane < D) {
            f.a = rx[ps * D + lane];
            f.b = rx[pc * D + lane];
        }
        f.lpo = ACCEPT ? rlp[ps] : 0.0;
        f.nacc = (ACCEPT && rnacc) ? rnacc[ps] : 0;
        return f;
    };
    Fetch pre{};
    int pf_draw = 0;   // a word of the next half-step's draw row, touched so it is L2-resident then
    if constexpr (FUSE) {
        const long long w0 = (long long)blockIdx.x * wb + wv;
        if constexpr (ACCEPT && !DIRECT) {
            // the same block index runs on the same XCD in the next launch of this grid
            if (sa.pre_next && wv < wb && w0 < n_walkers && lane == 0) {
                int zo = 0;
                asm volatile("" : "+v"(zo));   // a VGPR offset: a vector load, off the scalar waits
                pf_draw = *(const __attribute__((address_space(1))) int *)(
                    reinterpret_cast<const char *>(sa.pre_next + sa.j0 + w0) + zo);   // global_load, not flat
            }
        }
        if constexpr (RVK_FUSE_PROLOGUE) {
            static_assert(BLK >= kFuseMaxPFull && BLK >= kFuseMaxPrior, "one staging entry per thread");
            const int tid = threadIdx.x;
            const bool stc = tid < sa.pd.p_full, sts = tid < sa.pd.n_prior;
            int fc_r = 0;
            double ftm_r = 0.0;
            constexpr int SW = sizeof(PriorSlot) / 8;   // the slot as 8-byte words, in registers
            static_assert(sizeof(PriorSlot) % 8 == 0, "PriorSlot is whole 8-byte words");
            unsigned long long sw_r[SW];
            if (stc) {
                fc_r = sa.pd.colmap[tid];
                ftm_r = sa.pd.tmpl[tid];
            }
            if (sts) {
                const unsigned long long *src = reinterpret_cast<const unsigned long long *>(sa.pd.slots + tid);
#pragma unroll
                for (int k = 0; k < SW; ++k) sw_r[k] = src[k];
            }
            if (wv < wb && w0 < n_walkers) pre = fetch(w0);
            __builtin_amdgcn_sched_barrier(0);   // the stores below wait for their loads only
#if RVK_TAB_LDS
            if constexpr (TDEF) {
                if (tid < kTabN) tab_put(tab, tid, SC{tab_s, tab_c}, poison_arg());
            }
#endif
            if (stc) {
                fcol[tid] = fc_r;
                ftm[tid] = ftm_r;
            }
            if (sts) {
                unsigned long long *dst = reinterpret_cast<unsigned long long *>(fsl + tid);
#pragma unroll
                for (int k = 0; k < SW; ++k) dst[k] = sw_r[k];
            }
        } else {
            if (wv < wb && w0 < n_walkers) pre = fetch(w0);
            for (int i = threadIdx.x; i < sa.pd.p_full; i += BLK) {
                fcol[i] = sa.pd.colmap[i];
                ftm[i] = sa.pd.tmpl[i];
            }
            for (int i = threadIdx.x; i < sa.pd.n_prior; i += BLK) fsl[i] = sa.pd.slots[i];
        }
        __syncthreads();   // (also publishes the table)
    }
    LL_MARK(0);
    LL_MARK(1);
    for (long long base = (long long)blockIdx.x * wb; base < n_walkers; base += (long long)gridDim.x * wb) {
        const int nb = (int)((n_walkers - base) < wb ? (n_walkers - base) : wb);
        // prep (the table fill above lands under the same barrier)
        if constexpr (!FUSE) {
        static_assert(WB * NPA <= BLK, "the prep gives each thread at most one (walker, planet)");
        const int k = threadIdx.x;
        const bool has = k < nb * np;
        const int j = has ? k / np : 0, p = has ? k - j * np : 0;
        const double *p5 = theta + (base + j) * stride + 5 * p;
        if constexpr (TP && RVK_PREP_TAB && RVK_TAB_LDS && RVK_PREP_GTAB) {
            if (has) {   // sin/cos(w) from the global (L2-resident) table: no barrier before the prep
                PlanetK pk;
                okp[j][p] = planet_consts_t<0, true>(p5, pk, 0, d.tab);
                pks[j][p] = pk;
            }
        } else if constexpr (TP && RVK_PREP_TAB && RVK_TAB_LDS) {
            // "P K e w Tp" inline; its sin/cos(w) reads the LDS table that all waves fill: the row
            // is loaded first, then the block barrier publishes the table (the first pass; later
            // passes follow the end-of-pass barrier), so the two loads' latencies overlap
            double r5[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
            if (has) {
#pragma unroll
                for (int c = 0; c < 5; ++c) r5[c] = p5[c];
            }
            if (base == (long long)blockIdx.x * wb) __syncthreads();
            if (has) {
                PlanetK pk;
                okp[j][p] = planet_consts_t<0, true>(r5, pk, 0, tab);
                pks[j][p] = pk;
            }
        } else if (has) {
            PlanetK pk;
            // "P K e w Tp" inline (no call, no scratch); the others out of line
            const bool ok = TP ? planet_consts_t<0, RVK_PREP_TAB>(p5, pk, 0, tab) : planet_consts(d.par, p5, pk);
            pks[j][p] = pk;
            okp[j][p] = ok;
        }
#if RVK_TAB_LDS
        if constexpr (TDEF) {
            if (base == (long long)blockIdx.x * wb && threadIdx.x < kTabN)
                tab_put(tab, threadIdx.x, SC{tab_s, tab_c}, poison_arg());
        }
#endif
        LL_MARK(2);
        __syncthreads();
        }
        LL_MARK(3);
        for (int j = wv; j < nb; j += BLK / 64) {
            const long long w = base + j;
            const double *row = FUSE ? ff[j] : theta + w * stride;
            // log-prior (posterior / sampler mode)
            double lpw = FUSE ? 0.0 : (post.lp ? post.lp[w] : 0.0);
            // SAMPLE: the accept test's operands are loaded before the epoch loop, so their latency
            // (sidx -> lp[sidx] is a dependent pair) hides under the loop instead of the wave's tail
            long long sw_s = 0, nacc_s = 0;
            double lp_old_s = 0.0, fac_s = 0.0, lau_s = 0.0;
            if constexpr (FUSE) {   // this wave's proposal (StretchMove.get_proposal + fit.py:3461-3482)
                // Lane-parallel and register-resident: lane c < D holds q_c, lane k < p_full the
                // full row's column k (a ds_bpermute of q), lane k < n_prior its prior term; only
                // the planet constants and the row go through LDS, for the epoch loop.
                const PostDev &pd = sa.pd;
                const int D = pd.n_free;
                const Fetch f = (base == (long long)blockIdx.x * wb && j == wv) ? pre : fetch(w);
                lp_old_s = f.lpo;                         // (needed only in the epilogue)
                // this lane's prior slot (kind, source column, constants) read from LDS into registers
                // up front: the kind's formula then waits on no LDS read of its own
                PriorSlot ps_r{};
                if (RVK_FUSE_SLOTREG && lane < pd.n_prior) {
                    ps_r.kind = fsl[lane].kind;
                    ps_r.src = fsl[lane].src;
#pragma unroll
                    for (int i = 0; i < RVK_PRIOR_NPAR; ++i) ps_r.p[i] = fsl[lane].p[i];
                }
                const double q_s = lane < D ? (DIRECT ? f.a : stretch_q(f.b, f.a, f.z)) : 0.0;
                if (ACCEPT && lane < D) {                 // parked for the epilogue (read back by the same lane)
                    fq[j][lane] = q_s;
                    fx[j][lane] = f.a;
                }
                const int fc = lane < pd.p_full ? fcol[lane] : 0;
                double fv = shfl_d(q_s, fc < 0 ? 0 : fc);
                if (lane < pd.p_full) {
                    if (fc < 0) fv = ftm[lane];
                    ff[j][lane] = fv;
                }
                // column c of the full row, per lane: RVK_FUSE_COMPOSE reads it from q through the
                // composed map (one bpermute level on the chain to the planet constants and the
                // priors instead of q -> row -> operand); same values as reading the row fv
                auto col = [&](int c) -> double {
                    if constexpr (RVK_FUSE_COMPOSE) {
                        const int m = fcol[c];
                        const double v = shfl_d(q_s, m < 0 ? 0 : m);
                        return m < 0 ? ftm[c] : v;
                    } else {
                        return shfl_d(fv, c);
                    }
                };
                const int ioff = 5 * pd.n_planets + pd.n_inst;
                const double jv = col(ioff + (lane < pd.n_inst ? lane : 0));
                bool dead0 = lane < pd.n_inst && jv < 0.0;                                    // fit.py:3465-3468
                double term = 0.0;
                {
                    const int pl = lane < NP ? lane : 0;
                    double p5[5];
#pragma unroll
                    for (int k = 0; k < 5; ++k) p5[k] = col(5 * pl + k);
                    // the prior-side conversion (Case 3, fit.py:3418-3446): lane p < NP converts
                    // planet p; a ValueError rejects the walker; a slot with src < 0 reads it
                    const int src = lane < pd.n_prior ? (RVK_FUSE_SLOTREG ? ps_r.src : fsl[lane].src) : 0;
                    double xv = col(src < 0 ? 0 : src);
                    if constexpr (EXT) {
                        double d5[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
                        if (CONV && lane < NP) dead0 |= !to_default_call(pd.par, p5, d5);
                        if (CONV) {
                            const int di = src < 0 ? -src - 1 : 0, dp = di / 5, dj = di - 5 * dp;
#pragma unroll
                            for (int k = 0; k < 5; ++k) {
                                const double v = shfl_d(d5[k], dp);
                                if (src < 0 && dj == k) xv = v;
                            }
                        }
                        if (lane < pd.n_prior) term = RVK_FUSE_SLOTREG ? prior_lp(ps_r, xv) : prior_lp(fsl[lane], xv);
                    } else {
                        if (lane < pd.n_prior)
                            term = RVK_FUSE_SLOTREG ? prior_lp_basic(ps_r.kind, ps_r.p, xv)
                                                    : prior_lp_basic(fsl[lane].kind, fsl[lane].p, xv);
                    }
                    if (lane < NP) {
                        PlanetK pk;
                        const bool ok = TP ? planet_consts_t<0, RVK_PREP_TAB>(p5, pk, 0, tab) : planet_consts(d.par, p5, pk);
                        pks[j][lane] = pk;
                        okp[j][lane] = ok;
                    }
                }
                bool dead = __builtin_amdgcn_ballot_w64(dead0) != 0;
                double lp = 0.0;
                // the reference's key order; lanes >= n_prior hold +0.0, and lp (from +0.0) is never
                // -0.0, so the padding to a multiple of 8 adds exactly nothing
                for (int k0 = 0; k0 < pd.n_prior; k0 += 8) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) lp += readlane_d(term, k0 + k);
                }
                if (!isfinite(lp)) dead = true;                                                // fit.py:3481-3482
                lpw = dead ? -INFINITY : lp;
                fac_s = f.fac;
                lau_s = f.lau;
                sw_s = f.s;
                nacc_s = f.nacc;
                wave_lds_sync();                          // pks / ff of this walker, for the epoch loop
                LL_MARK(2);
            } else if constexpr (SAMPLE != 0) {
                sw_s = sa.sidx[w];
                // (a global-address-space load: a flat one would also hold lgkmcnt, which the
                // epoch loop's LDS reads wait on)
                lp_old_s = *(const __attribute__((address_space(1))) double *)(sa.run->lp + sw_s);
                fac_s = sa.fac[w];
                lau_s = sa.lau[w];
            }
            bool all_ok = true;
            if constexpr (NP > 0) {
#pragma unroll
                for (int p = 0; p < NP; ++p) all_ok &= okp[j][p] != 0;
            } else {
                for (int p = 0; p < np; ++p) all_ok &= okp[j][p] != 0;
            }
            double res = -INFINITY;
            if (all_ok && lpw != -INFINITY) {
            const double *g = row + 5 * np;
            const double *jit = g + n_inst;
            PlanetK pk[NP > 0 ? NP : 1];
#pragma unroll
            for (int p = 0; p < NP; ++p) pk[p] = NP >= RVK_PK_SGPR ? uniform_pk(pks[j][p]) : pks[j][p];
            const double tot = epoch_sum<NP, MULTI, SOLVER>(d, n_epochs, n_inst, g, jit, pk, pks[j], np, tab, t_1, v_1,
                                                            s_1, i_1, lane);
            LL_MARK(5);
            res = -0.5 * (tot + (double)n_epochs * kLog2Pi);
            if (FUSE || post.lp) res = ((res + lpw) + post.jac) + post.renorm;   // fit.py:3492-3494
            }
            if constexpr (ACCEPT) {   // RedBlueMove: accept if (ndim-1) log z + lp(q) - lp(s) > log u'
                const RunArgs &run = *sa.run;
                const int D = sa.D;
                const long long sw = sw_s;
                const double lp_old = lp_old_s;
                const bool acc = stretch_accept(fac_s, res, lp_old, lau_s);
                double *xs = run.x + sw * D;
                const long long W2 = 2 * sa.hfull;
                double *chain = run.chain ? run.chain + (long long)sa.step * W2 * D : nullptr;
                if (lane == 0 && isnan(res)) atomicOr(run.status, 1);
                if constexpr (FUSE) {             // D <= kFuseMaxD < 64: lane c holds coordinate c
                    if (lane < D) {
                        const double v = acc ? fq[j][lane] : fx[j][lane];
                        if (acc) xs[lane] = v;
                        if (chain) chain[sw * D + lane] = v;
                    }
                } else {
                const double *qw = sa.q + w * D;
                for (int c = lane; c < D; c += 64) {
                    const double v = acc ? qw[c] : xs[c];
                    if (acc) xs[c] = v;
                    if (chain) chain[sw * D + c] = v;
                }
                }
                if (lane == 0) {
                    if (acc) {
                        run.lp[sw] = res;
                        if (run.nacc) run.nacc[sw] = (FUSE ? nacc_s : run.nacc[sw]) + 1;
                    }
                    if (run.lnpc) run.lnpc[(long long)sa.step * W2 + sw] = acc ? res : lp_old;
                }
            } else {
                if (lane == 0) (MODE == 3 ? sa.out : out)[w] = res;
                LL_MARK(6);
            }
        }
        if (base + (long long)gridDim.x * wb < n_walkers) __syncthreads();   // LDS rows are rewritten next pass
    }
    LL_MARK(7);
    if constexpr (FUSE && ACCEPT && !DIRECT) {   // a use of the prefetched word (a no-op if it ever fires)
        asm volatile("" : "+v"(pf_draw));   // the word is consumed here, at the end, not earlier
        if (pf_draw == 0x7fc0dead && lane == 0) atomicOr(sa.run->status, 0);
    }
}

// Segmented variant: LPW lanes per walker, SEG = 64 / LPW walkers per wave (production
// solver, no sampler epilogue).  For few epochs per walker the fixed costs of a wave
// (constants, the per-walker setup, the log and the reduction) are shared by SEG walkers.
// Per-walker values live in VGPRs (they differ between segments); the epoch loop is the
// same, lanes stride their walker's epochs by LPW; each segment is summed with the row
// butterflies and v_readlane of its rows.
template <int NP, bool MULTI, bool TP, int LPW>
__global__ __launch_bounds__(kBlock, (NP >= 3 ? RVK_SEG_LB3 : 4)) void loglike_seg_kernel(EpochData d, int n_epochs, int n_inst,
                                                                 const double *__restrict__ theta,
                                                                 long long n_walkers, long long stride, int wb,
                                                                 double *__restrict__ out, PostArgs post) {
    constexpr int SEG = 64 / LPW;
    constexpr int WB = PassCfg<NP>::WB;
    static_assert(WB % (kWavesPerBlock * SEG) == 0, "pass size must be a multiple of the block's walkers");
    __shared__ PlanetK pks[WB][NP];
    __shared__ int okp[WB][NP];
    __shared__ SC tab[kTabN];
    const int lane = threadIdx.x & 63, seg = lane / LPW, li = lane % LPW;
    double t_1 = 0.0, v_1 = 0.0, s_1 = 1.0;
    int i_1 = 0;
    if (li < n_epochs) {
        t_1 = d.t[li]; v_1 = d.vel[li]; s_1 = d.s2[li];
        if (MULTI) i_1 = d.inst[li];
    }
    for (int i = threadIdx.x; i < kTabN; i += kBlock) tab_put(tab, i, d.tab[i], poison_arg());
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (long long base = (long long)blockIdx.x * wb; base < n_walkers; base += (long long)gridDim.x * wb) {
        const int nb = (int)((n_walkers - base) < wb ? (n_walkers - base) : wb);
        static_assert(WB * NP <= kBlock, "the prep gives each thread at most one (walker, planet)");
        const int k = threadIdx.x;
        const bool has = k < nb * NP;
        const int jp = has ? k / NP : 0, pp = has ? k - jp * NP : 0;
        const double *p5 = theta + (base + jp) * stride + 5 * pp;
        if constexpr (TP && RVK_PREP_TAB && RVK_PREP_GTAB) {
            if (has) {   // sin/cos(w) from the global table (the LDS copy is not yet published)
                PlanetK pk;
                okp[jp][pp] = planet_consts_t<0, true>(p5, pk, 0, d.tab);
                pks[jp][pp] = pk;
            }
        } else if constexpr (TP && RVK_PREP_TAB) {
            // as in loglike_kernel: the row first, then the barrier that publishes the LDS table
            double r5[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
            if (has) {
#pragma unroll
                for (int c = 0; c < 5; ++c) r5[c] = p5[c];
            }
            if (base == (long long)blockIdx.x * wb) __syncthreads();
            if (has) {
                PlanetK pk;
                okp[jp][pp] = planet_consts_t<0, true>(r5, pk, 0, tab);
                pks[jp][pp] = pk;
            }
        } else if (has) {
            PlanetK pk;
            const bool ok = TP ? planet_consts_t<0, RVK_PREP_TAB>(p5, pk, 0, tab) : planet_consts(d.par, p5, pk);
            pks[jp][pp] = pk;
            okp[jp][pp] = ok;
        }
        __syncthreads();
        for (int j0 = wv * SEG; j0 < nb; j0 += kWavesPerBlock * SEG) {
            const bool have = j0 + seg < nb;
            const int j = have ? j0 + seg : j0;                  // this lane's walker slot
            const long long w = base + j;
            const double *row = theta + w * stride;
            const double lpw = post.lp ? post.lp[w] : 0.0;
            bool ok = have && lpw != -INFINITY;
#pragma unroll
            for (int p = 0; p < NP; ++p) ok &= okp[j][p] != 0;
            const double *g = row + 5 * NP;
            const double *jit = g + n_inst;
            const double gd = jit[n_inst], gdd = jit[n_inst + 1];
            const double g0 = g[0], j0sq = jit[0] * jit[0];
            PlanetK pk[NP];
#pragma unroll
            for (int p = 0; p < NP; ++p) pk[p] = pks[j][p];
            // A = 64 / LPW accumulators per lane: accumulator a of lane li holds exactly what lane
            // li + LPW a of the one-wave-per-walker kernel holds (epochs li + LPW a + 64 k, in
            // order), and the segment total is formed from their 16-lane row sums in that
            // kernel's order ((r0 + r1) + (r2 + r3)) -- so a walker's log-likelihood has the same
            // bits whatever the layout, batch size or shard (tests/test_gpu_layout.py).
            constexpr int A = 64 / LPW;
            auto one_acc = [&](int vl, double t_f, double v_f, double s_f, int i_f, auto trend_c) -> double {
                constexpr bool TREND = decltype(trend_c)::value;
                double chi2 = 0.0, prod = 0.5;   // prod * 2^expo = running product of s^2
                int expo = 1;
                double tn = t_f, vn = v_f, sn = s_f;
                int in_ = i_f;
                // off = 8 (i + 64), the next epoch's byte offset (as in loglike_kernel)
                const unsigned lim = 8u * (unsigned)n_epochs;
                for (unsigned off = 8u * (unsigned)(vl + 64); off < lim + 512u; off += 512u) {
                    const double t = tn, vel = vn, s2b = sn;
                    const int ii = in_;
                    if (off < lim) {
                        tn = ld_off(d.t, off); vn = ld_off(d.vel, off); sn = ld_off(d.s2, off);
                        if (MULTI) in_ = ld_off(d.inst, off >> 1);
                    }
                    double gam = g0, jj = j0sq;
                    if (MULTI) {
                        for (int k = 1; k < n_inst; ++k) {
                            if (ii == k) { gam = g[k]; jj = jit[k] * jit[k]; }
                        }
                    }
                    double rv = gam - vel;   // the residual itself (as in loglike_kernel)
#pragma unroll
                    for (int p = 0; p < NP; ++p) rv = planet_rv<0>(pk[p], t, tab, rv);
                    if (TREND) {
                        const double dt = t - d.t0;
                        rv += __builtin_fma(gd, dt, gdd * (dt * dt));
                    }
                    const double s2 = s2b + jj;
                    const double r = rv;
                    chi2 = __builtin_fma(r * r, rcp_nr1(s2), chi2);
                    prod *= s2;
                    int ex;
                    prod = __builtin_frexp(prod, &ex);
                    expo += ex;
                }
                double lsum = log_frexp(prod, expo);
                if (!(prod >= 0.5 && prod < 1.0)) lsum = prod == 0.0 ? -INFINITY : prod;
                return chi2 + lsum;
            };
            // R[r][k]: row r of segment k's one-wave layout (its lanes 16r .. 16r+15), which is
            // accumulator 16r / LPW at segment offset 16r % LPW.  The accumulators run one after
            // another (a runtime loop: one copy of the epoch loop, no extra live state but the
            // uniform row sums).
            constexpr int RPA = LPW / 16;                        // rows per accumulator
            double R[4][SEG];
            const bool trend = __builtin_amdgcn_ballot_w64((gd != 0.0) | (gdd != 0.0)) != 0;
#pragma unroll 1
            for (int a = 0; a < A; ++a) {
                const int vl = li + LPW * a;                     // the one-wave kernel's lane
                double t_f = t_1, v_f = v_1, s_f = s_1;
                int i_f = i_1;
                if (a > 0) {
                    t_f = 0.0; v_f = 0.0; s_f = 1.0; i_f = 0;
                    if (vl < n_epochs) {
                        t_f = d.t[vl]; v_f = d.vel[vl]; s_f = d.s2[vl];
                        if (MULTI) i_f = d.inst[vl];
                    }
                }
                double x = 0.0;
                if (ok) {
                    if (trend) x = one_acc(vl, t_f, v_f, s_f, i_f, std::true_type{});
                    else x = one_acc(vl, t_f, v_f, s_f, i_f, std::false_type{});
                }
                x = row_sum(x);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (r / RPA == a) {
#pragma unroll
                        for (int k = 0; k < SEG; ++k) R[r][k] = readlane_d(x, k * LPW + 16 * (r % RPA));
                    }
                }
            }
            const unsigned long long okm = __builtin_amdgcn_ballot_w64(ok);
            double res[SEG];
#pragma unroll
            for (int k = 0; k < SEG; ++k) {
                const double tot = (R[0][k] + R[1][k]) + (R[2][k] + R[3][k]);
                res[k] = -0.5 * (tot + (double)n_epochs * kLog2Pi);
                if (post.lp) res[k] = ((res[k] + readlane_d(lpw, k * LPW)) + post.jac) + post.renorm;
            }
            if (lane == 0) {
#pragma unroll
                for (int k = 0; k < SEG; ++k) {
                    if (j0 + k >= nb) break;
                    out[base + j0 + k] = ((okm >> (k * LPW)) & 1ull) ? res[k] : -INFINITY;
                }
            }
        }
        if (base + (long long)gridDim.x * wb < n_walkers) __syncthreads();
    }
}

// Posterior predictive (fit.py:2690-2939): one wave per sample, lanes over times.  `sel`: bit p
// = planet p included; NP = the selected count (1..8 specialised, 0 = any count, the planet
// constants in LDS).
template <int NP, int SOLVER>
__global__ __launch_bounds__(kBlock) void predict_kernel(const double *__restrict__ tq, const int32_t *__restrict__ iq,
                                                         long long n_t, int n_planets_total, int n_inst, int par,
                                                         double t0, const double *__restrict__ theta,
                                                         long long n_samples, long long stride, unsigned what,
                                                         unsigned long long sel, const SC *__restrict__ gtab,
                                                         double *__restrict__ out, int poison) {
    __shared__ SC tab[kTabN];
    __shared__ PlanetK pkl[kWavesPerBlock][NP == 0 ? RVK_MAX_PLANETS : NP];
    load_tab(tab, gtab, poison);
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long wave0 = (long long)blockIdx.x * kWavesPerBlock + wv;
    const long long nwaves = (long long)gridDim.x * kWavesPerBlock;
    const int nsel = __builtin_popcountll(sel);
    for (long long s = wave0; s < n_samples; s += nwaves) {
        const double *row = theta + s * stride;
        // lane q < nsel: the q-th selected planet (q-th set bit of `sel`), written straight into
        // LDS by the out-of-line conversion (a PlanetK on the stack would be 64 B/lane of scratch
        // stores per sample -- half the output's bytes again in WRITE_SIZE)
        int okq = 1;
        if (lane < nsel) {
            unsigned long long m = sel;
            for (int k = 0; k < lane; ++k) m &= m - 1ull;
            okq = planet_consts_lds(par, row + 5 * __builtin_ctzll(m), &pkl[wv][lane]);
        }
        const bool ok = __builtin_amdgcn_ballot_w64(!okq) == 0;
        wave_lds_sync();
        PlanetK pk[NP > 0 ? NP : 1];
        if constexpr (NP > 0) {
#pragma unroll
            for (int q = 0; q < NP; ++q) pk[q] = pkl[wv][q];
        }
        const double *g = row + 5 * n_planets_total;
        const double *jit = g + n_inst;
        const double gd = jit[n_inst], gdd = jit[n_inst + 1];
        for (long long j = lane; j < n_t; j += 64) {
            double v = 0.0;
            const double t = tq[j];
            if constexpr (NP > 0) {
#pragma unroll
                for (int p = 0; p < NP; ++p) v = planet_rv<SOLVER>(pk[p], t, tab, v);
            } else {
                for (int p = 0; p < nsel; ++p) v = planet_rv<SOLVER>(pkl[wv][p], t, tab, v);
            }
            if (what & RVK_PRED_TREND) {
                const double dt = t - t0;
                v += __builtin_fma(gd, dt, gdd * (dt * dt));
            }
            if (what & RVK_PRED_GAMMA) v += g[iq ? iq[j] : 0];
            out[s * n_t + j] = ok ? v : NAN;
        }
        wave_lds_sync();   // pkl is rewritten for the wave's next sample
    }
}

template <int SOLVER>
__global__ __launch_bounds__(256) void kepler_kernel(const double *__restrict__ M, const double *__restrict__ e,
                                                     long long n, const SC *__restrict__ gtab,
                                                     double *__restrict__ cosE, double *__restrict__ sinE) {
    __shared__ SC tab[kTabN];
    load_tab(tab, gtab);
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        double c, s;
        const double ee = e[i];
        if (SOLVER == 1) solve_kepler_ref(M[i], ee, c, s);
        else solve_kepler_fast(M[i], ee, 6.0 * ee * ee * ee, tab, c, s);
        cosE[i] = c;
        sinE[i] = s;
    }
}

thread_local std::string g_err;

// Grid: one pass per block when W is small (4 walkers per block = 1 per wave);
// for large W at most kMaxBlocks blocks, each looping over passes of <= WB walkers.
#ifndef RVK_LL_MAXBLOCKS
#define RVK_LL_MAXBLOCKS 2048
#endif
constexpr long long kMaxBlocks = RVK_LL_MAXBLOCKS;

template <int NP>
void ll_grid(long long W, long long &blocks, int &wb, int wpb = kWavesPerBlock) {
    constexpr int WB = PassCfg<NP>::WB;
    blocks = (W + wpb - 1) / wpb;
    wb = wpb;
    if (blocks > kMaxBlocks) {
        long long per = (W + kMaxBlocks - 1) / kMaxBlocks;                 // walkers per block
        per = ((per + wpb - 1) / wpb) * wpb;
        wb = (int)(per < WB ? per : WB);
        blocks = (W + wb - 1) / wb;
        if (blocks > kMaxBlocks) blocks = kMaxBlocks;
    }
}

template <int NP, bool MULTI, bool TP, int LPW>
void launch_seg(hipStream_t st, EpochData d, int n, int ni, const double *th, long long W, long long stride,
                double *out, PostArgs post) {
    constexpr int SEG = 64 / LPW, PER = kWavesPerBlock * SEG, WB = PassCfg<NP>::WB;
    long long blocks = (W + PER - 1) / PER;
    int wb = PER;
    if (blocks > kMaxBlocks) {
        long long per = (W + kMaxBlocks - 1) / kMaxBlocks;
        per = ((per + PER - 1) / PER) * PER;
        wb = (int)(per < WB ? per : WB);
        blocks = (W + wb - 1) / wb;
        if (blocks > kMaxBlocks) blocks = kMaxBlocks;
    }
    hipLaunchKernelGGL((loglike_seg_kernel<NP, MULTI, TP, LPW>), dim3((unsigned)blocks), dim3(kBlock), 0, st, d, n,
                       ni, th, W, stride, wb, out, post);
}

// Lanes per walker for a launch.  Measured on MI355X (tools/kbench.py, KB_LPW): 32 lanes
// win when there are walkers enough for >= 4 waves per SIMD at two walkers per wave
// (W >= 8192: -2 .. -8 % on configs 3 and 4), tie at W = 4096 with one planet and lose
// at W = 4096 with three; 16 lanes lose everywhere.  NP > 3 spills at 32 lanes.
inline int choose_lpw(int forced, int np, int n, long long W) {
    (void)n;
    if (forced) return forced;
    return (np <= 3 && W >= 8192) ? 32 : 64;
}

template <int NP, bool MULTI, int SOLVER, bool TP>
void launch_ll(hipStream_t st, EpochData d, int n, int ni, const double *th, long long W, long long stride,
               double *out, PostArgs post) {
    if constexpr (SOLVER == 0 && NP > 0) {   // (the generic NP = 0 kernel has the one-wave layout only)
        const int lpw = choose_lpw(d.lpw, NP, n, W);
        if (lpw == 32) return launch_seg<NP, MULTI, TP, 32>(st, d, n, ni, th, W, stride, out, post);
        if (lpw == 16) return launch_seg<NP, MULTI, TP, 16>(st, d, n, ni, th, W, stride, out, post);
    }
    long long blocks;
    int wb;
    if (NP == 1 && RVK_LL_BLOCK > kBlock && W >= 256LL * (RVK_LL_BLOCK / 64)) {   // >= one block per CU
        ll_grid<NP>(W, blocks, wb, RVK_LL_BLOCK / 64);
        hipLaunchKernelGGL((loglike_kernel<NP, MULTI, SOLVER, TP, 0, RVK_LL_BLOCK>), dim3((unsigned)blocks),
                           dim3(RVK_LL_BLOCK), 0, st, d, n, ni, th, W, stride, wb, out, post, SampleArgs{});
        return;
    }
    ll_grid<NP>(W, blocks, wb);
    hipLaunchKernelGGL((loglike_kernel<NP, MULTI, SOLVER, TP, 0>), dim3((unsigned)blocks), dim3(kBlock), 0, st, d,
                       n, ni, th, W, stride, wb, out, post, SampleArgs{});
}

// The fused stretch-move half-step over the H walkers of the active half (SOLVER 0 only).
template <int NP, bool MULTI, bool TP>
void launch_sample(hipStream_t st, EpochData d, int n, int ni, const double *rows, long long H, long long stride,
                   PostArgs post, const SampleArgs &sa) {
    long long blocks;
    int wb;
    ll_grid<NP>(H, blocks, wb);
    hipLaunchKernelGGL((loglike_kernel<NP, MULTI, 0, TP, 1>), dim3((unsigned)blocks), dim3(kBlock), 0, st, d, n,
                       ni, rows, H, stride, wb, nullptr, post, sa);
}

// The same with the proposals made in the kernel's prep (SAMPLE == 2; rows unused), or only the
// proposals' log-posteriors (SAMPLE == 3, rvk_stretch_propose).
template <int NP, bool MULTI, bool TP, int SAMPLE>
void launch_sample_fused(hipStream_t st, EpochData d, int n, int ni, const double *rows, long long H, long long stride,
                         PostArgs post, const SampleArgs &sa) {
    // one walker per wave per pass (the kernel's fused LDS rows are per wave); grid-stride beyond
    constexpr int wb = RVK_SAMPLE_BLOCK / 64;
    long long blocks = (H + wb - 1) / wb;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL((loglike_kernel<NP, MULTI, 0, TP, SAMPLE, RVK_SAMPLE_BLOCK>), dim3((unsigned)blocks),
                       dim3(RVK_SAMPLE_BLOCK), 0, st, d, n, ni, rows, H, stride, wb, nullptr, post, sa);
}

template <bool MULTI, int SOLVER, bool TP>
loglike_launch_t pick_ll_s(int np) {
    switch (np) {
        case 1: return launch_ll<1, MULTI, SOLVER, TP>;
        case 2: return launch_ll<2, MULTI, SOLVER, TP>;
        case 3: return launch_ll<3, MULTI, SOLVER, TP>;
        case 4: return launch_ll<4, MULTI, SOLVER, TP>;
        case 5: return launch_ll<5, MULTI, SOLVER, TP>;
        case 6: return launch_ll<6, MULTI, SOLVER, TP>;
        case 7: return launch_ll<7, MULTI, SOLVER, TP>;
        case 8: return launch_ll<8, MULTI, SOLVER, TP>;
        default: return np <= RVK_MAX_PLANETS ? launch_ll<0, MULTI, SOLVER, TP> : nullptr;
    }
}

template <int SOLVER, bool TP>
loglike_launch_t pick_ll_t(int np, bool multi) {
    return multi ? pick_ll_s<true, SOLVER, TP>(np) : pick_ll_s<false, SOLVER, TP>(np);
}

#if !RVK_TU_SAMPLE   // (this would instantiate every likelihood kernel in rvk_sample.hip's build too)
loglike_launch_t pick_ll(int np, bool multi, int solver, bool tp) {
    if (solver == 1) return tp ? pick_ll_t<1, true>(np, multi) : pick_ll_t<1, false>(np, multi);
    return tp ? pick_ll_t<0, true>(np, multi) : pick_ll_t<0, false>(np, multi);
}
#endif

// MODE 1: propose_kernel + the likelihood with the accept / reject; 2: one fused half-step;
// 3: fused proposals, log-posterior out (the fused modes: NP <= 4); | 4: every prior kind;
// | 8: and the prior-side conversion in the fused prep.
template <bool MULTI, bool TP, int MODE>
sample_launch_t pick_sample_s(int np) {
    if constexpr (MODE == 1) {
        switch (np) {
            case 1: return launch_sample<1, MULTI, TP>;
            case 2: return launch_sample<2, MULTI, TP>;
            case 3: return launch_sample<3, MULTI, TP>;
            case 4: return launch_sample<4, MULTI, TP>;
            case 5: return launch_sample<5, MULTI, TP>;
            case 6: return launch_sample<6, MULTI, TP>;
            case 7: return launch_sample<7, MULTI, TP>;
            case 8: return launch_sample<8, MULTI, TP>;
            default: return np <= RVK_MAX_PLANETS ? launch_sample<0, MULTI, TP> : nullptr;
        }
    } else {
        // one planet with the basic priors (MODE 2 / 3) is rvk_sample1.hip's (RVK_TU_SAMPLE 2), the
        // other shapes rvk_sample.hip's (RVK_TU_SAMPLE 1): each build instantiates only its own
        constexpr bool NP1 = MODE == 2 || MODE == 3;
        if constexpr (RVK_TU_SAMPLE == 2) {
            return np == 1 && NP1 ? launch_sample_fused<1, MULTI, TP, MODE> : nullptr;
        } else {
            switch (np) {
                case 1:
                    if constexpr (NP1 && RVK_TU_SAMPLE == 1) return nullptr;
                    else return launch_sample_fused<1, MULTI, TP, MODE>;
                case 2: return launch_sample_fused<2, MULTI, TP, MODE>;
                case 3: return launch_sample_fused<3, MULTI, TP, MODE>;
                case 4: return launch_sample_fused<4, MULTI, TP, MODE>;
                default: return nullptr;
            }
        }
    }
}

template <int MODE>
sample_launch_t pick_sample(int np, bool multi, bool tp) {
    if (multi) return tp ? pick_sample_s<true, true, MODE>(np) : pick_sample_s<true, false, MODE>(np);
    return tp ? pick_sample_s<false, true, MODE>(np) : pick_sample_s<false, false, MODE>(np);
}

#if RVK_TU_SAMPLE
}  // namespace

// rvk_sample.hip and rvk_sample1.hip compile this file again with RVK_TU_SAMPLE 1 / 2: only the
// kernels that make their own stretch-move proposals (MODE 2 / 3, | 4, | 8), under other machine
// schedulers (Makefile).  Measured (sessions r5flags / r5tu / r5st, tools/sampler_variants.py, 3
// interleaved reps): iterative-ILP makes the half-steps 1.6 % (uniform priors) to 7 % (VanEylen)
// faster, max-ILP the one-planet basic-prior half-step (the config-2 sampler) 2.7 % faster again but
// the others ~1 % slower; the plain likelihood kernels lose 1-3.5 % under either (tools/kbench.py),
// so they keep the default scheduler in rvk.hip.
#if RVK_TU_SAMPLE == 2
#if RVK_LL_TRACE
// the phase stamps of THIS build's kernels (each translation unit has its own g_ll_trace)
extern "C" int rvk_ll_trace_dump_s1(unsigned long long *host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ll_trace), sizeof(g_ll_trace)) == hipSuccess ? 0 : -1;
}
#endif
rvk::sample_launch_t rvk::pick_sample_fused_np1(int mode, bool multi, bool tp) {
    switch (mode) {
        case 2: return pick_sample<2>(1, multi, tp);
        case 3: return pick_sample<3>(1, multi, tp);
        default: return nullptr;
    }
}
#else
rvk::sample_launch_t rvk::pick_sample_fused(int mode, int np, bool multi, bool tp) {
    switch (mode) {
        case 2: return pick_sample<2>(np, multi, tp);
        case 3: return pick_sample<3>(np, multi, tp);
        case 6: return pick_sample<6>(np, multi, tp);
        case 7: return pick_sample<7>(np, multi, tp);
        case 14: return pick_sample<14>(np, multi, tp);
        case 15: return pick_sample<15>(np, multi, tp);
        default: return nullptr;
    }
}
#endif
#else

int check_gfx950(int dev) {
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, dev));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(RVK_E_NODEV, std::string("device is ") + prop.gcnArchName + ", librvk is built for gfx950 only");
    return RVK_OK;
}

std::vector<SC> host_table() {
    std::vector<SC> t(kTabN);
    for (int j = -kTabHalf; j <= kTabHalf; ++j) {
        const double a = (double)j * kTabH;   // identical rounding to the device's jj * kTabH
        t[j + kTabHalf] = SC{std::sin(a), std::cos(a)};
    }
    return t;
}

int upload_table(SC **d_tab) {
    std::vector<SC> t = host_table();
    HIPCHK(hipMalloc(d_tab, sizeof(SC) * kTabN));
    HIPCHK(hipMemcpy(*d_tab, t.data(), sizeof(SC) * kTabN, hipMemcpyHostToDevice));
    return RVK_OK;
}

dim3 wave_grid(long long items) {
    long long blocks = (items + kWavesPerBlock - 1) / kWavesPerBlock;
    if (blocks > (1LL << 20)) blocks = 1LL << 20;
    if (blocks < 1) blocks = 1;
    return dim3((unsigned)blocks);
}

}  // namespace

int rvk::fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

int rvk::grow_dev(void **p, size_t *cap, size_t need) {
    if (need <= *cap && *p) return RVK_OK;
    if (*p) HIPCHK(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    HIPCHK(hipMalloc(p, need > 0 ? need : 1));
    *cap = need;
    return RVK_OK;
}

// ---- host-buffer transport (rvk_internal.h HostIO, RVK_OPT_HOSTIO) ------------------------
void rvk::HostIO::release() {
    if (h) (void)hipHostFree(h);
    (void)hipFree(d);
    h = hd = d = nullptr;
    hcap = dcap = 0;
}

static size_t io_align(size_t b) { return (b + 255) & ~size_t(255); }

int rvk::HostIO::begin(int opt, hipStream_t st, int n_in, const void *const *src, const size_t *bytes,
                       size_t out_bytes, const void **dev_in, void **dev_out) {
    size_t total_in = 0, off[kHostIoMaxIn];
    for (int i = 0; i < n_in; ++i) {
        off[i] = total_in;
        total_in += io_align(bytes[i]);
    }
    off_out = total_in;
    const size_t total = total_in + io_align(out_bytes);
    mode = opt == RVK_HOSTIO_AUTO ? (total_in <= kZeroCopyMaxBytes ? RVK_HOSTIO_ZEROCOPY : RVK_HOSTIO_PINNED) : opt;
    if (mode != RVK_HOSTIO_ZEROCOPY) {
        int rc = grow_dev((void **)&d, &dcap, total);
        if (rc) return rc;
    }
    if (mode == RVK_HOSTIO_PAGEABLE) {
        for (int i = 0; i < n_in; ++i) {
            HIPCHK_SYNC(st, hipMemcpyAsync(d + off[i], src[i], bytes[i], hipMemcpyHostToDevice, st));
            dev_in[i] = d + off[i];
        }
        *dev_out = d + off_out;
        return RVK_OK;
    }
    if (total > hcap) {
        if (h) HIPCHK(hipHostFree(h));
        h = hd = nullptr;
        hcap = 0;
        // fine-grained (coherent) pinned memory: the kernels may read and write it in place
        HIPCHK(hipHostMalloc((void **)&h, total, hipHostMallocCoherent | hipHostMallocMapped));
        hcap = total;
        void *dp = nullptr;
        HIPCHK(hipHostGetDevicePointer(&dp, h, 0));
        hd = (char *)dp;
    }
    for (int i = 0; i < n_in; ++i) std::memcpy(h + off[i], src[i], bytes[i]);
    if (mode == RVK_HOSTIO_ZEROCOPY) {
        for (int i = 0; i < n_in; ++i) dev_in[i] = hd + off[i];
        *dev_out = hd + off_out;
        return RVK_OK;
    }
    if (total_in) HIPCHK_SYNC(st, hipMemcpyAsync(d, h, total_in, hipMemcpyHostToDevice, st));   // one DMA
    for (int i = 0; i < n_in; ++i) dev_in[i] = d + off[i];
    *dev_out = d + off_out;
    return RVK_OK;
}

int rvk::HostIO::end(hipStream_t st, void *out, size_t out_bytes) {
    if (mode == RVK_HOSTIO_PAGEABLE) {
        HIPCHK_SYNC(st, hipMemcpyAsync(out, d + off_out, out_bytes, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        return RVK_OK;
    }
    if (mode == RVK_HOSTIO_PINNED)
        HIPCHK_SYNC(st, hipMemcpyAsync(h + off_out, d + off_out, out_bytes, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    std::memcpy(out, h + off_out, out_bytes);
    return RVK_OK;
}

int rvk::shared_table(int device, const SC **tab) {
    static std::mutex mu;
    static SC *tabs[64] = {};
    if (device < 0 || device >= 64) return fail(RVK_E_ARG, "device ordinal out of range");
    std::lock_guard<std::mutex> lk(mu);
    if (!tabs[device]) {
        SC *t = nullptr;
        int rc = upload_table(&t);
        if (rc) {
            (void)hipFree(t);
            return rc;
        }
        tabs[device] = t;
    }
    *tab = tabs[device];
    return RVK_OK;
}


extern "C" {

#if RVK_LL_TRACE
int rvk_ll_trace_dump(unsigned long long *host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ll_trace), sizeof(g_ll_trace)) == hipSuccess ? 0 : -1;
}
#endif

int rvk_version(void) { return 103; }

const char *rvk_last_error(void) { return g_err.c_str(); }

int rvk_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

static int grow(double **p, size_t *cap, size_t need) { return grow_dev((void **)p, cap, need); }

static void free_handle(rvk_handle *h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    (void)hipFree(h->d_t);       // one block: t | vel | s2 | inst (rvk_create)
    (void)hipFree(h->d_tab);
    (void)hipFree(h->d_theta);
    (void)hipFree(h->d_out);
    (void)hipFree(h->d_tq);
    (void)hipFree(h->d_iq);
    h->io.release();
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

static int create_impl(rvk_handle *h, const double *time, const double *vel, const double *velerr,
                       const int32_t *inst_idx, int32_t n, int32_t n_inst, int32_t n_planets, int32_t par,
                       double t0, int32_t device) {
    if (n < 0 || (n > 0 && (!time || !vel || !velerr)))
        return fail(RVK_E_ARG, "n_epochs must be >= 0 with non-NULL data (0 = model-only handle for rvk_predict)");
    if (n_planets < 1 || n_planets > RVK_MAX_PLANETS) return fail(RVK_E_ARG, "n_planets must be in [1, 32]");
    if (n_inst < 1 || n_inst > RVK_MAX_INST) return fail(RVK_E_ARG, "n_inst must be in [1, 64]");
    if (par < 0 || par > 3) return fail(RVK_E_ARG, "unknown parameterisation code");
    if (n > 0 && n_inst > 1 && !inst_idx) return fail(RVK_E_ARG, "inst_idx is required when n_inst > 1");
    std::vector<int32_t> inst((size_t)n, 0);
    if (inst_idx && n > 0)
        for (int i = 0; i < n; ++i) {
            if (inst_idx[i] < 0 || inst_idx[i] >= n_inst) return fail(RVK_E_ARG, "inst_idx out of range");
            inst[i] = inst_idx[i];
        }
    int ndev = rvk_device_count();
    if (ndev < 1) return fail(RVK_E_NODEV, "no HIP device visible");
    if (device < 0) HIPCHK(hipGetDevice(&device));
    if (device >= ndev) return fail(RVK_E_ARG, "device ordinal out of range");
    int rc = check_gfx950(device);
    if (rc) return rc;
    h->device = device;
    h->n = n;
    h->n_inst = n_inst;
    h->n_planets = n_planets;
    h->par = par;
    h->t0 = t0;
    h->launch = pick_ll(n_planets, n_inst > 1, 0, RVK_TP_INLINE && par == RVK_PAR_PKEWTP);
    h->sample = pick_sample<1>(n_planets, n_inst > 1, RVK_TP_INLINE && par == RVK_PAR_PKEWTP);
    // (the proposal-making modes live in rvk_sample.hip's and rvk_sample1.hip's builds of this file)
    const bool multi = n_inst > 1, tpi = RVK_TP_INLINE && par == RVK_PAR_PKEWTP;
    auto fused = [&](int mode) {
        return n_planets == 1 && (mode == 2 || mode == 3) ? pick_sample_fused_np1(mode, multi, tpi)
                                                          : pick_sample_fused(mode, n_planets, multi, tpi);
    };
    h->sample_fused[0] = fused(2);
    h->sample_eval[0] = fused(3);
    h->sample_fused[1] = fused(6);
    h->sample_eval[1] = fused(7);
    h->sample_fused[2] = fused(14);
    h->sample_eval[2] = fused(15);
    h->sample_direct[0] = pick_sample<19>(n_planets, n_inst > 1, RVK_TP_INLINE && par == RVK_PAR_PKEWTP);
    h->sample_direct[1] = pick_sample<23>(n_planets, n_inst > 1, RVK_TP_INLINE && par == RVK_PAR_PKEWTP);
    h->sample_direct[2] = pick_sample<31>(n_planets, n_inst > 1, RVK_TP_INLINE && par == RVK_PAR_PKEWTP);
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    if ((rc = upload_table(&h->d_tab))) return rc;
    if (n == 0) return RVK_OK;                                      // model-only handle
    // The epoch arrays carry kEpochPad entries of padding (finite values no result reads), so the
    // likelihood kernel's prefetch of epoch i + 64 is in bounds for every lane without a per-lane
    // guard (epoch_sum, RVK_EPOCH_UNI).
    const size_t np_ = (size_t)n + kEpochPad;
    std::vector<double> s2(np_, 1.0), tp(np_, time[n - 1]), vp(np_, 0.0);
    std::vector<int32_t> ip(np_, 0);
    h->s2ok = 1;
    for (int i = 0; i < n; ++i) {
        s2[i] = velerr[i] * velerr[i];                              // velerr ** 2 (fit.py:3598)
        if (!(s2[i] >= 0x1p-500 && s2[i] <= 0x1p500)) h->s2ok = 0;
        tp[i] = time[i];
        vp[i] = vel[i];
        ip[i] = inst[i];
    }
    // One allocation, t | vel | s2 | inst (each padded): the likelihood kernel addresses all four
    // through one buffer descriptor based at t (epoch_sum, RVK_EPOCH_UNI).
    const size_t bd = sizeof(double) * np_;
    char *blk = nullptr;
    HIPCHK(hipMalloc(&blk, 3 * bd + sizeof(int32_t) * np_));
    h->d_t = reinterpret_cast<double *>(blk);
    h->d_vel = reinterpret_cast<double *>(blk + bd);
    h->d_s2 = reinterpret_cast<double *>(blk + 2 * bd);
    h->d_inst = reinterpret_cast<int32_t *>(blk + 3 * bd);
    HIPCHK(hipMemcpy(h->d_t, tp.data(), bd, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->d_vel, vp.data(), bd, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->d_s2, s2.data(), bd, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->d_inst, ip.data(), sizeof(int32_t) * np_, hipMemcpyHostToDevice));
    return RVK_OK;
}

rvk_handle *rvk_create(const double *time, const double *vel, const double *velerr, const int32_t *inst_idx,
                       int32_t n_epochs, int32_t n_inst, int32_t n_planets, int32_t parameterisation, double t0,
                       int32_t device) {
    rvk_handle *h = new (std::nothrow) rvk_handle();
    if (!h) {
        fail(RVK_E_NOMEM, "out of host memory");
        return nullptr;
    }
    if (create_impl(h, time, vel, velerr, inst_idx, n_epochs, n_inst, n_planets, parameterisation, t0, device)) {
        free_handle(h);
        return nullptr;
    }
    return h;
}

void rvk_destroy(rvk_handle *h) { free_handle(h); }

void *rvk_stream(rvk_handle *h) { return h ? (void *)h->stream : nullptr; }

int rvk_set_option(rvk_handle *h, int32_t key, int32_t value) {
    if (!h) return fail(RVK_E_ARG, "NULL handle");
    if (key == RVK_OPT_SOLVER) {
        if (value != 0 && value != 1) return fail(RVK_E_ARG, "solver must be 0 (fast) or 1 (reference Halley)");
        h->solver = value;
        h->launch = pick_ll(h->n_planets, h->n_inst > 1, value, RVK_TP_INLINE && h->par == RVK_PAR_PKEWTP);
        return RVK_OK;
    }
    if (key == RVK_OPT_LPW) {
        if (value != 0 && value != 16 && value != 32 && value != 64) return fail(RVK_E_ARG, "lpw must be 0, 16, 32 or 64");
        h->lpw = value;
        return RVK_OK;
    }
    if (key == RVK_OPT_GRAPH) {
        if (value != 0 && value != 1) return fail(RVK_E_ARG, "graph must be 0 or 1");
        h->graph = value;
        return RVK_OK;
    }
    if (key == RVK_OPT_HOSTIO) {
        if (value < RVK_HOSTIO_AUTO || value > RVK_HOSTIO_ZEROCOPY) return fail(RVK_E_ARG, "unknown RVK_HOSTIO mode");
        h->hostio = value;
        return RVK_OK;
    }
    if (key == RVK_OPT_LDS_POISON) {
        if (value < 0 || value > 2) return fail(RVK_E_ARG, "lds poison must be 0, 1 or 2");
        h->poison = value;
        return RVK_OK;
    }
    return fail(RVK_E_ARG, "unknown option key");
}

int rvk_sync(rvk_handle *h) {
    if (!h) return fail(RVK_E_ARG, "NULL handle");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipStreamSynchronize(h->stream));
    return RVK_OK;
}

static int check_rows(rvk_handle *h, int64_t W, int64_t stride) {
    if (!h) return fail(RVK_E_ARG, "NULL handle");
    if (W < 0) return fail(RVK_E_ARG, "negative row count");
    long long pfull = 5LL * h->n_planets + 2LL * h->n_inst + 2;
    if (stride < pfull) return fail(RVK_E_ARG, "row_stride < P_full = 5*n_planets + 2*n_inst + 2");
    return RVK_OK;
}

int rvk_reserve(rvk_handle *h, int64_t max_walkers) {
    // The launch path allocates nothing (no workspace since the conversion moved into the
    // kernel's prep phase); kept so callers can size for graph capture unconditionally.
    if (!h || max_walkers < 0) return fail(RVK_E_ARG, "bad arguments");
    return RVK_OK;
}

int rvk_loglike_device(rvk_handle *h, const double *d_theta, int64_t W, int64_t stride, double *d_out,
                       void *stream) {
    int rc = check_rows(h, W, stride);
    if (rc) return rc;
    if (h->n < 1) return fail(RVK_E_ARG, "model-only handle (n_epochs = 0) has no data to evaluate");
    if (W == 0) return RVK_OK;
    if (!d_theta || !d_out) return fail(RVK_E_ARG, "NULL device buffer");
    hipStream_t st = (hipStream_t)stream;   // used as given: NULL is HIP's default stream
    HIPCHK(hipSetDevice(h->device));
    h->launch(st, h->epochs(), h->n, h->n_inst, d_theta, W, stride, d_out, PostArgs{nullptr, 0.0, 0.0});
    HIPCHK(hipGetLastError());
    return RVK_OK;
}

int rvk_loglike(rvk_handle *h, const double *theta, int64_t W, int64_t stride, double *out) {
    int rc = check_rows(h, W, stride);
    if (rc) return rc;
    if (W == 0) return RVK_OK;
    if (!theta || !out) return fail(RVK_E_ARG, "NULL host buffer");
    if (h->n < 1) return fail(RVK_E_ARG, "model-only handle (n_epochs = 0) has no data to evaluate");
    std::lock_guard<std::mutex> lock(h->mu);   // one blocking call per handle at a time (rvk.h, threading)
    HIPCHK(hipSetDevice(h->device));
    const void *src = theta, *d_theta = nullptr;
    void *d_out = nullptr;
    const size_t bt = sizeof(double) * (size_t)W * (size_t)stride, bo = sizeof(double) * (size_t)W;
    if ((rc = h->io.begin(h->hostio, h->stream, 1, &src, &bt, bo, &d_theta, &d_out))) return rc;
    if ((rc = rvk_loglike_device(h, (const double *)d_theta, W, stride, (double *)d_out, h->stream))) {
        (void)hipStreamSynchronize(h->stream);
        return rc;
    }
    return h->io.end(h->stream, out, bo);
}

int rvk_predict_device(rvk_handle *h, const double *d_theta, int64_t S, int64_t stride, const double *d_t,
                       const int32_t *d_inst, int64_t n_t, uint32_t what, double *d_out, void *stream) {
    int rc = check_rows(h, S, stride);
    if (rc) return rc;
    if (S == 0 || n_t == 0) return RVK_OK;
    if (!d_theta || !d_t || !d_out) return fail(RVK_E_ARG, "NULL device buffer");
    if ((what & RVK_PRED_GAMMA) && h->n_inst > 1 && !d_inst) return fail(RVK_E_ARG, "inst required for GAMMA");
    // planet selection: bits 0-7, every planet, or one planet by index (include/rvk.h)
    const unsigned long long all = (1ull << h->n_planets) - 1ull;
    unsigned long long sel = (unsigned long long)(what & RVK_PRED_PLANETS);
    if (what & RVK_PRED_ALL_PLANETS) sel = all;
    if (what & 0x0800u) {
        const unsigned p = (what >> 16) & 0xFFu;
        if ((int)p >= h->n_planets) return fail(RVK_E_ARG, "RVK_PRED_PLANET index out of range");
        sel |= 1ull << p;
    }
    sel &= all;
    const int nsel = __builtin_popcountll(sel);
    hipStream_t st = (hipStream_t)stream;
    HIPCHK(hipSetDevice(h->device));
    dim3 grid = wave_grid(S);
#define PRED_LAUNCH(K)                                                                                          \
    do {                                                                                                        \
        if (h->solver == 1)                                                                                     \
            hipLaunchKernelGGL((predict_kernel<K, 1>), grid, dim3(kBlock), 0, st, d_t, d_inst, (long long)n_t,   \
                               h->n_planets, h->n_inst, h->par, h->t0, d_theta, (long long)S, (long long)stride, \
                               what, sel, h->d_tab, d_out, h->poison);                                          \
        else                                                                                                    \
            hipLaunchKernelGGL((predict_kernel<K, 0>), grid, dim3(kBlock), 0, st, d_t, d_inst, (long long)n_t,   \
                               h->n_planets, h->n_inst, h->par, h->t0, d_theta, (long long)S, (long long)stride, \
                               what, sel, h->d_tab, d_out, h->poison);                                          \
    } while (0)
    switch (nsel) {
        case 1: PRED_LAUNCH(1); break;
        case 2: PRED_LAUNCH(2); break;
        case 3: PRED_LAUNCH(3); break;
        case 4: PRED_LAUNCH(4); break;
        case 5: PRED_LAUNCH(5); break;
        case 6: PRED_LAUNCH(6); break;
        case 7: PRED_LAUNCH(7); break;
        case 8: PRED_LAUNCH(8); break;
        default: PRED_LAUNCH(0); break;   // none selected (trend / gamma only), or more than 8
    }
#undef PRED_LAUNCH
    HIPCHK(hipGetLastError());
    return RVK_OK;
}

int rvk_predict(rvk_handle *h, const double *theta, int64_t S, int64_t stride, const double *t,
                const int32_t *inst, int64_t n_t, uint32_t what, double *out) {
    int rc = check_rows(h, S, stride);
    if (rc) return rc;
    if (S == 0 || n_t == 0) return RVK_OK;
    if (!theta || !t || !out) return fail(RVK_E_ARG, "NULL host buffer");
    if ((what & RVK_PRED_GAMMA) && h->n_inst > 1 && !inst) return fail(RVK_E_ARG, "inst required for GAMMA");
    std::lock_guard<std::mutex> lock(h->mu);   // one blocking call per handle at a time (rvk.h, threading)
    HIPCHK(hipSetDevice(h->device));
    // samples in chunks so the device output block stays <= 2^25 doubles (256 MB); the device
    // buffers are the handle's (grown on demand, kept across calls, freed by rvk_destroy)
    long long chunk = (1LL << 25) / n_t;
    if (chunk < 1) chunk = 1;
    if (chunk > S) chunk = S;
    if ((rc = grow(&h->d_theta, &h->cap_theta, sizeof(double) * (size_t)chunk * (size_t)stride)) ||
        (rc = grow(&h->d_out, &h->cap_out, sizeof(double) * (size_t)chunk * (size_t)n_t)) ||
        (rc = grow(&h->d_tq, &h->cap_tq, sizeof(double) * (size_t)n_t)) ||
        (inst && (rc = grow_dev((void **)&h->d_iq, &h->cap_iq, sizeof(int32_t) * (size_t)n_t))))
        return rc;
    if (inst)
        HIPCHK_SYNC(h->stream, hipMemcpyAsync(h->d_iq, inst, sizeof(int32_t) * n_t, hipMemcpyHostToDevice, h->stream));
    HIPCHK_SYNC(h->stream, hipMemcpyAsync(h->d_tq, t, sizeof(double) * n_t, hipMemcpyHostToDevice, h->stream));
    for (long long s0 = 0; s0 < S; s0 += chunk) {
        const long long ns = (S - s0) < chunk ? (S - s0) : chunk;
        HIPCHK_SYNC(h->stream, hipMemcpyAsync(h->d_theta, theta + s0 * stride, sizeof(double) * ns * stride,
                                              hipMemcpyHostToDevice, h->stream));
        if ((rc = rvk_predict_device(h, h->d_theta, ns, stride, h->d_tq, inst ? h->d_iq : nullptr, n_t, what,
                                     h->d_out, h->stream))) {
            (void)hipStreamSynchronize(h->stream);
            return rc;
        }
        HIPCHK_SYNC(h->stream, hipMemcpyAsync(out + s0 * n_t, h->d_out, sizeof(double) * ns * n_t,
                                              hipMemcpyDeviceToHost, h->stream));
    }
    HIPCHK(hipStreamSynchronize(h->stream));
    return RVK_OK;
}

}  // extern "C"

namespace {
// Owns a device allocation for the length of one call (freed on every return path).
struct DevBuf {
    void *p = nullptr;
    ~DevBuf() { (void)hipFree(p); }
    template <class T> T *as() const { return static_cast<T *>(p); }
};
struct OwnedStream {
    hipStream_t s = nullptr;
    ~OwnedStream() {
        if (s) {
            (void)hipStreamSynchronize(s);
            (void)hipStreamDestroy(s);
        }
    }
};
}  // namespace

extern "C" {

int rvk_solve_kepler(const double *M, const double *e, int64_t n, double *cosE, double *sinE, int32_t device,
                     int32_t solver) {
    if (n < 0 || (n > 0 && (!M || !e || !cosE || !sinE))) return fail(RVK_E_ARG, "bad arguments");
    if (n == 0) return RVK_OK;
    if (rvk_device_count() < 1) return fail(RVK_E_NODEV, "no HIP device visible");
    if (device < 0) HIPCHK(hipGetDevice(&device));
    int rc = check_gfx950(device);
    if (rc) return rc;
    HIPCHK(hipSetDevice(device));
    const SC *dtab = nullptr;
    if ((rc = shared_table(device, &dtab))) return rc;
    // RAII: every buffer and the call's own stream are released on every return path (the
    // stream is drained first, so no copy into the caller's arrays is left in flight)
    DevBuf dM, de, dc, ds;
    OwnedStream st;
    const size_t b = sizeof(double) * (size_t)n;
    HIPCHK(hipMalloc(&dM.p, b));
    HIPCHK(hipMalloc(&de.p, b));
    HIPCHK(hipMalloc(&dc.p, b));
    HIPCHK(hipMalloc(&ds.p, b));
    HIPCHK(hipStreamCreateWithFlags(&st.s, hipStreamNonBlocking));
    HIPCHK(hipMemcpyAsync(dM.p, M, b, hipMemcpyHostToDevice, st.s));
    HIPCHK(hipMemcpyAsync(de.p, e, b, hipMemcpyHostToDevice, st.s));
    const dim3 grid((unsigned)((n + 255) / 256));
    if (solver == 1)
        hipLaunchKernelGGL(kepler_kernel<1>, grid, dim3(256), 0, st.s, dM.as<double>(), de.as<double>(), (long long)n,
                           dtab, dc.as<double>(), ds.as<double>());
    else
        hipLaunchKernelGGL(kepler_kernel<0>, grid, dim3(256), 0, st.s, dM.as<double>(), de.as<double>(), (long long)n,
                           dtab, dc.as<double>(), ds.as<double>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(cosE, dc.p, b, hipMemcpyDeviceToHost, st.s));
    HIPCHK(hipMemcpyAsync(sinE, ds.p, b, hipMemcpyDeviceToHost, st.s));
    HIPCHK(hipStreamSynchronize(st.s));
    return RVK_OK;
}

}  // extern "C"
#endif  // RVK_TU_SAMPLE
