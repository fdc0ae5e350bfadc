// rvk_math.h -- fp64 device math for the Kepler/RV hot path on gfx950.
//
// Everything here is wave64 VALU code: no LDS, no MFMA (the path has no dense
// contraction).  Two Kepler solvers, both for E - e sin E = M:
//
//  * solve_kepler_ref  -- ravest's _solve_kepler (src/ravest/model.py:23-70)
//    restated: Halley seeded at E0 = M, stop at |E_new - E| < 1.48e-8, at most
//    50 iterations, result sin/cos(E_new), in a 2*pi-reduced frame.  Halley is
//    2*pi-equivariant, so iterates and iteration counts are the reference's
//    shifted by 2*pi*k; only rounding at the |M|*eps level differs (the
//    reference carries that rounding in E itself).  Selected with
//    RVK_OPT_SOLVER = 1.
//
//  * solve_kepler_fast -- the production solver (default).  It converges to
//    the same root to ~1 ulp, so cos E / sin E match the reference's converged
//    values within the stated fp64 tolerance:
//      1. r = M reduced to [-pi, pi] (Cody-Waite, FMA); planet_rv instead reduces the
//         phase u = (t - Tp) / P exactly, r = 2 pi (u - rint u);
//      2. e <= 0.18: the e^4 Lagrange series (seed_series), else
//         fp32 Halley seed from E0 = r with the hardware v_sin_f32/v_cos_f32
//         (accurate fp32 polynomials when e > 0.95, wave-uniform branch),
//         started from the series E0 = r + e sin r (1 + e cos r); per-lane exit
//         once an update is < 1e-2 (Halley is cubic: the error after it is
//         ~K d^3, ~1e-6); at most 8 iterations.  The large early steps cost
//         fp32 issue slots, not fp64 ones;
//      3. sin/cos of the fp32 root in fp64 from an LDS table of sin/cos at
//         j*pi/32 plus a degree-7/8 Taylor rotation (|d| <= pi/64);
//      4. Householder order-3 steps (quartic convergence) with sin/cos carried
//         by short-series rotation, until the local error bound
//         (e/f')^3 d^4 < 1e-17: one step whenever the seed is within 1e-5 and
//         e <= 0.9, which is the common case.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rvk {

constexpr double kPi      = 3.141592653589793;        // == np.pi
constexpr double kTwoPi   = 6.283185307179586;        // == 2*np.pi (exact doubling)
constexpr double kInv2Pi  = 0.15915494309189535;
constexpr double k2PiHi   = 6.283185307179586232e+00; // 0x401921FB54442D18
constexpr double k2PiMi   = 2.449293598294706414e-16; // 0x3CB1A62633145C07
constexpr double k2PiLo   = -5.989539619436679332e-33;
constexpr double k2OverPi = 0.6366197723675814;
constexpr double kPio2Hi  = 1.5707963267948966e+00;   // 0x3FF921FB54442D18
constexpr double kPio2Mi  = 6.123233995736766e-17;    // 0x3C91A62633145C07
constexpr double kPio2Lo  = -1.4973849048591698e-33;
constexpr double kLn2     = 0.6931471805599453;
constexpr double kLog2Pi  = 1.8378770664093453;       // == np.log(2*np.pi)

// Reduce x by 2*pi: r = x - k*2*pi, |r| <= pi (+ulp), abs error ~1e-15 for |x| < 2^50.
// Beyond 2^50 rad (ulp(M) > 2^-3: no phase information left; e.g. P = 1 d with
// |t - Tp| > 1.8e14 d) the result is defined as 0: finite, unspecified physically
// (the reference returns equally meaningless finite values there).
__device__ __forceinline__ double reduce_2pi(double x) {
    x = (__builtin_fabs(x) >= 0x1p50 && __builtin_fabs(x) < __builtin_inf()) ? 0.0 : x;   // NaN, inf propagate
    double k = __builtin_rint(x * kInv2Pi);
    double r = __builtin_fma(-k, k2PiHi, x);
    r = __builtin_fma(-k, k2PiMi, r);
    return __builtin_fma(-k, k2PiLo, r);
}

// sin and cos of a moderate argument (|x| < ~1e5) in one pass: quadrant
// reduction by pi/2 (3-part Cody-Waite with FMA) and the classic fdlibm
// minimax kernels (__kernel_sin / __kernel_cos coefficients, < 1 ulp on
// [-pi/4, pi/4]).  Branch-free: the quadrant is applied with selects.
__device__ __forceinline__ void sincos_mod(double x, double &s, double &c) {
    constexpr double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                     S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                     S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    constexpr double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                     C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                     C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double k = __builtin_rint(x * k2OverPi);
    double y = __builtin_fma(-k, kPio2Hi, x);
    y = __builtin_fma(-k, kPio2Mi, y);
    y = __builtin_fma(-k, kPio2Lo, y);
    int q = (int)k;
    double z = y * y;
    double rs = __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, S6, S5), S4), S3), S2);
    double sn = __builtin_fma(z * y, __builtin_fma(z, rs, S1), y);
    double rc = z * __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, C6, C5), C4), C3), C2), C1);
    double hz = 0.5 * z;
    double w = 1.0 - hz;
    double cs = w + (((1.0 - w) - hz) + z * rc);
    double ss = (q & 1) ? cs : sn;
    double cc = (q & 1) ? sn : cs;
    s = (q & 2) ? -ss : ss;
    c = ((q + 1) & 2) ? -cc : cc;
}

// fp32 sin/cos for the seed stage, |x| <~ 10: quadrant reduction + short
// minimax polynomials (abs error ~1e-7, relative near 0).
__device__ __forceinline__ void sincos_f32(float x, float &s, float &c) {
    float k = __builtin_rintf(x * 0.636619772f);
    float y = __builtin_fmaf(-k, 1.57079637f, x);
    y = __builtin_fmaf(-k, -4.37113883e-8f, y);
    int q = (int)k;
    float z = y * y;
    float sn = __builtin_fmaf(z * y, __builtin_fmaf(z, __builtin_fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f),
                                                    -1.6666654611e-1f), y);
    float cs = __builtin_fmaf(z, __builtin_fmaf(z, __builtin_fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f),
                                                4.166664568298827e-2f), -0.5f);
    cs = __builtin_fmaf(z, cs, 1.0f);
    float ss = (q & 1) ? cs : sn;
    float cc = (q & 1) ? sn : cs;
    s = (q & 2) ? -ss : ss;
    c = ((q + 1) & 2) ? -cc : cc;
}

// 1/b with one Newton-Raphson step on v_rcp_f64 (~2^-50 relative): enough for a
// summand such as r^2/s^2, whose rounding is below the reduction's own.
__device__ __forceinline__ double rcp_nr1(double b) {
    double r = __builtin_amdgcn_rcp(b);
    // fmin drops the NaN that -inf * 0 makes for b = inf, so 1/inf = 0 as in IEEE division
    return __builtin_fma(r, __builtin_fmin(__builtin_fma(-b, r, 1.0), 1.0), r);
}

// rcp_nr1 for a finite positive normal b, where its fmin is a no-op (1 - b r is tiny): the
// same bits without it.
__device__ __forceinline__ double rcp_nr1_finite(double b) {
    double r = __builtin_amdgcn_rcp(b);
    return __builtin_fma(r, __builtin_fma(-b, r, 1.0), r);
}

// 1/b to ~1 ulp: v_rcp_f64 + two Newton-Raphson steps (finite, normal b).
__device__ __forceinline__ double rcp_nr(double b) {
    double r = __builtin_amdgcn_rcp(b);
    double t = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, t, r);
    t = __builtin_fma(-b, r, 1.0);
    return __builtin_fma(r, t, r);
}

// ---- reference-faithful solver (RVK_OPT_SOLVER = 1) ---------------------------------
__device__ __forceinline__ void solve_kepler_ref(double M, double e, double &cosE, double &sinE) {
    const double tol = 1.48e-08;
    const double r = reduce_2pi(M);
    double E = r, s = 0.0, c = 0.0;
    bool done = false;
#pragma unroll 1
    for (int it = 0; it < 50; ++it) {
        sincos_mod(E, s, c);
        double f = E - e * s - r;
        double fp = 1.0 - e * c;
        double fpp = e * s;
        double En = E - f / (fp - (f * fpp) / (2.0 * fp));
        bool conv = __builtin_fabs(En - E) < tol;
        E = En;
        if (conv) { done = true; break; }
    }
    if (done) sincos_mod(E, s, c);   // sin/cos(E_new); else last iterate's (maxiter semantics)
    cosE = c;
    sinE = s;
}

// ---- production solver -------------------------------------------------------------
// sin/cos table for step 3: entries j = -kTabHalf..kTabHalf at a_j = j*kTabH
// (a_j rounded exactly as the device's jj*kTabH), filled by the host with libm.
#ifndef RVK_TAB_FINE
#define RVK_TAB_FINE 1
#endif
#if RVK_TAB_FINE
// Spacing pi/128: |d| <= pi/256, so the sin series to d^5 leaves <= 8.5e-18 and the cos series
// to d^6 <= 1.3e-20 (both far below 1 ulp) -- two FMAs fewer per lookup than pi/32 with series
// to d^7 / d^8.  321 entries (5 KB of LDS) cover |E| <= 3.93: every E of a mean anomaly
// reduced to [-pi, pi] (|E| <= pi) and every w in [-pi, pi), with margin for a seed's overshoot.
constexpr int kTabHalf = 160;
constexpr double kTabH = 0.09817477042468103 / 4;      // == np.pi / 128 (exact: a power-of-2 scaling)
constexpr double kTabInvH = 10.185916357881302 * 4;    // == 128 / np.pi
#else
// Spacing pi/32: |d| <= pi/64, so the sin series to d^7 leaves <= 4.4e-18 and the
// cos series to d^8 <= 2.3e-20 (both far below 1 ulp); 125 entries = 2 KB of LDS.
constexpr int kTabHalf = 62;                  // covers |E| <= 6.04
constexpr double kTabH = 0.09817477042468103;  // == np.pi / 32
constexpr double kTabInvH = 10.185916357881302;  // == 32 / np.pi
#endif
constexpr int kTabN = 2 * kTabHalf + 1;

struct SC { double s, c; };

// a * b + c as one VOP3 v_fma_f64 with the constant c in SGPRs.  A Horner step
// fma(z, p, c) otherwise comes out as the two-address v_fmac_f64, which needs c
// copied into the destination first (an extra v_mov_b64 per coefficient).
__device__ __forceinline__ double fma_s(double a, double b, double c) {
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
}

__device__ __forceinline__ void sincos_tab(double E, const SC *tab, double &S, double &C) {
    const double jj = __builtin_rint(E * kTabInvH);
    const double a = jj * kTabH;                 // same rounding as the host's j*h
    const double d = E - a;                      // exact (Sterbenz)
    // only the index is clamped (one v_med3_i32): |E| <= pi + 1e-6 for every finite solve;
    // a NaN/inf E gives a NaN d, a garbage one a garbage value, never an out-of-table read.
    // v_cvt_i32_f64 itself saturates and maps NaN to 0 (asm: no C++ out-of-range conversion).
    int ji;
    asm("v_cvt_i32_f64 %0, %1" : "=v"(ji) : "v"(jj));
    ji = ji < -kTabHalf ? -kTabHalf : (ji > kTabHalf ? kTabHalf : ji);
    const SC sc = tab[ji + kTabHalf];
    const double z = d * d;
#if RVK_TAB_FINE
    const double sd = __builtin_fma(d * z, fma_s(z, 1.0 / 120.0, -1.0 / 6.0), d);
    const double cm = z * __builtin_fma(z, fma_s(z, -1.0 / 720.0, 1.0 / 24.0), -0.5);
#else
    const double sd = __builtin_fma(d * z, fma_s(z, fma_s(z, -1.0 / 5040.0, 1.0 / 120.0), -1.0 / 6.0), d);
    const double cm = z * __builtin_fma(z, fma_s(z, fma_s(z, 1.0 / 40320.0, -1.0 / 720.0), 1.0 / 24.0), -0.5);
#endif
    S = __builtin_fma(sc.s, cm, __builtin_fma(sc.c, sd, sc.s));
    C = __builtin_fma(sc.c, cm, __builtin_fma(-sc.s, sd, sc.c));
}

#ifndef RVK_SEED_START
#define RVK_SEED_START 1      // 0: E0 = r (ravest's seed); 1: E0 = r + e sin r (1 + e cos r)
#endif
#ifndef RVK_SEED_THR
#define RVK_SEED_THR 1e-2f    // exit once a Halley update is below this (error ~ K d^3 after it)
#endif

template <bool PRECISE32>
__device__ __forceinline__ void sincos_seed(float x, float &s, float &c) {
    if (PRECISE32) {
        sincos_f32(x, s, c);
    } else {
        const float rev = x * 0.159154943f;   // v_sin/v_cos take revolutions
        s = __builtin_amdgcn_sinf(rev);
        c = __builtin_amdgcn_cosf(rev);
    }
}

template <bool PRECISE32>
__device__ __forceinline__ float seed_f32(float rf, float ef) {
    float Ef = rf;
    if (RVK_SEED_START == 1) {               // second-order series starter: ~1 Halley step fewer
        float s0, c0;
        sincos_seed<PRECISE32>(rf, s0, c0);
        Ef = __builtin_fmaf(ef * s0, __builtin_fmaf(ef, c0, 1.0f), rf);
    }
#pragma unroll 1
    for (int it = 0; it < 8; ++it) {
        float s, c;
        sincos_seed<PRECISE32>(Ef, s, c);
        const float f = Ef - ef * s - rf;
        const float fp = 1.0f - ef * c;
        const float fpp = ef * s;
        const float den = __builtin_fmaf(-0.5f * f, fpp, fp * fp);
        const float d = f * fp * __builtin_amdgcn_rcpf(den);
        Ef -= d;
        if (__builtin_fabsf(d) < RVK_SEED_THR) break;
    }
    return Ef;
}

#ifndef RVK_SERIES_E
#define RVK_SERIES_E 0.18f    // e <= this: the seed is the e^4 Lagrange series, no fp32 Halley step
#endif
// E = r + s [e + e^2 c + e^3 (1 - 3/2 s^2) + e^4 c (1 - 8/3 s^2)] + O(e^5), s, c = sin r, cos r
// (Lagrange's inversion of Kepler's equation to 4th order).  The e^5 remainder is at most
// 0.54 e^5: <= 1.0e-4 for e <= 0.18 (2.5e-5 at e = 0.136), so one Householder step ends the
// solve (error <= (e/f')^3 d^4 <= 0.0106 d^4 < 1e-17 for |d| <= 1.7e-4) at the cost of two
// v_sin/v_cos and ~10 fp32 ops instead of the starter plus a Halley iteration.
__device__ __forceinline__ float seed_series(float rf, float ef) {
    float s, c;
    sincos_seed<false>(rf, s, c);
    const float s2 = s * s;
    const float a4 = c * __builtin_fmaf(-2.66666667f, s2, 1.0f);
    float q = __builtin_fmaf(ef, a4, __builtin_fmaf(-1.5f, s2, 1.0f));
    q = __builtin_fmaf(ef, q, c);
    q = __builtin_fmaf(ef, q, 1.0f);
    return __builtin_fmaf(s, ef * q, rf);
}

// The solver's e-dependent choices for one planet when e is the same in every lane of the wave
// (one walker per wave): made once per walker, before the epoch loop, as wave-uniform bools
// (readfirstlane: scalar branches in the loop, not per-lane masks re-materialised every solve).
struct KFlags {
    bool series, precise, le09, le05;
};
__device__ __forceinline__ KFlags kflags_uniform(double e) {
    const float ef = (float)e;
    auto uni = [](bool b) -> bool { return __builtin_amdgcn_readfirstlane((int)b) != 0; };
    return KFlags{uni(ef <= RVK_SERIES_E), uni(ef > 0.95f), uni(e <= 0.9), uni(e <= 0.5)};
}

// r = the mean anomaly reduced to [-pi, pi]; e6e3 = 6*e^3 (per planet, precomputed).
// UNI: the choices come from kf (kflags_uniform of this e), else they are made per lane.
template <bool UNI = false>
__device__ __forceinline__ void solve_kepler_fast_r(double r, double e, double e6e3, const SC *tab, double &cosE,
                                                    double &sinE, KFlags kf = {}) {
    const float rf = (float)r, ef = (float)e;
#ifndef RVK_SEED_HW
#define RVK_SEED_HW 1
#endif
#ifndef RVK_ABLATE
#define RVK_ABLATE 0   // timing experiments only (wrong results): 1 = no fp64 stage, 2 = no fp32 seed, 3 = neither
#endif
    const bool series = UNI ? kf.series : ef <= RVK_SERIES_E;
    const float Ef = (RVK_ABLATE & 2) ? rf
                   : series ? seed_series(rf, ef)
                   : ((!RVK_SEED_HW || (UNI ? kf.precise : ef > 0.95f)) ? seed_f32<true>(rf, ef)
                                                                         : seed_f32<false>(rf, ef));
    double E = (double)Ef, S, C;
    sincos_tab(E, tab, S, C);
    if (RVK_ABLATE & 1) { cosE = C; sinE = S; return; }
#ifndef RVK_HH_SINGLE
#define RVK_HH_SINGLE 1
#endif
#ifndef RVK_HALLEY_LOWE
#define RVK_HALLEY_LOWE 0   // 1: e <= 0.5 takes a Halley first fp64 step (cubic, 6 fewer fp64 ops);
                            // measured a wash (-1.6 % .. +4 % over the kbench cases), so off
#endif
    // One step from (E, S = sin E, C = cos E), Halley's (hal) or Householder's of order 3;
    // returns the step d and leaves t ~ 1/den for the error estimate.  Only num/den sit under
    // the branch, so a wave whose lanes disagree on hal runs the shared rest once.
    auto step = [&](bool hal, double &t) -> double {
        const double f = E - e * S - r;
        const double f1 = 1.0 - e * C;
        const double f2 = e * S;
        double num, den;
        if (hal) {
            num = f * f1;                                                            // f f1 / (f1^2 - f f2 / 2)
            den = __builtin_fma(-0.5 * f, f2, f1 * f1);
        } else {
            const double f3 = e * C;
            const double f11 = f1 * f1;
            num = f * __builtin_fma(-3.0 * f, f2, 6.0 * f11);                        // f (6 f1^2 - 3 f f2)
            den = __builtin_fma(f * f, f3, 6.0 * f1 * __builtin_fma(-f, f2, f11));  // 6f1^3 - 6 f f1 f2 + f^2 f3
        }
        t = __builtin_amdgcn_rcp(den);
        t = __builtin_fma(t, __builtin_fma(-den, t, 1.0), t);
        const double d = -num * t;
        E += d;
        if (__builtin_fabs(d) > 1e-4) {    // too far for the short series: re-anchor on the table
            sincos_tab(E, tab, S, C);
        } else {                           // |d| <= 1e-4: sin d = d - d^3/6 (+8e-23), cos d = 1 - d^2/2 (+4e-18)
            const double z = d * d;
            const double sd = __builtin_fma(d * z, -1.0 / 6.0, d);
            const double cm = -0.5 * z;
            const double Sn = __builtin_fma(S, cm, __builtin_fma(C, sd, S));
            const double Cn = __builtin_fma(C, cm, __builtin_fma(-S, sd, C));
            S = Sn;
            C = Cn;
        }
        return d;
    };
    // next error ~ (e/f1)^3 d^4.  For e <= 0.9, (e/f1)^3 <= 729, so |d| <= 1e-5 already
    // bounds it by 7.3e-18 (one compare); otherwise estimate it as 6 e^3 d^4 / den.
    const bool e_le_09 = UNI ? kf.le09 : e <= 0.9;
    auto converged = [&](double d, double t) -> bool {
        if (RVK_HH_SINGLE && e_le_09) return __builtin_fabs(d) <= 1e-5;
        const double z2 = (d * d) * (d * d);
        return z2 * e6e3 * __builtin_fabs(t) < 1e-17;
    };
    // The first step is peeled (no loop-carried register shuffles on the common one-step path).
    // Halley's next error is c d^3 with |c| = |f2^2 / (4 f1^2) - f3 / (6 f1)| <= 0.42 for
    // e <= 0.5 (f1 >= 1/2, |f2|, |f3| <= 1/2): |d| <= 2.8e-6 bounds it by 9.2e-18.
    const bool hal = RVK_HALLEY_LOWE && (UNI ? kf.le05 : e <= 0.5);
    double t;
    double d = step(hal, t);
    bool done;
    if constexpr (UNI) {
        // one compare against a wave-uniform threshold (no select between per-lane bools, which
        // the compiler lowers through a VGPR and back every solve); the same tests as below
        if (hal) {
            done = __builtin_fabs(d) <= 2.8e-6;
        } else if (series || (RVK_HH_SINGLE && e_le_09)) {
            done = __builtin_fabs(d) <= (series ? 1.7e-4 : 1e-5);
        } else {
            done = converged(d, t);
        }
    } else {
        done = hal ? __builtin_fabs(d) <= 2.8e-6 : series ? __builtin_fabs(d) <= 1.7e-4 : converged(d, t);
    }
    if (!done) {
#pragma unroll 1
        for (int it = 1; it < 8; ++it) {
            d = step(false, t);
            if (converged(d, t)) break;
        }
    }
    cosE = C;
    sinE = S;
}

template <bool UNI = false>
__device__ __forceinline__ void solve_kepler_fast(double M, double e, double e6e3, const SC *tab, double &cosE,
                                                  double &sinE, KFlags kf = {}) {
    solve_kepler_fast_r<UNI>(reduce_2pi(M), e, e6e3, tab, cosE, sinE, kf);
}

// ---- register-light atan / atan2 / tan for the Tc and secosw/sesinw conversions ----
// fdlibm's s_atan.c algorithm (< 1 ulp): argument reduction to |x| < 7/16 against
// atan(0.5), atan(1), atan(1.5), atan(inf), then an 11-term odd polynomial.  Used by
// the in-kernel conversion instead of OCML's atan/atan2/tan.
__device__ __forceinline__ double atan_fd(double x) {
    constexpr double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
                     aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
                     aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
                     aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
                     aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
                     aT10 = 1.62858201153657823623e-02;
    const double ax = __builtin_fabs(x);
    // reduction: id = -1 (none), 0..3
    double num, den, hi, lo;
    int id;
    if (ax < 0.4375) { id = -1; num = ax; den = 1.0; hi = 0.0; lo = 0.0; }
    else if (ax < 0.6875) { id = 0; num = 2.0 * ax - 1.0; den = 2.0 + ax;
                            hi = 4.63647609000806093515e-01; lo = 2.26987774529616870924e-17; }
    else if (ax < 1.1875) { id = 1; num = ax - 1.0; den = ax + 1.0;
                            hi = 7.85398163397448278999e-01; lo = 3.06161699786838301793e-17; }
    else if (ax < 2.4375) { id = 2; num = ax - 1.5; den = 1.0 + 1.5 * ax;
                            hi = 9.82793723247329054082e-01; lo = 1.39033110312309984516e-17; }
    else { id = 3; num = -1.0; den = ax; hi = 1.57079632679489655800e+00; lo = 6.12323399573676603587e-17; }
    const double xr = (id < 0) ? ax : num / den;
    const double z = xr * xr, w = z * z;
    const double s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const double s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    double r;
    if (id < 0) r = xr - xr * (s1 + s2);
    else r = hi - ((xr * (s1 + s2) - lo) - xr);
    if (!(ax == ax)) r = x;                   // NaN propagates
    return __builtin_copysign(r, x);
}

// atan2 with C99 / numpy signed-zero semantics; atan2(+0, u < 0) == pi exactly
// (ravest then rejects w == pi, param.py:80-86).
__device__ __forceinline__ double atan2_fd(double y, double x) {
    constexpr double pi_lo = 1.2246467991473531772e-16;
    if (y == 0.0) {
        const bool xneg = (x < 0.0) || (x == 0.0 && __builtin_signbit(x));
        return xneg ? __builtin_copysign(kPi, y) : y;
    }
    if (x == 0.0) return __builtin_copysign(kPi / 2, y);
    const double z = atan_fd(__builtin_fabs(y / x));
    if (x > 0.0) return __builtin_copysign(z, y);
    return __builtin_copysign(kPi - (z - pi_lo), y);
}

__device__ __forceinline__ double tan_fd(double x) {
    double s, c;
    sincos_mod(x, s, c);
    return s / c;
}

// Per-planet constants in the default "P K e w Tp" form (model.py:199-206,
// model.py:302 n = 2*pi/P).  ok == false exactly where Planet() raises.
// rv = K * (inv * ((cosE - e) * cw - sinE * sqsw) + ecw),  inv = 1 / (1 - e cosE)
// (= K (cos f cos w - sin f sin w + e cos w), model.py:119-121,170; K stays the
// outer factor so K = inf gives +-inf like the reference, not inf - inf)
#ifndef RVK_PHASE
#define RVK_PHASE 1   // planet_rv reduces the phase (t - Tp) / P rather than M = n (t - Tp)
#endif
struct PlanetK {
    double n, Tp, e, K, cw, sqsw, ecw, e6e3;   // n = 1 / P (RVK_PHASE) or 2 pi / P
};

// param.py:88-105 (NaN passes the '<=' tests, as in the reference)
__device__ __forceinline__ bool valid_default(double P, double K, double e, double w) {
    return !(P <= 0.0) && !(K <= 0.0) && !(e < 0.0) && !(e >= 1.0) && (-kPi <= w && w < kPi);
}

// Conversion to the default parameterisation (param.py:299-362, 198-234).
// PAR >= 0: compile-time parameterisation (PAR = 0 needs no atan/tan/atan2);
// PAR = -1: runtime `par`.
// One planet's parameters in parameterisation `par` -> the default "P K e w Tp"
// (param.py:159-297, convert_pars_to_default_parameterisation).  Returns false
// exactly where that conversion raises (Tc -> Tp validates e, param.py:208-209).
template <int PAR>
__device__ __forceinline__ bool to_default_t(const double *p5, double &P, double &K, double &e, double &w,
                                             double &Tp, int par = PAR) {
    if (PAR >= 0) par = PAR;
    P = p5[0];
    K = p5[1];
    if (par >= 2) {                       // secosw/sesinw -> e, w  (param.py:217-234)
        double u = p5[2], v = p5[3];
        e = u * u + v * v;
        w = atan2_fd(v, u);
    } else {
        e = p5[2];
        w = p5[3];
    }
    bool ok = true;
    if (par == 1 || par == 3) {           // Tc -> Tp  (param.py:198-215)
        if (e < 0.0 || e >= 1.0) {
            ok = false;
            Tp = 0.0;
        } else {
            double theta_tc = (kPi / 2) - w;
            double E = 2 * atan_fd(sqrt((1 - e) / (1 + e)) * tan_fd(theta_tc / 2));
            double sE, cE;
            sincos_mod(E, sE, cE);
            double Mc = E - (e * sE);
            Tp = p5[4] - (P / kTwoPi) * Mc;
        }
    } else {
        Tp = p5[4];
    }
    return ok;
}

// TAB: sin/cos(w) from the LDS table `tab` (w is in [-pi, pi) for a valid planet;
// an invalid one is masked and w = 0 is used), sharing the epoch loop's constants
// instead of holding fdlibm's coefficients for the prep alone.
template <int PAR, bool TAB = false>
__device__ __forceinline__ bool planet_consts_t(const double *p5, PlanetK &pk, int par = PAR,
                                                const SC *tab = nullptr) {
    double P, K, e, w, Tp;
    bool ok = to_default_t<PAR>(p5, P, K, e, w, Tp, par);
    ok = ok && valid_default(P, K, e, w);
    if (!ok) {                            // keep the masked walker's arithmetic finite
        P = 1.0; e = 0.0; w = 0.0;
    }
    pk.n = RVK_PHASE ? 1.0 / P : kTwoPi / P;
    pk.Tp = Tp;
    pk.e = e;
    double sw, cw;
    if (TAB) sincos_tab(w, tab, sw, cw);
    else sincos_mod(w, sw, cw);
    pk.K = K;
    pk.cw = cw;
    pk.sqsw = sqrt(1.0 - e * e) * sw;
    pk.ecw = e * cw;
    pk.e6e3 = 6.0 * e * e * e;
    return ok;
}

// Out of line on purpose: an inlined conversion (atan/tan/sqrt/division chains) would
// set the whole kernel's VGPR budget; as a call it costs registers only while it runs.
__device__ __attribute__((noinline)) bool planet_consts(int par, const double *p5, PlanetK &pk) {
    return planet_consts_t<-1>(p5, pk, par);
}

// The same, storing into an LDS slot through a shared-address-space pointer (no caller stack
// object: the posterior predictive's per-sample prep, one planet per lane; dst is an LDS slot).
__device__ __attribute__((noinline)) bool planet_consts_lds(int par, const double *p5,
                                                            PlanetK *dst) {
    PlanetK pk;
    const bool ok = planet_consts_t<-1>(p5, pk, par);
    *dst = pk;
    return ok;
}

// One planet's RV at time t (model.py:327, 119-121, 170).  e == 0 takes the
// same arithmetic (the solvers return E = M), so there is no branch.
template <int SOLVER, bool UNI = false>
// acc + (this planet's RV at t).  UNI: pk is the same in every lane (solve_kepler_fast_r).  1/(1 - e cos E) with one Newton step on v_rcp_f64
// (<= 2.2e-15 relative, like the chi^2 terms); the divisor is in (0, 2).
__device__ __forceinline__ double planet_rv(const PlanetK &pk, double t, const SC *tab, double acc, KFlags kf = {}) {
    double cE, sE;
    if (SOLVER == 1) {
        const double M = RVK_PHASE ? kTwoPi * (pk.n * (t - pk.Tp)) : pk.n * (t - pk.Tp);
        solve_kepler_ref(M, pk.e, cE, sE);
    } else if (RVK_PHASE) {
        // orbits since periastron u = (t - Tp) / P: u - rint(u) is exact, so r = 2 pi (u - rint u)
        // is M reduced to [-pi, pi] to |M| 2.2e-16 + ulp(pi) (|u| >= 2^52: r = 0), in 5 VALU
        // instructions instead of M and a Cody-Waite reduction's 12.  Not contracted: fusing the
        // product into the subtraction would leave its rounding error, ~ulp(u), in the fraction.
#pragma clang fp contract(off)
        const double u = pk.n * (t - pk.Tp);
        solve_kepler_fast_r<UNI>(kTwoPi * (u - __builtin_rint(u)), pk.e, pk.e6e3, tab, cE, sE, kf);
    } else {
        solve_kepler_fast<UNI>(pk.n * (t - pk.Tp), pk.e, pk.e6e3, tab, cE, sE, kf);
    }
    const double b = 1.0 - pk.e * cE;
    double inv = __builtin_amdgcn_rcp(b);
    inv = __builtin_fma(inv, __builtin_fma(-b, inv, 1.0), inv);
    return __builtin_fma(pk.K, __builtin_fma(inv, __builtin_fma(cE - pk.e, pk.cw, -sE * pk.sqsw), pk.ecw), acc);
}

// Wave64 sum in a fixed order (bitwise reproducible): DPP butterflies inside each
// 16-lane row (quad_perm 1032, quad_perm 2301, row_half_mirror, row_mirror), then the
// four row totals read with v_readlane and added on the VALU.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, 0xF, 0xF, true);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)b, lane);
    const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(b >> 32), lane);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// v from lane `src` (0..63) of this wave, per lane (two ds_bpermute_b32; no LDS allocation)
__device__ __forceinline__ double shfl_d(double v, int src) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const int addr = src << 2;
    const unsigned lo = __builtin_amdgcn_ds_bpermute(addr, (int)(unsigned)b);
    const unsigned hi = __builtin_amdgcn_ds_bpermute(addr, (int)(unsigned)(b >> 32));
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// ln(m * 2^k) for a frexp mantissa m in [0.5, 1): fdlibm e_log.c's reduction and
// kernel (m -> [sqrt(1/2), sqrt(2)), s = f / (2 + f), degree-14 polynomial in s),
// ~1 ulp, about a quarter of the generic log's instructions.  Callers route
// m outside [0.5, 1) (0, inf, NaN) to log().
__device__ __forceinline__ double log_frexp(double m, int k) {
    constexpr double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                     Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                     Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                     Lg7 = 1.479819860511658591e-01;
    constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const bool lo = m < 0.70710678118654752440;
    m = lo ? 2.0 * m : m;
    k -= lo ? 1 : 0;
    const double f = m - 1.0;
    const double hfsq = 0.5 * f * f;
    const double s = f * rcp_nr(2.0 + f);
    const double z = s * s, w = z * z;
    const double t1 = w * fma_s(w, __builtin_fma(w, Lg6, Lg4), Lg2);
    const double t2 = z * fma_s(w, fma_s(w, __builtin_fma(w, Lg7, Lg5), Lg3), Lg1);
    const double R = t2 + t1;
    const double dk = (double)k;
    return dk * ln2_hi - ((hfsq - __builtin_fma(s, hfsq + R, dk * ln2_lo)) - f);
}

__device__ __forceinline__ double uniform_d(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = __builtin_amdgcn_readfirstlane((int)(unsigned)b);
    const unsigned hi = __builtin_amdgcn_readfirstlane((int)(unsigned)(b >> 32));
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// A wave-uniform PlanetK (read from LDS with a uniform address) moved to SGPRs:
// the 8 constants stay out of the VGPR budget of the epoch loop.
__device__ __forceinline__ PlanetK uniform_pk(const PlanetK &q) {
    PlanetK pk;
    pk.n = uniform_d(q.n); pk.Tp = uniform_d(q.Tp); pk.e = uniform_d(q.e); pk.K = uniform_d(q.K);
    pk.cw = uniform_d(q.cw); pk.sqsw = uniform_d(q.sqsw); pk.ecw = uniform_d(q.ecw);
    pk.e6e3 = uniform_d(q.e6e3);
    return pk;
}

// Every lane gets the sum of its 16-lane row (the DPP butterflies of wave_sum).
__device__ __forceinline__ double row_sum(double v) {
    v += dpp_d<0xB1>(v);    // quad_perm [1,0,3,2]
    v += dpp_d<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp_d<0x141>(v);   // row_half_mirror
    v += dpp_d<0x140>(v);   // row_mirror
    return v;
}

__device__ __forceinline__ double wave_sum(double v) {
    v += dpp_d<0xB1>(v);    // quad_perm [1,0,3,2]
    v += dpp_d<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp_d<0x141>(v);   // row_half_mirror
    v += dpp_d<0x140>(v);   // row_mirror
    return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
}

}  // namespace rvk
