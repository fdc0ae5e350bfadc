// gp64_accum_probe.hip -- what rate does the fp64 GP accumulation loop reach on one CU?
// (timing probe for DESIGN §9.1; the loop shape of rvk_gp64.hip accum_span: per register set a
// quarter tile of the shared A operand L(k+1, j) and of R row operands L(bi, j), 8 R
// v_mfma_f64_16x16x4_f64, a ring of 2 sets: the next set's loads in flight while one is consumed)
//
// One 512-thread workgroup (8 waves, 2 per SIMD) per CU, 256 workgroups.  Per wave: NS sets,
// s_memtime around the loop.  Variants:
//   src   0 = operands from a 64 KB block-private region (L2 / L1 resident), 1 = from a 1.1 MB
//         block-private workspace (the walker's tiles: MALL / HBM), 2 = no loads (registers only),
//         3 = operands from LDS (the same fragment layout staged once)
//   act   active waves: 8, 4 (one per SIMD: waves 0-3) or 1
//   R     rows per wave (1-3)
// Output: median cycles per set per active wave, and the implied fraction of the SIMD's fp64
// MFMA issue (64 cycles per MFMA; act = 8 puts two waves on each SIMD).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

using f64x4 = __attribute__((ext_vector_type(4))) double;
constexpr int TILE = 1024;           // doubles per 32 x 32 tile
constexpr int NS = 256;              // sets per wave (64 tile products of 4 quarters)

template <int R>
struct Ops {
    double2 a[2], b[R][2];
};

template <int R, int SRC>
__global__ __launch_bounds__(512, 1) void accum(const double *__restrict__ work, long long stride, int act,
                                                 double *out, long long *cyc) {
    extern __shared__ double lds[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const double *wk = work + (long long)blockIdx.x * stride;
    if (SRC == 3) {
        for (int i = threadIdx.x; i < 8 * TILE; i += 512) lds[i] = wk[i];
        __syncthreads();
    }
    if (wv >= act) return;
    f64x4 acc[R][2][2];
    for (int r = 0; r < R; ++r)
        for (int p = 0; p < 2; ++p)
            for (int q = 0; q < 2; ++q) acc[r][p][q] = f64x4{0.0, 0.0, 0.0, 0.0};
    // tile offsets (doubles): A = tile j of row "k+1", B = tile j of this wave's rows
    // SRC 0: 8 tiles per block reused; SRC 1: distinct tiles over ~1.1 MB (j strides a row's tiles)
    auto atile = [&](int j) -> long long { return SRC == 1 ? (long long)(j % 16) * TILE : 0; };
    auto btile = [&](int r, int j) -> long long {
        return SRC == 1 ? (long long)(16 + (wv * 3 + r) * 16 + (j % 16)) * TILE : (long long)(1 + (wv + r) % 7) * TILE;
    };
    Ops<R> X, Y;
    auto issue = [&](Ops<R> &o, int hx) {
        hx = hx < NS ? hx : NS - 1;
        const int j = hx >> 2, part = hx & 3;
        if constexpr (SRC == 2) {
            o.a[0] = o.a[1] = double2{1.0 + hx, 2.0};
            for (int r = 0; r < R; ++r) o.b[r][0] = o.b[r][1] = double2{0.5, 1.0 * r};
            return;
        }
        const int off = part * 64 + lane;    // double2 units
        if constexpr (SRC == 3) {
            const double2 *la = reinterpret_cast<const double2 *>(lds);
            o.a[0] = la[off];
            o.a[1] = la[off + 256];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const double2 *lb = reinterpret_cast<const double2 *>(lds + (1 + (wv + r) % 7) * TILE);
                o.b[r][0] = lb[off];
                o.b[r][1] = lb[off + 256];
            }
            return;
        }
        const double2 *ta = reinterpret_cast<const double2 *>(wk + atile(j));
        o.a[0] = ta[off];
        o.a[1] = ta[off + 256];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const double2 *tb = reinterpret_cast<const double2 *>(wk + btile(r, j));
            o.b[r][0] = tb[off];
            o.b[r][1] = tb[off + 256];
        }
    };
    auto consume = [&](const Ops<R> &o) {
#pragma unroll
        for (int cmp = 0; cmp < 2; ++cmp)
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int p = 0; p < 2; ++p)
#pragma unroll
                    for (int q = 0; q < 2; ++q)
                        acc[r][p][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(cmp ? o.a[p].y : o.a[p].x,
                                                                            cmp ? o.b[r][q].y : o.b[r][q].x, acc[r][p][q], 0, 0, 0);
    };
    const long long t0 = __builtin_amdgcn_s_memtime();
    issue(X, 0);
    for (int hx = 0; hx < NS; hx += 2) {
        issue(Y, hx + 1);
        __builtin_amdgcn_sched_barrier(0);
        consume(X);
        __builtin_amdgcn_sched_barrier(0);
        issue(X, hx + 2);
        __builtin_amdgcn_sched_barrier(0);
        consume(Y);
        __builtin_amdgcn_sched_barrier(0);
    }
    double s = 0.0;
    for (int r = 0; r < R; ++r)
        for (int p = 0; p < 2; ++p)
            for (int q = 0; q < 2; ++q) s += acc[r][p][q][0] + acc[r][p][q][3];
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[(long long)blockIdx.x * 512 + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * 8 + wv] = t1 - t0;
}

template <int R, int SRC>
static void run(const double *work, long long stride, double *out, long long *cyc, int act) {
    const size_t lds = SRC == 3 ? 8 * TILE * sizeof(double) : 0;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL((accum<R, SRC>), dim3(256), dim3(512), lds, 0, work, stride, act, out, cyc);
        CK(hipDeviceSynchronize());
    }
    std::vector<long long> h(256 * 8);
    CK(hipMemcpy(h.data(), cyc, h.size() * sizeof(long long), hipMemcpyDeviceToHost));
    std::vector<double> v;
    for (int b = 0; b < 256; ++b)
        for (int w = 0; w < act; ++w) v.push_back((double)h[b * 8 + w] / NS);
    std::sort(v.begin(), v.end());
    const double med = v[v.size() / 2];
    const int per_simd = act == 8 ? 2 : 1;
    const double util = 8.0 * R * 64.0 * per_simd / med;   // the SIMD's MFMA issue busy fraction
    static const char *src_name[] = {"l2", "workspace", "registers", "lds"};
    std::printf("{\"R\": %d, \"src\": \"%s\", \"active_waves\": %d, \"cycles_per_set\": %.0f, \"p90\": %.0f, "
                "\"mfma_busy\": %.3f}\n", R, src_name[SRC], act, med, v[v.size() * 9 / 10], util);
}

int main() {
    const long long stride = (16 + 8 * 3 * 16 + 16) * (long long)TILE;   // doubles per block (~3.3 MB)
    double *work = nullptr, *out = nullptr;
    long long *cyc = nullptr;
    CK(hipMalloc((void **)&work, (size_t)stride * 256 * sizeof(double)));
    CK(hipMemset(work, 0, (size_t)stride * 256 * sizeof(double)));
    CK(hipMalloc((void **)&out, 256 * 512 * sizeof(double)));
    CK(hipMalloc((void **)&cyc, 256 * 8 * sizeof(long long)));
    for (int act : {8, 4, 1}) {
        run<1, 2>(work, stride, out, cyc, act);
        run<1, 0>(work, stride, out, cyc, act);
        run<1, 1>(work, stride, out, cyc, act);
        run<1, 3>(work, stride, out, cyc, act);
        run<2, 2>(work, stride, out, cyc, act);
        run<2, 0>(work, stride, out, cyc, act);
        run<2, 1>(work, stride, out, cyc, act);
        run<2, 3>(work, stride, out, cyc, act);
        run<3, 2>(work, stride, out, cyc, act);
        run<3, 0>(work, stride, out, cyc, act);
        run<3, 1>(work, stride, out, cyc, act);
        run<3, 3>(work, stride, out, cyc, act);
    }
    return 0;
}
