// Diagnostic: accuracy of v_rcp_f64 / v_rcp_f32 / v_sin_f32 / v_cos_f32 on gfx950.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
__global__ void k(const double *x, double *r0, double *r1, float *sf, float *cf, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double b = x[i];
    double r = __builtin_amdgcn_rcp(b);
    r0[i] = r;
    r1[i] = __builtin_fma(r, __builtin_fma(-b, r, 1.0), r);
    float a = (float)(x[i] - 3.0);                      // angle in [-3, 3.x]
    sf[i] = __builtin_amdgcn_sinf(a * 0.159154943f);
    cf[i] = __builtin_amdgcn_cosf(a * 0.159154943f);
}
int main() {
    const int n = 1 << 20;
    std::vector<double> x(n);
    for (int i = 0; i < n; ++i) x[i] = 0.5 + 6.0 * (i + 0.5) / n;
    double *dx, *d0, *d1; float *ds, *dc;
    hipMalloc(&dx, n * 8); hipMalloc(&d0, n * 8); hipMalloc(&d1, n * 8); hipMalloc(&ds, n * 4); hipMalloc(&dc, n * 4);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dx, d0, d1, ds, dc, n);
    std::vector<double> r0(n), r1(n); std::vector<float> s(n), c(n);
    hipMemcpy(r0.data(), d0, n * 8, hipMemcpyDeviceToHost); hipMemcpy(r1.data(), d1, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(s.data(), ds, n * 4, hipMemcpyDeviceToHost); hipMemcpy(c.data(), dc, n * 4, hipMemcpyDeviceToHost);
    double e0 = 0, e1 = 0, es = 0, ec = 0, esr = 0;
    for (int i = 0; i < n; ++i) {
        double t = 1.0 / x[i];
        e0 = fmax(e0, fabs(r0[i] - t) / t); e1 = fmax(e1, fabs(r1[i] - t) / t);
        double a = (double)(float)(x[i] - 3.0);
        es = fmax(es, fabs(s[i] - sin(a))); ec = fmax(ec, fabs(c[i] - cos(a)));
        if (fabs(a) < 0.3 && a != 0) esr = fmax(esr, fabs(s[i] - sin(a)) / fabs(sin(a)));
    }
    printf("{\"rcp_f64_rel\": %.3e, \"rcp_f64_1nr_rel\": %.3e, \"sin_f32_abs\": %.3e, \"cos_f32_abs\": %.3e, \"sin_f32_rel_small\": %.3e}\n", e0, e1, es, ec, esr);
    return 0;
}
