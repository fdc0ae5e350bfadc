// Probe: cycles per v_mfma_f32_32x32x2_f32 for one dependent accumulator chain vs 2 / 4
// interleaved chains, one wave per SIMD (4 waves per block, 1 block per CU) and 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
using f32x16 = __attribute__((ext_vector_type(16))) float;

template <int CH>
__global__ __launch_bounds__(256) void chain(const float *in, float *out, long long *cyc, int iters) {
    f32x16 acc[CH];
    for (int q = 0; q < CH; ++q) acc[q] = f32x16{};
    float a = in[threadIdx.x], b = in[threadIdx.x + 256];
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k)
#pragma unroll
            for (int q = 0; q < CH; ++q) acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[q], 0, 0, 0);
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int q = 0; q < CH; ++q) for (int r = 0; r < 16; ++r) s += acc[q][r];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CH>
void run(int blocks, const float *in, float *out, long long *cyc) {
    const int iters = 64;
    hipLaunchKernelGGL(chain<CH>, dim3(blocks), dim3(256), 0, 0, in, out, cyc, iters);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(chain<CH>, dim3(blocks), dim3(256), 0, 0, in, out, cyc, iters);
    hipDeviceSynchronize();
    long long h[1024];
    hipMemcpy(h, cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < blocks; ++i) m += h[i];
    m /= blocks;
    printf("chains=%d blocks=%d: %.1f cycles per MFMA per wave (%.1f per MFMA issued on the SIMD)\n", CH, blocks,
           m / (iters * 16.0 * CH), m / (iters * 16.0 * CH) / (blocks > 256 ? 2.0 : 1.0));
}

int main() {
    float *in, *out;
    long long *cyc;
    hipMalloc(&in, 4096 * sizeof(float));
    hipMalloc(&out, 1024 * 256 * sizeof(float));
    hipMalloc(&cyc, 1024 * sizeof(long long));
    hipMemset(in, 0, 4096 * sizeof(float));
    for (int blocks : {256, 512}) {
        run<1>(blocks, in, out, cyc);
        run<2>(blocks, in, out, cyc);
        run<4>(blocks, in, out, cyc);
    }
    return 0;
}
