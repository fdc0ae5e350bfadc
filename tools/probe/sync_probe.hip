// sync_probe.hip -- how long does the host wait for a short kernel, by completion mechanism?
// (timing probe for the host-buffer entry points' launch + synchronize floor)
//
// Modes, each median over N round trips of one launch of a kernel that runs ~T us on a
// 256-block grid (1024 threads) and writes one double per block to fine-grained host memory:
//   sync   hipStreamSynchronize
//   query  spin on hipStreamQuery
//   flag   the last block (a device-scope counter) publishes a sequence number to a host flag
//          at system scope; the host spins on it (hipStreamQuery every 256 polls as the
//          fault / error escape), then reads the outputs
//   event  hipEventRecord after the launch + hipEventSynchronize
// argv: mode [spin] -- "spin" sets hipDeviceScheduleSpin before the first HIP call.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

__global__ __launch_bounds__(1024) void work(double *out, unsigned long long ticks, unsigned long long *ctr,
                                             unsigned int *flag, unsigned long long expect, unsigned int seq) {
    const unsigned long long t0 = wall_clock64();   // 100 MHz
    double acc = threadIdx.x;
    while (wall_clock64() - t0 < ticks) acc = acc * 0.999 + 1.0;
    __syncthreads();
    if (threadIdx.x == 0) {
        out[blockIdx.x] = acc;
        if (flag) {
            __threadfence_system();
            const unsigned long long old = __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            if (old == expect) {
                __threadfence_system();
                __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "sync";
    const bool spin = argc > 2 && !std::strcmp(argv[2], "spin");
    const double kernel_us = argc > 3 ? std::atof(argv[3]) : 7.0;
    if (spin) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    CK(hipSetDevice(0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const int blocks = 256;
    double *out = nullptr;
    unsigned int *flag = nullptr;
    unsigned long long *ctr = nullptr;
    CK(hipHostMalloc((void **)&out, blocks * sizeof(double), hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc((void **)&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipMalloc((void **)&ctr, sizeof(unsigned long long)));
    CK(hipMemset(ctr, 0, sizeof(unsigned long long)));
    *flag = 0;
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const unsigned long long ticks = (unsigned long long)(kernel_us * 100.0);
    const bool use_flag = !std::strcmp(mode, "flag");
    const int N = 3000, warm = 300;
    std::vector<double> t;
    t.reserve(N);
    unsigned long long launches = 0;
    for (int i = 0; i < N + warm; ++i) {
        const unsigned int seq = (unsigned int)(i + 1);
        const double a = now_us();
        hipLaunchKernelGGL(work, dim3(blocks), dim3(1024), 0, st, out, ticks, ctr, use_flag ? flag : nullptr,
                           (launches + 1) * blocks - 1, seq);
        ++launches;
        if (!std::strcmp(mode, "sync")) {
            CK(hipStreamSynchronize(st));
        } else if (!std::strcmp(mode, "query")) {
            hipError_t e;
            while ((e = hipStreamQuery(st)) == hipErrorNotReady) {
            }
            CK(e);
        } else if (!std::strcmp(mode, "event")) {
            CK(hipEventRecord(ev, st));
            CK(hipEventSynchronize(ev));
        } else if (use_flag) {
            int polls = 0;
            while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
                if (++polls % 256 == 0) {
                    hipError_t e = hipStreamQuery(st);
                    if (e != hipErrorNotReady && e != hipSuccess) CK(e);
                    if (e == hipSuccess && __atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
                        std::fprintf(stderr, "stream idle but flag %u != %u\n", *flag, seq);
                        return 1;
                    }
                }
            }
        } else {
            std::fprintf(stderr, "unknown mode %s\n", mode);
            return 2;
        }
        volatile double sink = out[blocks - 1];
        (void)sink;
        const double b = now_us();
        if (i >= warm) t.push_back(b - a);
    }
    CK(hipStreamSynchronize(st));
    std::sort(t.begin(), t.end());
    std::printf("{\"mode\": \"%s\", \"spin\": %s, \"kernel_us\": %.1f, \"p10_us\": %.2f, \"median_us\": %.2f, \"p90_us\": %.2f}\n",
                mode, spin ? "true" : "false", kernel_us, t[N / 10], t[N / 2], t[N * 9 / 10]);
    return 0;
}
