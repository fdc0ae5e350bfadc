// rvk_internal.h -- declarations shared by the translation units of librvk.so
// (rvk.hip: log-likelihood / predictive / Kepler; rvk_post.hip: device
// log-posterior and stretch-move sampler).  Not part of the C-ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <string>

#include "../../include/rvk.h"
#include "rvk_math.h"
#include "rvk_post_dev.h"

namespace rvk {

constexpr int kBlock = 256;                    // 4 waves
constexpr int kWavesPerBlock = kBlock / 64;
constexpr int kEpochPad = 64;                  // padding entries after the device epoch arrays (rvk_create)

// Per-epoch data: SoA, device-resident for the handle's lifetime.
struct EpochData {
    const double *t;      // time
    const double *vel;
    const double *s2;     // velerr^2 (fit.py:3598)
    const int32_t *inst;  // instrument index (fit.py:3586)
    const SC *tab;        // sin/cos table (rvk_math.h, kTabN entries)
    double t0;            // Trend reference time (model.py:486,491)
    int par;              // parameterisation code (RVK_PAR_*)
    int lpw;              // lanes per walker: 0 = chosen per launch, else 64 / 32 / 16 (RVK_OPT_LPW)
    int np;               // planets (the generic kernels' runtime count; the others are specialised)
    int poison;           // RVK_OPT_LDS_POISON: tab_put writes NaN first (tests only)
    int s2ok;             // every velerr^2 in [2^-500, 2^500] (rvk_create): epoch_sum may renormalise less often
};

// Store entry i of an LDS copy of the sin/cos table.  poison (RVK_OPT_LDS_POISON, tests only):
// NaN first, the real value ~10 us later (the compiler barrier keeps the first store), so a
// reader not ordered after the publishing barrier sees NaN.  poison == 2 (the tests' positive
// control): the real value is never stored, so every table read is NaN -- a kernel the option
// reaches then returns NaN walkers, which shows the equality tests run poisoned.
__device__ __forceinline__ void tab_put(SC *tab, int i, SC v, int poison) {
    if (poison) {
        tab[i] = SC{__builtin_nan(""), __builtin_nan("")};
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        for (int k = 0; k < 3; ++k) __builtin_amdgcn_s_sleep(127);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        if (poison > 1) return;
    }
    tab[i] = v;
}

// Optional log-posterior epilogue of the log-likelihood kernel (fit.py:3461-3495):
// lp == nullptr: out = log-likelihood.  Otherwise lp[w] is the walker's log-prior
// (-inf = rejected before the likelihood: negative jitter, a prior-side conversion
// error or a non-finite prior), and out = ((ll + lp) + jac) + renorm in the
// reference's order; a rejected walker skips its epoch loop.
struct PostArgs {
    const double *lp;
    double jac;
    double renorm;
};

typedef void (*loglike_launch_t)(hipStream_t, EpochData, int, int, const double *, long long, long long, double *,
                                 PostArgs);

typedef void (*sample_launch_t)(hipStream_t, EpochData, int, int, const double *, long long, long long, PostArgs,
                                const SampleArgs &);
// the launcher of the fused half-step kernels of one MODE (2, 3, 6, 7, 14, 15: rvk.hip's
// pick_sample_s), defined in rvk_sample.hip's build of rvk.hip; nullptr when the shape has none
sample_launch_t pick_sample_fused(int mode, int np, bool multi, bool tp);
// MODE 2 / 3 with one planet, from rvk_sample1.hip's build
sample_launch_t pick_sample_fused_np1(int mode, bool multi, bool tp);

int fail(int code, const std::string &msg);

// Grow a device buffer to >= need bytes (contents dropped); the caller owns *p and frees it.
int grow_dev(void **p, size_t *cap, size_t need);

// Per-device copy of the sin/cos table, uploaded once per process (never freed).
int shared_table(int device, const SC **tab);

// Host-buffer transport of the blocking entry points (rvk_loglike, rvk_logpost, rvk_gp_logpost,
// rvk_gp_loglike; RVK_OPT_HOSTIO).  One call: up to kHostIoMaxIn caller input buffers and one
// output buffer.  Modes:
//   RVK_HOSTIO_PAGEABLE  hipMemcpyAsync straight from / to the caller's (pageable) buffers;
//   RVK_HOSTIO_PINNED    one memcpy into a pinned staging buffer, ONE DMA of all inputs into a
//                        device buffer of the same layout, the kernels, one DMA of the output back;
//   RVK_HOSTIO_ZEROCOPY  memcpy into the (fine-grained, device-visible) pinned staging buffer and
//                        the kernels read their inputs from it and write their output into it
//                        over PCIe -- no copy engine on the call's path;
//   RVK_HOSTIO_AUTO      zero-copy up to kZeroCopyMaxBytes of input, pinned DMA above.
// Staging and device buffers belong to the owning object and grow on demand.
constexpr int kHostIoMaxIn = 2;
constexpr size_t kZeroCopyMaxBytes = size_t(1) << 20;
struct HostIO {
    char *h = nullptr;          // pinned staging (hipHostMallocCoherent)
    char *hd = nullptr;         // its device-visible address
    size_t hcap = 0;
    char *d = nullptr;          // device copy of the inputs and the output (PAGEABLE / PINNED)
    size_t dcap = 0;
    int mode = 0;               // resolved mode of the call in flight
    size_t off_out = 0;         // output offset in h / d
    void release();
    // Stage the inputs; on return dev_in[i] / *dev_out are what the kernels use.
    int begin(int opt, hipStream_t st, int n_in, const void *const *src, const size_t *bytes, size_t out_bytes,
              const void **dev_in, void **dev_out);
    // Wait for the stream and deliver the output into the caller's buffer.
    int end(hipStream_t st, void *out, size_t out_bytes);
};

// Draw blocks (and the device stretch move's cached graphs) are a multiple of this many steps.
constexpr int kStepsPerGraph = 8;

// The stretch move's device draws (split_draws_kernel) for a block of steps: table[s][half][j]
// for steps step0 .. step0 + steps - 1, plus the kernel's scratch.  Owned by a posterior.
struct DrawTable {
    PreDraw *block = nullptr;
    uint32_t *keys = nullptr;
    int32_t *sets = nullptr;
    size_t cap_block = 0, cap_keys = 0, cap_sets = 0;   // bytes
    long long H = 0;                                     // walkers per half of the current content
    int steps = 0;
    void release();
};

// Fill `t` with the draws of n_steps steps from global step step0 (RVK_STRETCH_* flags), stream-ordered;
// with host draws (run.set != NULL) from those instead.
int draws_fill(DrawTable &t, hipStream_t st, long long H, int n_steps, int D, uint64_t seed, uint64_t step0, double a,
               int flags);
int draws_fill_host(DrawTable &t, hipStream_t st, long long H, int n_steps, int D, const RunArgs &run);
// Steps per draw block for H walkers per half: a multiple of kStepsPerGraph, table <= 256 MB.
int draws_block_steps(long long H);

}  // namespace rvk

// As HIPCHK, but first drains `stream`, so no async copy into a caller's buffer is still in
// flight when the error is returned (the host-buffer entry points).
#define HIPCHK_SYNC(stream, expr)                                                             \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess) {                                                               \
            (void)hipStreamSynchronize(stream);                                               \
            return rvk::fail(RVK_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));   \
        }                                                                                     \
    } while (0)

#define HIPCHK(expr)                                                                          \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess)                                                                 \
            return rvk::fail(RVK_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));   \
    } while (0)

struct rvk_handle {
    int device = 0;
    hipStream_t stream = nullptr;
    int n = 0, n_inst = 1, n_planets = 1, par = 0;
    double t0 = 0.0;
    double *d_t = nullptr, *d_vel = nullptr, *d_s2 = nullptr;
    rvk::SC *d_tab = nullptr;
    int32_t *d_inst = nullptr;
    // scratch for the host-buffer entry points (rvk_loglike, rvk_predict), grown on demand
    double *d_theta = nullptr, *d_out = nullptr, *d_tq = nullptr;
    int32_t *d_iq = nullptr;
    size_t cap_theta = 0, cap_out = 0, cap_tq = 0, cap_iq = 0;
    rvk::loglike_launch_t launch = nullptr;
    rvk::sample_launch_t sample = nullptr;   // fused stretch-move half-step (production solver)
    // ... with the proposals made in the same kernel, and proposals + log-posterior only
    // (rvk_stretch_propose); [1]: every prior kind, [2]: + the prior-side conversion in the prep
    rvk::sample_launch_t sample_fused[3] = {nullptr, nullptr, nullptr};
    rvk::sample_launch_t sample_eval[3] = {nullptr, nullptr, nullptr};
    // ... and the given free coordinates' log-posteriors (rvk_logpost_device in one kernel)
    rvk::sample_launch_t sample_direct[3] = {nullptr, nullptr, nullptr};
    int solver = 0;
    int graph = 0;                           // RVK_OPT_GRAPH
    int lpw = 0;                             // RVK_OPT_LPW
    int hostio = RVK_HOSTIO_AUTO;            // RVK_OPT_HOSTIO, shared by the posteriors built on the handle
    int poison = 0;                          // RVK_OPT_LDS_POISON
    int s2ok = 0;                            // EpochData::s2ok
    rvk::HostIO io;                          // rvk_loglike's transport
    // Held by every blocking (host-buffer) entry point of this handle and of the posteriors /
    // GP objects built on it: they share the handle's stream and staging (include/rvk.h).
    std::mutex mu;

    rvk::EpochData epochs() const { return rvk::EpochData{d_t, d_vel, d_s2, d_inst, d_tab, t0, par, lpw, n_planets, poison, s2ok}; }
    int p_full() const { return 5 * n_planets + 2 * n_inst + 2; }
};
