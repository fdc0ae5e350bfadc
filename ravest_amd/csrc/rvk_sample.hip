// rvk_sample.hip -- the fused stretch-move half-step kernels (the loglike_kernel instantiations that
// make their own proposals: MODE 2 / 3 and their all-priors / conversion forms) as a translation unit
// of their own, so the Makefile can give them a different machine scheduler than the plain
// likelihood kernels (rvk.hip, which is this file's source: see its RVK_TU_SAMPLE section).
#define RVK_TU_SAMPLE 1
#include "rvk.hip"
