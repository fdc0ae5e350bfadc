// rvk_sample1.hip -- the one-planet fused stretch-move half-step kernels with the basic priors
// (MODE 2 / 3: the config-2 sampler) as a translation unit of their own, under the max-ILP machine
// scheduler (Makefile); rvk.hip is the source (its RVK_TU_SAMPLE section), rvk_sample.hip builds the
// other proposal-making shapes.
#define RVK_TU_SAMPLE 2
#include "rvk.hip"
