#!/bin/bash
# The fused half-step / DIRECT log-posterior kernels after a change: their GPU tests, then the sampler
# steps of every bench posterior (tools/sampler_ab.sh against varlib/librvk_*.so, if any).
TAG=${1:?tag}; REPS=${2:-2}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_posterior.py tests/test_gpu_sampler_api.py tests/test_gpu_sampling.py \
  tests/test_gpu_sharded_sampler.py tests/test_gpu_posterior.py tests/test_gpu_lds_poison.py -m gpu -x -q --timeout 180 \
  --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
echo "tests: $(tail -1 $O/pytest.log)"
bash tools/sampler_ab.sh $TAG $REPS uniform beta vaneylen cfg3 cfg4
