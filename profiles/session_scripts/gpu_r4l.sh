#!/bin/bash
TAG=${1:-r4l}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gp64.py tests/test_gpu_gp.py tests/test_gpu_hostpath.py tests/test_gpu_sampling.py tests/test_gpu_device_posterior.py tests/test_gpu_sampler_api.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "^FAILED|Error" $O/pytest.log | head -5; [ $rc -eq 0 ] || exit 1
REPS=3 SKIPTEST=1 bash tools/gp64_ab.sh ${TAG}_g64 fp64 || exit 1
for rep in 1 2 3; do
  for so in ravest_amd/lib/librvk.so varlib/samp/librvk_*.so; do
    v=$(basename $so .so); [ "$so" = ravest_amd/lib/librvk.so ] && v=main
    echo "$v $(RAVEST_AMD_LIB=$(realpath $so) timeout -k 10 200 python tools/sampler_bench.py 4096 400 raw 2>/dev/null | tail -1 | cut -c1-400)"
  done
done
