#!/bin/bash
# sampler parity + fused half-step A/B (prologue ordering, draw prefetch)
O=gpurun_out/r4o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_device_posterior.py tests/test_gpu_sampler_api.py tests/test_gpu_sampling.py tests/test_gpu_hostpath.py tests/test_gpu_sharded_sampler.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "^FAILED|Error" $O/pytest.log | head -5; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for so in ravest_amd/lib/librvk.so varlib/samp/librvk_*.so; do
    v=$(basename $so .so); [ "$so" = ravest_amd/lib/librvk.so ] && v=main
    echo "$v $(RAVEST_AMD_LIB=$(realpath $so) timeout -k 10 200 python tools/sampler_bench.py 4096 400 raw 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: round(v*1e3, 3) for k, v in d.items() if k.startswith("raw_ms")})')"
  done
done
