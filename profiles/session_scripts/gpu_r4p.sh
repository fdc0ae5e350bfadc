#!/bin/bash
# likelihood parity + kbench A/B of varlib/ll variants (3 interleaved reps) + sampler raw step
O=gpurun_out/r4p; mkdir -p $O/kb
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py tests/test_gpu_posterior.py tests/test_gpu_device_posterior.py tests/test_gpu_hostpath.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "^FAILED|Error" $O/pytest.log | head -5; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for so in ravest_amd/lib/librvk.so varlib/ll/librvk_*.so; do
    v=$(basename $so .so); [ "$so" = ravest_amd/lib/librvk.so ] && v=librvk_main
    RAVEST_AMD_LIB=$(realpath $so) timeout -k 10 200 python tools/kbench.py > $O/kb/kb_${v}_$rep.log 2>&1 || { echo "fail $v"; tail -3 $O/kb/kb_${v}_$rep.log; exit 1; }
    echo "$v sampler $(RAVEST_AMD_LIB=$(realpath $so) timeout -k 10 200 python tools/sampler_bench.py 4096 400 raw 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: round(v*1e3, 3) for k, v in d.items() if k.startswith("raw_ms")})')"
  done
done
python tools/ab_summary.py $O/kb
