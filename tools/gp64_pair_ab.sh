#!/bin/bash
# fp64 config-5 timing, base vs varlib/librvk_<v>.so (3 reps interleaved); when the variant is >= 3 % faster,
# its GP parity tests.  usage: bash tools/gp64_pair_ab.sh TAG v
O=gpurun_out/${1:-pair}; v=${2:-pair}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  timeout -k 10 120 python tools/gp_bench.py 4096 512 fp64 > $O/base_$rep.json 2>/dev/null || { echo "fail base"; exit 1; }
  RAVEST_AMD_LIB=varlib/librvk_$v.so timeout -k 10 120 python tools/gp_bench.py 4096 512 fp64 > $O/${v}_$rep.json 2>$O/${v}_$rep.err || { echo "fail $v"; tail -5 $O/${v}_$rep.err; exit 1; }
  python -c "import json; a=json.load(open('$O/base_$rep.json')); b=json.load(open('$O/${v}_$rep.json')); print('base', round(a['ms_per_eval'],3), '$v', round(b['ms_per_eval'],3), 'err', b['max_rel_err_vs_fp64_oracle_64w'], b['mask_identical'])"
done
win=$(python -c "
import json, numpy as np
a=np.median([json.load(open('$O/base_%d.json'%r))['ms_per_eval'] for r in (1,2,3)])
b=np.median([json.load(open('$O/${v}_%d.json'%r))['ms_per_eval'] for r in (1,2,3)])
print(1 if b < 0.97*a else 0)")
echo "win=$win"
if [ "$win" = 1 ]; then
  RAVEST_AMD_LIB=varlib/librvk_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_gp64.py tests/test_gpu_gp.py tests/test_gpu_predictive.py -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v tests: $(tail -1 $O/pytest_$v.log)"
fi
echo done
