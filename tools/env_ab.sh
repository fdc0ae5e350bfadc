O=gpurun_out/env1; mkdir -p $O
OFF="--no-cpu-baseline --no-gp --no-predictive --no-host-path --no-sampler --no-configs"
for rep in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 $OFF > $O/base_$rep.json 2>/dev/null || exit 1
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 $OFF > $O/kern_$rep.json 2>/dev/null || exit 1
  HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 python bench.py --steps 20 --warmup 5 $OFF > $O/nokern_$rep.json 2>/dev/null || exit 1
done
for f in $O/*.json; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step']*1e3,3), round(d['kernel_ms']*1e3,3))"; done
