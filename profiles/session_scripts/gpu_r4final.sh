#!/bin/bash
# Round-4 closing session: GPU tests, smoke, the driver's bench line, the same command under
# rocprofv3 --kernel-trace --stats (stats kept, raw traces dropped), and the N>1 path on a
# world-size-1 RCCL group.  Usage: bash profiles/session_scripts/gpu_r4final.sh TAG
TAG=${1:-r4final}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" $O/pytest_gpu.log | head; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 > $O/bench_under_rocprof.json 2> $O/rocprof.err || { tail -20 $O/rocprof.err; exit 1; }
find $O/prof -type f ! -name "*stats*" -delete
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29561 --log-dir $O/tr_logs --redirects 3 --tee 3 bench.py --group --steps 20 --warmup 5 --no-cpu-baseline --no-gp --no-predictive --no-host-path > $O/bench_group.out 2> $O/bench_group.err || { tail -30 $O/bench_group.err; exit 1; }
python - "$O" <<'PY'
import json, sys, glob
O = sys.argv[1]
lines = [l.split("]:", 1)[1] if l.startswith("[default") else l for l in open(O + "/bench_group.out")]
js = [l for l in lines if l.lstrip().startswith("{")]
json.dump(json.loads(js[-1]), open(O + "/bench_group.json", "w"), indent=1)
d = json.load(open(O + "/bench.json"))
g = json.load(open(O + "/bench_group.json"))
print("value", d["value"], "ms/step", d["ms_per_step"] * 1e3, "kernel us", d["kernel_ms"] * 1e3, "host call us", d["host_path_ms_per_call"] * 1e3)
print("roofline", d["roofline"])
print("sampler", {k: v for k, v in d.get("sampler", {}).items() if "ms" in k})
print("gp", d["gp_config5"]["ms_per_eval"], d["gp_config5"]["fp64"]["ms_per_eval"])
print("group", g.get("process_group"), g["value"], g["logprob_agreement"]["ranks_bitwise_identical"])
PY
echo done
