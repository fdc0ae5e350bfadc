export TMPDIR=/tmp
O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -k "predict" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/host_phase_probe.py 4096 > $O/phase4096.json 2>$O/phase.err && timeout -k 10 120 python tools/host_phase_probe.py 2048 > $O/phase2048.json 2>>$O/phase.err || { tail $O/phase.err; exit 1; }
cat $O/phase4096.json $O/phase2048.json
bash tools/pmc_write_probe.sh $O/wp || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sampler --no-gp --no-configs --no-host-path > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(json.dumps(d.get('predictive'))[:600])"
