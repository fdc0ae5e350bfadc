O=gpurun_out/abl
mkdir -p $O
for v in abl1 abl2 abl3; do
  RAVEST_AMD_LIB=build/variants/librvk_$v.so timeout -k 10 100 python tools/gp_bench.py > $O/$v.json 2>/dev/null || echo fail $v
  echo "$v $(cut -c1-160 $O/$v.json)"
done
RAVEST_AMD_LIB=build/variants/librvk_trabl1.so timeout -k 10 100 python tools/gp_trace.py > $O/trabl1.txt 2>&1
