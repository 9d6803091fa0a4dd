# A/B of an experiment variant against base on cfg2 and cfg3 (parity suites on the variant first)
set -e
V=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${2:-r03ao}
mkdir -p $O
cd $R
BLT_LIB_PATH=$R/build/exp/libblt_bpe_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_byte_tokenizer.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_$V.log 2>&1 || { tail -40 $O/tests_$V.log; exit 1; }
tail -1 $O/tests_$V.log
run() {  # name lib workload
  BLT_LIB_PATH=$R/build/exp/libblt_bpe_$2.so timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extra --workload $3 > $O/bench_$1.json 2> $O/bench_$1.err
  python -c "import json;d=json.load(open('$O/bench_$1.json'));r=d['roofline'];print('$1',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'])"
}
for k in 1 2 3; do
  run cfg2_base_$k base cfg2
  run cfg2_${V}_$k $V cfg2
done
for k in 1 2; do
  run cfg3_base_$k base cfg3
  run cfg3_${V}_$k $V cfg3
done
echo done
