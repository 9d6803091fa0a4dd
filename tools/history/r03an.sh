# small-map table fill: parity suites on the product build, then cfg2 / cfg3 A/B (list fill vs whole-table copy)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03an}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_byte_tokenizer.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name lib workload
  BLT_LIB_PATH=$R/build/exp/libblt_bpe_$2.so timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extra --workload $3 > $O/bench_$1.json 2> $O/bench_$1.err
  python -c "import json;d=json.load(open('$O/bench_$1.json'));r=d['roofline'];print('$1',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'])"
}
for k in 1 2 3; do
  run cfg2_nosp_$k nosp cfg2
  run cfg2_sp_$k sp cfg2
done
run cfg3_nosp nosp cfg3
run cfg3_sp sp cfg3
echo done
