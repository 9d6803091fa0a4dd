# static first tickets in both scan kernels: full GPU suite on the product build, then prev/new A/B
# on cfg2, cfg3 and f2 (fused_rate multi: fused and two-kernel chains)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03ap}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
run() {  # name lib workload
  BLT_LIB_PATH=$R/build/exp/libblt_bpe_$2.so timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extra --workload $3 > $O/bench_$1.json 2> $O/bench_$1.err
  python -c "import json;d=json.load(open('$O/bench_$1.json'));r=d['roofline'];print('$1',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'])"
}
for k in 1 2; do
  for v in prev new; do
    run cfg2_${v}_$k $v cfg2
    run cfg3_${v}_$k $v cfg3
    BLT_LIB_PATH=$R/build/exp/libblt_bpe_$v.so timeout -k 10 200 python3 tools/fused_rate.py > $O/f2_${v}_$k.jsonl 2> $O/f2_${v}_$k.err
    sed "s/^/f2 $v $k /" $O/f2_${v}_$k.jsonl
  done
done
echo done
