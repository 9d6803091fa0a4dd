# prev/new A/B on cfg3 (4 alternating runs each) and cfg5 (2 each)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03aq}
mkdir -p $O
cd $R
run() {  # name lib workload
  BLT_LIB_PATH=$R/build/exp/libblt_bpe_$2.so timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extra --workload $3 > $O/bench_$1.json 2> $O/bench_$1.err
  python -c "import json;d=json.load(open('$O/bench_$1.json'));r=d['roofline'];print('$1',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'])"
}
for k in 1 2 3 4; do
  run cfg3_prev_$k prev cfg3
  run cfg3_new_$k new cfg3
done
for k in 1 2; do
  run cfg5_prev_$k prev cfg5
  run cfg5_new_$k new cfg5
done
echo done
