# A/B on one box: byte kernel without the self-reset tail (reset every step) vs with it
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03ah}
mkdir -p $O
cd $R
run() {  # name lib extra-args
  BLT_LIB_PATH=$R/build/exp/libblt_bpe_$2.so timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extra $3 > $O/bench_$1.json 2> $O/bench_$1.err
  python -c "import json;d=json.load(open('$O/bench_$1.json'));r=d['roofline'];print('$1',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'])"
}
for k in 1 2 3; do
  run nosr_reset_$k nosr --reset-each-step
  run sr_reset_$k sr --reset-each-step
  run sr_$k sr ""
done
echo done
