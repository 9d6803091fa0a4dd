set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03m
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --only-configs multi,selfval,chain > $O/bench_f2.json 2> $O/bench_f2.err
python -c "import json;d=json.load(open('$O/bench_f2.json'));print({k:(v['ms'],v['frac'],v['u16_passes']) for k,v in d['configs'].items()})"
for r in 1 2; do
for f in "--events-outside-timed-loop" ""; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline $f > $O/b.json 2> $O/b.err
python -c "import json;d=json.load(open('$O/b.json'));print('$f', d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
done
done
