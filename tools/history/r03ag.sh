# self-resetting byte kernels: targeted tests, bench A/B (reset every step vs one reset), kernel trace
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03ag}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_new_$r.json 2> $O/bench_new_$r.err
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --reset-each-step > $O/bench_old_$r.json 2> $O/bench_old_$r.err
done
for f in $O/bench_*.json; do python -c "import json,sys;d=json.load(open('$f'));r=d['roofline'];print('$f'.split('/')[-1],d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'])"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg3 -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/prof_cfg3.log 2>&1
echo done
