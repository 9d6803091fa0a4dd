# Round-3 final measurements (final kernel source): tests, smoke, the driver's bench command,
# rocprofv3 kernel stats, PMC traffic + instruction counters for cfg3/cfg5/cfg2 and traffic for
# cfg4's per-rank shard sizes at N = 2/4/8 (4/2/1 GiB)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03ad}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
python -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print(d['value'],r['kernel_ms'],r['frac'],r['traffic'],{k:v.get('frac') for k,v in d['configs'].items()})"
cd /tmp && export TMPDIR=/tmp
for w in cfg3 cfg5 cfg2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --workload $w > $O/prof_$w.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_f2 -o run -- python3 $R/tools/config_rates.py > $O/prof_f2.log 2>&1
cd $R
for w in cfg3 cfg5 cfg2; do
  timeout -k 10 600 python tools/pmc_profile.py $O/pmc_$w --groups fetch,write,insts -- --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $O/pmc_$w.log 2>&1
done
for g in 1 2 4; do
  timeout -k 10 600 python tools/pmc_profile.py $O/pmc_cfg4_$g --groups fetch,write -- --workload cfg4 --total-bytes $((g << 30)) --steps 3 --warmup 1 --no-cpu-baseline --no-extra > $O/pmc_cfg4_$g.log 2>&1
done
echo done
