# final check of the round's tree: GPU tests, smoke, the driver's bench command
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03af
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
python -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print(d['value'],r['kernel_ms'],r['frac'],r['traffic'],r.get('traffic_source'),{k:v.get('frac') for k,v in d['configs'].items()}, d['cli_end_to_end']['value'])"
