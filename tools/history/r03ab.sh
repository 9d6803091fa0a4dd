# fused kernel: fused tests, general-map tests, f2 rows (async ms / sync ms)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03ab
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fused or token_scan or general or chained or wrapping or self_valued or live" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --only-configs multi,selfval,chain --steps 5 --warmup 2 > $O/b.json 2> $O/b.err
python -c "
import json;d=json.load(open('$O/b.json'))
print({k:(v.get('ms'), v.get('sync_ms'), v.get('sync_path'), v.get('bit_exact_vs_oracle')) for k,v in d['configs'].items()})"
