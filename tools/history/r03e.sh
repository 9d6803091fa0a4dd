set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03e
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q ${TESTSEL:+-k "$TESTSEL"} --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 200 python tools/kbench.py --only cfg2,cfg3,cfg5 > $O/kb.jsonl 2>> $O/kb.err; cat $O/kb.jsonl
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --only-configs multi,wrap,selfval,chain > $O/bench_f2.json 2> $O/bench_f2.err
python -c "import json;d=json.load(open('$O/bench_f2.json'));print(json.dumps(d['configs'],indent=1))"
