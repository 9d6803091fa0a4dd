set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03j
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for r in 1 2 3; do
for v in noearly early; do
  BLT_LIB_PATH=$R/build/exp/libblt_bpe_$v.so timeout -k 10 180 python tools/kbench.py --only cfg2,cfg3,cfg5,text1 --reps 30 --tag $v >> $O/kb.jsonl 2>> $O/kb.err
done
done
python - <<'PY'
import json,collections
d=collections.defaultdict(list)
for l in open("gpurun_out/r03j/kb.jsonl"):
    j=json.loads(l); d[(j["tag"],j["cfg"])].append(j["ms"])
for k in sorted(d): print(k, [round(x,4) for x in d[k]])
PY
