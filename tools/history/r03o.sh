# bisect the round-3 cfg3 kernel time across this round's kernel commits (kbench A/B, interleaved)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03o
mkdir -p $O
cd $R
for r in 1 2 3; do
for v in r02 caa0ee79 c042c0d4 c1de22a4 c0398e33 cur; do
  BLT_LIB_PATH=$R/build/exp/libblt_bpe_$v.so timeout -k 10 180 python tools/kbench.py --only cfg2,cfg3,cfg5 --reps 30 --tag $v >> $O/kb.jsonl 2>> $O/kb.err
done
done
python - <<'PY'
import json,collections
d=collections.defaultdict(list)
for l in open("gpurun_out/r03o/kb.jsonl"):
    j=json.loads(l); d[(j["tag"],j["cfg"])].append(j["ms"])
for k in sorted(d): print(k, [round(x,4) for x in d[k]], round(sum(d[k])/len(d[k]),4))
PY
