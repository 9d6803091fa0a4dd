# Sparse-emission ablations (timing only, wrong output): 1 no stage writes, 2 no stage reads,
# 4 no copy-out stores, 8 no sparse emission at all; 0 = the product
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03v
mkdir -p $O
cd $R
for r in 1 2; do
for v in abl0 abl1 abl2 abl4 abl8; do
  BLT_LIB_PATH=$R/build/exp/libblt_bpe_$v.so timeout -k 10 180 python tools/kbench.py --only cfg2,cfg3,cfg5 --reps 30 --tag $v >> $O/kb.jsonl 2>> $O/kb.err
done
done
python - <<'PY'
import json,collections
d=collections.defaultdict(list)
for l in open("gpurun_out/r03v/kb.jsonl"):
    j=json.loads(l); d[(j["tag"],j["cfg"])].append(j["ms"])
for k in sorted(d): print(k, [round(x,4) for x in d[k]], round(sum(d[k])/len(d[k]),4))
PY
