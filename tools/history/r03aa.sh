# A/B: ticket claimed by the look-back wave beside its status loads (tk1) vs wave 1 at the
# iteration start (tk0, the product)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03aa
mkdir -p $O
cd $R
BLT_LIB_PATH=$R/build/exp/libblt_bpe_tk1.so timeout -k 10 300 python tools/kbench.py --only cfg2,cfg3,cfg5 --reps 5 --check --tag chk_tk1 > $O/chk.jsonl 2>> $O/kb.err
cat $O/chk.jsonl
for r in 1 2 3; do
for v in tk0 tk1; do
  BLT_LIB_PATH=$R/build/exp/libblt_bpe_$v.so timeout -k 10 180 python tools/kbench.py --only cfg2,cfg3,cfg5 --reps 30 --tag $v >> $O/kb.jsonl 2>> $O/kb.err
done
done
python - <<'PY'
import json,collections
d=collections.defaultdict(list)
for l in open("gpurun_out/r03aa/kb.jsonl"):
    j=json.loads(l); d[(j["tag"],j["cfg"])].append(j["ms"])
for k in sorted(d): print(k, [round(x,4) for x in d[k]], round(sum(d[k])/len(d[k]),4))
PY
