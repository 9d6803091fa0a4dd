# A/B: loop-head vmcnt(0) (ev0, the round-3 product) vs the wait ahead of the emission stores
# (ev1) and with the ticket atomic left alone by the atomic optimizer (ev2); kbench + f2 multi
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03t
mkdir -p $O
cd $R
for v in ev1 ev2; do
  BLT_LIB_PATH=$R/build/exp/libblt_bpe_$v.so timeout -k 10 300 python tools/kbench.py --only cfg2,cfg3,cfg5 --reps 5 --check --tag chk_$v >> $O/chk.jsonl 2>> $O/kb.err
done
cat $O/chk.jsonl
for r in 1 2 3; do
for v in ev0 ev1 ev2; do
  BLT_LIB_PATH=$R/build/exp/libblt_bpe_$v.so timeout -k 10 180 python tools/kbench.py --only cfg2,cfg3,cfg5 --reps 30 --tag $v >> $O/kb.jsonl 2>> $O/kb.err
  BLT_LIB_PATH=$R/build/exp/libblt_bpe_$v.so timeout -k 10 180 python tools/config_rates.py --only multi > $O/multi_$v.json 2>>$O/kb.err; python -c "
import json;d=json.load(open('$O/multi_$v.json'));print('$v multi', d if not isinstance(d,dict) else {k:d[k] for k in d if k in ('ms','frac','bit_exact','multi')})" >> $O/multi.txt
done
done
cat $O/multi.txt
python - <<'PY'
import json,collections
d=collections.defaultdict(list)
for l in open("gpurun_out/r03t/kb.jsonl"):
    j=json.loads(l); d[(j["tag"],j["cfg"])].append(j["ms"])
for k in sorted(d): print(k, [round(x,4) for x in d[k]], round(sum(d[k])/len(d[k]),4))
PY
