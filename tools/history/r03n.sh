set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03n
mkdir -p $O
cd $R
for w in 5 20 60 5; do
timeout -k 10 300 python bench.py --steps 20 --warmup $w --no-extra --no-cpu-baseline > $O/b.json 2> $O/b.err
python -c "import json;d=json.load(open('$O/b.json'));print('w=$w', d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
done
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-extra --no-cpu-baseline > $O/b.json 2> $O/b.err
python -c "import json;d=json.load(open('$O/b.json'));print('steps100', d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
for r in 1 2; do
for v in r02 cur; do
  BLT_LIB_PATH=$R/build/exp/libblt_bpe_$v.so timeout -k 10 180 python tools/kbench.py --only cfg2,cfg3,cfg5 --reps 30 --tag $v >> $O/kb.jsonl 2>> $O/kb.err
done
done
python - <<'PY'
import json,collections
d=collections.defaultdict(list)
for l in open("gpurun_out/r03n/kb.jsonl"):
    j=json.loads(l); d[(j["tag"],j["cfg"])].append(j["ms"])
for k in sorted(d): print(k, [round(x,4) for x in d[k]])
PY
