set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03k
mkdir -p $O
cd $R
for r in 1 2; do
for f in "--events-outside-timed-loop" ""; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline $f > $O/b.json 2> $O/b.err
python -c "import json;d=json.load(open('$O/b.json'));print('$f', d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
done
done
