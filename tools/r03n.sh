set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03n
mkdir -p $O
cd $R
for w in 5 20 60 5; do
timeout -k 10 300 python bench.py --steps 20 --warmup $w --no-extra --no-cpu-baseline --events-in-timed-loop > $O/b.json 2> $O/b.err
python -c "import json;d=json.load(open('$O/b.json'));print('w=$w', d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
done
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-extra --no-cpu-baseline --events-in-timed-loop > $O/b.json 2> $O/b.err
python -c "import json;d=json.load(open('$O/b.json'));print('steps100', d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
