# rocprofv3 kernel stats of the f2 config rows (multi, wrap, selfval, chain) on the current kernel source
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03ar}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_f2 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --only-configs multi,wrap,selfval,chain > $O/bench_f2.json 2> $O/bench_f2.err
find $O/prof_f2 -name '*kernel_stats.csv' -exec cut -c1-160 {} \;
