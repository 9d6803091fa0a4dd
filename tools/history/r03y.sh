# fused passes 1 + 2 vs two kernels: wall-clock rate and rocprofv3 kernel stats
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03y
mkdir -p $O
cd $R
timeout -k 10 300 python tools/fused_rate.py --map multi > $O/rate_multi.jsonl 2> $O/rate.err
cat $O/rate_multi.jsonl
timeout -k 10 300 python tools/fused_rate.py --map selfval > $O/rate_selfval.jsonl 2>> $O/rate.err
cat $O/rate_selfval.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/fused_rate.py --map multi --reps 10 > $O/prof.log 2>&1
head -12 $O/prof/run_kernel_stats.csv | cut -c1-160
