set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03ac
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/fused_rate.py --map chain --reps 3 > $O/prof.log 2>&1
head -14 $O/prof/run_kernel_stats.csv | cut -c1-150
