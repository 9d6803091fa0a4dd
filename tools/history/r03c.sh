set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03c
mkdir -p $O
cd $R
for m in 128 256 512 1024 2048 4096; do
  timeout -k 10 200 python tools/kbench.py --only cfg3,cfg5 --mib $m --tag m$m >> $O/kb_sizes.jsonl 2>> $O/kb.err
done
cat $O/kb_sizes.jsonl
timeout -k 10 300 python tools/host_path_rate.py --gpus 1,8 --no-cfg2 > $O/host_path.json 2> $O/host_path.err
cat $O/host_path.json
timeout -k 10 300 python tools/cli_rate.py --mib 2048 --gpus 1,8 > $O/cli.json 2> $O/cli.err
cat $O/cli.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_f2 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --only-configs multi,wrap,selfval,chain > $O/prof_f2.log 2>&1
find $O/prof_f2 -name '*kernel_stats.csv' -exec cat {} \;
cd $R
timeout -k 10 600 python tools/pmc_profile.py $O/pmc_cfg3 --groups fetch,write > $O/pmc_cfg3.log 2>&1
cat $O/pmc_cfg3/traffic.json
