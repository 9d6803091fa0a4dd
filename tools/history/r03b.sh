set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03b
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python tools/host_path_rate.py --gpus 1,2,8 --no-cfg2 > $O/host_path.json 2> $O/host_path.err
cat $O/host_path.json
timeout -k 10 300 python tools/cli_rate.py --mib 2048 --gpus 1,2,8 > $O/cli.json 2> $O/cli.err
cat $O/cli.json
BLT_BENCH_BACKEND=gloo BLT_BENCH_DEVICE=0 timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 > $O/rehearse_n2.json 2> $O/rehearse_n2.err || { tail -30 $O/rehearse_n2.err; exit 1; }
cat $O/rehearse_n2.json
