set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03a
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python tools/host_path_rate.py --gpus 1,2,8 --no-cfg2 > $O/host_path.json 2> $O/host_path.err
cat $O/host_path.json
timeout -k 10 300 python tools/cli_rate.py --mib 2048 --gpus 1,8 > $O/cli.json 2> $O/cli.err
cat $O/cli.json
