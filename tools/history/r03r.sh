# CLI phase timing (BLT_CLI_TIMING) on tmpfs, 1 and 2 GiB
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03r
mkdir -p $O
cd $R
for m in 1024 2048; do
  BLT_CLI_TIMING=1 timeout -k 10 300 python tools/cli_rate.py --mib $m --dir /dev/shm --gpus 1 --no-oracle-time > $O/cli_$m.json 2> $O/cli_$m.err
  python -c "
import json;d=json.load(open('$O/cli_$m.json'))
for k,v in d['runs'].items(): print($m, k, v['cli_seconds'], v['cli_input_GBps']); print(v['phases'])"
done
