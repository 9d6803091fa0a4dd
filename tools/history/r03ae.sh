# CLI A/B on one box: device setup beside the mmap (default) vs after it (BLT_NO_PREWARM=1)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03ae
mkdir -p $O
cd $R
for r in 1 2; do
for mode in pre nopre; do
  if [ $mode = nopre ]; then export BLT_NO_PREWARM=1; else unset BLT_NO_PREWARM; fi
  BLT_CLI_TIMING=1 timeout -k 10 300 python tools/cli_rate.py --mib 1024 --dir /dev/shm --gpus 1 --no-oracle-time > $O/cli_$mode.json 2> $O/cli_$mode.err
  python -c "
import json;d=json.load(open('$O/cli_$mode.json'))
for k,v in d['runs'].items(): print('$mode', v['cli_seconds'], v['cli_input_GBps'], v['phases'].replace(chr(10),' | ')[:400])"
done
done
