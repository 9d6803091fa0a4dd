#!/bin/bash
# GPU box: the general multi-pass map rate (tools/config_rates.py --only multi) per variant build.
#   gpurun -- 'bash tools/multi_run.sh TAG tw4 tw2'
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for v in "$@"; do
  BLT_LIB_PATH=$R/build/exp/libblt_bpe_$v.so timeout -k 10 200 python tools/config_rates.py --only multi > "$O/multi_$v.json" 2>&1
  echo "$v $(grep -E '"ms"|bit_exact' "$O/multi_$v.json" | tr -d ' \n')"
done
