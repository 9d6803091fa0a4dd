#!/bin/bash
# GPU box: the general-map GPU tests, then the multi-pass rate of each variant build.
#   gpurun -- 'bash tools/toks_run.sh TAG "v1 v2"'
set -e
TAG=$1; VARS=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "token_scan or general or chained or wrapping or pipeline_text or multipass" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for v in $VARS; do
  if [ "$v" = product ]; then L=$R/blt_amd/libblt_bpe.so; else L=$R/build/exp/libblt_bpe_$v.so; fi
  BLT_LIB_PATH=$L timeout -k 10 200 python tools/config_rates.py --only multi > $O/multi_$v.json 2>&1
  echo "$v $(grep -E '"ms"|bit_exact' $O/multi_$v.json | tr -d ' \n')"
done
