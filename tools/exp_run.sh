#!/bin/bash
# GPU box: byte-pass kernel timings (tools/kbench.py), the general multi-pass rate
# (tools/config_rates.py --only multi) and u16-pass phase timing (tools/tok_timing.py, timing builds)
# for a list of variant builds build/xp/libblt_bpe_NAME.so.
#   gpurun -- 'bash tools/exp_run.sh TAG "base tke" "timing timingtke"'
set -e
TAG=$1; VARS=$2; TVARS=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for v in $VARS; do
  BLT_LIB_PATH=$R/build/xp/libblt_bpe_$v.so timeout -k 10 180 python tools/kbench.py --only ${KB_ONLY:-cfg2,cfg3,cfg5} --tag "$v" ${KB_ARGS:-} >> "$O/kb.jsonl" 2>> "$O/kb.err"
  BLT_LIB_PATH=$R/build/xp/libblt_bpe_$v.so timeout -k 10 200 python tools/config_rates.py --only multi > "$O/multi_$v.json" 2>&1
  echo "$v multi $(grep -E '"ms"|bit_exact' "$O/multi_$v.json" | tr -d ' \n')"
done
cat "$O/kb.jsonl"
for v in $TVARS; do
  BLT_LIB_PATH=$R/build/xp/libblt_bpe_$v.so timeout -k 10 200 python tools/tok_timing.py > "$O/tok_$v.txt" 2>&1
  echo "== $v"; tail -17 "$O/tok_$v.txt"
done
