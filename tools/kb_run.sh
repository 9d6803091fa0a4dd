#!/bin/bash
# GPU box: tools/kbench.py for each variant build/xp/libblt_bpe_NAME.so (kernel timings only).
#   gpurun -- 'bash tools/kb_run.sh TAG "cfg2,cfg3,cfg5" base e2 ...'
set -e
TAG=$1; ONLY=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for v in "$@"; do
  BLT_LIB_PATH=$R/build/xp/libblt_bpe_$v.so timeout -k 10 180 python tools/kbench.py --only "$ONLY" --tag "$v" ${KB_ARGS:-} >> "$O/kb.jsonl" 2>> "$O/kb.err"
done
cat "$O/kb.jsonl"
