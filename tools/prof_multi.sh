#!/bin/bash
# GPU box: rocprofv3 kernel trace + stats of the general multi-pass map (tools/config_rates.py --only multi)
# and a kernel-time size sweep of cfg2's text (tools/kbench.py textN).
#   gpurun -- 'bash tools/prof_multi.sh TAG'
set -e
TAG=${1:-multi}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 200 python tools/kbench.py --only ${KB_ONLY:-text1,text4,text16,text50,text100,text400} > "$O/kb_sizes.jsonl" 2> "$O/kb_sizes.err"
cat "$O/kb_sizes.jsonl"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_multi" -o run -- python3 "$R/tools/config_rates.py" --only multi > "$O/prof_multi.log" 2>&1
find "$O/prof_multi" -name '*kernel_stats.csv' -exec cat {} \;
