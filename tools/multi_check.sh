#!/bin/bash
# GPU box: the GPU test suite, then the general multi-pass map rate and its rocprofv3 kernel stats.
#   gpurun -- 'bash tools/multi_check.sh TAG'
set -e
TAG=${1:-multi}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$O/gpu_tests.log" 2>&1 || { tail -40 "$O/gpu_tests.log"; exit 1; }
tail -3 "$O/gpu_tests.log"
timeout -k 10 200 python tools/config_rates.py --only multi > "$O/multi.json" 2>&1
cat "$O/multi.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_multi" -o run -- python3 "$R/tools/config_rates.py" --only multi > "$O/prof_multi.log" 2>&1
find "$O/prof_multi" -name '*kernel_stats.csv' -exec cat {} \;
