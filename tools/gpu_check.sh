#!/bin/bash
# One GPU call: parity tests, smoke, bench, rocprofv3 kernel stats of the bench command.
#   gpurun --timeout 900 -- 'bash tools/gpu_check.sh TAG [pmc GROUPS]'
# Every GPU step runs under its own time limit; the chain stops at the first failure.
set -e
TAG=${1:-check}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { tail -40 "$O/gpu_tests.log"; exit 1; }
tail -3 "$O/gpu_tests.log"
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > "$O/smoke.log" 2>&1
tail -1 "$O/smoke.log"
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
cd /tmp && export TMPDIR=/tmp
for w in cfg3 cfg5 cfg2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$w" -o run -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-extra --workload $w > "$O/prof_$w.log" 2>&1
  find "$O/prof_$w" -name '*kernel_stats.csv' -exec head -3 {} \;
done
if [ "${2:-}" = pmc ]; then
  cd "$R"
  timeout -k 10 600 python tools/pmc_profile.py "$O/pmc" --groups ${3:-fetch,write} > "$O/pmc.log" 2>&1
  tail -5 "$O/pmc.log"
fi
