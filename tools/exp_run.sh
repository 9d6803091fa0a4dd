#!/bin/bash
# Timing experiments on the GPU box: the timing build's per-wave phase table, then the kernel
# time of each experiment build (parts of the work removed; wrong output by construction).
#   make exp EXPS="1 2 4 8"; gpurun -- 'bash tools/exp_run.sh TAG 1 2 4 8'
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 200 python tools/tile_timing.py > "$O/tile_timing.txt" 2>&1
head -20 "$O/tile_timing.txt"
for e in "$@"; do
  lib=build/exp/libblt_bpe_$e.so
  [ -f "$lib" ] || lib=build/exp/libblt_bpe_exp$e.so
  BLT_LIB_PATH=$R/$lib timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$O/bench_$e.json" 2> "$O/bench_$e.err" || true
  python - "$e" "$O/bench_$e.json" <<'PY'
import json, sys
try:
    j = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    print(f"exp {sys.argv[1]:>10s}: kernel {j['roofline']['kernel_ms']:.4f} ms  value {j['value']:.1f} GB/s")
except Exception as ex:
    print(f"exp {sys.argv[1]}: failed ({ex})")
PY
done
