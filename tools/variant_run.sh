#!/bin/bash
# GPU box: parity tests + bench for each experiment variant build/xp/libblt_bpe_NAME.so.
#   gpurun -- 'bash tools/variant_run.sh TAG base pf ...'   (NAME:t = tile timing of that build,
#   NAME:b = bench only)
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for v in "$@"; do
  case $v in
    *:t) n=${v%:t}; BLT_LIB_PATH=$R/build/xp/libblt_bpe_$n.so timeout -k 10 200 python tools/tile_timing.py > "$O/timing_$n.txt" 2>&1
         head -18 "$O/timing_$n.txt"; continue;;
    *:tr) n=${v%:tr}; BLT_LIB_PATH=$R/build/xp/libblt_bpe_$n.so timeout -k 10 200 python tools/tile_timing.py --random > "$O/timing_r_$n.txt" 2>&1
         head -18 "$O/timing_r_$n.txt"; continue;;
  esac
  notest=0
  case $v in *:b) v=${v%:b}; notest=1;; esac   # NAME:b = bench only (timing experiments with wrong output)
  export BLT_LIB_PATH=$R/build/xp/libblt_bpe_$v.so
  if [ $notest = 0 ] && ! timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/tests_$v.log" 2>&1; then
    echo "variant $v: TESTS FAILED"; tail -30 "$O/tests_$v.log"; exit 1
  fi
  for k in 1 2; do
    timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > "$O/bench_${v}_$k.json" 2> "$O/bench_${v}_$k.err"
    python - "$v" "$O/bench_${v}_$k.json" <<'PY'
import json, sys
j = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"variant {sys.argv[1]:>10s}: kernel {j['roofline']['kernel_ms']:.4f} ms  value {j['value']:.1f} GB/s  frac {j['roofline']['frac']}")
PY
  done
  unset BLT_LIB_PATH
done
