#!/bin/bash
# GPU box: the GPU tests, then bench.py; prints the host-path rates of the bench line.
#   gpurun -- 'bash tools/stage_check.sh TAG'
set -e
TAG=${1:-stage}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
print(d["value"], d["end_to_end"], d["per_chunk_path"])
PY
