# fused passes 1 + 2: parity tests, then the general-map tests, then f2 rows fused vs two kernels
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03x
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/fused_tests.log 2>&1 || { tail -40 $O/fused_tests.log; exit 1; }
tail -1 $O/fused_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
