# failure pattern of an experiment variant across the GPU parity suites (no -x)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${2:-r03ak}
mkdir -p $O
cd $R
BLT_LIB_PATH=$R/build/exp/libblt_bpe_$1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_byte_tokenizer.py -m gpu -q --timeout 120 --timeout-method thread -p no:randomly > $O/tests_$1.log 2>&1
grep -E "FAILED|passed|failed" $O/tests_$1.log | tail -40
exit 0
