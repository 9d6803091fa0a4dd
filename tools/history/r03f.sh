set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03f
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for r in 1 2; do
for v in nooob oob; do
  BLT_LIB_PATH=$R/build/exp/libblt_bpe_$v.so timeout -k 10 180 python tools/kbench.py --only cfg2,cfg3,cfg5 --tag $v >> $O/kb.jsonl 2>> $O/kb.err
  BLT_LIB_PATH=$R/build/exp/libblt_bpe_$v.so timeout -k 10 180 python tools/config_rates.py --only multi > $O/multi_$v.json 2>>$O/kb.err; grep -E '"ms"|frac' $O/multi_$v.json | tr -d '\n'; echo " $v"
done
done
cat $O/kb.jsonl
