set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r02s4_toks; mkdir -p $O; cd $R
PYTEST_K=token_scan timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "token_scan or general or chained or wrapping or pipeline_text or multipass" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for v in toks2 toks1 toks2 toks1; do
  BLT_LIB_PATH=$R/build/exp/libblt_bpe_$v.so timeout -k 10 200 python tools/config_rates.py --only multi > $O/multi_$v.json 2>&1
  echo "$v $(grep -E '"ms"|bit_exact' $O/multi_$v.json | tr -d ' \n')"
done
BLT_LIB_PATH=$R/build/exp/libblt_bpe_timing2.so timeout -k 10 200 python tools/tok_timing.py > $O/tok2.txt 2>&1; tail -18 $O/tok2.txt
