set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/v33
bash tools/variant_run.sh v33 w16 w8
for v in w16 w8; do BLT_LIB_PATH=$R/build/exp/libblt_bpe_$v.so timeout -k 10 200 python tools/config_rates.py --only cfg2,cfg5 > gpurun_out/v33/rates_$v.json 2>&1; echo $v $(grep '"ms"' gpurun_out/v33/rates_$v.json); done
