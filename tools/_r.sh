set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/v29
bash tools/variant_run.sh v29 co
BLT_LIB_PATH=$R/build/exp/libblt_bpe_co.so timeout -k 10 200 python tools/config_rates.py --only cfg2,cfg5 > gpurun_out/v29/rates.json 2>&1; grep '"ms"\|input_GBps' gpurun_out/v29/rates.json
