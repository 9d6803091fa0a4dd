set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/v25
bash tools/variant_run.sh v25 st stt:tr
BLT_LIB_PATH=$R/build/exp/libblt_bpe_st.so timeout -k 10 200 python tools/config_rates.py --only cfg2,cfg5 > gpurun_out/v25/rates.json 2>&1; grep '"ms"\|input_GBps' gpurun_out/v25/rates.json
