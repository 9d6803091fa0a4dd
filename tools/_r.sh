set -e
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu_check.sh r01s2d pmc fetch,write,time,insts
timeout -k 10 400 python tools/config_rates.py > gpurun_out/r01s2d/rates.json 2>&1
grep -c bit_exact gpurun_out/r01s2d/rates.json
