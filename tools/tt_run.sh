set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r02s4_tt; mkdir -p $O; cd $R
timeout -k 10 200 python tools/tile_timing.py 1024 > $O/cfg3.txt 2>&1
timeout -k 10 200 python tools/tile_timing.py 1024 --random > $O/cfg5.txt 2>&1
BLT_LIB_PATH=$R/build/exp/libblt_bpe_timingdn.so timeout -k 10 200 python tools/tile_timing.py 1024 > $O/cfg3dn.txt 2>&1
head -20 $O/cfg3.txt $O/cfg5.txt $O/cfg3dn.txt
