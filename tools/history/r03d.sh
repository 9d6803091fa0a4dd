set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03d
mkdir -p $O
cd $R
timeout -k 10 120 python tools/launch_floor.py > $O/floor.json 2>$O/floor.err; cat $O/floor.json
timeout -k 10 200 python tools/tile_timing.py 1024 > $O/tt_cfg3.txt 2>&1; head -24 $O/tt_cfg3.txt
timeout -k 10 200 python tools/tile_timing.py 100 --cfg2 > $O/tt_cfg2.txt 2>&1; head -24 $O/tt_cfg2.txt
timeout -k 10 200 python tools/tile_timing.py 1024 --random > $O/tt_cfg5.txt 2>&1; head -24 $O/tt_cfg5.txt
