set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03g
mkdir -p $O
cd $R
timeout -k 10 200 python tools/tok_timing.py 256 > $O/tok.txt 2>&1; cat $O/tok.txt | grep -v amdgpu.ids
timeout -k 10 200 python tools/tile_timing.py 256 --few > $O/few.txt 2>&1; head -22 $O/few.txt | grep -v amdgpu.ids
