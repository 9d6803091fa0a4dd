# tmpfs output-write microbenchmark on the GPU box's host (CPU only): pwrite vs mmap copies
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03s
mkdir -p $O
gcc -O2 -pthread -o $O/w $R/tools/tmpfs_write.c
for m in 0 1 2 3; do for t in 1 4 8 16; do timeout -k 5 60 $O/w 1024 $t $m; done; done 2>&1 | tee $O/w.txt
