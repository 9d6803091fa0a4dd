# u16 merge pass with its chunk starts from an LDS list (BLT_BND_LDS=1, the product build) against
# the global-memory walk (bnd0): GPU parity suite on the product library, then the f2 chain /
# selfval / multi rows on both builds, alternating
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03as}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for k in 1 2; do
  for v in bnd0 bnd1; do
    BLT_LIB_PATH=$R/build/exp/libblt_bpe_$v.so timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --only-configs chain,selfval,multi > $O/bench_${v}_$k.json 2> $O/bench_${v}_$k.err
    python -c "
import json;d=json.loads(open('$O/bench_${v}_$k.json').read().strip().splitlines()[-1])
print('$v', ' '.join(f\"{k}: {c['ms']} / {c['sync_ms']} ms {c['bit_exact_vs_oracle']}\" for k,c in d['configs'].items()))"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_chain -o run -- python3 $R/bench.py --steps 3 --warmup 1 --only-configs chain > $O/prof_chain.log 2>&1
find $O/prof_chain -name '*kernel_stats.csv' -exec cut -c1-140 {} \;
