# HBM traffic (PMC) of the fused kernel and of the two-kernel chain on f2's multi workload
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03z
mkdir -p $O
cd $R
for k in "scan_tokens_kernel<2, true>" "scan_tokens_kernel<2, false>" "scan_bytes_kernel<true, 1"; do
  tag=$(echo "$k" | tr -c 'a-z0-9' '_')
  timeout -k 10 300 python tools/pmc_profile.py $O/pmc_$tag --groups fetch,write --kernel "$k" --script tools/fused_rate.py -- --map multi --reps 3 > $O/pmc_$tag.log 2>&1
  python -c "import json;d=json.load(open('$O/pmc_$tag/pmc_summary.json'));print('$k', d.get('hbm_bytes_per_launch'), d['dispatches'])"
done
