#!/bin/bash
# One GPU call made of named steps (the maintained runner; round 3's one-off scripts are in
# tools/history/).  Every GPU step runs under its own time limit and the chain stops at the first
# failure (set -e), so a fault or a hang ends the call there.
#
#   gpurun --timeout 1200 -- 'bash tools/round.sh TAG STEP [STEP ...]'
#
# Steps (outputs under gpurun_out/TAG/):
#   tests              pytest -m gpu (every parity test), tests.log
#   smoke              __graft_entry__.smoke(), smoke.log
#   bench              the driver's command: bench.py --gpus 1 --steps 20 --warmup 5, bench.json
#   bench:ARGS         bench.py with extra arguments (+ for spaces), bench_<n>.json
#   benche:NAME=VALUE:ARGS  bench.py with one environment setting
#   benchlib:LIBTAG:ARGS  bench.py on build/xp/libblt_bpe_LIBTAG.so
#   kbench[:LIBTAG]    tools/kbench.py on cfg2/cfg3/cfg5 (LIBTAG: build/xp/libblt_bpe_LIBTAG.so)
#   tim:LIBTAG[:ARGS]  tools/tile_timing.py on a timing build (build/xp/libblt_bpe_LIBTAG.so)
#   prof:WL            rocprofv3 --kernel-trace --stats of bench.py --workload WL (cfg2|cfg3|cfg5)
#   proff2[:ROWS]      rocprofv3 kernel stats of the f2 rows (bench.py --only-configs ROWS)
#   pmc:WL[:GROUPS]    tools/pmc_profile.py on bench.py --workload WL (groups default fetch,write,insts)
#   pmc4:G             PMC traffic of cfg4's per-rank shard of G GiB (N = 8/4/2: G = 1/2/4)
#   pmcf2:ROW[:GROUPS] PMC of one f2 row (tools/f2_row.py: every kernel of its calls, traffic per call)
#   cli[:ENV]          tools/cli_phases.py: the CLI's BLT_CLI_TIMING phases on 1 GiB, the HIP start-up probe
#   copyprobe          tools/copy_probe.cpp: host<->device copy rates by kind of host memory
#   rehearse:N         bench.py --gpus N, every rank on device 0 over gloo (multi-rank logic rehearsal)
#   py:SCRIPT[:ARGS]   a tool script under its own time limit
#   resources          -Rpass-analysis=kernel-resource-usage of the kernel source (CPU only)
set -e
TAG=${1:?tag}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
nb=0
for st in "$@"; do
  IFS=: read -r kind a b <<< "$st"
  echo "== $st $(date +%T)"
  case $kind in
    tests)
      # tests[:K] runs only the tests whose names match K (pytest -k; + for spaces)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=8 --timeout 300 --timeout-method thread ${a:+-k "${a//+/ }"} \
        > "$O/tests${a:+_$a}.log" 2>&1 || { tail -40 "$O/tests${a:+_$a}.log"; exit 1; }
      tail -2 "$O/tests${a:+_$a}.log" ;;
    smoke)
      timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > "$O/smoke.log" 2>&1
      tail -1 "$O/smoke.log" ;;
    bench)
      if [ -z "$a" ]; then
        timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
        python tools/summarize_bench.py "$O/bench.json"
      else
        nb=$((nb + 1))
        timeout -k 10 400 python bench.py ${a//+/ } > "$O/bench_$nb.json" 2> "$O/bench_$nb.err"
        python tools/summarize_bench.py "$O/bench_$nb.json"
      fi ;;
    benche)
      # bench.py with one environment setting: benche:NAME=VALUE:ARGS (ARGS + for spaces)
      nb=$((nb + 1))
      ( export "$a" && timeout -k 10 400 python bench.py ${b//+/ } > "$O/bench_${a//=/}_$nb.json" 2> "$O/bench_${a//=/}_$nb.err" )
      echo "[$a]"; python tools/summarize_bench.py "$O/bench_${a//=/}_$nb.json" ;;
    benchlib)
      # bench.py on an experiment build: benchlib:LIBTAG:ARGS (ARGS + for spaces)
      nb=$((nb + 1))
      BLT_LIB_PATH=$R/build/xp/libblt_bpe_$a.so timeout -k 10 400 python bench.py ${b//+/ } > "$O/bench_${a}_$nb.json" 2> "$O/bench_${a}_$nb.err"
      echo "[$a]"; python tools/summarize_bench.py "$O/bench_${a}_$nb.json" ;;
    kbench)
      lib=""; [ -n "$a" ] && lib="$R/build/xp/libblt_bpe_$a.so"
      BLT_LIB_PATH=$lib timeout -k 10 300 python tools/kbench.py --check >> "$O/kbench.jsonl" 2> "$O/kbench.err"
      tail -3 "$O/kbench.jsonl" ;;
    tim)
      # per-wave phase timing of a timing build (-DBLT_TIMING): tim:LIBTAG[:ARGS] (ARGS + for spaces)
      nb=$((nb + 1))
      BLT_LIB_PATH=$R/build/xp/libblt_bpe_$a.so timeout -k 10 300 python tools/tile_timing.py ${b//+/ } \
        > "$O/tim_${a}_$nb.txt" 2>&1
      head -22 "$O/tim_${a}_$nb.txt" | grep -E "^256|exit|publishes|wave  0|wave  8|wave 12|spins|rounds" ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$O/prof_$a" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-extra \
        --workload "$a" > "$O/prof_$a.log" 2>&1)
      find "$O/prof_$a" -name '*kernel_stats.csv' -exec head -4 {} \; | cut -c1-160 ;;
    proff2)
      # proff2[:ROWS[:ENV]]  (ENV: NAME=VALUE for the profiled run)
      rows=${a:-multi,wrap,selfval,chain}
      bt=${b##*/}; pd=prof_f2${a:+_${a//,/_}}${b:+_${bt//[=.]/_}}
      (cd /tmp && export TMPDIR=/tmp && { [ -z "$b" ] || export "$b"; } && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$O/$pd" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --only-configs "$rows" \
        > "$O/$pd.log" 2>&1)
      find "$O/$pd" -name '*kernel_stats.csv' -exec head -12 {} \; | cut -c1-160 ;;
    pmc)
      timeout -k 10 900 python tools/pmc_profile.py "$O/pmc_$a" --groups "${b:-fetch,write,insts}" -- \
        --workload "$a" --steps 5 --warmup 2 --no-cpu-baseline --no-extra > "$O/pmc_$a.log" 2>&1
      tail -3 "$O/pmc_$a.log" ;;
    pmc4)
      # cfg4's per-rank shard of G GiB (the N = 8/4/2 shard sizes 1/2/4 GiB): pmc4:G
      timeout -k 10 900 python tools/pmc_profile.py "$O/pmc_cfg4_$a" --groups fetch,write -- \
        --workload cfg4 --total-bytes $((a << 30)) --steps 3 --warmup 1 --no-cpu-baseline --no-extra > "$O/pmc_cfg4_$a.log" 2>&1
      tail -2 "$O/pmc_cfg4_$a.log" ;;
    pmcf2)
      # 5 asynchronous calls (tools/f2_row.py): traffic per call = totals / 5
      timeout -k 10 900 python tools/pmc_profile.py "$O/pmc_$a" --kernel "" --script tools/f2_row.py --calls 5 \
        --groups "${b:-fetch,write}" -- --row "$a" --reps 5 > "$O/pmc_$a.log" 2>&1
      grep -E "hbm_bytes_per_call|calls" "$O/pmc_$a/pmc_summary.json" ;;
    cli)
      # BLT_CLI_TIMING phases of the CLI on 1 GiB (tools/cli_phases.py), cli:ENV (NAME=VALUE, commas)
      [ -x build/hip_init_probe ] || /opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 tools/hip_init_probe.cpp -o build/hip_init_probe
      echo "shmem THP: $(cat /sys/kernel/mm/transparent_hugepage/shmem_enabled 2>/dev/null)" 
      nb=$((nb + 1))
      timeout -k 10 300 python tools/cli_phases.py --out "$O/cli_phases_$nb.json" ${a:+--env "$a"} > "$O/cli_$nb.log" 2>&1
      python -c "import json;d=json.load(open('$O/cli_phases_$nb.json'));print(d.get('hip_init_probe'));[print(r['wall_s'],r['GBps']) for r in d['runs']]" ;;
    copyprobe)
      # host<->device copy rates from the CLI's kinds of host memory (tools/copy_probe.cpp)
      [ -x build/copy_probe ] || /opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 tools/copy_probe.cpp -o build/copy_probe
      timeout -k 10 120 build/copy_probe > "$O/copy_probe.txt" 2>&1
      cat "$O/copy_probe.txt" ;;
    rehearse)
      # rehearse:N  bench.py at --gpus N with every rank on device 0 over gloo (the multi-rank logic on a
      # one-GPU box; its value is no scaling figure), rehearse_N.json
      BLT_BENCH_BACKEND=gloo BLT_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node "$a" --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus "$a" --steps 5 --warmup 2 \
        --no-cpu-baseline --no-extra > "$O/rehearse_$a.json" 2> "$O/rehearse_$a.err"
      tail -c 600 "$O/rehearse_$a.json" ;;
    py)
      # any tool script: py:tools/x.py[:ARGS] (ARGS + for spaces), output py_<n>.log
      nb=$((nb + 1))
      timeout -k 10 300 python -u "$a" ${b//+/ } > "$O/py_$nb.log" 2>&1 || { tail -30 "$O/py_$nb.log"; exit 1; }
      tail -60 "$O/py_$nb.log" ;;
    resources)
      /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -c blt_amd/csrc/bpe_kernels.hip -o /tmp/rk.o \
        -Rpass-analysis=kernel-resource-usage > "$O/resources.txt" 2>&1
      grep -E "Function Name|VGPRs:|SGPRs Spill|VGPRs Spill" "$O/resources.txt" | sed 's/.*remark: *//' ;;
    *)
      echo "unknown step $st"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
