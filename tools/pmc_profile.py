"""Collects rocprofv3 PMC counters for the merge-scan kernel, one counter group per pass.

    python tools/pmc_profile.py OUTDIR [--groups A,B,...] [--kernel NAME] [--script S] [-- args]

(--script: the profiled program instead of bench.py, e.g. tools/config_rates.py with
`-- --only multi` for the u16 scan kernel of the general map.)

Each group runs `rocprofv3 --pmc <counters> --kernel-trace --output-format csv -- python
bench.py ...` as a child process (counters in their own passes, never with sys/runtime
traces), then averages every counter per dispatch of the kernels whose name contains
--kernel (default scan_bytes_kernel).  Writes OUTDIR/pmc_summary.json, including the HBM
traffic per launch corrected as MI355X_MICROARCH.md prescribes for gfx950: FETCH_SIZE counts
half of a wide streaming read (doubled here), WRITE_SIZE is exact; both are in KiB.
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GIB = 1 << 30
CHUNK = 16 << 20   # bench.py's --chunksize

GROUPS = {
    "time": ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
             "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA"],
    "insts": ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
              "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_INST_LDS"],
    "misc": ["SQ_WAVES", "SQ_INSTS_BRANCH", "SQ_INSTS_SMEM", "SQ_ACTIVE_INST_VMEM", "SQ_INST_CYCLES_VMEM_RD",
             "SQ_INST_CYCLES_VMEM_WR", "SQ_LDS_UNALIGNED_STALL", "GRBM_GUI_ACTIVE"],
    "fetch": ["FETCH_SIZE"],
    "write": ["WRITE_SIZE"],
}


def run_group(outdir, name, counters, bench_args, kernel, script="bench.py"):
    d = os.path.join(outdir, name)
    os.makedirs(d, exist_ok=True)
    cmd = ["rocprofv3", "--pmc", *counters, "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run",
           "--", sys.executable, os.path.join(ROOT, script), *bench_args]
    print("+", " ".join(cmd), flush=True)
    with open(os.path.join(d, "log.txt"), "w") as log:
        rc = subprocess.run(cmd, stdout=log, stderr=subprocess.STDOUT, timeout=900).returncode
    if rc != 0:
        raise SystemExit(f"rocprofv3 pass {name} failed with {rc} (see {d}/log.txt)")
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    sums, disp = {}, {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if kernel not in row.get("Kernel_Name", ""):
                    continue
                cname = row["Counter_Name"]
                sums[cname] = sums.get(cname, 0.0) + float(row["Counter_Value"])
                disp.setdefault(cname, set()).add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    return {k: sums[k] / max(1, len(disp[k])) for k in sums}, {k: len(v) for k, v in disp.items()}, sums


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--groups", default=",".join(GROUPS))
    ap.add_argument("--kernel", default="scan_bytes_kernel")
    ap.add_argument("--script", default="bench.py")
    ap.add_argument("--calls", type=int, default=0,
                    help="calls the script makes (f2 rows: several kernels per call): also report totals / calls")
    argv = sys.argv[1:]
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    a = ap.parse_args(argv)
    bench_args = extra or ["--steps", "5", "--warmup", "2", "--no-cpu-baseline", "--no-extra"]
    os.makedirs(a.outdir, exist_ok=True)
    result = {"kernel": a.kernel, "bench_args": bench_args, "per_dispatch": {}, "dispatches": {}, "totals": {}}
    for g in a.groups.split(","):
        vals, nd, tot = run_group(a.outdir, g, GROUPS[g], bench_args, a.kernel, a.script)
        result["per_dispatch"].update(vals)
        result["dispatches"].update(nd)
        result["totals"].update(tot)
    if a.calls and "FETCH_SIZE" in result["totals"] and "WRITE_SIZE" in result["totals"]:
        t = result["totals"]
        result["calls"] = a.calls
        result["hbm_bytes_per_call"] = int((2.0 * t["FETCH_SIZE"] + t["WRITE_SIZE"]) * 1024 / a.calls)
    pd = result["per_dispatch"]
    if "FETCH_SIZE" in pd and "WRITE_SIZE" in pd and a.script == "bench.py":
        result["hbm_bytes_per_launch"] = int((2.0 * pd["FETCH_SIZE"] + pd["WRITE_SIZE"]) * 1024)
        result["traffic_note"] = "(2 x FETCH_SIZE + WRITE_SIZE) KiB: gfx950 FETCH_SIZE counts half of wide reads"
        # what bench.py reports as roofline.traffic for the same workload
        sys.path.insert(0, ROOT)
        import bench
        per_gpu, total, wl = GIB, 0, "cfg3"
        for i, x in enumerate(bench_args):
            if x == "--bytes-per-gpu":
                per_gpu = int(bench_args[i + 1])
            if x == "--workload":
                wl = bench_args[i + 1]
            if x == "--total-bytes":
                total = int(bench_args[i + 1])
        # the bytes one launch processes at N = 1 (bench.workload's shapes)
        n = 100 << 20 if wl == "cfg2" else per_gpu if wl == "cfg3" else (total or bench.STRONG_TOTAL[wl])
        with open(os.path.join(a.outdir, "traffic.json"), "w") as f:
            json.dump({"workload": wl, "bytes_per_gpu": n, "chunk_size": CHUNK, "kernel": a.kernel,
                       "kernel_source_sha256": bench.kernel_source_sha(),
                       "hbm_bytes_per_launch": result["hbm_bytes_per_launch"], "note": result["traffic_note"]}, f,
                      indent=1)
    with open(os.path.join(a.outdir, "pmc_summary.json"), "w") as f:
        json.dump(result, f, indent=1, sort_keys=True)
    print(json.dumps(result, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
