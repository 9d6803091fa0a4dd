"""Merges the PMC traffic records of one tools/pmc_profile.py run per workload into
profiles/traffic.json (the record bench.py reads for roofline.traffic), and copies each
pmc_summary.json to profiles/ under the round's name.

    python tools/merge_traffic.py gpurun_out/TAG r03

Looks for TAG/pmc_cfg3, pmc_cfg5, pmc_cfg2 and pmc_cfg4_{1,2,4} (tools/r03ad.sh's layout).  A
record is taken only if it names the current kernel source's sha256 (bench.kernel_source_sha).
"""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    src, tag = sys.argv[1], sys.argv[2]
    import bench
    sha = bench.kernel_source_sha()
    path = os.path.join(ROOT, "profiles", "traffic.json")
    with open(path) as f:
        tj = json.load(f)
    runs = [("cfg3", "pmc_cfg3", "cfg3"), ("cfg5", "pmc_cfg5", "cfg5"), ("cfg2", "pmc_cfg2", "cfg2"),
            ("cfg4@1GiB", "pmc_cfg4_1", "cfg4_1"), ("cfg4@2GiB", "pmc_cfg4_2", "cfg4_2"),
            ("cfg4@4GiB", "pmc_cfg4_4", "cfg4_4")]
    for key, d, name in runs:
        rec_path = os.path.join(src, d, "traffic.json")
        if not os.path.exists(rec_path):
            print(f"{key}: no record in {d}")
            continue
        with open(rec_path) as f:
            rec = json.load(f)
        if rec.get("kernel_source_sha256") != sha:
            print(f"{key}: record is for another kernel source, skipped")
            continue
        dst = os.path.join(ROOT, "profiles", f"{tag}_pmc_{name}.json")
        shutil.copy(os.path.join(src, d, "pmc_summary.json"), dst)
        tj["workloads"][key] = {"workload": rec["workload"], "bytes_per_gpu": rec["bytes_per_gpu"],
                                "chunk_size": rec["chunk_size"], "hbm_bytes_per_launch": rec["hbm_bytes_per_launch"],
                                "kernel_source_sha256": sha,
                                "source": f"profiles/{tag}_pmc_{name}.json (tools/pmc_profile.py)"}
        print(f"{key}: {rec['hbm_bytes_per_launch']} B per launch -> {os.path.relpath(dst, ROOT)}")
    with open(path, "w") as f:
        json.dump(tj, f, indent=1)


if __name__ == "__main__":
    main()
