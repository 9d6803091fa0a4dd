"""End-to-end rate of the `blt` command-line drop-in on the GPU box (file -> mmap -> GPU -> file).

    python tools/cli_rate.py [--mib 2048] [--dir /tmp]

Writes cfg3's text (seed 3) and the 50k merges file, runs
`blt_amd/blt -i IN -o OUT --merges M --chunksize 16MB --type text --gpus G` for each --gpus value
three times (the best of the last two is timed: files in the page cache, as the reference's own
benchmarks run), checks OUT against the C oracle's stream byte for byte, and times the oracle
restatement on the same file for comparison.  Prints one JSON object.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=2048)
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp"))
    ap.add_argument("--gpus", default="1", help="comma list of --gpus values to time")
    ap.add_argument("--no-oracle-time", action="store_true")
    a = ap.parse_args()
    from blt_amd import synth
    from oracle import oracle as O
    n = a.mib << 20
    d = os.path.join(a.dir, f"blt_cli_rate_{os.getpid()}")
    os.makedirs(d, exist_ok=True)
    fin, fout, fm = os.path.join(d, "in.txt"), os.path.join(d, "out.bin"), os.path.join(d, "merges.txt")
    try:
        text = synth.text(n, seed=3)
        text.tofile(fin)
        pairs = synth.text_merges_50k(synth.text(64 << 20, seed=3), seed=3)
        with open(fm, "w") as f:
            f.write(synth.merges_file_text(pairs))
        m = synth.merges_dict(pairs)
        threads = min(16, os.cpu_count() or 1)
        c0 = time.perf_counter()
        exp = O.COracle(m).run(text, 16 << 20, content_type="text", threads=threads)
        cpu_s = time.perf_counter() - c0
        res = {"bytes": n, "oracle_seconds": round(cpu_s, 4), "oracle_threads": threads,
               "oracle_input_GBps": round(n / cpu_s / 1e9, 3), "runs": {}}
        for g in a.gpus.split(","):
            cmd = [os.path.join(ROOT, "blt_amd", "blt"), "-i", fin, "-o", fout, "--merges", fm, "--chunksize", "16MB",
                   "--type", "text", "--gpus", g]
            subprocess.run(cmd, check=True)
            best = None
            for _ in range(2):
                os.remove(fout)   # a fresh output file: truncating the last run's pages is not blt's cost
                t0 = time.perf_counter()
                r = subprocess.run(cmd, check=True, stderr=subprocess.PIPE, env=dict(os.environ, BLT_CLI_TIMING="1"))
                dt = time.perf_counter() - t0
                if best is None or dt < best[0]:
                    best = (dt, r.stderr.decode().strip())
            got = np.fromfile(fout, dtype=np.uint8)
            res["runs"][g] = {"cli_seconds": round(best[0], 4), "cli_input_GBps": round(n / best[0] / 1e9, 3),
                              "bit_exact": bool(np.array_equal(got, exp)), "phases": best[1]}
        print(json.dumps(res, indent=1))
    finally:
        for f in (fin, fout, fm):
            if os.path.exists(f):
                os.remove(f)
        os.rmdir(d)


if __name__ == "__main__":
    main()
