"""Phases of the `blt` CLI drop-in on cfg3's 1 GiB (tmpfs in, tmpfs out): wall time of each run
and the BLT_CLI_TIMING stamps (exec -> main, merges loaded, mmap, HIP runtime up, device setup,
windows, writer waits, output closed), plus the HIP start-up probe (build/hip_init_probe).

    python tools/cli_phases.py [--mib 1024] [--runs 4] [--out profiles/r04_cli_phases.json]
    python tools/cli_phases.py --variants ";BLT_PREALLOC_AT=1" --runs 8   (A/B: runs alternate)
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--runs", type=int, default=4)
    ap.add_argument("--out", default="")
    ap.add_argument("--env", default="", help="extra environment for the CLI, NAME=VALUE[,NAME=VALUE]")
    ap.add_argument("--variants", default=None,
                    help="';'-separated environments (NAME=VALUE[,NAME=VALUE], empty = default) run in turn")
    a = ap.parse_args()
    from blt_amd import synth
    base = "/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir()
    d = tempfile.mkdtemp(prefix="blt_cli_phases_", dir=base)
    fin, fout, fm = (os.path.join(d, x) for x in ("in.txt", "out.bin", "merges.txt"))
    res = {"mib": a.mib, "tmpfs": base, "runs": []}
    try:
        synth.text(a.mib << 20, seed=3).tofile(fin)
        with open(fm, "w") as f:
            f.write(synth.merges_file_text(synth.text_merges_50k(synth.text(64 << 20, seed=3), seed=3)))
        probe = os.path.join(ROOT, "build", "hip_init_probe")
        if os.path.exists(probe):
            res["hip_init_probe"] = json.loads(subprocess.run([probe], capture_output=True, text=True,
                                                              timeout=60).stdout.strip().splitlines()[-1])
        def env_of(spec):
            env = dict(os.environ, BLT_CLI_TIMING="1")
            for kv in filter(None, spec.split(",")):
                k, v = kv.split("=", 1)
                env[k] = v
            return env
        cmd = [os.path.join(ROOT, "blt_amd", "blt"), "-i", fin, "-o", fout, "--merges", fm, "--chunksize", "16MB",
               "--type", "text", "--gpus", "1"]

        def run(env):
            if os.path.exists(fout):
                os.remove(fout)
            t0 = time.perf_counter()
            p = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=env)
            dt = time.perf_counter() - t0
            return dt, p
        if a.variants is None:
            env = env_of(a.env)
            for _ in range(a.runs):
                dt, p = run(env)
                res["runs"].append({"wall_s": round(dt, 4), "GBps": round((a.mib << 20) / dt / 1e9, 3), "rc": p.returncode,
                                    "stamps": [ln for ln in p.stderr.splitlines() if ln.startswith("blt timing")]})
        else:
            from bench import cli_phases
            specs = a.variants.split(";")
            run(env_of(""))   # warm (page cache of the binary and libraries)
            res["variants"] = {sp or "default": {"wall_s": [], "phases": [], "rc": []} for sp in specs}
            for _ in range(a.runs):
                for sp in specs:
                    dt, p = run(env_of(sp))
                    r = res["variants"][sp or "default"]
                    r["wall_s"].append(round(dt, 4))
                    r["rc"].append(p.returncode)
                    r["phases"].append(cli_phases(p.stderr, dt))
                    print(sp or "default", round(dt, 4), flush=True)
            for r in res["variants"].values():
                w = sorted(r["wall_s"])
                r["median_s"], r["best_s"] = w[len(w) // 2], w[0]
    finally:
        for f in (fin, fout, fm):
            if os.path.exists(f):
                os.remove(f)
        os.rmdir(d)
    js = json.dumps(res, indent=1)
    print(js)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js + "\n")


if __name__ == "__main__":
    main()
