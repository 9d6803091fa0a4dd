"""One-line summary of a bench.py JSON output file (its last JSON line): value, kernel time,
roofline fraction, traffic and each `configs` row's fraction / time and bit-exact flag.

    python tools/summarize_bench.py gpurun_out/TAG/bench.json
"""
import json
import sys


def main(path):
    lines = [ln for ln in open(path).read().splitlines() if ln.startswith("{")]
    if not lines:
        print(f"{path}: no JSON line")
        return 1
    d = json.loads(lines[-1])
    r = d["roofline"]
    print(f"value {d['value']} GB/s  kernel {r['kernel_ms']} ms  frac {r['frac']}  traffic {r['traffic']}  "
          f"exact {d.get('bit_exact_vs_oracle')}  cpu {(d.get('cpu_baseline') or {}).get('value')}")
    for k, c in d.get("configs", {}).items():
        t = c.get("kernel_ms", c.get("ms"))
        extra = f" sync {c['sync_ms']} ({c['sync_path']})" if "sync_ms" in c else ""
        print(f"  {k:8s} frac {c.get('frac')}  ms {t}{extra}  exact {c.get('bit_exact_vs_oracle')}")
    for k in ("end_to_end", "per_chunk_path", "cli_end_to_end"):
        if k in d:
            print(f"  {k}: {d[k].get('value')} GB/s")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
