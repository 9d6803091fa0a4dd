"""Static instruction mix of one kernel in a hipcc -save-temps .s file (VALU / SALU / LDS / VMEM
per basic block and in total), plus the resource lines (VGPRs, SGPRs, scratch).

    python tools/isa_mix.py FILE.s scan_bytes_kernelILb1ELb1 [--blocks]
"""
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    blocks = "--blocks" in sys.argv
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^_Z\S*" + re.escape(pat) + r"\S*:", l) and start is None:
            start = i
        elif start is not None and l.startswith(".Lfunc_end"):
            end = i
            break
    body = lines[start:end]
    tot = {}
    cur, cur_cnt = "entry", {}
    out = []

    def flush():
        if cur_cnt:
            out.append((cur, dict(cur_cnt)))

    for l in body:
        t = l.strip()
        if re.match(r"^\.LBB\S+:", t):
            flush()
            cur, cur_cnt = t.split(":")[0], {}
            continue
        if not t or t.startswith((".", ";")):
            continue
        op = t.split()[0]
        k = ("VALU" if op.startswith("v_") else "SALU" if op.startswith("s_") and not op.startswith(("s_waitcnt", "s_cbranch", "s_branch", "s_nop", "s_sleep", "s_setprio", "s_barrier"))
             else "CTRL" if op.startswith("s_") else "LDS" if op.startswith("ds_") else "VMEM" if op.startswith(("buffer_", "global_", "flat_", "scratch_")) else "other")
        cur_cnt[k] = cur_cnt.get(k, 0) + 1
        tot[k] = tot.get(k, 0) + 1
        if "scratch" in op or ("buffer_" in op and "off," in t and "s[0:3]" in t):
            cur_cnt["spill"] = cur_cnt.get("spill", 0) + 1
    flush()
    print("total", tot)
    if blocks:
        for name, c in out:
            print(f"{name:>12s} {c}")
    for l in lines[end:end + 80]:
        if re.search(r"num_vgpr|numbered_sgpr|private_seg_size|spill", l):
            print(l.strip())


if __name__ == "__main__":
    main()
