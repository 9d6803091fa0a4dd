"""Register and LDS use of every kernel in bpe_kernels.hip, from the compiler's
-Rpass-analysis=kernel-resource-usage remarks (device compile only, no GPU needed).

    python tools/resources.py [out.txt]      # a table: kernel, VGPRs, SGPRs, spills, waves/SIMD, LDS

tests/test_resources.py uses parse() to keep spills out of the product kernels.
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "blt_amd", "csrc", "bpe_kernels.hip")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FIELDS = {"TotalSGPRs": "sgprs", "VGPRs": "vgprs", "ScratchSize [bytes/lane]": "scratch",
          "Occupancy [waves/SIMD]": "waves", "SGPRs Spill": "sgpr_spill", "VGPRs Spill": "vgpr_spill",
          "LDS Size [bytes/block]": "lds"}


def remarks(extra=()):
    """The compiler's resource remarks for the kernel source (a ~30 s device-only compile)."""
    with tempfile.TemporaryDirectory() as d:
        cmd = [HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only", "-c", SRC,
               "-o", os.path.join(d, "k.o"), "-Rpass-analysis=kernel-resource-usage", *extra]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(r.stderr[-4000:])
        return r.stderr


def parse(text):
    """{mangled kernel name: {field: int}}"""
    out, cur = {}, None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark: ([^:]+): (\S+) \[-Rpass", line)
        if cur is not None and m and m.group(1).strip() in FIELDS:
            v = m.group(2)
            cur[FIELDS[m.group(1).strip()]] = int(v) if v.lstrip("-").isdigit() else v
    return out


def demangle(name):
    try:
        return subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    except OSError:
        return name


def table(res):
    rows = ["%-72s %5s %5s %6s %6s %7s %5s %7s" % ("kernel", "VGPR", "SGPR", "vspill", "sspill", "scratch", "waves",
                                                     "LDS")]
    for k in sorted(res, key=demangle):
        r = res[k]
        rows.append("%-72s %5s %5s %6s %6s %7s %5s %7s" % (demangle(k)[:72], r.get("vgprs"), r.get("sgprs"),
                                                              r.get("vgpr_spill"), r.get("sgpr_spill"), r.get("scratch"),
                                                              r.get("waves"), r.get("lds")))
    return "\n".join(rows)


if __name__ == "__main__":
    t = table(parse(remarks()))
    print(t)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(t + "\n")
