"""Per-kernel register / spill / LDS / occupancy of the HIP sources, from
hipcc's -Rpass-analysis=kernel-resource-usage (gfx950).  A spill or scratch
use in a hot kernel shows here before any GPU run.
usage: python tools/kernel_resources.py [source.hip ...] [--grep PATTERN]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "fishnet_amd", "csrc")
KEYS = {"VGPRs": "vgpr", "VGPRs Spill": "spill", "ScratchSize [bytes/lane]": "scratch",
        "Occupancy [waves/SIMD]": "occ", "LDS Size [bytes/block]": "lds"}


def resources(src: str):
    out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                          "-c", src, "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage"],
                         capture_output=True, text=True, cwd=SRC).stderr
    name, rec = None, {}
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            if name:
                yield name, rec
            name, rec = m.group(1), {}
            continue
        m = re.search(r"remark:\s+(.+?): (\d+)\s", line + " ")
        if m and m.group(1) in KEYS:
            rec[KEYS[m.group(1)]] = int(m.group(2))
    if name:
        yield name, rec


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    pat = sys.argv[sys.argv.index("--grep") + 1] if "--grep" in sys.argv else ""
    if pat in args:
        args.remove(pat)
    srcs = args or ["ft_segments.hip", "ft_sliced.hip", "kernels.hip", "variant.hip"]
    for s in srcs:
        for name, r in resources(s):
            dn = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
            dn = re.sub(r"fnnue::|\(anonymous namespace\)::|void ", "", dn)
            dn = re.sub(r"\(.*", "", dn)
            if pat and not re.search(pat, dn):
                continue
            print(f"{dn[:70]:70s} vgpr={r.get('vgpr')} spill={r.get('spill')} scratch={r.get('scratch')} "
                  f"occ={r.get('occ')} lds={r.get('lds')}")


if __name__ == "__main__":
    main()
