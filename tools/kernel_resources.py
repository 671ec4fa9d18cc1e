#!/usr/bin/env python3
"""Per-kernel register / LDS / occupancy table of a HIP source compiled for
gfx950 (clang's kernel-resource-usage remarks), demangled names.

  python tools/kernel_resources.py csrc/hip/fft_passes.hip [name-filter]"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def main() -> None:
    src = Path(sys.argv[1]).resolve()
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--offload-device-only",
           "-c", str(src), "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage", *sys.argv[3:]]
    r = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp")
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
        if not m:
            continue
        txt = m.group(1)
        if txt.startswith("Function Name:"):
            cur = {"name": txt.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in txt:
            k, v = txt.split(":", 1)
            cur[k.strip()] = v.strip()
    names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                           text=True).stdout.splitlines()
    print(f"{'kernel':70s} {'VGPR':>5s} {'AGPR':>5s} {'spill':>5s} {'LDS':>7s} {'occ':>4s}")
    for r, n in zip(rows, names):
        n = n.replace("brp::hipk::(anonymous namespace)::", "")
        n = re.sub(r"\(.*", "", n)
        if pat and pat not in n:
            continue
        print(f"{n[:70]:70s} {r.get('VGPRs', '?'):>5s} {r.get('AGPRs', '?'):>5s} {r.get('VGPRs Spill', '?'):>5s} "
              f"{r.get('LDS Size [bytes/block]', '?'):>7s} {r.get('Occupancy [waves/SIMD]', '?'):>4s}")


if __name__ == "__main__":
    main()
