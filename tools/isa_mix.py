#!/usr/bin/env python3
"""Instruction mix per kernel of a HIP source compiled for gfx950 (static
counts in the generated ISA: VALU, packed-FP32 VALU, LDS, global memory,
scalar), demangled names.

  python tools/isa_mix.py csrc/hip/fft_passes.hip ["filter|filter"] [-- extra hipcc flags]"""
import re
import subprocess
import sys
from collections import Counter
from pathlib import Path


def main() -> None:
    args = sys.argv[1:]
    extra = []
    if "--" in args:
        i = args.index("--")
        args, extra = args[:i], args[i + 1:]
    src = Path(args[0]).resolve()
    pat = args[1] if len(args) > 1 else ""
    out = Path("/tmp") / (src.stem + ".isa.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                    "--offload-device-only", "-S", str(src), "-o", str(out), *extra], check=True, cwd="/tmp",
                   capture_output=True)
    text = out.read_text()
    funcs = {}
    cur = None
    for line in text.splitlines():
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1)
            funcs[cur] = Counter()
            continue
        if cur is None:
            continue
        if line.startswith("\t.end_amdhsa") or line.startswith(".Lfunc_end"):
            cur = None
            continue
        t = line.strip()
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        funcs[cur][t.split()[0]] += 1
    names = list(funcs)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    print(f"{'kernel':58s} {'VALU':>6s} {'v_pk':>5s} {'LDS':>5s} {'VMEM':>5s} {'SALU':>5s}")
    for n, d in zip(names, dem):
        d = d.replace("brp::hipk::(anonymous namespace)::", "")
        d = re.sub(r"\(.*", "", d)
        if pat and not any(x in d for x in pat.split("|")):
            continue
        c = funcs[n]
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        pk = sum(v for k, v in c.items() if k.startswith("v_pk_"))
        lds = sum(v for k, v in c.items() if k.startswith("ds_"))
        vmem = sum(v for k, v in c.items() if k.startswith(("global_", "buffer_", "flat_")))
        salu = sum(v for k, v in c.items() if k.startswith("s_"))
        print(f"{d[:58]:58s} {valu:6d} {pk:5d} {lds:5d} {vmem:5d} {salu:5d}")


if __name__ == "__main__":
    main()
