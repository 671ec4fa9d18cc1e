"""Generate the CPU golden-model results for the benchmark work unit.

The reference publishes no result file for its test WU, so recall is measured
against this framework's double-precision CPU golden model (csrc/core,
reference-order float semantics), run over the full template bank with the
benchmark flags (-A 0.08 -P 3.0 -f 400.0 -W). Output (tracked in git):
  data/golden/bench_wu_cpu_results.txt   result file (no comment header)
  data/golden/bench_wu_cpu_table.bin     the final 5x100 CP_cand table (24000 B)
  data/golden/bench_wu_cpu_meta.json     template range, timing
The reference's smoke target (debian/patches/benchmark.patch: first 200
templates at -A 0.04 -P 3.0 -W -z, default -f 250) has its own golden files:
  python tools/make_golden.py --end 200 --fA 0.04 --f0 250   (suffix _first200_A0.04_f250)
Reference-legal inputs outside the benchmark flags (the GPU's bounded-output
and wide-key paths, tests/test_gpu_bounded.py):
  python tools/make_golden.py --end 20 --no-white              (raw powers: every bin above chi^2)
  python tools/make_golden.py --end 6 --padding 5 --f0 8000 --fA 0.9999   (fundamental_idx_hi > 2^23)
Usage: python tools/make_golden.py [--threads 8] [--end N] [--fA 0.08] [--f0 400] [--padding 3] [--no-white]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--end", type=int, default=0, help="templates [0, end) (0: whole bank)")
    ap.add_argument("--fA", type=float, default=0.08, help="false-alarm rate -A")
    ap.add_argument("--f0", type=float, default=400.0, help="maximum signal frequency -f")
    ap.add_argument("--padding", type=float, default=3.0, help="padding factor -P")
    ap.add_argument("--no-white", action="store_true",
                    help="no whitening (no -W); the padding mean is then taken in double precision "
                         "(BRP_CPU_MEAN=double: the GPU / CUDA-build semantics, see cpu_backend.cpp)")
    ap.add_argument("--out", default=str(ROOT / "data" / "golden"))
    a = ap.parse_args()
    os.environ["BRP_NO_RESULT_HEADER"] = "1"
    if a.no_white:
        os.environ["BRP_CPU_MEAN"] = "double"
    import boinc_app_eah_brp_amd as pkg
    from boinc_app_eah_brp_amd.models import SearchConfig

    brp = pkg.native()
    D = ROOT / "data" / "testwu"
    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    suffix = (("" if a.end == 0 else f"_first{a.end}") + ("" if a.fA == 0.08 else f"_A{a.fA:g}") +
              ("" if a.f0 == 400.0 else f"_f{a.f0:g}") + ("" if a.padding == 3.0 else f"_P{a.padding:g}") +
              ("_noW" if a.no_white else ""))
    cfg = SearchConfig.benchmark(str(D / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000_1099.bin4"),
                                 str(D / "stochastic_full.bank"),
                                 str(D / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000.zap"),
                                 outputfile=str(out / f"bench_wu_cpu_results{suffix}.txt"), batch=1, use_cpu=True)
    cfg.fA = a.fA
    cfg.f0 = a.f0
    cfg.padding = a.padding
    cfg.white = not a.no_white
    t0 = time.time()
    r = brp.run_search(cfg.options(), 0, a.end, True, False, a.threads)
    dt = time.time() - t0
    (out / f"bench_wu_cpu_table{suffix}.bin").write_bytes(bytes(r["table"].to_bytes()))
    meta = dict(templates=r["templates_run"], templates_total=r["templates_total"], seconds=dt, threads=a.threads,
                flags=f"-A {a.fA:g} -P {a.padding:g} -f {a.f0:g}" + (" (accurate padding mean)" if a.no_white else " -W"), backend="cpu golden (double FFT, reference float order)")
    (out / f"bench_wu_cpu_meta{suffix}.json").write_text(json.dumps(meta, indent=1) + "\n")
    print(json.dumps(meta))


if __name__ == "__main__":
    main()
