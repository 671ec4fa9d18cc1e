"""Plan-wisdom generator, the counterpart of the reference's FFTW wisdom script
(debian/extra/create_wisdomf_eah_brp.sh): measures the template pipeline of
the benchmark geometry on this GPU for candidate kernel settings and writes the
fastest into data/wisdom/mi355x.json, which the HIP engine reads at setup
(csrc/core/wisdom.cpp; BRP_PERSIST still overrides).

Stage 1 (sequential pipeline time per template from HipEngine.benchmark_stages):
pass-2 persistent workgroups per CU. Stage 2 (concurrency, bench.py on a bank
prefix with the stage-1 winner): templates per batch x pipelines per GPU;
recorded in the file for the application defaults. (The two-pass FFT and the
harmonic-sum variants were measured slower and are not product options:
profiles/README.md, tools/experiments/.)

  python tools/tune_plan.py [--templates 2000] [--out data/wisdom/mi355x.json]
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
D = ROOT / "data" / "testwu"
WU = D / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000_1099.bin4"
ZAP = D / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000.zap"
BANK = D / "stochastic_full.bank"


def stage_time(brp, geom, series, zaps, tin, env: dict, batch: int = 4, reps: int = 10) -> float:
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        eng = brp.HipEngine()
        eng.init(0, batch)
        eng.setup(geom, series, float(np.mean(series)))
        opt = dict(f0=400.0, padding=3.0, fA=0.08, window=1000, white=True)
        eng.whiten(opt, zaps, series.copy())
        res = eng.benchmark_stages(*tin, reps)
        return res["batch"] / batch
    finally:
        for k in env:
            os.environ.pop(k, None)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--templates", type=int, default=2000, help="bank prefix for the concurrency stage")
    ap.add_argument("--out", default=str(ROOT / "data" / "wisdom" / "mi355x.json"))
    args = ap.parse_args()
    os.environ["BRP_WISDOM"] = "/nonexistent"  # measure without the current wisdom
    import torch

    import boinc_app_eah_brp_amd as pkg

    brp = pkg.native()
    brp.set_log_level(2)
    arch = torch.cuda.get_device_properties(0).gcnArchName.split(":")[0]
    hdr, series, _ = brp.read_work_unit(str(WU))
    opt = dict(f0=400.0, padding=3.0, fA=0.08, window=1000, white=True)
    geom = brp.derive_geometry(hdr, opt)
    M = geom["nsamples"] // 2
    zaps = brp.read_zaplist(str(ZAP))
    P, tau, psi = (np.asarray(v, dtype=np.float32) for v in brp.read_template_bank(str(BANK)))
    tin = (P[:4], tau[:4], psi[:4])

    # stage 1: kernel variants
    results = []
    for persist in (0, 2, 3, 4, 6, 8):
        env = {"BRP_PERSIST": persist}
        us = stage_time(brp, geom, series, zaps, tin, env)
        results.append(dict(persist_per_cu=persist, us_per_template=round(us, 2)))
        print(json.dumps(results[-1]), flush=True)
    best = min(results, key=lambda r: r["us_per_template"])

    # stage 2: batch x pipelines with the stage-1 winner (subprocess bench runs)
    env = dict(os.environ, BRP_PERSIST=str(best["persist_per_cu"]))
    conc = []
    for batch, pipes in ((1, 2), (1, 3), (1, 4), (2, 2), (2, 3)):
        r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "2", "--warmup", "1", "--templates",
                            str(args.templates), "--batch", str(batch), "--streams", str(pipes)],
                           env=env, capture_output=True, text=True, timeout=600)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if r.returncode != 0 or not line:
            print(r.stderr[-2000:], file=sys.stderr)
            return 1
        v = json.loads(line[-1])["value"]
        conc.append(dict(batch=batch, pipelines=pipes, templates_per_s=v))
        print(json.dumps(conc[-1]), flush=True)
    bc = max(conc, key=lambda r: r["templates_per_s"])

    entry = dict(arch=arch, M=int(M), persist_per_cu=best["persist_per_cu"], batch=bc["batch"],
                 pipelines=bc["pipelines"], us_per_template_sequential=best["us_per_template"],
                 templates_per_s=bc["templates_per_s"], date=datetime.date.today().isoformat(), stage1=results,
                 stage2=conc)
    out = Path(args.out)
    doc = {"entries": []}
    if out.exists():
        doc = json.loads(out.read_text())
    doc["entries"] = [e for e in doc.get("entries", []) if not (e.get("arch") == arch and e.get("M") == int(M))]
    doc["entries"].append(entry)
    out.parent.mkdir(parents=True, exist_ok=True)
    # one flat object per entry line (the C++ reader scans flat objects):
    # the per-candidate measurements go to a sibling file
    flat = [{k: v for k, v in e.items() if k not in ("stage1", "stage2", "stage3")} for e in doc["entries"]]
    out.write_text("{\"entries\": [\n" + ",\n".join("  " + json.dumps(e) for e in flat) + "\n]}\n")
    out.with_suffix(".measurements.json").write_text(json.dumps(doc, indent=1) + "\n")
    print(f"wrote {out}: {json.dumps(flat[-1])}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
