#!/usr/bin/env python3
"""Benchmark: templates/s of one full BRP work unit on N MI355X GPUs.

Reproduces the reference benchmark configuration
(debian/extra/einstein_bench/bench_single.sh:28):
  -i p2030.20151015.G187.41-00.88.N.b2s0g0.00000_1099.bin4  (2^22 samples)
  -t stochastic_full.bank (6662 templates) -l <zaplist>
  -A 0.08 -P 3.0 -f 400.0 -W
One step = the whole work unit: device whitening/zapping, every template of
the bank (sharded over the ranks in contiguous blocks), one RCCL all-gather of
the 24 KB candidate tables and the exact merge. Strong scaling: the total work
per step is fixed, `value` is templates/s of the whole job.

  python bench.py --gpus 1 --steps 3 --warmup 1
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
      --master-port 29500 bench.py --gpus 8 --steps 3 --warmup 1
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "templates/sec (whole node), 2^22-sample WU at 1/2/4/8 MI355X; candidate recall"
DATA = ROOT / "data" / "testwu"
WU = DATA / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000_1099.bin4"
BANK = DATA / "stochastic_full.bank"
ZAP = DATA / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000.zap"
GOLDEN = ROOT / "data" / "golden" / "bench_wu_cpu_results.txt"  # tools/make_golden.py (CPU golden model)


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    # 1 template x 3 pipelines keeps every pipeline's FFT buffers (71 MB each) resident in the
    # 256 MB Infinity Cache between passes: +7-8 % over 8 x 2 (profiles/README.md)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("BRP_BATCH", "1")))
    ap.add_argument("--streams", type=int, default=int(os.environ.get("BRP_STREAMS", "3")),
                    help="independent pipelines (stream + buffers) per GPU; >1 overlaps host sync with compute")
    ap.add_argument("--templates", type=int, default=0, help="limit the bank (0 = all 6662)")
    ap.add_argument("--ps-fp16", action="store_true",
                    help="config 5: fp16 power spectrum (precision/throughput trade; recall is reported)")
    ap.add_argument("--wus", type=int, default=1,
                    help="work units resident per GPU (config 4): the reference WU + synthetic WUs of its shape")
    ap.add_argument("--synthetic", action="store_true", help="synthetic WU/bank of the benchmark shape")
    ap.add_argument("--padding", type=float, default=3.0,
                    help="-P (3.0 = the headline config; other values measure e.g. the chirp-z path, not the metric)")
    ap.add_argument("--write-output", default="", help="rank 0 writes the result file of the last step here")
    ap.add_argument("--shard-of", default="",
                    help="N:R = time only rank R's template block of an N-rank run on this one GPU "
                         "(compute-only scaling proxy; no collectives; not the driver's metric)")
    ap.add_argument("--cpu", action="store_true",
                    help="rehearsal of the multi-rank path without GPUs: gloo collectives, CPU golden backend, "
                         "small synthetic WU (not a benchmark; used by tests/test_bench_cpu.py)")
    return ap.parse_args()


def synthetic_inputs(workdir: Path):
    from boinc_app_eah_brp_amd.utils import synth

    case = synth.synthetic_case(workdir, n=1 << 22, n_templates=6661,
                                inj=synth.Injection(f0=123.4, P_orb=1500.0, tau=0.1, psi0=1.0, amplitude=0.2))
    return Path(case["wu"]), Path(case["bank"]), Path(case["zap"])


GOLDEN_TABLE = ROOT / "data" / "golden" / "bench_wu_cpu_table.bin"


def recall_vs_golden(table, geom) -> dict | None:
    """Candidate recall against the CPU golden model run of the whole bank
    (tools/make_golden.py):
      results: fraction of the golden result-file lines (top <= 100 by
               significance, one per frequency) whose (f0 bin, n_harm) appears
               among this run's result lines;
      table:   fraction of the golden 5x100 table entries (level, bin) present
               in this run's table."""
    if not GOLDEN.exists():
        return None
    import tempfile

    from boinc_app_eah_brp_amd import native

    brp = native()
    t_obs = geom["t_obs_d"]

    def lines_of(path):
        out = set()
        with open(path) as fh:
            for line in fh:
                if line.startswith("%") or not line.strip():
                    continue
                f = line.split()
                out.add((round(float(f[0]) * t_obs), int(f[6])))
        return out

    golden = lines_of(GOLDEN)
    with tempfile.TemporaryDirectory() as d:
        p = Path(d) / "ours.cand"
        brp.write_results(str(p), table, t_obs, False)
        ours = lines_of(p)
    rec = {"results": round(len(golden & ours) / max(1, len(golden)), 4), "golden_lines": len(golden)}
    if GOLDEN_TABLE.exists():
        import numpy as np

        gt = brp.CandidateTable()
        gt.from_bytes(np.frombuffer(GOLDEN_TABLE.read_bytes(), dtype=np.uint8).copy())

        def keyset(t):
            ent = t.entries()
            return {(k // 100, int(e[0])) for k, e in enumerate(ent) if e[5] > 0}

        g, o = keyset(gt), keyset(table)
        rec["table"] = round(len(g & o) / max(1, len(g)), 4)
        rec["golden_entries"] = len(g)
    return rec


def visible_gpus(topology: str = "/sys/class/kfd/kfd/topology/nodes", dev_dir: str = "/dev/dri") -> int:
    """GPUs this process may use, counted without any HIP call (so the bench
    parent never creates a HIP context its rank processes could inherit, and
    never depends on whether torch.cuda.device_count() falls back to
    hipGetDeviceCount): KFD topology nodes with a non-zero gfx_target_version
    whose DRM render node is present and accessible, then narrowed by
    ROCR_VISIBLE_DEVICES and HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES in the
    runtime's order (each list indexes the devices the previous one left; the
    list ends at its first invalid entry; an empty list hides every device)."""
    try:
        nodes = sorted(os.listdir(topology), key=lambda x: int(x) if x.isdigit() else 1 << 30)
    except OSError:
        return 0
    n = 0
    for node in nodes:
        try:
            with open(os.path.join(topology, node, "properties")) as fh:
                props = dict(ln.split(None, 1) for ln in fh.read().splitlines() if len(ln.split(None, 1)) == 2)
        except (OSError, ValueError):
            continue
        try:
            if int(props.get("gfx_target_version", "0")) == 0:
                continue  # a CPU node
            minor = int(props.get("drm_render_minor", "-1"))
        except ValueError:
            continue
        render = os.path.join(dev_dir, f"renderD{minor}")
        if minor >= 0 and os.path.exists(render) and not os.access(render, os.R_OK | os.W_OK):
            continue  # present in the topology, not ours (device cgroup / permissions)
        n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        val = os.environ.get(var)
        if val is None:
            continue
        if var == "CUDA_VISIBLE_DEVICES" and os.environ.get("HIP_VISIBLE_DEVICES") is not None:
            continue  # HIP's own variable wins
        kept, seen = 0, set()
        for tok in (t.strip() for t in val.split(",")):
            if not tok:
                break
            if tok.isdigit():
                if int(tok) >= n or tok in seen:
                    break
                seen.add(tok)
            kept += 1  # a UUID (ROCR) names one device
        n = min(n, kept)
    return n


def share_device() -> bool:
    """BRP_BENCH_SHARE_DEVICE=1 (tests only): every rank runs on device 0 and
    the ranks talk over gloo, so the self-launched multi-rank path (rank
    processes, floor exchange, all-gather, merge) runs on a one-GPU box. Not a
    throughput measurement: the JSON line says so."""
    return os.environ.get("BRP_BENCH_SHARE_DEVICE") == "1"


def launch_ranks(args) -> int:
    """`--gpus N` (N > 1) without a launcher environment: start the N rank
    processes here, one per GPU, the way torch.distributed.run would
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT).
    Nothing in this process touches the GPU (the devices are counted from
    sysfs, visible_gpus), so no rank inherits a HIP context. Rank 0 prints the
    JSON line. Fewer visible devices than N is an error, never a silent 1-GPU
    run (BRP_BENCH_SHARE_DEVICE=1: one device is enough, see share_device)."""
    import socket
    import subprocess

    n = args.gpus
    if not args.cpu:
        need = 1 if share_device() else n
        have = visible_gpus()
        if have < need:
            # second opinion from the runtime, in a child process (this parent
            # must stay free of HIP): the sysfs view can miss devices on hosts
            # that expose them differently
            try:
                r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                                   capture_output=True, text=True, timeout=300)
                have = max(have, int(r.stdout.strip().splitlines()[-1]))
            except (OSError, ValueError, IndexError, subprocess.SubprocessError):
                pass
        if have < need:
            print(f"[bench] error: --gpus {n} but only {have} HIP device(s) are visible", file=sys.stderr)
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), BRP_BENCH_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *sys.argv[1:]], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                print(f"[bench] rank process {procs.index(p)} exited with {code}; stopping the others",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


def main() -> int:
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and not args.shard_of:
        return launch_ranks(args)
    import torch  # noqa: F401  (loads the HIP runtime first; RCCL backend)

    from boinc_app_eah_brp_amd import native
    from boinc_app_eah_brp_amd.parallel import ShardedSearch, barrier, init_distributed, max_over_ranks

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if not args.shard_of and world_env != args.gpus:
        print(f"[bench] error: --gpus {args.gpus} but WORLD_SIZE={world_env}", file=sys.stderr)
        return 2
    shared = share_device() and not args.cpu and world_env > 1
    if not args.cpu and not args.shard_of and not shared and torch.cuda.device_count() < world_env:
        print(f"[bench] error: {world_env} ranks but only {torch.cuda.device_count()} HIP device(s)", file=sys.stderr)
        return 2
    ctx = init_distributed("gloo" if (args.cpu or shared) else None)
    if args.shard_of:
        from boinc_app_eah_brp_amd.parallel import DistContext

        n_of, r_of = (int(x) for x in args.shard_of.split(":"))
        ctx = DistContext(rank=r_of, world=n_of, local_rank=ctx.local_rank, backend="none", solo_shard=True)
    use_gpu = torch.cuda.is_available() and not args.cpu
    world = 1 if ctx.solo_shard else ctx.world
    brp = native()
    brp.set_log_level(2)
    wu, bank, zap = WU, BANK, ZAP
    data_desc = "real: reference test WU p2030...b2s0g0.00000_1099.bin4 (2^22 4-bit samples) + stochastic_full.bank"
    window = 1000
    if args.cpu:
        from boinc_app_eah_brp_amd.utils import synth

        case = synth.synthetic_case(Path(os.environ.get("TMPDIR", "/tmp")) / f"brp_bench_cpu_{ctx.rank}", n=1 << 15,
                                    n_templates=24,
                                    inj=synth.Injection(f0=211.0, P_orb=900.0, tau=0.03, psi0=0.7, amplitude=3.0))
        wu, bank, zap = Path(case["wu"]), Path(case["bank"]), Path(case["zap"])
        window = 100
        data_desc = "synthetic CPU rehearsal of the multi-rank path (2^15 samples, 25 templates; not a benchmark)"
    elif args.synthetic or not WU.exists():
        wu, bank, zap = synthetic_inputs(Path(os.environ.get("TMPDIR", "/tmp")) / f"brp_bench_{ctx.rank}")
        data_desc = "synthetic: 2^22-sample 4-bit WU with an injected binary pulsar + random 6662-template bank"
    opts = dict(inputfile=str(wu), templatebank=str(bank), zaplistfile=str(zap), f0=400.0, padding=args.padding, fA=0.08,
                window=window, white=True, batch=args.batch, outputfile=args.write_output, ps_fp16=args.ps_fp16)
    n_wus = max(1, args.wus)
    if n_wus > 1:
        from boinc_app_eah_brp_amd.models import MultiWUSearch, SearchConfig
        from boinc_app_eah_brp_amd.models.multi import same_shape_synthetic_wus

        hdr, _, _ = brp.read_work_unit(str(wu))
        if ctx.rank == 0:
            print(f"[bench] preparing {n_wus - 1} synthetic WUs", file=sys.stderr, flush=True)
        extra = same_shape_synthetic_wus(Path(os.environ.get("TMPDIR", "/tmp")) / "brp_bench_wus", hdr, n_wus - 1)
        cfg = SearchConfig.benchmark(str(wu), str(bank), str(zap), batch=args.batch, ps_fp16=args.ps_fp16)
        search = MultiWUSearch([str(wu)] + extra, cfg, pipelines=args.streams, ctx=ctx)
        data_desc += f" + {n_wus - 1} synthetic WUs of the same shape (noise + injected binary pulsars)"
    else:
        search = ShardedSearch(opts, ctx, device=0 if shared else None, streams=1 if args.cpu else args.streams,
                               use_cpu=args.cpu)
    limit = args.templates if args.templates > 0 else search.total

    def first_table(t):
        return t[0] if isinstance(t, list) else t
    if use_gpu:
        torch.cuda.synchronize()

    lead = ctx.rank == 0 or ctx.solo_shard

    def progress(msg):
        # long runs (config 4 at many WUs) stay visibly alive on stderr; stdout keeps the one JSON line
        if lead:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    table = None
    for w in range(args.warmup):
        progress(f"warmup step {w + 1}/{args.warmup}")
        table = search.step(limit)
    first = bytes(first_table(table).to_bytes()) if table is not None else None
    barrier(ctx)
    if use_gpu:
        torch.cuda.synchronize()
    search.timings.clear()
    progress(f"timing {args.steps} step(s)")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        table = search.step(limit)
    barrier(ctx)
    if use_gpu:
        torch.cuda.synchronize()
    elapsed = max_over_ranks(time.perf_counter() - t0, ctx)

    tables = table if isinstance(table, list) else [table]
    table = tables[0]
    if args.write_output and n_wus == 1:
        search.write_output(table, limit)
    stats = search.session.stats()
    if lead:
        geom = search.session.geometry()
        work = limit
        if ctx.solo_shard:
            from boinc_app_eah_brp_amd.parallel import shard_range

            lo, hi = shard_range(limit, ctx.rank, ctx.world)
            work = hi - lo
        total = work * args.steps * n_wus
        value = total / elapsed
        n_cands = sum(1 for e in table.entries() if e[5] > 0)
        rec = (recall_vs_golden(table, geom) if limit == search.total and not args.cpu and not ctx.solo_shard
               and args.padding == 3.0 else None)
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "templates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "baseline_note": "reference publishes no templates/s; BASELINE.md derives ~2.1 templates/s per CPU core",
            "vs_derived_cpu_core": round(value / 2.1, 1),
            "dtype": "fp32 FFT, fp16 power spectrum (inexact experiment mode)" if args.ps_fp16 else "fp32",
            "data": data_desc,
            "recall_vs_golden": rec,
            "candidates_in_table": n_cands,
            "collective_failure_degraded": ctx.degraded,
            "floor_sync_rounds_last_step": getattr(search, "floor_rounds", None),
            "launched_by": "bench.py" if os.environ.get("BRP_BENCH_LAUNCHED") else
                           ("torch.distributed.run" if world > 1 else "single process"),
            "table_identical_to_warmup": (first == bytes(table.to_bytes())) if first is not None else None,
            "table_sha256": hashlib.sha256(bytes(table.to_bytes())).hexdigest(),
            "busy_span_ms_rank0": round(stats["busy_span_ms"], 3),
            "device_candidates_per_template_rank0": round(stats.get("candidates", 0) / max(1, stats["templates"]), 2),
            "bounded_output_batches_rank0": stats.get("select_batches", 0),
            "whiten_ms_rank0": round(stats["whiten_ms"], 3),
            "phase_ms_per_step_rank0": {k: round(1e3 * v / args.steps, 2) for k, v in search.timings.items()},
            "config": {
                "model": f"Einstein@Home BRP4 search (-P {args.padding:g} -f 400 -A 0.08 -W): resample + "
                         f"{int(geom['nsamples'])}-pt real FFT + 16-harmonic sum + top-100 per level",
                "global_batch": limit,
                "seq_len": int(geom["n_unpadded"]),
                "fft_len": int(geom["nsamples"]),
                "parallelism": f"dp{world} (template-bank sharding, RCCL all-gather of candidate tables)",
                "device_batch": args.batch,
                "pipelines_per_gpu": args.streams,
                "work_units": n_wus,
            },
        }
        if shared:
            out["shared_device"] = ("all ranks ran on device 0 over gloo (BRP_BENCH_SHARE_DEVICE=1): a test of the "
                                    "multi-rank launch, not a multi-GPU throughput")
        if ctx.solo_shard:
            out["shard_of"] = {"world": ctx.world, "rank": ctx.rank, "templates": work,
                               "note": "compute-only timing of one rank's block on one GPU (no collectives)"}
        print(json.dumps(out), flush=True)
    if ctx.distributed:
        import torch.distributed as dist

        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
