"""High-level search pipelines ("models" of this framework).

`BRPSearch` is the Einstein@Home binary-radio-pulsar search of one work unit
(reference MAIN, demod_binary.c:117-1695): optional whitening + RFI zapping,
then for every orbital template resampling -> real FFT -> power spectrum ->
1/2/4/8/16-harmonic sums -> top-100 candidates per harmonic level, checkpoint
and result file. Backends: "hip" (MI355X kernels) or "cpu" (golden model).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, field
from pathlib import Path

from .. import native


@dataclass
class SearchConfig:
    inputfile: str
    templatebank: str
    outputfile: str = ""
    checkpointfile: str = ""
    zaplistfile: str = ""
    f0: float = 250.0        # -f
    padding: float = 1.0     # -P
    fA: float = 0.04         # -A
    window: int = 1000       # -B
    white: bool = False      # -W
    debug: bool = False      # -z
    device: int = -1         # -D
    batch: int = 4           # templates per device batch
    use_cpu: bool = False
    ps_fp16: bool = False    # fp16 power spectrum (config 5 precision/throughput trade; needs white)

    @classmethod
    def benchmark(cls, wu: str, bank: str, zap: str, **kw) -> "SearchConfig":
        """The reference benchmark flags: -A 0.08 -P 3.0 -f 400.0 -W."""
        return cls(inputfile=wu, templatebank=bank, zaplistfile=zap, fA=0.08, padding=3.0, f0=400.0, white=True, **kw)

    def options(self) -> dict:
        return {k: v for k, v in asdict(self).items()}


@dataclass
class SearchOutput:
    table: object
    geometry: dict
    templates_total: int
    templates_run: int
    interrupted: bool
    timings: dict = field(default_factory=dict)
    stats: dict = field(default_factory=dict)  # backend counters (bounded-output re-runs, ...)

    def candidates(self):
        """Table entries (f0 bin, power, P_b, tau, Psi, n_harm) with n_harm > 0."""
        return [e for e in self.table.entries() if e[5] > 0]


class BRPSearch:
    """Search one work unit with the native driver (C++ host loop, HIP kernels)."""

    def __init__(self, config: SearchConfig, gpus: int = 1, pipelines: int = 1):
        self.config = config
        self.gpus = gpus            # devices (CPU backend: worker threads)
        self.pipelines = pipelines  # HIP pipelines (stream + buffers + host thread) per device
        self.brp = native()

    def run(self, begin: int = 0, end: int = 0, write_output: bool = True, use_checkpoint: bool = True) -> SearchOutput:
        r = self.brp.run_search(self.config.options(), begin, end, write_output, use_checkpoint, self.gpus,
                                self.pipelines)
        return SearchOutput(table=r["table"], geometry=r["geometry"], templates_total=r["templates_total"],
                            templates_run=r["templates_run"], interrupted=r["interrupted"],
                            timings=dict(setup=r["t_setup"], templates=r["t_templates"], total=r["t_total"],
                                         busy_span_ms=r["busy_span_ms"], whiten_ms=r["whiten_ms"]),
                            stats=dict(overflow_reruns=r["overflow_reruns"], select_batches=r["select_batches"],
                                       select_exits=r["select_exits"], tie_reruns=r["tie_reruns"]))

    def results(self):
        lines, done = self.brp.read_results(self.config.outputfile)
        return lines, done

    @staticmethod
    def command_line(args: list[str]) -> int:
        """Run the MAIN-compatible command line parser (e.g. ['prog', '-i', ...])."""
        return native().search_main([str(a) for a in args])


def app_binary() -> Path:
    """Path of the BOINC application executable (built in-tree)."""
    from .._build import app_path

    return app_path()
