"""Every reference-legal input on the GPU (pytest -m gpu): the bounded
candidate output and the geometry-sized candidate keys (hip_engine.cpp,
harmonic_sum.hip launch_harmonic_sum_select).

The reference's CPU path inserts any number of above-threshold bins per
template (demod_binary.c:1310-1397, hs_common.c:95-99); the device list of a
batch has a fixed number of slots. A batch that overflows it is re-run with
the bounded output (per template and level only the values >= the 100th
largest), which gives the in-order applier exactly the same table. Golden
tables come from the CPU golden model (tools/make_golden.py)."""
from pathlib import Path

import numpy as np
import pytest

from boinc_app_eah_brp_amd.models import BRPSearch, SearchConfig
from boinc_app_eah_brp_amd.utils import synth

from conftest import BANK, ROOT, WU, ZAP
from test_gpu_search import _cfg, _compare_tables

pytestmark = pytest.mark.gpu

GOLDEN = ROOT / "data" / "golden"
INJ = synth.Injection(f0=211.0, P_orb=900.0, tau=0.03, psi0=0.7, amplitude=3.0)


@pytest.fixture(scope="module")
def case(tmp_path_factory):
    return synth.synthetic_case(tmp_path_factory.mktemp("bcase"), n=1 << 16, n_templates=37, inj=INJ)


def _golden(name):
    brp = __import__("boinc_app_eah_brp_amd").native()
    t = brp.CandidateTable()
    t.from_bytes(np.frombuffer((GOLDEN / name).read_bytes(), dtype=np.uint8).copy())
    return t


def _run(cfg, monkeypatch=None, pipelines=1, **env):
    if monkeypatch is not None:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
    return BRPSearch(cfg, pipelines=pipelines).run(write_output=False, use_checkpoint=False)


def test_bounded_output_equals_compacting_path(brp, gpu, case, tmp_path, monkeypatch):
    """BRP_HS_SELECT=1 (the bounded output for every batch) gives the table of
    the compacting path byte for byte, whitened and raw series."""
    for white in (True, False):
        ref = _run(_cfg(case, tmp_path / f"c{white}", white=white, batch=4))
        monkeypatch.setenv("BRP_HS_SELECT", "1")
        sel = _run(_cfg(case, tmp_path / f"s{white}", white=white, batch=4))
        monkeypatch.delenv("BRP_HS_SELECT")
        assert sel.stats["select_batches"] > 0
        assert bytes(sel.table.to_bytes()) == bytes(ref.table.to_bytes()), white


def test_small_list_overflow_reruns_exactly(brp, gpu, case, tmp_path, monkeypatch):
    """Fault injection: a small list (BRP_HS_CAP; the engine keeps it at the
    bounded output's size, 8 templates x 5 levels x 128 slots) overflows at
    -A 1; those batches are re-run with the bounded output and the table is
    the default run's (whose 2^20-slot lists hold everything), byte for byte.
    Three pipelines, two batches in flight each."""
    # -A 1: zero thresholds, every bin of [w2, fhi) is above them (~25 k values per template)
    ref = _run(_cfg(case, tmp_path / "a", fA=1.0, batch=2), pipelines=3)
    monkeypatch.setenv("BRP_HS_CAP", "64")
    small = _run(_cfg(case, tmp_path / "b", fA=1.0, batch=2), pipelines=3)
    assert small.stats["overflow_reruns"] > 0, small.stats
    assert bytes(small.table.to_bytes()) == bytes(ref.table.to_bytes())


def test_reference_wu_without_whitening_vs_cpu_golden(brp, gpu, tmp_path):
    """The shipped WU without -W (raw powers ~1.4e6: 329 049 of 329 052
    fundamental bins of template 0 exceed thr1): first 20 templates against
    the CPU golden model (tools/make_golden.py --end 20 --no-white, which pads
    with the accurate mean like the device: on a raw series the reference
    CPU build's serial float mean is ~2 % off, cpu_backend.cpp)."""
    cfg = SearchConfig(inputfile=str(WU), templatebank=str(BANK), zaplistfile=str(ZAP), fA=0.08, padding=3.0,
                       f0=400.0, white=False, batch=1)
    g = BRPSearch(cfg, pipelines=3).run(begin=0, end=20, write_output=False, use_checkpoint=False)
    assert g.templates_run == 20
    assert g.stats["overflow_reruns"] + g.stats["select_batches"] > 0, g.stats
    gold = _golden("bench_wu_cpu_table_first20_noW.bin")
    assert sum(1 for e in gold.entries() if e[5] > 0) == 500
    _compare_tables(g.table, gold)


def test_high_f0_and_padding_wide_keys_vs_cpu_golden(brp, gpu, tmp_path):
    """-P 5 -f 8000 on the shipped WU: fundamental_idx_hi = 10 485 261 > 2^23
    (the previous key layout's limit) with a 5 * 2^22-point FFT; -A 0.9999 so
    that every level has candidates. First 6 templates against the CPU golden
    model (tools/make_golden.py --end 6 --padding 5 --f0 8000 --fA 0.9999)."""
    cfg = SearchConfig(inputfile=str(WU), templatebank=str(BANK), zaplistfile=str(ZAP), fA=0.9999, padding=5.0,
                       f0=8000.0, white=True, batch=1)
    g = BRPSearch(cfg, pipelines=2).run(begin=0, end=6, write_output=False, use_checkpoint=False)
    assert g.geometry["fundamental_idx_hi"] > (1 << 23)
    gold = _golden("bench_wu_cpu_table_first6_A0.9999_f8000_P5.bin")
    assert sum(1 for e in gold.entries() if e[5] > 0) > 50
    _compare_tables(g.table, gold)


@pytest.mark.parametrize("fA", [0.9999, 1.0])
def test_false_alarm_near_one(brp, gpu, case, tmp_path, fA):
    """-A 0.9999 and -A 1 (probability 1: thresholds 0, every bin a
    candidate) on the GPU against the CPU golden model."""
    g = _run(_cfg(case, tmp_path / "g", fA=fA, batch=4))
    c = BRPSearch(_cfg(case, tmp_path / "c", fA=fA, use_cpu=True)).run(write_output=False, use_checkpoint=False)
    _compare_tables(g.table, c.table)



def test_bounded_output_overflow_reruns_exactly(brp, gpu, case, tmp_path, monkeypatch):
    """The last GPU-fatal input class: the bounded output itself overflowing
    (more values >= a 100th place than list slots, a storm of exact ties).
    Forced with a list smaller than one template's bounded output
    (BRP_FAULT=hs_cap_raw, BRP_HS_CAP=64, BRP_HS_SELECT=1, -A 1): every batch
    is re-run into a list sized to its count, and the table equals the default
    run's and the CPU golden model's, never RADPUL_HIP_CAND_OVERFLOW."""
    ref = _run(_cfg(case, tmp_path / "a", fA=1.0, batch=2), pipelines=2)
    for k, v in dict(BRP_FAULT="hs_cap_raw", BRP_HS_CAP="64", BRP_HS_SELECT="1").items():
        monkeypatch.setenv(k, v)
    tie = _run(_cfg(case, tmp_path / "b", fA=1.0, batch=2), pipelines=2)
    assert tie.stats["tie_reruns"] > 0, tie.stats
    assert bytes(tie.table.to_bytes()) == bytes(ref.table.to_bytes())
    for k in ("BRP_FAULT", "BRP_HS_CAP", "BRP_HS_SELECT"):
        monkeypatch.delenv(k)
    c = BRPSearch(_cfg(case, tmp_path / "c", fA=1.0, use_cpu=True)).run(write_output=False, use_checkpoint=False)
    _compare_tables(tie.table, c.table)
