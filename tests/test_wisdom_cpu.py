"""Plan wisdom (csrc/core/wisdom.cpp): entry lookup by (arch, M) with the
gcnArchName feature suffix ignored, missing files/entries, and the committed
MI355X wisdom file parses."""
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def test_wisdom_lookup(brp, tmp_path):
    p = tmp_path / "w.json"
    p.write_text('{"entries": [\n'
                 '  {"arch": "gfx942", "M": 6291456, "persist_per_cu": 2},\n'
                 '  {"arch": "gfx950", "M": 6291456, "persist_per_cu": 6,'
                 ' "batch": 1, "pipelines": 3, "date": "2026-10-16"},\n'
                 '  {"arch": "gfx950", "M": 2097152, "persist_per_cu": 8}\n]}\n')
    w = brp.load_wisdom(str(p), "gfx950:sramecc+:xnack-", 6291456)
    assert w["found"] and w["persist_per_cu"] == 6
    assert w["batch"] == 1 and w["pipelines"] == 3
    w = brp.load_wisdom(str(p), "gfx950", 2097152)
    assert w["found"] and w["persist_per_cu"] == 8 and w["batch"] == -1
    assert not brp.load_wisdom(str(p), "gfx950", 123)["found"]
    assert not brp.load_wisdom(str(tmp_path / "missing.json"), "gfx950", 6291456)["found"]


def test_repository_wisdom_parses(brp):
    p = ROOT / "data" / "wisdom" / "mi355x.json"
    assert brp.wisdom_path() == str(p) or brp.wisdom_path()  # BRP_WISDOM may override
    if p.exists():
        w = brp.load_wisdom(str(p), "gfx950", 6291456)
        assert w["found"] and w["persist_per_cu"] >= 0 and w["pipelines"] >= 1
