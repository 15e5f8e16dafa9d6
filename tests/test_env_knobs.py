"""The shipped library's environment surface: the set of
DIPS_* variables the sources in dips_amd/csrc read equals the table in
INTEGRATION.md's "Environment knobs" section, and every parity test that
table names exists.  Alternative kernel forms are handle flags
(DIPS_FLAG_CROSSCHECK, DIPS_FLAG_GRAY_*_TABLE), not variables."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dips_amd", "csrc")


def _read_vars():
    found = set()
    for fn in os.listdir(CSRC):
        if fn.endswith((".hip", ".h", ".cpp")):
            with open(os.path.join(CSRC, fn)) as f:
                found |= set(re.findall(r'getenv\(\s*"(DIPS_[A-Z0-9_]+)"\s*\)', f.read()))
    return found


def _table():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## Environment knobs"):]
    nxt = sec.find("\n## ", 3)
    sec = sec if nxt < 0 else sec[:nxt]
    rows = re.findall(r"^\| `(DIPS_[A-Z0-9_]+)` \|(.*)$", sec, flags=re.M)
    return {name: rest for name, rest in rows}


def test_library_reads_exactly_the_documented_knobs():
    read = _read_vars()
    table = _table()
    assert read == set(table), {"undocumented": sorted(read - set(table)), "not read": sorted(set(table) - read)}
    assert len(read) <= 6, read  # deployment sizing only


def test_every_knob_names_an_existing_parity_test():
    table = _table()
    for name, rest in table.items():
        cites = re.findall(r"`(tests/[\w/]+\.py)(?:::(\w+))?`", rest)
        assert cites, name
        for path, func in cites:
            src = open(os.path.join(ROOT, path)).read()
            assert name in src, (name, path)
            if func:
                assert f"def {func}(" in src, (name, path, func)
