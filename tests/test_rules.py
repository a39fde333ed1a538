"""coll/tuned's dynamic rules file as coll/mi355x reads it (host logic, no GPU).

The reader restates ompi/mca/coll/tuned/coll_tuned_dynamic_file.c:56-283 and the lookups
coll_tuned_dynamic_rules.c:287-393: numbers read like fscanf("%li") (decimal, hex, octal),
'#' comments, per-communicator-size rule = last one whose size <= n (else the first), per-message
rule = last one whose size <= m, and the file is rejected (with its line) when a section is short
or when a communicator rule does not start at message size 0.
"""
from __future__ import annotations

import pytest

from conftest import load_pkg

RULES = """# two collectives
2
2            # ALLREDUCE (coll_tuned.h:44)
2            # two communicator sizes
4 3          # comm size 4: three message sizes
0     3 0 0  # recursive doubling from 0 B
0x2000 4 0 0 # ring from 8 KiB (hex, as %li reads it)
1048576 5 0 65536
16 2
0 4 0 0
010 2 0 0    # octal 8 -> 8 B: nonoverlapping
11           # REDUCE (coll_tuned.h:53)
1
1 2
0 2 4 0
65536 3 1 32768
"""


@pytest.fixture()
def rules(tmp_path):
    pkg = load_pkg()
    f = tmp_path / "rules.conf"
    f.write_text(RULES)
    r = pkg.Rules(str(f))
    yield pkg, r
    r.destroy()


def test_counts_and_lookups(rules):
    pkg, r = rules
    AR, RED = pkg.COLL["ALLREDUCE"], pkg.COLL["REDUCE"]
    assert r.ncoll == 2
    # comm size 4 rule
    assert r.decide(AR, 4, 0)[0] == 3
    assert r.decide(AR, 4, 8191)[0] == 3
    assert r.decide(AR, 4, 8192)[0] == 4
    assert r.decide(AR, 4, 1 << 20) == (5, 0, 65536)
    # comm sizes 5..15 still use the size-4 rule; 16 and above the size-16 rule
    assert r.decide(AR, 15, 1 << 30)[0] == 5
    assert r.decide(AR, 16, 7)[0] == 4
    assert r.decide(AR, 64, 8)[0] == 2
    # smaller than every communicator rule: the first rule (get_com_rule_ptr starts there)
    assert r.decide(AR, 2, 100)[0] == 3
    # reduce: fan-in/out and segment size come with the rule
    assert r.decide(RED, 8, 100) == (2, 4, 0)
    assert r.decide(RED, 8, 65536) == (3, 1, 32768)
    # collectives without rules -> 0 (no rule)
    assert r.decide(pkg.COLL["BCAST"], 4, 100)[0] == 0
    assert r.decide(pkg.COLL["REDUCESCATTER"], 4, 100)[0] == 0


@pytest.mark.parametrize("text,what", [
    ("", "number of collectives"),
    ("17\n", "more collectives"),
    ("1\n16 0\n", "collective id out of range"),
    ("1\n2 1\n4 1\n8 3 0 0\n", "must be 0"),
    ("1\n2 1\n4 2\n0 3 0 0\n", "message size"),
    ("1\n2 1\n4 1\n0 3 0\n", "segment size"),
])
def test_rejected_files(tmp_path, text, what):
    pkg = load_pkg()
    f = tmp_path / "bad.conf"
    f.write_text(text)
    with pytest.raises(pkg.MI355XError, match=what):
        pkg.Rules(str(f))


def test_missing_file(tmp_path):
    pkg = load_pkg()
    with pytest.raises(pkg.MI355XError, match="cannot read"):
        pkg.Rules(str(tmp_path / "nope.conf"))
