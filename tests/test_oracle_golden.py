"""Pin the CPU oracle against the reference's own fixtures (CPU only).

* index64.json — the BitScan De Bruijn table the reference loads
  (modules/BitScan.cpp:32-49); the oracle derives its table from the De Bruijn
  constant of Iptables_BitScan_dp.c:97, so equality pins the bit scan.
* scenarios.json — the reference's integration tests (local_test*.sh) as
  probes with the scripts' own pass/fail assertions (make_scenarios.py).
"""
import json
import os
import random

import pytest

from helpers import GOLDEN, OracleCube, load_scenarios
from oracle.ffi import Oracle, index64


def test_index64_matches_reference_table():
    with open(os.path.join(GOLDEN, "index64.json")) as fh:
        ref = json.load(fh)["index64"]
    assert index64() == ref


def test_debruijn_scan_is_ctz():
    tab = index64()
    rnd = random.Random(7)
    vals = [1 << p for p in range(64)] + [rnd.getrandbits(64) | 1 << rnd.randrange(64) for _ in range(2000)]
    for b in vals:
        idx = (((b ^ (b - 1)) * 0x03F79D71B4CB0A89) & (2**64 - 1)) >> 58
        assert tab[idx] == (b & -b).bit_length() - 1


SCEN = load_scenarios()


@pytest.mark.parametrize("sc", SCEN["scenarios"], ids=[s["name"] for s in SCEN["scenarios"]])
def test_reference_scenarios_on_oracle(sc):
    cube = OracleCube(Oracle(), SCEN["ports"], SCEN["localip"])
    for k, st in enumerate(sc["steps"]):
        for op in st["ops"]:
            cube.op(op)
        if "probe" not in st:
            continue
        verdicts = cube.probe(st["probe"])
        got = "pass" if all(v == 1 for v in verdicts) else "fail"
        assert got == st["expect"], f"{sc['name']} step {k} ({st.get('ref_line', '')}): {verdicts}"
        if "counters" in st:
            c = st["counters"]
            chain = {"INPUT": 0, "FORWARD": 1, "OUTPUT": 2}[c["chain"]]
            pk, _, _, _ = cube.o.read_counters(chain, c["rule"] + 1)
            assert pk[c["rule"]] == c["pkts"]
