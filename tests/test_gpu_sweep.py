"""Seeded, bounded subsets of the randomised parity sweep (tools/parity_sweep.py)
in the driver's `-m gpu` suite, ~60 s together.

Each trial compares verdicts, rule ids and every counter of the product library
with the oracle (stateful trials also the whole session table):
- chains of 4,100-8,000 rules in every chain (2-4 summary blocks: the two-item
  deal and the global counter atomics past the LDS bins), pcn-iptables and
  pcn-firewall in conntrack modes DISABLED / MANUAL / AUTOMATIC, generic kernel
  and chain programs; two seeds whose chains the reference's LPM trie cannot
  hold (> 1,024 prefixes, Iptables_IpLookup_dp.c:54-55): the product must refuse
  them with -ENOSPC and "LPM trie full" at apply_rules, where the reference's map
  push throws (modules/IpLookup.cpp:130-140, libs/polycube/src/table.cpp:61-66);
- small quirky chains with edge-case frames (both hooks, both directions,
  labels, in_port, fixed and variable lengths);
- stateful multi-batch flows through the GPU connection table.
The seeds are fixed, so a failure reproduces with
`python tools/parity_sweep.py [--big|--stateful] --seed0 S --trials 1`."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import parity_sweep  # noqa: E402

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

# 90000-90023 cover pcn-iptables with and without chain programs and pcn-firewall
# in each conntrack mode with and without them (the first two draws of each seed);
# 80106 (pcn-iptables) and 80170 (pcn-firewall, AUTOMATIC) draw chains past the
# trie capacity (profiles/r04_sweep2/sweep_big.log)
BIG_SEEDS = list(range(90000, 90024)) + [80106, 80170]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _check(r):
    assert r["mismatches"] == 0 and r["counters_equal"], r


@pytest.fixture
def big():
    parity_sweep.BIG = True
    yield
    parity_sweep.BIG = False


@pytest.mark.parametrize("part", range(4))
def test_big_chain_sweep(dev, big, part):
    seen = []
    for seed in BIG_SEEDS[part::4]:
        r = parity_sweep.trial(seed, torch, dev)
        _check(r)
        seen.append(r)
    # what the slice covered (the whole list: every service x program choice, 2 refusals)
    refused = [r for r in seen if "oracle_refused" in r]
    for r in refused:
        assert r["product_refused"] and "LPM trie full" in r["product_error"], r


def test_big_chain_sweep_covers_every_mode():
    """The seed list itself (CPU, no trial run): both services, every firewall conntrack
    mode, chain programs on and off."""
    import numpy as np
    combos = set()
    for seed in BIG_SEEDS[:24]:
        rng = np.random.default_rng(seed)
        fw_mode = int(rng.integers(-1, 3))
        jit = int(rng.choice([1, 1, -1]))
        combos.add((fw_mode, jit))
    assert combos == {(m, j) for m in (-1, 0, 1, 2) for j in (1, -1)}


@pytest.mark.parametrize("part", range(2))
def test_quirky_chain_sweep(dev, part):
    for seed in range(1000 + 30 * part, 1030 + 30 * part):
        _check(parity_sweep.trial(seed, torch, dev))


@pytest.mark.parametrize("part", range(2))
def test_stateful_sweep(dev, part):
    fused = 0
    for seed in range(5000 + 20 * part, 5020 + 20 * part):
        r = parity_sweep.stateful_trial(seed, torch, dev)
        _check(r)
        assert r["tables_equal"], r
        fused += r["fused_batches"]
    # half the trials run 64-byte frames of one length: the fused stage A (its walk
    # records and stale ports) is in the sweep wherever the chain has no conntrack rules
    assert fused > 0, "no trial took the fused stage A"
