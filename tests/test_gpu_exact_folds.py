"""The exact in-order folds of k_step (getBrokerLoad / getUnbalanceBL, utils.go:92-143)
at every broker count the chain's batching can split differently.

exact_unbalance_wave runs the additions as a broadcast-LDS chain in batches of 16
elements, then a tail, per 64-element chunk, and substitutes the moved broker's two
loads (ps / pt) through a per-wave LDS row only in the chunks that hold them.  With
`exact_unbalance=True` every move() decision folds, so each plan below exercises
n mod 16 and n mod 64 tails, substitutions inside a tail, and (past 1024 brokers)
more brokers than k_step has threads.  Bar: the oracle's plan, su / cu bit for bit
(assert_same_plan checks exact decisions bitwise).
"""
import random

import pytest

from kafkabalancer_amd import engine as E

from test_gpu_parity_data import random_plist
from helpers import assert_same_plan, default_cfg, oracle_plan

pytestmark = pytest.mark.gpu

BROKERS = [1, 2, 3, 15, 16, 17, 31, 63, 64, 65, 79, 127, 128, 129, 255, 1023, 1025, 1500]


@pytest.mark.parametrize("B", BROKERS)
@pytest.mark.parametrize("weights", ["int", "zipf"])
def test_exact_folds_vs_oracle(B, weights):
    rng = random.Random(9100 + B * 3 + (weights == "zipf"))
    # the oracle scores every candidate with a full O(B) fold: past 255 brokers
    # 400 partitions and 10 steps keep it to a few seconds
    P, steps = (max(40, 3 * B), 30) if B <= 255 else (400, 10)
    pl = random_plist(rng, P, B, weights, "none", False, False)
    cfg = default_cfg(allow_leader=B % 2 == 1, min_unbalance=0.0)
    eng = E.Engine(pl, cfg, exact_unbalance=True)
    ech, eerr = eng.plan(steps)
    och, oerr, opl = oracle_plan(pl, cfg, steps)
    assert_same_plan(ech, eerr, och, oerr)
    moves = [c for c in ech if c["step"] in ("MoveLeaders", "MoveNonLeaders")]
    assert all(c.get("exact") for c in moves), "a move() decision was not folded"
    if oerr is None:
        assert eng.state() == opl.state()
    eng.close()
