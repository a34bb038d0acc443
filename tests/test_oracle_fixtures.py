"""The CPU oracle reproduces its committed self-consistency fixtures (tests/golden/oracle_scenarios.json,
written by tests/golden/make_oracle_fixtures.py): per-step view/deadline digests, protocol counters
and the running hash of the ordered MembershipEvent stream, for every scenario of tests/scenarios.py."""
import json
import os

import pytest

import scenarios

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "oracle_scenarios.json")))["scenarios"]


@pytest.mark.parametrize("name", sorted(FIX))
def test_oracle_matches_fixture(name):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_oracle_fixtures

    got = make_oracle_fixtures.trace(name)
    want = FIX[name]
    assert (got["n"], got["seed"]) == (want["n"], want["seed"])
    assert len(got["steps"]) == len(want["steps"])
    for i, (g, w) in enumerate(zip(got["steps"], want["steps"])):
        assert g == w, f"{name}: step {i} differs from the fixture"


def test_fixture_covers_every_scenario():
    assert set(FIX) == set(scenarios.SCENARIOS)
