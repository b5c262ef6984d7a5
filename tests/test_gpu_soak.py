"""A short run of the randomised soak (scripts/soak.py): drawn configurations (R 1-8, payloads 0-256 B
and longer caller Cmds, loss, snapshots, CRC-32C, partial memberships; one engine, every message
through the wire, or 2-4 ranks), every input kind at random, the GPU engine equal to the C oracle
after every tick. The long runs are in profiles/r05*_soak.log."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))


@pytest.mark.parametrize("seed", [7, 1003, 2011, 3001, 4007, 5003])
def test_soak_configuration(seed):
    import soak
    assert soak.run(seed, 120)
