import os
import sys

# Kernel arguments in host memory (HIP_FORCE_DEV_KERNARG=0), set before anything initialises HIP.
# Device-memory kernel arguments are the suspected cause of the intermittent control-kernel
# faults (DESIGN.md §3 "The control-kernel fault"). An explicit setting in the environment wins.
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "0")

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP engine)")
    config.addinivalue_line("markers", "slow: longer CPU cross-checks")
