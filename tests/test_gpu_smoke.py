"""The driver's round-end smoke() (one small hot-path run on cuda:0 checked against the oracle),
run in the GPU suite so a change of the pipeline's contract shows up here first."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_graft_entry_smoke():
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import __graft_entry__ as g
    g.smoke()
