"""The end-to-end example (host tables -> GPU projection -> H -> MLPCONV) learns the task."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_geolocate_pipeline(cuda, monkeypatch, capsys):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples"))
    import geolocate_pipeline as gp
    monkeypatch.setattr(sys, "argv", ["geolocate_pipeline.py", "--users", "3000", "--epochs", "60"])
    acc = gp.main()
    assert acc > 0.5  # 12 regions: chance is 0.083
