"""MLPCONV's default layer-2 order (CPU: a pure rule, no device work)."""
import pytest

from graphconvgeo_amd import dense
from graphconvgeo_amd.mlpconv import MLPCONV, trainer_order


def test_auto_order_rule():
    """'auto' runs propagate-first wherever the fused MFMA output layer takes the classes or the
    SpMM is narrower that way: Twitter-US (K = 300, C = 256) and Twitter-World (C = 930) both
    measured faster propagate-first (profiles/r06); the reference association only past the
    fused layer's width with C <= K."""
    assert trainer_order("auto", 300, 256) == "propagate_first"    # Twitter-US
    assert trainer_order("auto", 300, 930) == "propagate_first"    # Twitter-World
    assert trainer_order("auto", 2000, 1500) == "reference"        # > FUSED_MAX_COLS, C <= K
    assert trainer_order("auto", 500, 1500) == "propagate_first"   # C > K
    assert dense.FUSED_MAX_COLS == 1024
    for explicit in ("reference", "propagate_first"):
        assert trainer_order(explicit, 300, 256) == explicit


def test_mlpconv_default_is_auto_and_validates():
    assert MLPCONV(hidden_layer_size=8, device="cpu").order == "auto"
    with pytest.raises(ValueError):
        MLPCONV(hidden_layer_size=8, device="cpu", order="sideways")
