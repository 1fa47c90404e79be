"""Random image and token-row graphs over the planner's op set (models/fuzz.py) all plan for the device, in both
precisions, and run on the CPU executor (the oracle of tests/test_gpu_fuzz.py)."""
import os

import numpy as np
import pytest

SEEDS = list(range(30))


@pytest.mark.parametrize("seed", SEEDS)
def test_random_graph_plans(native, tmp_path, seed):
    from die_amd.models import fuzz

    blob, shp, used = fuzz.build_random(seed)
    p = str(tmp_path / ("f%d.onnx" % seed))
    open(p, "wb").write(blob)
    for prec in ("fp32", "bf16"):
        r = native.plan_report(p, prec)
        assert r["supported"], (seed, used, r["text"])
    x = np.random.default_rng(seed).standard_normal((2,) + shp).astype(np.float32)
    y = native.cpu_run(p, x)
    assert y.shape[0] == 2 and np.isfinite(y).all()


def test_fuzz_covers_every_block_kind():
    from die_amd.models import fuzz

    kinds = set()
    for seed in SEEDS:
        kinds.update(fuzz.build_random(seed)[2])
    assert kinds >= {"stem", "conv", "down", "residual", "se", "pool", "padconv", "resize", "convT", "unary", "concat",
                     "where", "mbconv"}, kinds


@pytest.mark.parametrize("seed", SEEDS)
def test_random_rows_graph_plans(native, tmp_path, seed):
    from die_amd.models import fuzz

    blob, shp, used = fuzz.build_random_rows(seed)
    p = str(tmp_path / ("r%d.onnx" % seed))
    open(p, "wb").write(blob)
    for prec in ("fp32", "bf16"):
        r = native.plan_report(p, prec)
        assert r["supported"], (seed, used, r["text"])
    x = np.random.default_rng(seed).standard_normal((2,) + shp).astype(np.float32)
    y = native.cpu_run(p, x)
    assert y.shape[0] == 2 and np.isfinite(y).all()


def test_rows_fuzz_covers_every_block_kind():
    from die_amd.models import fuzz

    kinds = set()
    for seed in SEEDS:
        kinds.update(fuzz.build_random_rows(seed)[2])
    assert kinds >= {"linear", "ln", "residual", "gate", "mix", "splitcat", "attn"}, kinds


def test_reshape_element_count_is_checked(native, tmp_path):
    """A request whose width does not match the graph's Reshape target fails instead of reading past
    the input."""
    from die_amd.models import fuzz

    blob, shp, _ = fuzz.build_random_rows(18)
    p = str(tmp_path / "r.onnx")
    open(p, "wb").write(blob)
    x = np.zeros((1, shp[0] - 8), np.float32)
    with pytest.raises(Exception, match="element count"):
        native.cpu_run(p, x)
