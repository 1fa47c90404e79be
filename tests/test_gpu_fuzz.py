"""Differential test of the whole HIP compile path on random image and token-row graphs (models/fuzz.py): planner
fusion passes + kernels vs the fp32 CPU executor, fp32 (split) mode at rel-L2 <= 2e-4 with the same
top-1, bf16 at <= 5e-2, at batch 1 and a padded bucket."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]

SEEDS = list(range(30))


def _rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("kind,seed", [("image", s) for s in SEEDS] + [("rows", s) for s in SEEDS])
def test_random_graph_matches_cpu_executor(native, tmp_path, kind, seed):
    from die_amd.models import fuzz

    blob, shp, used = (fuzz.build_random if kind == "image" else fuzz.build_random_rows)(seed)
    p = str(tmp_path / ("f%d.onnx" % seed))
    open(p, "wb").write(blob)
    for prec, tol in (("fp32", 2e-4), ("bf16", 5e-2)):
        eng = native.Engine(p, device="hip", max_batch=4, precision=prec, autotune=False)
        try:
            assert eng.refresh_info()["name"].startswith("hip:gfx950"), (seed, used)
            for B in (1, 3):
                x = np.random.default_rng(seed * 7 + B).standard_normal((B,) + shp).astype(np.float32)
                ref = native.cpu_run(p, x).reshape(B, -1)
                got = eng.run(x.reshape(B, -1))
                err = _rel(got, ref)
                assert np.isfinite(got).all() and err <= tol, (seed, used, prec, B, err)
                if prec == "fp32":
                    assert (got.argmax(1) == ref.argmax(1)).all(), (seed, used)
        finally:
            eng.close()
