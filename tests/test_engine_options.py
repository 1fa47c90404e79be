"""Engine option semantics that hold on any host: precision routing (fp32 never silently runs on
the bf16 HIP kernels) and option validation."""
import numpy as np
import pytest


def test_fp32_precision_routes_to_cpu_executor(native, models):
    path, _, _ = models["tiny"]
    e = native.Engine(path, device="auto", precision="fp32", max_batch=2)
    try:
        assert e.info["device"].startswith("cpu"), e.info["device"]
        x = np.random.default_rng(0).random((2, e.input_numel), dtype=np.float32)
        y = e.run(x)
        assert y.shape == (2, e.output_numel) and np.isfinite(y).all()
    finally:
        e.close()


def test_fp32_on_hip_is_rejected(native, models):
    path, _, _ = models["tiny"]
    with pytest.raises(Exception, match="fp32"):
        native.Engine(path, device="hip", precision="fp32")


def test_unknown_precision_is_rejected(native, models):
    path, _, _ = models["tiny"]
    with pytest.raises(Exception, match="precision"):
        native.Engine(path, device="cpu", precision="fp8")
