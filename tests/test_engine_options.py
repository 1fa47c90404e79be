"""Engine option semantics that hold on any host: precision selection (fp32 is the default, bf16
the opt-in fast mode) and option validation."""
import numpy as np
import pytest


def test_fp32_precision_on_cpu_executor(native, models):
    path, _, _ = models["tiny"]
    e = native.Engine(path, device="cpu", precision="fp32", max_batch=2)
    try:
        assert e.info["device"].startswith("cpu"), e.info["device"]
        x = np.random.default_rng(0).random((2, e.input_numel), dtype=np.float32)
        y = e.run(x)
        assert y.shape == (2, e.output_numel) and np.isfinite(y).all()
    finally:
        e.close()


def test_hip_without_gpu_fails_loudly(native, models):
    from conftest import gpu_available

    if gpu_available():
        pytest.skip("a GPU is visible")
    path, _, _ = models["tiny"]
    with pytest.raises(Exception, match="HIP engine unavailable"):
        native.Engine(path, device="hip", precision="fp32")


def test_unknown_precision_is_rejected(native, models):
    path, _, _ = models["tiny"]
    with pytest.raises(Exception, match="precision"):
        native.Engine(path, device="cpu", precision="fp8")


def test_hip_hw_queue_env_rule():
    """GPU_MAX_HW_QUEUES below 8 (HIP's / the boxes' default 4) is raised to 8; DIE_HIP_HW_QUEUES
    sets it explicitly; larger explicit values stay (profiles/r3_rccl_hw_queues.md)."""
    import die_amd

    for given, want in (({}, "8"), ({"GPU_MAX_HW_QUEUES": "4"}, "8"), ({"GPU_MAX_HW_QUEUES": "16"}, "16"),
                        ({"GPU_MAX_HW_QUEUES": "4", "DIE_HIP_HW_QUEUES": "4"}, "4"),
                        ({"DIE_HIP_HW_QUEUES": "6"}, "6"), ({"GPU_MAX_HW_QUEUES": "junk"}, "8")):
        env = dict(given)
        die_amd.configure_hip_env(env)
        assert env["GPU_MAX_HW_QUEUES"] == want, (given, env)
        assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
