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


def test_efficient_batch_policy(native):
    """EngineOptions::efficient_batch: a batch is cut below the queue only when a smaller
    size is cheaper per image by more than the margin.  A flat curve (one bucket, replay noise) never
    trims; a real step (ResNet50 fp32: B = 21 spills a tile round, +19 % for +5 % images) does."""
    # one bucket of 24 whose forward costs the same at every live size, +-0.4 % noise
    rng = np.random.default_rng(1)
    flat = [1.40 * (1.0 + 0.004 * rng.standard_normal()) for _ in range(24)]
    for q in range(1, 25):
        assert native.pick_efficient_batch(flat, q) == q
    # per-image time falling with B, then a step at 21 (profiles/r5_batch_curve.md shape)
    step = [0.30 + 0.045 * b for b in range(1, 21)] + [1.46, 1.47, 1.455, 1.44]
    assert native.pick_efficient_batch(step, 20) == 20
    assert native.pick_efficient_batch(step, 21) == 20  # 69.5 vs 60.0 us per image: cut
    assert native.pick_efficient_batch(step, 23) == 20  # 63.3 vs 60.0: cut
    assert native.pick_efficient_batch(step, 24) == 24  # the bucket end is as cheap as B = 20
    # a step of 1.5 % per image is inside the 2 % margin: no cut; margin 0 (the strict argmin) cuts
    small = [1.0 * b for b in range(1, 20)] + [20 * 1.015]
    assert native.pick_efficient_batch(small, 20, margin=0.02) == 20
    assert native.pick_efficient_batch(small, 20, margin=0.0) == 19
    assert native.pick_efficient_batch(step, 0) == 1 and native.pick_efficient_batch(step, 99) == 24


def test_efficient_batch_bucket_ends(native):
    """efficient_batch_ends (default on): only the graph bucket sizes are cut targets.  Round-6 curve
    shape: the bucket-26 graph at 25 live looks cheaper per image than 24, yet a queue of 25 goes
    out as 24 (a batch of 25 broke the serving loop's 24-request rhythm); 26 queued runs whole."""
    ends = [1, 2, 4, 6, 8, 12, 16, 18, 20, 22, 24, 26, 28, 30, 32]
    curve = [0.62 + 0.03 * b for b in range(1, 21)]
    curve[19] = 1.17                                    # B = 20: 58.5 us / image
    curve += [1.366, 1.378, 1.389, 1.394, 1.429, 1.441]  # 21..26: step at 21, 24 = 58.1, 25 = 57.2, 26 = 55.4
    curve += [1.50] * 6
    assert native.pick_efficient_batch(curve, 25, margin=0.0) == 25           # any size: 25 wins
    assert native.pick_efficient_batch(curve, 25, margin=0.0, ends=ends) == 24
    assert native.pick_efficient_batch(curve, 23, margin=0.0, ends=ends) == 20
    assert native.pick_efficient_batch(curve, 26, margin=0.0, ends=ends) == 26
    assert native.pick_efficient_batch(curve, 24, margin=0.0, ends=ends) == 24
