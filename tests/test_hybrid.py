"""Hybrid HIP + CPU execution (engine/hybrid_engine.cpp): the reference's per-node EP fallback
(/root/reference/src/inference_engine.cpp:21-31 -- ORT runs the nodes the CUDA EP cannot take on
the CPU EP and keeps the rest on the GPU).  Partition checks run on the CPU; execution on the GPU."""
import numpy as np
import pytest

from conftest import gpu_available


def _odd_model(path):
    from test_plan_general import _unsupported_model

    _unsupported_model(path)


def test_partition_of_sin_cos_model(native, tmp_path):
    p = str(tmp_path / "odd.onnx")
    _odd_model(p)
    segs = native.hybrid_partition(p)
    assert [s["device"] for s in segs] == ["hip", "cpu"], segs
    assert segs[0]["ops"] == ["Conv"] and segs[0]["input"] == "x"
    assert sorted(segs[1]["ops"]) == ["Add", "Cos", "Relu", "Sin"]


@pytest.fixture(scope="module")
def injected_rn50(native, tmp_path_factory):
    from die_amd.models import resnet_v2 as r

    cfg = r.ResNetConfig()
    blob, w = r.build_onnx(cfg, inject_unit=4)  # stage 2, second unit (0-based unit index 4)
    p = str(tmp_path_factory.mktemp("hyb") / "rn50_sign.onnx")
    open(p, "wb").write(blob)
    return p, w, cfg


def test_partition_keeps_ninety_percent_of_resnet_convs_on_gpu(native, injected_rn50):
    path = injected_rn50[0]
    segs = native.hybrid_partition(path, 8)
    assert [s["device"] for s in segs] == ["hip", "cpu", "hip"], [(s["device"], s["gemm_nodes"]) for s in segs]
    gemm = sum(s["gemm_nodes"] for s in segs)
    on_gpu = sum(s["gemm_nodes"] for s in segs if s["device"] == "hip")
    assert gemm == 54 and on_gpu / gemm >= 0.9, (on_gpu, gemm)
    cpu = segs[1]
    assert "Sign" in cpu["ops"] and cpu["gemm_nodes"] == 3  # just the unit holding the Sign


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a GPU")
def test_hybrid_engine_sin_cos_model_matches_cpu_oracle(native, tmp_path):
    p = str(tmp_path / "odd.onnx")
    _odd_model(p)
    eng = native.Engine(p, device="auto", max_batch=4)
    try:
        info = eng.refresh_info()
        assert info["name"] == "hybrid(hip,cpu)", info["name"]
        x = np.random.default_rng(1).standard_normal((4, 3 * 8 * 8)).astype(np.float32)
        got = eng.run(x)
        ref = native.cpu_run(p, x.reshape(4, 3, 8, 8)).reshape(4, -1)
        err = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
        assert err <= 1e-5, err
    finally:
        eng.close()


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a GPU")
def test_hybrid_engine_resnet50_with_injected_op(native, injected_rn50):
    import torch

    from die_amd.models import resnet_v2 as r

    path, w, cfg = injected_rn50
    eng = native.Engine(path, device="auto", max_batch=8, precision="fp32")
    try:
        info = eng.refresh_info()
        assert info["name"] == "hybrid(hip,cpu,hip)", info["name"]
        st = info.get("engine_stats", info)
        for B in (1, 8):
            x = r.synthetic_input(B, cfg, seed=70 + B)
            with torch.no_grad():
                ref = r.torch_forward(w, x, cfg, device="cuda").double().cpu().numpy()  # relu * Sign(relu) = relu
            got = eng.run(x.reshape(B, -1)).astype(np.float64)
            err = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
            assert err <= 1e-4, (B, err)
            assert (got.argmax(1) == ref.argmax(1)).all()
    finally:
        eng.close()
