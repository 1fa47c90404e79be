"""Global pool + FC head in one launch (kernels/misc.hip gap_fc_kernel, planner pass fuse_gap_fc; opt-in:
EngineOptions::fuse_gap_fc, slower than the two-kernel head at ResNet50's shape, profiles/r4_gap_fc.md).
The fused kernel pools in fp32 and dots with the hi + lo weights on the VALU, summing the channel
slices' partial logits in a fixed order after a write-through hand-off, so it is compared with a
float64 torch reference (fp32 mode at rel <= 1e-5), with the two-kernel path, and run twice for
bitwise repeatability -- over mean / max pooling, class counts that are and are not multiples of 8
(the latter fuse the BF16_TO_F32 conversion as well), channel counts that pick different slice
widths, and batches above the 32-sample LDS chunk."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def _head_model(path, C, H, classes, pool, relu_out, seed=0):
    from die_amd.utils.onnx_writer import GraphBuilder

    rng = np.random.default_rng(seed)
    g = GraphBuilder(name="gap_fc")
    x = g.input("x", ["N", 3, H, H])
    w0 = (rng.standard_normal((C, 3, 1, 1)) / np.sqrt(3)).astype(np.float32)
    b0 = (0.1 * rng.standard_normal(C)).astype(np.float32)
    w1 = (rng.standard_normal((classes, C)) / np.sqrt(C)).astype(np.float32)
    b1 = (0.1 * rng.standard_normal(classes)).astype(np.float32)
    h = g.node("Conv", [x, g.init("w0", w0), g.init("b0", b0)], name="conv0", kernel_shape=[1, 1])
    h = g.node("Relu", [h], name="relu0")
    h = g.node("GlobalMaxPool" if pool == "max" else "GlobalAveragePool", [h], name="pool")
    h = g.node("Flatten", [h], name="flat", axis=1)
    h = g.node("Gemm", [h, g.init("w1", w1), g.init("b1", b1)], name="fc", transB=1)
    if relu_out:
        h = g.node("Relu", [h], name="relu1")
    g.output(h, ["N", classes])
    open(path, "wb").write(g.model_proto(opset=13))
    return w0, b0, w1, b1


def _ref(wts, x, pool, relu_out):
    w0, b0, w1, b1 = (v.astype(np.float64) for v in wts)
    h = np.einsum("bchw,oc->bohw", x.astype(np.float64), w0[:, :, 0, 0]) + b0[None, :, None, None]
    h = np.maximum(h, 0)
    p = h.max(axis=(2, 3)) if pool == "max" else h.mean(axis=(2, 3))
    y = p @ w1.T + b1
    return np.maximum(y, 0) if relu_out else y


@pytest.mark.parametrize("C,H,classes,pool,relu_out", [
    (256, 7, 1000, "mean", False),   # ResNet-like head, 32 slices of 8 channels
    (2048, 3, 1000, "mean", False),  # 32 slices of 64 channels (ResNet50's)
    (96, 5, 10, "mean", True),       # classes % 8 != 0: the BF16_TO_F32 op is fused too
    (40, 6, 7, "max", False),
])
def test_gap_fc_matches_reference_and_unfused(native, tmp_path, C, H, classes, pool, relu_out):
    p = str(tmp_path / "head.onnx")
    wts = _head_model(p, C, H, classes, pool, relu_out)
    s = native.plan_summary(p, 70, precision="fp32", fuse_gap_fc=True)
    kinds = [o["kind"] for o in s["ops"]]
    assert "gap_fc" in kinds and "gap" not in kinds and "bf16_to_f32" not in kinds, kinds
    for precision, tol in (("fp32", 1e-5), ("bf16", 3e-2)):
        fused = native.Engine(p, device="hip", max_batch=70, precision=precision, autotune=False, fuse_gap_fc=True)
        plain = native.Engine(p, device="hip", max_batch=70, precision=precision, autotune=False)
        try:
            assert fused.refresh_info()["options"]["fuse_gap_fc"] is True
            for B in (1, 5, 70):
                x = np.random.default_rng(B + C).standard_normal((B, 3, H, H)).astype(np.float32)
                a = fused.run(x.reshape(B, -1))
                np.testing.assert_array_equal(a, fused.run(x.reshape(B, -1)))  # deterministic slice order
                b = plain.run(x.reshape(B, -1))
                ref = _ref(wts, x, pool, relu_out)
                err = float(np.linalg.norm(a - ref) / np.linalg.norm(ref))
                assert err <= tol, (precision, B, err)
                err_plain = float(np.linalg.norm(b - ref) / np.linalg.norm(ref))
                assert err <= err_plain * 1.5 + 1e-7, (precision, B, err, err_plain)
        finally:
            fused.close()
            plain.close()


def test_resnet50_gap_fc_matches_unfused(native, tmp_path):
    from die_amd.models import resnet_v2 as r

    cfg = r.ResNetConfig()
    p = str(tmp_path / "rn50.onnx")
    open(p, "wb").write(r.build_onnx(cfg)[0])
    fused = native.Engine(p, device="hip", max_batch=20, precision="fp32", autotune=False, fuse_gap_fc=True)
    plain = native.Engine(p, device="hip", max_batch=20, precision="fp32", autotune=False)
    try:
        for B in (1, 20):
            x = r.synthetic_input(B, cfg, seed=60 + B).reshape(B, -1)
            a, b = fused.run(x), plain.run(x)
            err = float(np.linalg.norm(a - b) / np.linalg.norm(b))
            assert err <= 1e-5 and (a.argmax(1) == b.argmax(1)).all(), (B, err)
    finally:
        fused.close()
        plain.close()
