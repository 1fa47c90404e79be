"""Stem 7x7/2 + 3x3/2 max pool (+ the pooled value's BN/ReLU) in one kernel (kernels/stem.hip
stem_pool_nchw_kernel, planner pass fuse_stem_pool).  The fused kernel pools the stem's stored
representation in registers (DPP row shifts across the 16 columns of a wave, LDS across waves, a
carried row across pool rows, a recomputed halo row per segment), so it must equal the two-kernel
path bit for bit -- on ResNet50 at several batch sizes (segment lengths differ), and on odd image
sizes where the last stem row / column falls off the map.  Also checked against torch fp32."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def _stem_model(path, H, W, post_bn=True, seed=0):
    from die_amd.utils.onnx_writer import GraphBuilder

    rng = np.random.default_rng(seed)
    g = GraphBuilder(name="stem_pool")
    x = g.input("x", ["N", 3, H, W])
    wts = {}

    def bn(inp, name, c):
        ps = []
        for k, v in (("gamma", (1 + 0.2 * rng.standard_normal(c)).astype(np.float32)),
                     ("beta", (0.2 * rng.standard_normal(c)).astype(np.float32)),
                     ("mean", (0.1 * rng.standard_normal(c)).astype(np.float32)),
                     ("var", (0.5 + rng.random(c)).astype(np.float32))):
            wts[name + "." + k] = v
            ps.append(g.init(name + "." + k, v))
        return g.node("BatchNormalization", [inp] + ps, name=name, epsilon=1e-5)

    h = bn(x, "bn_in", 3)
    wts["conv0.weight"] = (rng.standard_normal((64, 3, 7, 7)) / np.sqrt(147)).astype(np.float32)
    w = g.init("conv0.weight", wts["conv0.weight"])
    h = g.node("Conv", [h, w], name="conv0", kernel_shape=[7, 7], strides=[2, 2], pads=[3, 3, 3, 3])
    h = g.node("Relu", [bn(h, "bn0", 64)], name="relu0")
    h = g.node("MaxPool", [h], name="pool0", kernel_shape=[3, 3], strides=[2, 2], pads=[1, 1, 1, 1])
    if post_bn:
        h = g.node("Relu", [bn(h, "bn1", 64)], name="relu1")
    Hs, Ws = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    g.output(h, ["N", 64, (Hs - 1) // 2 + 1, (Ws - 1) // 2 + 1])
    open(path, "wb").write(g.model_proto(opset=13))
    return wts


def _torch_ref(w, x):
    """The same graph in torch, float64 on the CPU, from the model's weights."""
    import torch
    import torch.nn.functional as F

    t = {k: torch.from_numpy(v).double() for k, v in w.items()}

    def bn(h, n):
        sc = t[n + ".gamma"] / torch.sqrt(t[n + ".var"] + 1e-5)
        return h * sc[None, :, None, None] + (t[n + ".beta"] - t[n + ".mean"] * sc)[None, :, None, None]

    h = bn(torch.from_numpy(x).double(), "bn_in")
    h = F.relu(bn(F.conv2d(h, t["conv0.weight"], stride=2, padding=3), "bn0"))
    h = F.max_pool2d(h, 3, 2, 1)
    if "bn1.gamma" in t:
        h = F.relu(bn(h, "bn1"))
    return h.numpy()


@pytest.mark.parametrize("H,W,post_bn", [(224, 224, True), (98, 77, True), (61, 130, False), (17, 9, True)])
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_stem_pool_fused_equals_unfused_and_torch(native, tmp_path, H, W, post_bn, precision):
    p = str(tmp_path / ("stem_%d_%d.onnx" % (H, W)))
    wts = _stem_model(p, H, W, post_bn)
    fused = native.Engine(p, device="hip", max_batch=8, precision=precision, autotune=False)
    plain = native.Engine(p, device="hip", max_batch=8, precision=precision, autotune=False, fuse_stem_pool=False)
    try:
        s = native.plan_summary(p, 8, precision=precision)
        assert s["ops"][0]["kind"] == "stem" and s["ops"][0]["pool_fused"], s["ops"][:2]
        assert "pool" not in [o["kind"] for o in s["ops"]]
        for B in (1, 3, 8):
            x = np.random.default_rng(B + H).standard_normal((B, 3, H, W)).astype(np.float32)
            a = fused.run(x.reshape(B, -1))
            b = plain.run(x.reshape(B, -1))
            np.testing.assert_array_equal(a, b)
            if precision == "fp32":
                ref = _torch_ref(wts, x).reshape(B, -1)
                err = float(np.linalg.norm(a - ref) / np.linalg.norm(ref))
                assert err <= 1e-5, (B, err)
    finally:
        fused.close()
        plain.close()


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_resnet50_stem_pool_fusion_bit_exact(native, tmp_path, precision):
    from die_amd.models import resnet_v2 as r

    cfg = r.ResNetConfig()
    p = str(tmp_path / "rn50.onnx")
    open(p, "wb").write(r.build_onnx(cfg)[0])
    fused = native.Engine(p, device="hip", max_batch=20, precision=precision, autotune=False)
    plain = native.Engine(p, device="hip", max_batch=20, precision=precision, autotune=False, fuse_stem_pool=False)
    try:
        assert fused.refresh_info()["options"]["fuse_stem_pool"] is True
        for B in (1, 7, 20):
            x = r.synthetic_input(B, cfg, seed=40 + B).reshape(B, -1)
            np.testing.assert_array_equal(fused.run(x), plain.run(x))
    finally:
        fused.close()
        plain.close()
