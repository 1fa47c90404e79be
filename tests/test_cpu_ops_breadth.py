"""CPU executor (engine/cpu_exec.cpp) on the wider op set, one op per model, against numpy.  The CPU
executor is the fp32 oracle the HIP engine is checked against (tests/test_gpu_general.py ops_zoo),
so each op it gained for that purpose is pinned here first.  The reference runs these ops through
ONNX Runtime (not importable here), so numpy's definition of each op is the check."""
import numpy as np
import pytest


def _one_op(tmp_path, op, x_shape, out_shape, consts=(), n_out=1, **attrs):
    from die_amd.utils.onnx_writer import GraphBuilder

    g = GraphBuilder(name=op.lower())
    x = g.input("x", list(x_shape))
    ins = [x] + [g.const(c, "c%d" % i) for i, c in enumerate(consts)]
    y = g.node(op, ins, name="op", n_out=n_out, **attrs)
    if n_out > 1:  # concatenate the parts back on axis 1 so the model has one output
        y = g.node("Concat", y, name="cat", axis=1)
    g.output(y, list(out_shape))
    p = str(tmp_path / (op + ".onnx"))
    open(p, "wb").write(g.model_proto(opset=13))
    return p


X = np.random.default_rng(3).standard_normal((2, 3, 5, 6)).astype(np.float32) * 3


@pytest.mark.parametrize("mode", ["constant", "reflect", "edge"])
def test_pad_modes(native, tmp_path, mode):
    pads = np.array([0, 0, 1, 2, 0, 0, 2, 1], np.int64)
    p = _one_op(tmp_path, "Pad", X.shape, (2, 3, 8, 9), consts=[pads], mode=mode)
    want = np.pad(X, ((0, 0), (0, 0), (1, 2), (2, 1)), mode=mode)
    np.testing.assert_array_equal(native.cpu_run(p, X), want)


def test_pad_constant_value_and_crop(native, tmp_path):
    pads = np.array([0, 0, 2, -1, 0, 0, 0, -2], np.int64)
    p = _one_op(tmp_path, "Pad", X.shape, (2, 3, 7, 3), consts=[pads, np.array(1.5, np.float32)])
    want = np.pad(X[:, :, :, 1:4], ((0, 0), (0, 0), (2, 0), (0, 0)), constant_values=1.5)
    np.testing.assert_array_equal(native.cpu_run(p, X), want)


@pytest.mark.parametrize("sizes", [None, [1, 2]])
def test_split(native, tmp_path, sizes):
    consts = [] if sizes is None else [np.array(sizes, np.int64)]
    p = _one_op(tmp_path, "Split", X.shape, X.shape, consts=consts, n_out=2 if sizes else 3, axis=1)
    np.testing.assert_array_equal(native.cpu_run(p, X), X)  # split then concat = identity


def test_split_equal_parts_last_smaller(native, tmp_path):
    from die_amd.utils.onnx_writer import GraphBuilder

    g = GraphBuilder(name="split3")
    x = g.input("x", [2, 3, 5, 6])
    a, b = g.node("Split", [x], name="sp", axis=3, n_out=2)  # 6 -> 3 + 3
    c, d = g.node("Split", [x], name="sp2", axis=2, n_out=2)  # 5 -> 3 + 2
    g.output(g.node("Add", [g.node("ReduceSum", [b, g.const(np.array([3], np.int64), "ax")], name="rs", keepdims=1),
                            g.node("ReduceMax", [d], name="rm", axes=[2], keepdims=1)], name="add"), [2, 3, 5, 6])
    p = str(tmp_path / "split3.onnx")
    open(p, "wb").write(g.model_proto(opset=13))
    # b: [2,3,5,3] summed over axis 3 -> [2,3,5,1]; d: [2,3,2,6] max over axis 2 -> [2,3,1,6]
    want = X[:, :, :, 3:].sum(3, keepdims=True) + X[:, :, 3:, :].max(2, keepdims=True)
    np.testing.assert_allclose(native.cpu_run(p, X), want, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("op,ref,attrs", [
    ("HardSigmoid", lambda v: np.clip(0.25 * v + 0.4, 0, 1), dict(alpha=0.25, beta=0.4)),
    ("HardSwish", lambda v: v * np.clip(v / 6 + 0.5, 0, 1), {}),
    ("Softplus", lambda v: np.log1p(np.exp(v)), {}),
    ("Sin", np.sin, {}), ("Cos", np.cos, {}), ("Sign", np.sign, {}), ("Floor", np.floor, {}),
    ("Ceil", np.ceil, {}), ("Round", np.round, {}),
])
def test_unary(native, tmp_path, op, ref, attrs):
    p = _one_op(tmp_path, op, X.shape, X.shape, **attrs)
    np.testing.assert_allclose(native.cpu_run(p, X), ref(X.astype(np.float64)), rtol=2e-6, atol=1e-6)


@pytest.mark.parametrize("stride,pads,opad,group,dil", [
    (2, [1, 1, 1, 1], [1, 1], 1, 1), (1, [0, 0, 0, 0], [0, 0], 1, 1), (3, [2, 0, 1, 1], [0, 2], 3, 1),
    (2, [1, 1, 1, 1], [0, 0], 1, 2)])
def test_conv_transpose_vs_torch(native, tmp_path, stride, pads, opad, group, dil):
    import torch
    import torch.nn.functional as F
    from die_amd.utils.onnx_writer import GraphBuilder

    rng = np.random.default_rng(5)
    x = rng.standard_normal((2, 6, 5, 7)).astype(np.float32)
    w = rng.standard_normal((6, 4, 3, 3)).astype(np.float32)
    b = rng.standard_normal(4 * group).astype(np.float32)
    ref = F.conv_transpose2d(torch.from_numpy(x).double(), torch.from_numpy(w).double(), torch.from_numpy(b).double(),
                             stride=stride, padding=0, output_padding=0, groups=group, dilation=dil).numpy()
    # ONNX pads crop the full output [top, left, bottom, right]; output_padding extends the bottom/right
    full = ref
    Hf, Wf = full.shape[2], full.shape[3]
    out = np.zeros((2, 4 * group, Hf + opad[0], Wf + opad[1]))
    out[:, :, :Hf, :Wf] = full
    if opad[0]:
        out[:, :, Hf:, :] = b.reshape(1, -1, 1, 1)
    if opad[1]:
        out[:, :, :, Wf:] = b.reshape(1, -1, 1, 1)
    want = out[:, :, pads[0]:out.shape[2] - pads[2], pads[1]:out.shape[3] - pads[3]]
    g = GraphBuilder(name="ct")
    xi = g.input("x", [2, 6, 5, 7])
    y = g.node("ConvTranspose", [xi, g.init("w", w), g.init("b", b)], name="ct", kernel_shape=[3, 3],
               strides=[stride, stride], pads=pads, output_padding=opad, group=group, dilations=[dil, dil])
    g.output(y, list(want.shape))
    p = str(tmp_path / "ct.onnx")
    open(p, "wb").write(g.model_proto(opset=13))
    np.testing.assert_allclose(native.cpu_run(p, x), want, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("mode,coord,scale,torch_kw", [
    ("nearest", "asymmetric", 2.0, dict(mode="nearest")),
    ("nearest", "asymmetric", 0.5, dict(mode="nearest")),
    ("linear", "half_pixel", 2.0, dict(mode="bilinear", align_corners=False)),
    ("linear", "pytorch_half_pixel", 0.5, dict(mode="bilinear", align_corners=False)),
    ("linear", "align_corners", 1.5, dict(mode="bilinear", align_corners=True)),
])
def test_resize_vs_torch(native, tmp_path, mode, coord, scale, torch_kw):
    import torch
    import torch.nn.functional as F
    from die_amd.utils.onnx_writer import GraphBuilder

    x = np.random.default_rng(6).standard_normal((2, 3, 8, 10)).astype(np.float32)
    want = F.interpolate(torch.from_numpy(x).double(), scale_factor=scale, **torch_kw).numpy()
    g = GraphBuilder(name="rs")
    xi = g.input("x", [2, 3, 8, 10])
    y = g.node("Resize", [xi, g.const(np.zeros(0, np.float32), "roi"), g.const(np.array([1, 1, scale, scale], np.float32), "sc")],
               name="rs", mode=mode, coordinate_transformation_mode=coord, nearest_mode="floor")
    g.output(y, list(want.shape))
    p = str(tmp_path / "rs.onnx")
    open(p, "wb").write(g.model_proto(opset=13))
    np.testing.assert_allclose(native.cpu_run(p, x), want, rtol=1e-5, atol=1e-6)


def test_where_compare_logic(native, tmp_path):
    from die_amd.utils.onnx_writer import GraphBuilder

    x = np.random.default_rng(7).standard_normal((2, 3, 4, 5)).astype(np.float32)
    g = GraphBuilder(name="wh")
    xi = g.input("x", [2, 3, 4, 5])
    zero = g.const(np.array(0.0, np.float32), "zero")
    half = g.const(np.array(0.5, np.float32), "half")
    m = g.node("Or", [g.node("Greater", [xi, half], name="gt"), g.node("LessOrEqual", [xi, g.node("Neg", [half], name="nh")],
                                                                     name="le")], name="or")
    m = g.node("And", [m, g.node("Not", [g.node("Equal", [xi, zero], name="eq")], name="ne")], name="and")
    y = g.node("Where", [m, xi, g.node("Mul", [g.node("Cast", [m], name="mf", to=1), zero], name="zeros")], name="wh")
    g.output(y, [2, 3, 4, 5])
    p = str(tmp_path / "wh.onnx")
    open(p, "wb").write(g.model_proto(opset=13))
    want = np.where(((x > 0.5) | (x <= -0.5)) & (x != 0), x, 0.0)
    np.testing.assert_array_equal(native.cpu_run(p, x), want)
