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
