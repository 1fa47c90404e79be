"""Generated models for the HIP planner's general path ("model-agnostic device execution").

The reference serves whatever single-input ONNX model it is given (input 0 / output 0,
/root/reference/src/inference_engine.cpp:33-69).  These generators build small models with the op
mix a ResNet / ViT never exercises, random weights, written by the in-tree ONNX writer:

* `mlp`       2-D input [N, F], Gemm (transB) / MatMul layers with Relu / Tanh / Sigmoid / LeakyRelu,
              hidden and output widths that are NOT multiples of 8, Softmax head;
* `bert`      2-D input [N, S*D] reshaped to [N, S, D], post-LN encoder layers (attention in the
              torch export pattern, erf-GELU FFN), mean-pool over tokens, 3-class head;
* `se_cnn`    an image CNN with 12 input channels (> 8), odd channel counts, a squeeze-excitation
              gate (GAP -> FC -> ReLU -> FC -> Sigmoid -> broadcast Mul), channel Concat and
              Slice, and a Flatten of a 4x4 map (NCHW order) into the classifier.
* `ratio_mlp` a Div of two activations of width 10 (stored with 16 channels) feeding a Gemm: the
              pad columns of both operands are 0, so 0/0 must not reach the next GEMM.
* `ops_zoo`   the elementwise / data-movement ops of the wider ONNX op set on an image and on rows:
              Pad folded into a conv, Pad before a MaxPool (a pad pass), HardSwish, channel Split,
              Abs / Neg / Exp / Softplus / HardSigmoid / Max / Min / Pow / Reciprocal / Log / Sqrt /
              Erf, ReduceMax / ReduceSum over the spatial axes, GlobalMaxPool, a rows Split.
* `upsample_net` a decoder-style CNN: ConvTranspose (stride 2, output_padding, 12 output channels),
              Resize nearest (asymmetric / floor, the torch export), Resize linear down (half_pixel)
              and up (align_corners), comparisons of two activations and with constants, Where
              with activation and scalar branches, Not / And / Or, Cast of masks to float.  Every
              mask multiplies a value that is 0 where the mask flips, so bf16 rounding near a
              threshold cannot change the output discontinuously.
* `token_mixer` data-dependent token mixing: MatMul of two activations outside the attention
              pattern (softmax(h W) [S, S] x h [S, D], and x g [S, 20]: inner size 24 and an
              output width that are not multiples of 8).
* `ln_wide`    LayerNormalization over 20 features (stored with 24: pad columns out of the
              statistics) and over 2560 features (wider than the register-resident kernels hold).
* `ln_offset`  pre-norm rows whose LayerNorm input carries a large DC offset (~60 on every channel,
              |mean| / std ~ 60 per row) before the LayerNorm -> MatMul: the case where folding the
              LayerNorm into the GEMM (x.W' - mean * colsum) cancels.
* `bert_long`  the `bert` encoder at 320 tokens: attention past 256 keys (streaming kernel).
* `bert_hd32`, `bert_hd128`  the `bert` encoder with head dim 32 (4 heads of 128 features, 40 tokens)
              and 128 (2 heads of 256 features, 24 tokens).
`synthetic_input(model, batch)` gives inputs of the right shape.  The CPU executor is the fp32
oracle for all of them (tests/test_gpu_general.py).
"""
from __future__ import annotations

import math
from typing import Dict, Tuple

import numpy as np

from ..utils.onnx_writer import GraphBuilder

SPECS = {
    "mlp": dict(in_features=300, hidden=(100, 60, 36), classes=10),
    "bert": dict(seq=32, dim=128, heads=2, ffn=256, layers=2, classes=3),
    "se_cnn": dict(in_ch=12, image=16, classes=10),
    "ratio_mlp": dict(in_features=40, hidden=10, classes=5),
    "ops_zoo": dict(in_ch=8, image=16, classes=10),
    "upsample_net": dict(in_ch=8, image=12, classes=10),
    "token_mixer": dict(seq=24, dim=40, classes=10),
    "ln_wide": dict(seq=6, dim=20, wide=2560, classes=10),
    "ln_offset": dict(seq=64, dim=128, hidden=256, classes=10),
    "bert_long": dict(seq=320, dim=128, heads=2, ffn=256, layers=1, classes=3),
    "bert_hd32": dict(seq=40, dim=128, heads=4, ffn=256, layers=2, classes=3),
    "bert_hd128": dict(seq=24, dim=256, heads=2, ffn=512, layers=2, classes=3),
}


def _rng(seed):
    return np.random.default_rng(seed)


def _lin(rng, fan_in, shape):
    return (rng.standard_normal(shape) / math.sqrt(fan_in)).astype(np.float32)


def build_mlp(seed: int = 0, opset: int = 13) -> Tuple[bytes, Dict[str, np.ndarray]]:
    s = SPECS["mlp"]
    rng = _rng(seed)
    g = GraphBuilder(name="mlp")
    x = g.input("features", ["N", s["in_features"]])
    h, fan = x, s["in_features"]
    acts = ["Relu", "Tanh", "LeakyRelu"]
    for i, width in enumerate(s["hidden"]):
        if i % 2 == 0:  # Gemm with transB (torch nn.Linear export)
            w = g.init("fc%d.weight" % i, _lin(rng, fan, (width, fan)))
            b = g.init("fc%d.bias" % i, (0.1 * rng.standard_normal(width)).astype(np.float32))
            h = g.node("Gemm", [h, w, b], name="fc%d" % i, transB=1)
        else:  # MatMul + Add (the other common export)
            w = g.init("fc%d.weight" % i, _lin(rng, fan, (fan, width)))
            b = g.init("fc%d.bias" % i, (0.1 * rng.standard_normal(width)).astype(np.float32))
            h = g.node("Add", [g.node("MatMul", [h, w], name="fc%d/MatMul" % i), b], name="fc%d/Add" % i)
        a = acts[i % len(acts)]
        h = g.node(a, [h], name="act%d" % i, **({"alpha": 0.1} if a == "LeakyRelu" else {}))
        fan = width
    # a sigmoid gate on the last hidden layer, then the classifier
    gate = g.node("Sigmoid", [h], name="gate")
    h = g.node("Mul", [h, gate], name="gated")
    w = g.init("head.weight", _lin(rng, fan, (s["classes"], fan)))
    b = g.init("head.bias", (0.1 * rng.standard_normal(s["classes"])).astype(np.float32))
    y = g.node("Gemm", [h, w, b], name="head", transB=1)
    y = g.node("Softmax", [y], name="prob", axis=-1)
    g.output(y, ["N", s["classes"]])
    return g.model_proto(opset=opset), {}


def build_bert(seed: int = 0, opset: int = 17, spec: str = "bert") -> Tuple[bytes, Dict[str, np.ndarray]]:
    s = SPECS[spec]
    rng = _rng(seed)
    S, D, H, F = s["seq"], s["dim"], s["heads"], s["ffn"]
    hd = D // H
    g = GraphBuilder(name="bert_encoder")
    x = g.input("embeddings", ["N", S * D])  # token embeddings, flattened (2-D input)
    h = g.node("Reshape", [x, g.const(np.array([0, S, D], np.int64), "seq_shape")], name="to_tokens")
    heads_shape = g.const(np.array([0, 0, H, hd], np.int64), "heads_shape")
    merge_shape = g.const(np.array([0, 0, D], np.int64), "merge_shape")
    scale = g.const(np.array(math.sqrt(hd), np.float32), "sqrt_d")
    sqrt2 = g.const(np.array(1.4142135381698608, np.float32), "sqrt2")
    one = g.const(np.array(1.0, np.float32), "one")
    half = g.const(np.array(0.5, np.float32), "half")

    def linear(inp, name, fin, fout):
        w = g.init(name + ".weight", _lin(rng, fin, (fin, fout)))
        b = g.init(name + ".bias", (0.02 * rng.standard_normal(fout)).astype(np.float32))
        return g.node("Add", [g.node("MatMul", [inp, w], name=name + "/MatMul"), b], name=name + "/Add")

    def ln(inp, name):
        gw = g.init(name + ".weight", (1.0 + 0.1 * rng.standard_normal(D)).astype(np.float32))
        gb = g.init(name + ".bias", (0.1 * rng.standard_normal(D)).astype(np.float32))
        return g.node("LayerNormalization", [inp, gw, gb], name=name, axis=-1, epsilon=1e-12)

    for i in range(s["layers"]):
        p = "layer%d." % i
        q = linear(h, p + "query", D, D)
        k = linear(h, p + "key", D, D)
        v = linear(h, p + "value", D, D)
        q = g.node("Transpose", [g.node("Reshape", [q, heads_shape], name=p + "q_heads")], name=p + "q_perm",
                   perm=[0, 2, 1, 3])
        k = g.node("Transpose", [g.node("Reshape", [k, heads_shape], name=p + "k_heads")], name=p + "k_perm",
                   perm=[0, 2, 3, 1])
        v = g.node("Transpose", [g.node("Reshape", [v, heads_shape], name=p + "v_heads")], name=p + "v_perm",
                   perm=[0, 2, 1, 3])
        sc = g.node("Div", [g.node("MatMul", [q, k], name=p + "scores"), scale], name=p + "scale")
        sc = g.node("Softmax", [sc], name=p + "softmax", axis=-1)
        c = g.node("MatMul", [sc, v], name=p + "context")
        c = g.node("Reshape", [g.node("Transpose", [c], name=p + "ctx_perm", perm=[0, 2, 1, 3]), merge_shape],
                   name=p + "ctx_merge")
        o = linear(c, p + "attn_out", D, D)
        h = ln(g.node("Add", [o, h], name=p + "residual1"), p + "ln1")  # post-LN (BERT)
        m = linear(h, p + "intermediate", D, F)
        t = g.node("Div", [m, sqrt2], name=p + "gelu/div")
        t = g.node("Add", [g.node("Erf", [t], name=p + "gelu/erf"), one], name=p + "gelu/add")
        t = g.node("Mul", [g.node("Mul", [m, t], name=p + "gelu/mul"), half], name=p + "gelu/half")
        o = linear(t, p + "output", F, D)
        h = ln(g.node("Add", [o, h], name=p + "residual2"), p + "ln2")
    pooled = g.node("ReduceMean", [h], name="mean_pool", axes=[1], keepdims=0)
    w = g.init("classifier.weight", _lin(rng, D, (s["classes"], D)))
    b = g.init("classifier.bias", (0.1 * rng.standard_normal(s["classes"])).astype(np.float32))
    y = g.node("Gemm", [pooled, w, b], name="classifier", transB=1)
    g.output(y, ["N", s["classes"]])
    return g.model_proto(opset=opset), {}


def build_se_cnn(seed: int = 0, opset: int = 13) -> Tuple[bytes, Dict[str, np.ndarray]]:
    s = SPECS["se_cnn"]
    rng = _rng(seed)
    g = GraphBuilder(name="se_cnn")
    x = g.input("image", ["N", s["in_ch"], s["image"], s["image"]])

    def conv(inp, name, cin, cout, k, stride=1, pad=None, bias=True):
        pad = k // 2 if pad is None else pad
        w = g.init(name + ".weight", _lin(rng, cin * k * k, (cout, cin, k, k)))
        ins = [inp, w]
        if bias:
            ins.append(g.init(name + ".bias", (0.1 * rng.standard_normal(cout)).astype(np.float32)))
        return g.node("Conv", ins, name=name, kernel_shape=[k, k], strides=[stride, stride], pads=[pad] * 4)

    def bn(inp, name, c):
        ps = [g.init(name + "." + k, v) for k, v in (
            ("gamma", (1 + 0.1 * rng.standard_normal(c)).astype(np.float32)),
            ("beta", (0.1 * rng.standard_normal(c)).astype(np.float32)),
            ("mean", (0.1 * rng.standard_normal(c)).astype(np.float32)),
            ("var", (0.5 + rng.random(c)).astype(np.float32)))]
        return g.node("BatchNormalization", [inp] + ps, name=name, epsilon=1e-5)

    h = g.node("Relu", [bn(conv(x, "conv1", s["in_ch"], 20, 3, bias=False), "bn1", 20)], name="relu1")  # 20 % 8 != 0
    h = g.node("Relu", [conv(h, "conv2", 20, 24, 3, stride=2)], name="relu2")  # 8x8
    # squeeze-excitation: GAP -> FC(24->6) -> ReLU -> FC(6->24) -> Sigmoid -> broadcast Mul
    z = g.node("Flatten", [g.node("GlobalAveragePool", [h], name="se_gap")], name="se_flat", axis=1)
    z = g.node("Relu", [g.node("Gemm", [z, g.init("se1.weight", _lin(rng, 24, (6, 24))),
                                         g.init("se1.bias", np.zeros(6, np.float32))], name="se1", transB=1)],
               name="se_relu")
    z = g.node("Sigmoid", [g.node("Gemm", [z, g.init("se2.weight", _lin(rng, 6, (24, 6))),
                                            g.init("se2.bias", np.zeros(24, np.float32))], name="se2", transB=1)],
               name="se_sigmoid")
    z = g.node("Reshape", [z, g.const(np.array([-1, 24, 1, 1], np.int64), "se_shape")], name="se_gate")
    h = g.node("Mul", [h, z], name="se_scale")
    # two branches joined on the channel axis, then a channel slice
    b1 = g.node("Relu", [conv(h, "branch1", 24, 16, 1)], name="b1_relu")
    b2 = g.node("Tanh", [conv(h, "branch2", 24, 12, 3)], name="b2_tanh")  # last input: 12 % 8 != 0
    h = g.node("Concat", [b1, b2], name="concat", axis=1)  # 28 channels
    h = g.node("Slice", [h, g.const(np.array([8], np.int64), "sl_start"), g.const(np.array([28], np.int64), "sl_end"),
                         g.const(np.array([1], np.int64), "sl_axes")], name="slice")  # 20 channels
    h = g.node("MaxPool", [h], name="pool", kernel_shape=[2, 2], strides=[2, 2])  # 4x4
    h = g.node("Flatten", [h], name="flatten", axis=1)  # NCHW order over a 4x4 map
    w = g.init("fc.weight", _lin(rng, 20 * 16, (s["classes"], 20 * 16)))
    y = g.node("Gemm", [h, w, g.init("fc.bias", (0.1 * rng.standard_normal(s["classes"])).astype(np.float32))],
               name="fc", transB=1)
    y = g.node("Softmax", [y], name="prob", axis=-1)
    g.output(y, ["N", s["classes"]])
    return g.model_proto(opset=opset), {}


def build_ratio_mlp(seed: int = 0, opset: int = 13) -> Tuple[bytes, Dict[str, np.ndarray]]:
    s = SPECS["ratio_mlp"]
    rng = _rng(seed)
    g = GraphBuilder(name="ratio_mlp")
    x = g.input("features", ["N", s["in_features"]])
    F, Hd = s["in_features"], s["hidden"]

    def fc(inp, name, fin, fout):
        w = g.init(name + ".weight", _lin(rng, fin, (fout, fin)))
        b = g.init(name + ".bias", (0.1 * rng.standard_normal(fout)).astype(np.float32))
        return g.node("Gemm", [inp, w, b], name=name, transB=1)

    num = g.node("Tanh", [fc(x, "num", F, Hd)], name="num_tanh")                       # pad columns 0
    den = g.node("Relu", [fc(x, "den", F, Hd)], name="den_relu")                       # pad columns 0
    den = g.node("Add", [den, g.const(np.array(1.0, np.float32), "one")], name="den_shift")  # >= 1, pads 0
    r = g.node("Div", [num, den], name="ratio")                                        # pads: 0 / 0
    y = fc(r, "head", Hd, s["classes"])
    g.output(y, ["N", s["classes"]])
    return g.model_proto(opset=opset), {}


def build_ops_zoo(seed: int = 0, opset: int = 13) -> Tuple[bytes, Dict[str, np.ndarray]]:
    s = SPECS["ops_zoo"]
    rng = _rng(seed)
    g = GraphBuilder(name="ops_zoo")
    x = g.input("image", ["N", s["in_ch"], s["image"], s["image"]])
    one = g.const(np.array(1.0, np.float32), "one")
    two = g.const(np.array(2.0, np.float32), "two")

    def conv(inp, name, cin, cout, k, pad):
        w = g.init(name + ".weight", _lin(rng, cin * k * k, (cout, cin, k, k)))
        b = g.init(name + ".bias", (0.1 * rng.standard_normal(cout)).astype(np.float32))
        return g.node("Conv", [inp, w, b], name=name, kernel_shape=[k, k], pads=[pad] * 4)

    # relu first so the graph input is materialised once; Pad(1) folded into the 3x3 conv (pads 0)
    h = g.node("Relu", [x], name="in_relu")
    h = g.node("Pad", [h, g.const(np.array([0, 0, 1, 1, 0, 0, 1, 1], np.int64), "pad1")], name="pad1", mode="constant")
    h = g.node("HardSwish", [conv(h, "conv1", s["in_ch"], 16, 3, 0)], name="hswish")
    # asymmetric Pad before a MaxPool: not foldable (zeros vs -inf) -> a pad pass; 17x17 -> 8x8
    h = g.node("Pad", [h, g.const(np.array([0, 0, 0, 1, 0, 0, 1, 0], np.int64), "pad2")], name="pad2", mode="constant")
    h = g.node("MaxPool", [h], name="pool", kernel_shape=[2, 2], strides=[2, 2])
    a, b = g.node("Split", [h, g.const(np.array([8, 8], np.int64), "split_sizes")], name="split", axis=1, n_out=2)
    a = g.node("Exp", [g.node("Neg", [g.node("Abs", [a], name="abs")], name="neg")], name="exp")  # (0, 1]
    sp = g.node("Softplus", [b], name="softplus")
    hs = g.node("HardSigmoid", [b], name="hsigmoid", alpha=0.25, beta=0.4)
    mx = g.node("Max", [a, sp], name="max")
    mn = g.node("Min", [a, hs], name="min")
    h = g.node("Concat", [mx, mn], name="cat", axis=1)  # 16 channels
    h = conv(h, "conv2", 16, 12, 1, 0)  # 12 % 8 != 0
    r = g.node("Reciprocal", [g.node("Add", [g.node("Pow", [h, two], name="pow"), one], name="pow1")], name="recip")
    h = g.node("Erf", [g.node("Log", [r], name="log")], name="erf")  # log of (0, 1]
    h = g.node("Sqrt", [g.node("Abs", [h], name="abs2")], name="sqrt")
    rmax = g.node("ReduceMax", [h], name="rmax", axes=[2, 3], keepdims=1)
    rsum = g.node("ReduceSum", [h, g.const(np.array([2, 3], np.int64), "rsum_axes")], name="rsum", keepdims=1)
    gmax = g.node("GlobalMaxPool", [h], name="gmax")
    z = g.node("Add", [g.node("Add", [rmax, rsum], name="pool_add"), gmax], name="pool_add2")
    z = g.node("Flatten", [z], name="flatten", axis=1)  # rows [N, 12]
    z = g.node("Gemm", [z, g.init("fc1.weight", _lin(rng, 12, (16, 12))),
                        g.init("fc1.bias", (0.1 * rng.standard_normal(16)).astype(np.float32))], name="fc1", transB=1)
    u, v = g.node("Split", [z], name="row_split", axis=1, n_out=2)  # equal parts of rows
    z = g.node("Concat", [g.node("HardSwish", [u], name="row_hswish"), g.node("Softplus", [v], name="row_softplus")],
               name="row_cat", axis=1)
    w = g.init("fc2.weight", _lin(rng, 16, (s["classes"], 16)))
    y = g.node("Gemm", [z, w, g.init("fc2.bias", np.zeros(s["classes"], np.float32))], name="fc2", transB=1)
    g.output(y, ["N", s["classes"]])
    return g.model_proto(opset=opset), {}


def build_upsample_net(seed: int = 0, opset: int = 13) -> Tuple[bytes, Dict[str, np.ndarray]]:
    s = SPECS["upsample_net"]
    rng = _rng(seed)
    g = GraphBuilder(name="upsample_net")
    x = g.input("image", ["N", s["in_ch"], s["image"], s["image"]])
    f32 = 1  # onnx FLOAT
    empty = g.const(np.zeros(0, np.float32), "no_roi")

    def c(v, name):
        return g.const(np.array(v, np.float32), name)

    w1 = g.init("conv1.weight", _lin(rng, 8 * 9, (16, 8, 3, 3)))
    h = g.node("Relu", [g.node("Conv", [x, w1, g.init("conv1.bias", (0.1 * rng.standard_normal(16)).astype(np.float32))],
                               name="conv1", kernel_shape=[3, 3], pads=[1, 1, 1, 1])], name="relu1")  # 12x12x16
    wt = g.init("up.weight", _lin(rng, 16 * 9 / 4, (16, 12, 3, 3)))  # ConvTranspose weight [Cin, Cout, kh, kw]
    d = g.node("ConvTranspose", [h, wt, g.init("up.bias", (0.1 * rng.standard_normal(12)).astype(np.float32))],
               name="up", kernel_shape=[3, 3], strides=[2, 2], pads=[1, 1, 1, 1], output_padding=[1, 1])  # 24x24x12
    u = g.node("Resize", [h, empty, g.const(np.array([1, 1, 2, 2], np.float32), "nn_scales")], name="nn_up",
               mode="nearest", coordinate_transformation_mode="asymmetric", nearest_mode="floor")  # 24x24x16
    u2 = g.node("Conv", [u, g.init("proj.weight", _lin(rng, 16, (12, 16, 1, 1)))], name="proj", kernel_shape=[1, 1])
    z = g.node("Where", [g.node("Greater", [d, u2], name="gt"), d, u2], name="pick_max")           # max(d, u2)
    z = g.node("Where", [g.node("Less", [z, c(0.0, "zero")], name="neg"), c(0.0, "zero_f"), z], name="relu_where")
    r = g.node("Resize", [z, empty, g.const(np.array([1, 1, 0.5, 0.5], np.float32), "down_scales")], name="down",
               mode="linear", coordinate_transformation_mode="half_pixel")                          # 12x12
    r2 = g.node("Resize", [r, empty, g.const(np.array([1, 1, 1.5, 1.5], np.float32), "up_scales")], name="up15",
                mode="linear", coordinate_transformation_mode="align_corners")                      # 18x18
    r2 = g.node("Sub", [r2, c(0.3, "shift")], name="center")
    m1 = g.node("And", [g.node("Greater", [r2, c(0.0, "zero2")], name="pos"),
                        g.node("Less", [c(50.0, "big"), r2], name="huge")], name="pos_and")  # r2 > 0 and 50 < r2: empty
    m1 = g.node("Or", [m1, g.node("Greater", [r2, c(0.0, "zero3")], name="pos2")], name="pos_or")  # = r2 > 0
    m2 = g.node("Not", [m1], name="nonpos")
    pos = g.node("Mul", [r2, g.node("Cast", [m1], name="m1f", to=f32)], name="pos_part")
    neg = g.node("Mul", [r2, g.node("Cast", [m2], name="m2f", to=f32)], name="neg_part")
    hsum = g.node("Sub", [pos, g.node("Mul", [neg, c(0.1, "slope")], name="leak")], name="leaky")  # leaky ReLU
    z = g.node("Flatten", [g.node("GlobalAveragePool", [hsum], name="gap")], name="flat", axis=1)
    w = g.init("fc.weight", _lin(rng, 12, (s["classes"], 12)))
    y = g.node("Gemm", [z, w, g.init("fc.bias", np.zeros(s["classes"], np.float32))], name="fc", transB=1)
    g.output(y, ["N", s["classes"]])
    return g.model_proto(opset=opset), {}


def build_token_mixer(seed: int = 0, opset: int = 13) -> Tuple[bytes, Dict[str, np.ndarray]]:
    s = SPECS["token_mixer"]
    rng = _rng(seed)
    S, D = s["seq"], s["dim"]
    g = GraphBuilder(name="token_mixer")
    x = g.input("tokens", ["N", S * D])
    h = g.node("Reshape", [x, g.const(np.array([0, S, D], np.int64), "seq_shape")], name="to_tokens")
    logits = g.node("MatMul", [h, g.init("mix.weight", _lin(rng, D, (D, S)))], name="mix_logits")  # [N, S, S]
    a = g.node("Softmax", [logits], name="mix_softmax", axis=-1)
    m = g.node("MatMul", [a, h], name="mix")                                                  # [S, S] x [S, D]
    h = g.node("Add", [m, h], name="mix_residual")
    gl = g.node("Add", [g.node("MatMul", [h, g.init("gate.weight", _lin(rng, D, (D, 20)))], name="gate/MatMul"),
                        g.init("gate.bias", (0.1 * rng.standard_normal(20)).astype(np.float32))], name="gate/Add")
    gl = g.node("Tanh", [gl], name="gate_tanh")                                               # [N, S, 20]
    m2 = g.node("MatMul", [a, gl], name="mix2")                                               # [S, S] x [S, 20]
    pooled = g.node("ReduceMean", [m2], name="pool", axes=[1], keepdims=0)                    # [N, 20]
    w = g.init("head.weight", _lin(rng, 20, (s["classes"], 20)))
    y = g.node("Gemm", [pooled, w, g.init("head.bias", np.zeros(s["classes"], np.float32))], name="head", transB=1)
    g.output(y, ["N", s["classes"]])
    return g.model_proto(opset=opset), {}


def build_ln_wide(seed: int = 0, opset: int = 17) -> Tuple[bytes, Dict[str, np.ndarray]]:
    s = SPECS["ln_wide"]
    rng = _rng(seed)
    S, D, Wd = s["seq"], s["dim"], s["wide"]
    g = GraphBuilder(name="ln_wide")
    x = g.input("tokens", ["N", S * D])
    h = g.node("Reshape", [x, g.const(np.array([0, S, D], np.int64), "seq_shape")], name="to_tokens")

    def ln(inp, name, c):
        gw = g.init(name + ".weight", (1.0 + 0.1 * rng.standard_normal(c)).astype(np.float32))
        gb = g.init(name + ".bias", (0.1 * rng.standard_normal(c)).astype(np.float32))
        return g.node("LayerNormalization", [inp, gw, gb], name=name, axis=-1, epsilon=1e-5)

    h = ln(h, "ln_in", D)  # 20 logical columns, 24 stored
    h = g.node("Add", [g.node("MatMul", [h, g.init("up.weight", _lin(rng, D, (D, Wd)))], name="up/MatMul"),
                       g.init("up.bias", (0.1 * rng.standard_normal(Wd)).astype(np.float32))], name="up/Add")
    h = g.node("Tanh", [ln(h, "ln_wide", Wd)], name="act")  # 2560 columns
    pooled = g.node("ReduceMean", [h], name="pool", axes=[1], keepdims=0)
    w = g.init("head.weight", _lin(rng, Wd, (s["classes"], Wd)))
    y = g.node("Gemm", [pooled, w, g.init("head.bias", np.zeros(s["classes"], np.float32))], name="head", transB=1)
    g.output(y, ["N", s["classes"]])
    return g.model_proto(opset=opset), {}


def build_ln_offset(seed: int = 0, opset: int = 17, offset: float = 60.0) -> Tuple[bytes, Dict[str, np.ndarray]]:
    """offset: the row-constant DC offset added before the LayerNorm, in units of the rows' own
    standard deviation (the tokens are N(0, 1))."""
    s = SPECS["ln_offset"]
    rng = _rng(seed)
    S, D, H = s["seq"], s["dim"], s["hidden"]
    g = GraphBuilder(name="ln_offset")
    x = g.input("tokens", ["N", S * D])
    h = g.node("Reshape", [x, g.const(np.array([0, S, D], np.int64), "seq_shape")], name="to_tokens")
    # a row-constant offset (the same for every channel): |mean| / std of each row ~ 60 -- the
    # cancellation case -- plus a small per-channel spread
    off = (offset + 0.5 * rng.standard_normal(D)).astype(np.float32)
    h = g.node("Add", [h, g.init("offset", off)], name="dc_offset")

    def ln(inp, name, c):
        gw = g.init(name + ".weight", (1.0 + 0.1 * rng.standard_normal(c)).astype(np.float32))
        gb = g.init(name + ".bias", (0.1 * rng.standard_normal(c)).astype(np.float32))
        return g.node("LayerNormalization", [inp, gw, gb], name=name, axis=-1, epsilon=1e-5)

    h = g.node("Add", [g.node("MatMul", [ln(h, "ln0", D), g.init("fc1.weight", _lin(rng, D, (D, H)))], name="fc1/MatMul"),
                       g.init("fc1.bias", (0.1 * rng.standard_normal(H)).astype(np.float32))], name="fc1/Add")
    h = g.node("Tanh", [h], name="act")
    pooled = g.node("ReduceMean", [h], name="pool", axes=[1], keepdims=0)
    w = g.init("head.weight", _lin(rng, H, (s["classes"], H)))
    y = g.node("Gemm", [pooled, w, g.init("head.bias", np.zeros(s["classes"], np.float32))], name="head", transB=1)
    g.output(y, ["N", s["classes"]])
    return g.model_proto(opset=opset), {}


BUILDERS = {"mlp": build_mlp, "bert": build_bert, "se_cnn": build_se_cnn, "ratio_mlp": build_ratio_mlp,
            "ops_zoo": build_ops_zoo, "upsample_net": build_upsample_net, "token_mixer": build_token_mixer,
            "ln_wide": build_ln_wide, "ln_offset": build_ln_offset,
            "bert_long": lambda seed=0: build_bert(seed, spec="bert_long"),
            "bert_hd32": lambda seed=0: build_bert(seed, spec="bert_hd32"),
            "bert_hd128": lambda seed=0: build_bert(seed, spec="bert_hd128")}


def build_onnx(name: str, seed: int = 0) -> bytes:
    return BUILDERS[name](seed)[0]


def input_shape(name: str):
    s = SPECS[name]
    if name in ("mlp", "ratio_mlp"):
        return (s["in_features"],)
    if name in ("bert", "bert_long", "bert_hd32", "bert_hd128", "token_mixer", "ln_wide", "ln_offset"):
        return (s["seq"] * s["dim"],)
    return (s["in_ch"], s["image"], s["image"])


def synthetic_input(name: str, batch: int, seed: int = 1) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return rng.standard_normal((batch,) + input_shape(name)).astype(np.float32)
