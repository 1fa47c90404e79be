"""Random image-model graphs over the HIP planner's op set, for differential tests of the whole
compile path (planner fusion passes + kernels) against the CPU executor (tests/test_plan_fuzz.py on
the CPU: every graph plans; tests/test_gpu_fuzz.py: every graph matches the fp32 oracle).

A graph is a chain of randomly chosen blocks on an NCHW image -- conv (1x1 / 3x3, stride 1 / 2,
optional BN, one of several activations), residual add, squeeze-excitation gate, max / average
pool, Pad + conv, nearest / linear resize, transposed conv, elementwise unary chains, channel
concat + slice, Where / comparison masks, inverted-residual blocks (1x1 expand, depthwise 3x3, SiLU
as x * Sigmoid(x), 1x1 project) -- then a global pool and a Gemm classifier.  Channel
counts include values that are not multiples of 8 where the planner allows them.  Deterministic in
the seed.
"""
from __future__ import annotations

import math
from typing import List, Tuple

import numpy as np

from ..utils.onnx_writer import GraphBuilder


def build_random(seed: int, blocks: int = 6) -> Tuple[bytes, Tuple[int, int, int], List[str]]:
    """-> (model bytes, input (C, H, W), the block kinds used)."""
    rng = np.random.default_rng(seed)
    C0 = int(rng.choice([3, 8, 12]))
    H = int(rng.choice([12, 16]))
    H0 = H
    g = GraphBuilder(name="fuzz%d" % seed)
    x = g.input("image", ["N", C0, H, H])
    used: List[str] = []
    k = [0]

    def nm(base):
        k[0] += 1
        return "%s%d" % (base, k[0])

    def const(v):
        return g.const(np.array(v, np.float32), nm("c"))

    def lin(shape, fan):
        return (rng.standard_normal(shape) / math.sqrt(fan)).astype(np.float32)

    def conv(inp, cin, cout, ks, stride, pad, bias=True):
        w = g.init(nm("w"), lin((cout, cin, ks, ks), cin * ks * ks))
        ins = [inp, w]
        if bias:
            ins.append(g.init(nm("b"), (0.1 * rng.standard_normal(cout)).astype(np.float32)))
        return g.node("Conv", ins, name=nm("conv"), kernel_shape=[ks, ks], strides=[stride, stride], pads=[pad] * 4)

    def bn(inp, c):
        ps = [g.init(nm("bn"), v) for v in ((1 + 0.1 * rng.standard_normal(c)).astype(np.float32),
                                           (0.1 * rng.standard_normal(c)).astype(np.float32),
                                           (0.1 * rng.standard_normal(c)).astype(np.float32),
                                           (0.5 + rng.random(c)).astype(np.float32))]
        return g.node("BatchNormalization", [inp] + ps, name=nm("bn"), epsilon=1e-5)

    def act(inp):
        a = str(rng.choice(["Relu", "Sigmoid", "Tanh", "LeakyRelu", "HardSwish", "Clip", "Softplus", "none"]))
        if a == "none":
            return inp
        if a == "LeakyRelu":
            return g.node(a, [inp], name=nm("act"), alpha=0.1)
        if a == "Clip":
            return g.node(a, [inp, const(0.0), const(6.0)], name=nm("act"))
        return g.node(a, [inp], name=nm("act"))

    # stem: a conv so the image becomes an NHWC activation with >= 8 channels
    C = int(rng.choice([8, 16, 24]))
    h = act(bn(conv(x, C0, C, 3, 1, 1, bias=False), C))
    used.append("stem")
    saved = [(h, C, H)]  # tensors a residual can join
    for _ in range(blocks):
        kinds = ["conv", "conv", "residual", "se", "pool", "padconv", "unary", "concat", "where", "mbconv"]
        if H >= 8:
            kinds += ["down"]
        if H <= 12:
            kinds += ["resize", "convT"]
        kind = str(rng.choice(kinds))
        if kind == "conv":
            cout = int(rng.choice([8, 12, 16, 20, 24, 32])) if C % 8 == 0 else C
            ks = int(rng.choice([1, 3]))
            h = conv(h, C, cout, ks, 1, ks // 2)
            if rng.random() < 0.5:
                h = bn(h, cout)
            h, C = act(h), cout
        elif kind == "down":
            cout = int(rng.choice([16, 24, 32]))
            h = act(conv(h, C, cout, 3, 2, 1))
            C, H = cout, (H + 1) // 2
        elif kind == "residual":
            same = [t for t in saved if t[1] == C and t[2] == H and t[0] != h]
            if not same:
                h2 = act(conv(h, C, C, 3, 1, 1))
                h = g.node("Add", [h2, h], name=nm("res"))
            else:
                h = g.node("Add", [h, same[int(rng.integers(len(same)))][0]], name=nm("res"))
            h = g.node("Relu", [h], name=nm("relu"))
        elif kind == "se":
            z = g.node("Flatten", [g.node("GlobalAveragePool", [h], name=nm("gap"))], name=nm("flat"), axis=1)
            r = max(4, C // 4)
            z = g.node("Relu", [g.node("Gemm", [z, g.init(nm("w"), lin((r, C), C)), g.init(nm("b"), np.zeros(r, np.float32))],
                                       name=nm("fc"), transB=1)], name=nm("relu"))
            z = g.node("Sigmoid", [g.node("Gemm", [z, g.init(nm("w"), lin((C, r), r)), g.init(nm("b"), np.zeros(C, np.float32))],
                                          name=nm("fc"), transB=1)], name=nm("sig"))
            z = g.node("Reshape", [z, g.const(np.array([-1, C, 1, 1], np.int64), nm("shape"))], name=nm("gate"))
            h = g.node("Mul", [h, z], name=nm("se"))
        elif kind == "pool":
            if H < 4:
                continue
            op = str(rng.choice(["MaxPool", "AveragePool"]))
            h = g.node(op, [h], name=nm("pool"), kernel_shape=[2, 2], strides=[2, 2])
            H //= 2
        elif kind == "padconv":
            if C % 8:
                continue
            p = g.node("Pad", [h, g.const(np.array([0, 0, 1, 1, 0, 0, 1, 1], np.int64), nm("pads"))], name=nm("pad"),
                       mode="constant")
            h = act(conv(p, C, C, 3, 1, 0))
        elif kind == "resize":
            if rng.random() < 0.5:
                h = g.node("Resize", [h, g.const(np.zeros(0, np.float32), nm("roi")),
                                      g.const(np.array([1, 1, 2, 2], np.float32), nm("sc"))], name=nm("rs"),
                           mode="nearest", coordinate_transformation_mode="asymmetric", nearest_mode="floor")
            else:
                h = g.node("Resize", [h, g.const(np.zeros(0, np.float32), nm("roi")),
                                      g.const(np.array([1, 1, 2, 2], np.float32), nm("sc"))], name=nm("rs"),
                           mode="linear", coordinate_transformation_mode="half_pixel")
            H *= 2
        elif kind == "convT":
            if C % 8:
                continue
            cout = int(rng.choice([8, 12, 16]))
            w = g.init(nm("wt"), lin((C, cout, 3, 3), C * 9 / 4))
            h = g.node("ConvTranspose", [h, w, g.init(nm("b"), (0.1 * rng.standard_normal(cout)).astype(np.float32))],
                       name=nm("convT"), kernel_shape=[3, 3], strides=[2, 2], pads=[1, 1, 1, 1], output_padding=[1, 1])
            h, C, H = act(h), cout, H * 2
        elif kind == "unary":
            chain = str(rng.choice(["expneg", "softsign", "sqrt"]))
            if chain == "expneg":  # exp(-|x|) in (0, 1]
                h = g.node("Exp", [g.node("Neg", [g.node("Abs", [h], name=nm("abs"))], name=nm("neg"))], name=nm("exp"))
            elif chain == "softsign":  # x / (1 + |x|)
                den = g.node("Add", [g.node("Abs", [h], name=nm("abs")), const(1.0)], name=nm("den"))
                h = g.node("Div", [h, den], name=nm("softsign"))
            else:  # sqrt(x^2 + 1) - 0.5 (not - 1: x^2 + 1 rounds to 1 in bf16 for |x| < 0.06, and the
                # cancellation made a bf16 engine's output 75 % off the fp32 oracle -- an ill-conditioned
                # graph, not a kernel error)
                h = g.node("Sub", [g.node("Sqrt", [g.node("Add", [g.node("Pow", [h, const(2.0)], name=nm("sq")),
                                                                  const(1.0)], name=nm("p1"))], name=nm("sqrt")),
                                   const(0.5)], name=nm("m1"))
        elif kind == "concat":
            if C % 8:
                continue
            b2 = act(conv(h, C, 8, 1, 1, 0))
            h = g.node("Concat", [h, b2], name=nm("cat"), axis=1)
            Cc = C + 8
            keep = int(rng.choice([8, 16])) if C >= 16 else 8
            h = g.node("Slice", [h, g.const(np.array([0], np.int64), nm("s0")), g.const(np.array([keep], np.int64), nm("s1")),
                                 g.const(np.array([1], np.int64), nm("ax"))], name=nm("slice"))
            C = keep if keep <= Cc else Cc
        elif kind == "mbconv":  # inverted residual (MobileNetV2 / EfficientNet): 1x1 expand, depthwise 3x3, SiLU, 1x1 project
            if C % 8:
                continue
            E = 2 * C

            def silu(t):
                return g.node("Mul", [t, g.node("Sigmoid", [t], name=nm("sg"))], name=nm("silu"))

            e = silu(bn(conv(h, C, E, 1, 1, 0, bias=False), E))
            wd = g.init(nm("dw"), lin((E, 1, 3, 3), 9))
            d = g.node("Conv", [e, wd], name=nm("dwconv"), kernel_shape=[3, 3], strides=[1, 1], pads=[1, 1, 1, 1], group=E)
            d = silu(bn(d, E))
            h = g.node("Add", [h, bn(conv(d, E, C, 1, 1, 0, bias=False), C)], name=nm("res"))
        elif kind == "where":  # max(h, g(h)) through a comparison mask (continuous)
            other = g.node("Tanh", [h], name=nm("tanh"))
            h = g.node("Where", [g.node("Greater", [h, other], name=nm("gt")), h, other], name=nm("where"))
        used.append(kind)
        saved.append((h, C, H))
    z = g.node("Flatten", [g.node("GlobalAveragePool", [h], name=nm("gap"))], name=nm("flat"), axis=1)
    classes = int(rng.choice([5, 10, 16]))
    y = g.node("Gemm", [z, g.init(nm("w"), lin((classes, C), C)), g.init(nm("b"), np.zeros(classes, np.float32))],
               name="head", transB=1)
    g.output(y, ["N", classes])
    return g.model_proto(opset=13), (C0, H0, H0), used


def build_random_rows(seed: int, blocks: int = 6) -> Tuple[bytes, Tuple[int], List[str]]:
    """Random token-row graphs: input [N, S*D] reshaped to [N, S, D], then linear layers with
    activations, LayerNorm, residuals, gated units, data-dependent token mixing (softmax(h W) h: a
    MatMul of two activations), multi-head self-attention (head dim 32 / 64 / 80), channel split /
    concat, and a mean over tokens into a classifier.
    -> (model bytes, input (S*D,), the block kinds used)."""
    rng = np.random.default_rng(10_000 + seed)
    S = int(rng.choice([5, 9, 16, 20]))
    D = int(rng.choice([16, 24, 32, 40]))
    D0 = D
    g = GraphBuilder(name="fuzzrows%d" % seed)
    x = g.input("tokens", ["N", S * D])
    h = g.node("Reshape", [x, g.const(np.array([0, S, D], np.int64), "seq_shape")], name="to_tokens")
    used: List[str] = []
    k = [0]

    def nm(base):
        k[0] += 1
        return "%s%d" % (base, k[0])

    def lin(shape, fan):
        return (rng.standard_normal(shape) / math.sqrt(fan)).astype(np.float32)

    def linear(inp, din, dout):
        w = g.init(nm("w"), lin((din, dout), din))
        b = g.init(nm("b"), (0.1 * rng.standard_normal(dout)).astype(np.float32))
        return g.node("Add", [g.node("MatMul", [inp, w], name=nm("mm")), b], name=nm("add"))

    def act(inp):
        a = str(rng.choice(["Relu", "Tanh", "Sigmoid", "Gelu", "none"]))
        if a == "none":
            return inp
        if a == "Gelu":  # the erf form as torch exports it
            t = g.node("Div", [inp, g.const(np.array(1.4142135381698608, np.float32), nm("c"))], name=nm("gd"))
            t = g.node("Add", [g.node("Erf", [t], name=nm("erf")), g.const(np.array(1.0, np.float32), nm("c"))],
                       name=nm("ga"))
            return g.node("Mul", [g.node("Mul", [inp, t], name=nm("gm")), g.const(np.array(0.5, np.float32), nm("c"))],
                          name=nm("gh"))
        return g.node(a, [inp], name=nm("act"))

    def ln(inp, c):
        return g.node("LayerNormalization", [inp, g.init(nm("g"), (1 + 0.1 * rng.standard_normal(c)).astype(np.float32)),
                                             g.init(nm("b"), (0.1 * rng.standard_normal(c)).astype(np.float32))],
                      name=nm("ln"), axis=-1, epsilon=1e-5)

    for _ in range(blocks):
        kind = str(rng.choice(["linear", "linear", "ln", "residual", "gate", "mix", "splitcat", "attn"]))
        if kind == "linear":
            d2 = int(rng.choice([16, 24, 32, 40, 48]))
            h, D = act(linear(h, D, d2)), d2
        elif kind == "ln":
            h = ln(h, D)
        elif kind == "residual":
            h = g.node("Add", [h, act(linear(h, D, D))], name=nm("res"))
        elif kind == "gate":
            h = g.node("Mul", [h, g.node("Sigmoid", [linear(h, D, D)], name=nm("sig"))], name=nm("gate"))
        elif kind == "mix":
            a = g.node("Softmax", [g.node("MatMul", [h, g.init(nm("wm"), lin((D, S), D))], name=nm("ml"))],
                       name=nm("sm"), axis=-1)
            h = g.node("MatMul", [a, h], name=nm("mix"))
        elif kind == "attn":
            # multi-head self-attention in the torch export's form (Q/K/V linears, head Reshape +
            # Transpose, MatMul -> Div -> Softmax -> MatMul, merge), head dim 32 / 64 / 80, then back
            # to D with an output linear and a residual
            hd = int(rng.choice([32, 64, 80]))
            nh = int(rng.choice([1, 2]))
            E = hd * nh
            heads = g.const(np.array([0, 0, nh, hd], np.int64), nm("hs"))
            merge = g.const(np.array([0, 0, E], np.int64), nm("ms"))
            qh, kh, vh = (g.node("Reshape", [linear(h, D, E), heads], name=nm("heads")) for _ in range(3))
            qh = g.node("Transpose", [qh], name=nm("qp"), perm=[0, 2, 1, 3])
            kh = g.node("Transpose", [kh], name=nm("kp"), perm=[0, 2, 3, 1])
            vh = g.node("Transpose", [vh], name=nm("vp"), perm=[0, 2, 1, 3])
            sc = g.node("Div", [g.node("MatMul", [qh, kh], name=nm("scores")),
                                g.const(np.array(math.sqrt(hd), np.float32), nm("c"))], name=nm("scale"))
            sc = g.node("Softmax", [sc], name=nm("softmax"), axis=-1)
            c = g.node("MatMul", [sc, vh], name=nm("context"))
            c = g.node("Reshape", [g.node("Transpose", [c], name=nm("cp"), perm=[0, 2, 1, 3]), merge], name=nm("merge"))
            h = g.node("Add", [h, linear(c, E, D)], name=nm("res"))
        elif kind == "splitcat":
            if D % 16:
                continue
            a, b = g.node("Split", [h], name=nm("split"), axis=2, n_out=2)
            h = g.node("Concat", [g.node("Tanh", [b], name=nm("t")), a], name=nm("cat"), axis=2)
        used.append(kind)
    pooled = g.node("ReduceMean", [h], name="pool", axes=[1], keepdims=0)
    classes = int(rng.choice([3, 7, 10]))
    y = g.node("Gemm", [pooled, g.init("head.w", lin((classes, D), D)), g.init("head.b", np.zeros(classes, np.float32))],
               name="head", transB=1)
    g.output(y, ["N", classes])
    return g.model_proto(opset=13), (S * D0,), used
