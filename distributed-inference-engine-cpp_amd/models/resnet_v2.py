"""ResNet-v2 (pre-activation) ONNX generator + torch fp32 reference.

Mirrors the topology of the ONNX model-zoo `resnet50-v2-7.onnx` the reference serves
(`src/worker_node.cpp:145-168`, README "models/resnet50-v2-7.onnx"; blob absent:
`.MISSING_LARGE_BLOBS:1`): gluoncv `resnet50_v2` exported at opset 7 with input `data`
[N,3,224,224] and output `resnetv24_dense0_fwd` [N,1000]:

    BN(data) -> Conv7x7/2 -> BN -> ReLU -> MaxPool3x3/2
    -> 4 stages of BottleneckV2 units   (pre-activation: BN->ReLU->conv, shortcut conv on the
       first unit of a stage takes the activated input)
    -> BN -> ReLU -> GlobalAveragePool -> Flatten -> Gemm

The weights are random (no network, no checkpoint).  `torch_forward` rebuilds the same network in
torch from the same numpy arrays and is the correctness oracle for the C++ CPU executor and for the
HIP engine.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..utils.onnx_writer import GraphBuilder

LAYERS = {
    18: ("basic", [2, 2, 2, 2]),
    34: ("basic", [3, 4, 6, 3]),
    50: ("bottleneck", [3, 4, 6, 3]),
    101: ("bottleneck", [3, 4, 23, 3]),
    152: ("bottleneck", [3, 8, 36, 3]),
}


@dataclass
class ResNetConfig:
    depth: int = 50
    num_classes: int = 1000
    image: int = 224
    in_ch: int = 3
    width: int = 64          # stem width; stage widths are width * (1, 2, 4, 8)
    layers: Optional[List[int]] = None  # override units per stage (tiny test models)
    block: Optional[str] = None
    seed: int = 0
    prefix: str = "resnetv24"


def _rng_bn(rng, c, prefix, w, input_bn=False):
    if input_bn:  # gluon BatchNorm(scale=False, center=False) on raw pixels in [0, 1)
        w[prefix + "_gamma"] = np.ones(c, np.float32)
        w[prefix + "_beta"] = np.zeros(c, np.float32)
        w[prefix + "_running_mean"] = np.full(c, 0.45, np.float32) + rng.normal(0, 0.02, c).astype(np.float32)
        w[prefix + "_running_var"] = np.full(c, 0.07, np.float32) + rng.uniform(0, 0.01, c).astype(np.float32)
        return
    w[prefix + "_gamma"] = rng.uniform(0.7, 1.3, c).astype(np.float32)
    w[prefix + "_beta"] = rng.normal(0, 0.1, c).astype(np.float32)
    w[prefix + "_running_mean"] = rng.normal(0, 0.1, c).astype(np.float32)
    w[prefix + "_running_var"] = rng.uniform(0.6, 1.4, c).astype(np.float32)


def _rng_conv(rng, cout, cin, k, prefix, w, gain=1.0):
    std = gain * math.sqrt(2.0 / (cin * k * k))
    w[prefix + "_weight"] = rng.normal(0, std, (cout, cin, k, k)).astype(np.float32)


def make_weights(cfg: ResNetConfig) -> Tuple[Dict[str, np.ndarray], list]:
    """Random weights + an op list describing the network (shared by ONNX and torch builders)."""
    block, layers = LAYERS[cfg.depth]
    if cfg.layers is not None:
        layers = cfg.layers
    if cfg.block is not None:
        block = cfg.block
    rng = np.random.default_rng(cfg.seed)
    p = cfg.prefix
    w: Dict[str, np.ndarray] = {}
    ops = []
    _rng_bn(rng, cfg.in_ch, p + "_batchnorm0", w, input_bn=True)
    _rng_conv(rng, cfg.width, cfg.in_ch, 7, p + "_conv0", w)
    _rng_bn(rng, cfg.width, p + "_batchnorm1", w)
    expansion = 4 if block == "bottleneck" else 1
    in_ch = cfg.width
    for s, n_units in enumerate(layers):
        sp = "%s_stage%d" % (p, s + 1)
        mid = cfg.width * (2 ** s)
        out_ch = mid * expansion
        bn_i = conv_i = 0
        for u in range(n_units):
            stride = 2 if (u == 0 and s > 0) else 1
            downsample = u == 0 and (stride != 1 or in_ch != out_ch)
            unit = {"stride": stride, "in": in_ch, "mid": mid, "out": out_ch, "block": block}
            names = {}
            names["bn1"] = "%s_batchnorm%d" % (sp, bn_i); bn_i += 1
            _rng_bn(rng, in_ch, names["bn1"], w)
            if block == "bottleneck":
                names["conv1"] = "%s_conv%d" % (sp, conv_i); conv_i += 1
                _rng_conv(rng, mid, in_ch, 1, names["conv1"], w)
                names["bn2"] = "%s_batchnorm%d" % (sp, bn_i); bn_i += 1
                _rng_bn(rng, mid, names["bn2"], w)
                names["conv2"] = "%s_conv%d" % (sp, conv_i); conv_i += 1
                _rng_conv(rng, mid, mid, 3, names["conv2"], w)
                names["bn3"] = "%s_batchnorm%d" % (sp, bn_i); bn_i += 1
                _rng_bn(rng, mid, names["bn3"], w)
                names["conv3"] = "%s_conv%d" % (sp, conv_i); conv_i += 1
                # small last-conv gain keeps the residual stream bounded over 16+ units
                _rng_conv(rng, out_ch, mid, 1, names["conv3"], w, gain=0.3)
            else:
                names["conv1"] = "%s_conv%d" % (sp, conv_i); conv_i += 1
                _rng_conv(rng, mid, in_ch, 3, names["conv1"], w)
                names["bn2"] = "%s_batchnorm%d" % (sp, bn_i); bn_i += 1
                _rng_bn(rng, mid, names["bn2"], w)
                names["conv2"] = "%s_conv%d" % (sp, conv_i); conv_i += 1
                _rng_conv(rng, out_ch, mid, 3, names["conv2"], w, gain=0.3)
            if downsample:
                names["ds"] = "%s_conv%d" % (sp, conv_i); conv_i += 1
                _rng_conv(rng, out_ch, in_ch, 1, names["ds"], w)
            unit["names"] = names
            unit["downsample"] = downsample
            unit["tag"] = "%s_unit%d" % (sp, u)
            ops.append(unit)
            in_ch = out_ch
    _rng_bn(rng, in_ch, p + "_batchnorm2", w)
    w[p + "_dense0_weight"] = rng.normal(0, 1.0 / math.sqrt(in_ch), (cfg.num_classes, in_ch)).astype(np.float32)
    w[p + "_dense0_bias"] = rng.normal(0, 0.01, cfg.num_classes).astype(np.float32)
    return w, ops


def build_onnx(cfg: ResNetConfig = ResNetConfig(), opset: int = 7, dynamic_batch: bool = True,
               initializers_as_inputs: bool = True, inject_unit: int = -1,
               inject_op: str = "Sign") -> Tuple[bytes, Dict[str, np.ndarray]]:
    """inject_unit >= 0: an `inject_op` node after that unit's second activation -- a node the HIP
    planner may not lower, for the hybrid HIP + CPU tests (engine/hybrid_engine.cpp).  Sign is
    applied as y * Sign(y), the identity on the ReLU output it follows; any other op is applied as
    is (it should be the identity on y >= 0, e.g. Abs), so the model's function is unchanged."""
    w, ops = make_weights(cfg)
    p = cfg.prefix
    g = GraphBuilder(name="resnet_v2", initializers_as_inputs=initializers_as_inputs)
    for k, v in w.items():
        g.init(k, v)
    N = "N" if dynamic_batch else 1
    x = g.input("data", [N, cfg.in_ch, cfg.image, cfg.image])
    bn_attrs = {"epsilon": 1e-5, "momentum": 0.9}
    if opset < 9:
        bn_attrs["spatial"] = 1

    def bn(inp, name):
        return g.node("BatchNormalization", [inp, name + "_gamma", name + "_beta", name + "_running_mean",
                                             name + "_running_var"], name=name + "_fwd", **bn_attrs)

    def conv(inp, name, k, stride, pad):
        return g.node("Conv", [inp, name + "_weight"], name=name + "_fwd", kernel_shape=[k, k],
                      strides=[stride, stride], pads=[pad, pad, pad, pad], dilations=[1, 1], group=1)

    x = bn(x, p + "_batchnorm0")
    x = conv(x, p + "_conv0", 7, 2, 3)
    x = bn(x, p + "_batchnorm1")
    x = g.node("Relu", [x], name=p + "_relu0_fwd")
    x = g.node("MaxPool", [x], name=p + "_pool0_fwd", kernel_shape=[3, 3], strides=[2, 2], pads=[1, 1, 1, 1])
    for i, u in enumerate(ops):
        n = u["names"]
        residual = x
        a = bn(x, n["bn1"])
        a = g.node("Relu", [a], name=u["tag"] + "_activation0")
        if u["downsample"]:
            residual = conv(a, n["ds"], 1, u["stride"], 0)
        if u["block"] == "bottleneck":
            y = conv(a, n["conv1"], 1, 1, 0)
            y = g.node("Relu", [bn(y, n["bn2"])], name=u["tag"] + "_activation1")
            y = conv(y, n["conv2"], 3, u["stride"], 1)
            y = g.node("Relu", [bn(y, n["bn3"])], name=u["tag"] + "_activation2")
            if i == inject_unit:
                z = g.node(inject_op, [y], name=u["tag"] + "_injected")
                y = g.node("Mul", [y, z], name=u["tag"] + "_injected_mul") if inject_op == "Sign" else z
            y = conv(y, n["conv3"], 1, 1, 0)
        else:
            y = conv(a, n["conv1"], 3, u["stride"], 1)
            y = g.node("Relu", [bn(y, n["bn2"])], name=u["tag"] + "_activation1")
            y = conv(y, n["conv2"], 3, 1, 1)
        x = g.node("Add", [y, residual], name=u["tag"] + "__plus0")
    x = bn(x, p + "_batchnorm2")
    x = g.node("Relu", [x], name=p + "_relu1_fwd")
    x = g.node("GlobalAveragePool", [x], name=p + "_pool1_fwd")
    x = g.node("Flatten", [x], name="flatten_473", axis=1)
    y = g.node("Gemm", [x, p + "_dense0_weight", p + "_dense0_bias"], name=p + "_dense0_fwd", alpha=1.0, beta=1.0,
               transA=0, transB=1)
    g.output(y, [N, cfg.num_classes])
    ir = 3 if opset <= 7 else 8
    return g.model_proto(opset=opset, ir_version=ir), w


def torch_forward(w: Dict[str, np.ndarray], x, cfg: ResNetConfig = ResNetConfig(), device="cpu",
                  dtype=None):
    """fp32 torch implementation of the generated graph (oracle)."""
    import torch
    import torch.nn.functional as F

    dtype = dtype or torch.float32
    _, ops = make_weights(cfg)  # topology only (weights regenerated identically, then ignored)
    p = cfg.prefix
    t = {k: torch.from_numpy(v).to(device=device, dtype=dtype) for k, v in w.items()}
    if not torch.is_tensor(x):
        x = torch.from_numpy(np.asarray(x, np.float32))
    x = x.to(device=device, dtype=dtype)

    def bn(v, name):
        return F.batch_norm(v, t[name + "_running_mean"], t[name + "_running_var"], t[name + "_gamma"],
                            t[name + "_beta"], False, 0.0, 1e-5)

    x = bn(x, p + "_batchnorm0")
    x = F.conv2d(x, t[p + "_conv0_weight"], stride=2, padding=3)
    x = F.relu(bn(x, p + "_batchnorm1"))
    x = F.max_pool2d(x, 3, 2, 1)
    for u in ops:
        n = u["names"]
        residual = x
        a = F.relu(bn(x, n["bn1"]))
        if u["downsample"]:
            residual = F.conv2d(a, t[n["ds"] + "_weight"], stride=u["stride"])
        if u["block"] == "bottleneck":
            y = F.conv2d(a, t[n["conv1"] + "_weight"])
            y = F.relu(bn(y, n["bn2"]))
            y = F.conv2d(y, t[n["conv2"] + "_weight"], stride=u["stride"], padding=1)
            y = F.relu(bn(y, n["bn3"]))
            y = F.conv2d(y, t[n["conv3"] + "_weight"])
        else:
            y = F.conv2d(a, t[n["conv1"] + "_weight"], stride=u["stride"], padding=1)
            y = F.relu(bn(y, n["bn2"]))
            y = F.conv2d(y, t[n["conv2"] + "_weight"], padding=1)
        x = y + residual
    x = F.relu(bn(x, p + "_batchnorm2"))
    x = x.mean(dim=(2, 3))
    return F.linear(x, t[p + "_dense0_weight"], t[p + "_dense0_bias"])


def tiny_config(seed: int = 0) -> ResNetConfig:
    """A small pre-activation bottleneck ResNet with every op kind of ResNet50-v2 (fast CPU tests)."""
    return ResNetConfig(depth=50, layers=[1, 2, 1, 1], width=16, image=64, num_classes=10, seed=seed)


def synthetic_input(batch: int, cfg: ResNetConfig = ResNetConfig(), seed: int = 1) -> np.ndarray:
    """Image-like values in [0, 1) with 4 decimals (what the benchmark payload carries)."""
    rng = np.random.default_rng(seed)
    x = rng.random((batch, cfg.in_ch, cfg.image, cfg.image), dtype=np.float32)
    return np.round(x, 4).astype(np.float32)
