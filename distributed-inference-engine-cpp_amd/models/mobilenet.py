"""MobileNetV2-style ONNX generator + torch fp32 reference (grouped-conv coverage of the HIP engine).

The reference engine binds input 0 / output 0 of ANY single-input ONNX model through ONNX Runtime
(/root/reference/src/inference_engine.cpp:31-69), so the in-tree engine must cover more than the
ResNet50 op set.  This family exercises what ResNet-v2 and ViT do not:
  * depthwise 3x3 convs (Conv with group = channels) folded with BatchNormalization,
  * Clip(0, 6) (ReLU6) given as opset-11 min/max inputs, fused into conv epilogues,
  * TF-style asymmetric "SAME" padding on the stride-2 depthwise convs (pads [0, 0, 1, 1]),
  * inverted-residual Adds, and an optional Softmax head on the logits.
Weights are random (no checkpoint offline); `torch_forward` rebuilds the network from the same
arrays and is the oracle.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Tuple

import numpy as np

from ..utils.onnx_writer import GraphBuilder

# (expansion t, channels c, repeats n, stride s) of MobileNetV2
SETTINGS = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2), (6, 320, 1, 1)]


@dataclass
class MobileNetConfig:
    width: float = 1.0
    image: int = 224
    in_ch: int = 3
    num_classes: int = 1000
    last: int = 1280
    softmax_head: bool = True
    asym_pad: bool = True  # stride-2 depthwise convs padded [0, 0, 1, 1] like a TF export
    seed: int = 0


def tiny_mobilenet_config(seed: int = 0) -> MobileNetConfig:
    return MobileNetConfig(width=0.5, image=64, num_classes=10, last=256, seed=seed)


def _div8(v: float) -> int:
    return max(8, int(v + 4) // 8 * 8)


def _blocks(cfg: MobileNetConfig) -> List[dict]:
    out, cin = [], _div8(32 * cfg.width)
    for t, c, n, s in SETTINGS:
        cout = _div8(c * cfg.width)
        for i in range(n):
            out.append({"t": t, "cin": cin, "cout": cout, "stride": s if i == 0 else 1, "hidden": cin * t})
            cin = cout
    return out


def make_weights(cfg: MobileNetConfig) -> Dict[str, np.ndarray]:
    rng = np.random.default_rng(cfg.seed)
    w: Dict[str, np.ndarray] = {}

    def conv(name, cout, cin_per_group, k, gain=1.0):
        std = gain * math.sqrt(2.0 / (cin_per_group * k * k))
        w[name + ".weight"] = rng.normal(0, std, (cout, cin_per_group, k, k)).astype(np.float32)

    def bn(name, c):
        w[name + ".gamma"] = rng.uniform(0.7, 1.3, c).astype(np.float32)
        w[name + ".beta"] = rng.normal(0, 0.1, c).astype(np.float32)
        w[name + ".mean"] = rng.normal(0, 0.1, c).astype(np.float32)
        w[name + ".var"] = rng.uniform(0.6, 1.4, c).astype(np.float32)

    c0 = _div8(32 * cfg.width)
    conv("stem", c0, cfg.in_ch, 3)
    bn("stem_bn", c0)
    for i, b in enumerate(_blocks(cfg)):
        p = "block%d." % i
        if b["t"] != 1:
            conv(p + "expand", b["hidden"], b["cin"], 1)
            bn(p + "expand_bn", b["hidden"])
        conv(p + "dw", b["hidden"], 1, 3)
        bn(p + "dw_bn", b["hidden"])
        conv(p + "project", b["cout"], b["hidden"], 1, gain=0.5)
        bn(p + "project_bn", b["cout"])
    cl = _blocks(cfg)[-1]["cout"]
    conv("head", cfg.last, cl, 1)
    bn("head_bn", cfg.last)
    w["fc.weight"] = rng.normal(0, 1.0 / math.sqrt(cfg.last), (cfg.num_classes, cfg.last)).astype(np.float32)
    w["fc.bias"] = rng.normal(0, 0.01, cfg.num_classes).astype(np.float32)
    return w


def build_onnx(cfg: MobileNetConfig = MobileNetConfig(), opset: int = 13) -> Tuple[bytes, Dict[str, np.ndarray]]:
    w = make_weights(cfg)
    g = GraphBuilder(name="mobilenet_v2")
    for k, v in w.items():
        g.init(k, v)
    lo = g.const(np.array(0.0, np.float32), "clip_min")
    hi = g.const(np.array(6.0, np.float32), "clip_max")
    x = g.input("input", ["N", cfg.in_ch, cfg.image, cfg.image])

    def conv_bn(inp, name, bn_name, k, stride, pads, group=1):
        y = g.node("Conv", [inp, name + ".weight"], name=name, kernel_shape=[k, k], strides=[stride, stride],
                   pads=pads, group=group)
        return g.node("BatchNormalization", [y, bn_name + ".gamma", bn_name + ".beta", bn_name + ".mean",
                                             bn_name + ".var"], name=bn_name, epsilon=1e-5)

    def relu6(inp, name):
        return g.node("Clip", [inp, lo, hi], name=name)

    h = relu6(conv_bn(x, "stem", "stem_bn", 3, 2, [1, 1, 1, 1]), "stem_relu6")
    for i, b in enumerate(_blocks(cfg)):
        p = "block%d." % i
        y = h
        if b["t"] != 1:
            y = relu6(conv_bn(y, p + "expand", p + "expand_bn", 1, 1, [0, 0, 0, 0]), p + "expand_relu6")
        pads = [0, 0, 1, 1] if (b["stride"] == 2 and cfg.asym_pad) else [1, 1, 1, 1]
        y = relu6(conv_bn(y, p + "dw", p + "dw_bn", 3, b["stride"], pads, group=b["hidden"]), p + "dw_relu6")
        y = conv_bn(y, p + "project", p + "project_bn", 1, 1, [0, 0, 0, 0])
        if b["stride"] == 1 and b["cin"] == b["cout"]:
            y = g.node("Add", [y, h], name=p + "residual")
        h = y
    h = relu6(conv_bn(h, "head", "head_bn", 1, 1, [0, 0, 0, 0]), "head_relu6")
    h = g.node("GlobalAveragePool", [h], name="gap")
    h = g.node("Flatten", [h], name="flatten", axis=1)
    y = g.node("Gemm", [h, "fc.weight", "fc.bias"], name="fc", transB=1)
    if cfg.softmax_head:
        y = g.node("Softmax", [y], name="prob", axis=-1)
    g.output(y, ["N", cfg.num_classes])
    return g.model_proto(opset=opset, ir_version=7), w


def torch_forward(w: Dict[str, np.ndarray], x, cfg: MobileNetConfig = MobileNetConfig(), device="cpu", dtype=None):
    import torch
    import torch.nn.functional as F

    dtype = dtype or torch.float32
    t = {k: torch.from_numpy(v).to(device=device, dtype=dtype) for k, v in w.items()}
    if not torch.is_tensor(x):
        x = torch.from_numpy(np.asarray(x, np.float32))
    x = x.to(device=device, dtype=dtype)

    def conv_bn(inp, name, bn, stride, pad, group=1, asym=False):
        if asym:
            inp = F.pad(inp, (0, 1, 0, 1))
            pad = 0
        y = F.conv2d(inp, t[name + ".weight"], stride=stride, padding=pad, groups=group)
        return F.batch_norm(y, t[bn + ".mean"], t[bn + ".var"], t[bn + ".gamma"], t[bn + ".beta"], False, 0.0, 1e-5)

    h = torch.clamp(conv_bn(x, "stem", "stem_bn", 2, 1), 0, 6)
    for i, b in enumerate(_blocks(cfg)):
        p = "block%d." % i
        y = h
        if b["t"] != 1:
            y = torch.clamp(conv_bn(y, p + "expand", p + "expand_bn", 1, 0), 0, 6)
        asym = b["stride"] == 2 and cfg.asym_pad
        y = torch.clamp(conv_bn(y, p + "dw", p + "dw_bn", b["stride"], 1, group=b["hidden"], asym=asym), 0, 6)
        y = conv_bn(y, p + "project", p + "project_bn", 1, 0)
        if b["stride"] == 1 and b["cin"] == b["cout"]:
            y = y + h
        h = y
    h = torch.clamp(conv_bn(h, "head", "head_bn", 1, 0), 0, 6)
    y = F.linear(h.mean(dim=(2, 3)), t["fc.weight"], t["fc.bias"])
    return torch.softmax(y, -1) if cfg.softmax_head else y


def synthetic_input(batch: int, cfg: MobileNetConfig = MobileNetConfig(), seed: int = 1) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return np.round(rng.random((batch, cfg.in_ch, cfg.image, cfg.image), dtype=np.float32), 4).astype(np.float32)
