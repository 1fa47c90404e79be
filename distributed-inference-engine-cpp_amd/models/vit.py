"""ViT-B/16 ONNX generator + torch fp32 reference (BASELINE.json config 5).

Graph layout follows a HuggingFace `ViTForImageClassification` export at opset 17:
  Conv16x16/16 (patch embed) -> Reshape[0,C,-1] -> Transpose[0,2,1] -> Concat(Expand(cls), .) -> +pos
  -> 12 x { LayerNormalization -> MatMul+Add (q, k, v) -> Reshape[0,0,H,D] -> Transpose
            -> MatMul(q, k^T) -> Div(sqrt(D)) -> Softmax -> MatMul(., v) -> Transpose -> Reshape
            -> MatMul+Add (proj) -> Add(residual)
            -> LayerNormalization -> MatMul+Add -> GELU(erf: Div, Erf, Add, Mul, Mul) -> MatMul+Add
            -> Add(residual) }
  -> LayerNormalization -> Gather(token 0) -> Gemm (classifier).
The batch dimension is dynamic (the cls-token Expand takes its shape from Shape(input)).  Weights
are random (no checkpoint offline); `torch_forward` is the fp32 oracle for both executors.

Export variants (op coverage of the HIP engine): `decomposed_ln` writes every LayerNormalization the
way torch exports it below opset 17 (ReduceMean, Sub, Pow, ReduceMean, Add, Sqrt, Div, Mul, Add),
`cls_slice` selects the cls token with Slice + Reshape instead of Gather, `softmax_head` appends a
Softmax to the logits.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Tuple

import numpy as np

from ..utils.onnx_writer import INT64, GraphBuilder


@dataclass
class ViTConfig:
    image: int = 224
    patch: int = 16
    in_ch: int = 3
    dim: int = 768
    depth: int = 12
    heads: int = 12
    mlp: int = 3072
    num_classes: int = 1000
    eps: float = 1e-12
    seed: int = 0
    decomposed_ln: bool = False
    cls_slice: bool = False
    softmax_head: bool = False


def tiny_vit_config(seed: int = 0) -> ViTConfig:
    # head dim 64 (the fused attention kernel's tile), 16 patches + cls = 17 tokens
    return ViTConfig(image=32, patch=8, dim=128, depth=2, heads=2, mlp=256, num_classes=16, seed=seed)


def make_weights(cfg: ViTConfig) -> Dict[str, np.ndarray]:
    rng = np.random.default_rng(cfg.seed)
    D, P = cfg.dim, cfg.patch
    S = (cfg.image // P) ** 2 + 1
    w: Dict[str, np.ndarray] = {}

    def lin(name, k, n, std=None):
        w[name + ".weight"] = rng.normal(0, std or 1.0 / math.sqrt(k), (k, n)).astype(np.float32)  # [in, out]
        w[name + ".bias"] = rng.normal(0, 0.02, n).astype(np.float32)

    w["embeddings.patch.weight"] = rng.normal(0, 1.0 / math.sqrt(cfg.in_ch * P * P), (D, cfg.in_ch, P, P)).astype(np.float32)
    w["embeddings.patch.bias"] = rng.normal(0, 0.02, D).astype(np.float32)
    w["embeddings.cls_token"] = rng.normal(0, 0.5, (1, 1, D)).astype(np.float32)
    w["embeddings.position_embeddings"] = rng.normal(0, 0.2, (1, S, D)).astype(np.float32)
    for i in range(cfg.depth):
        p = "encoder.layer.%d." % i
        for ln in ("layernorm_before", "layernorm_after"):
            w[p + ln + ".weight"] = rng.uniform(0.8, 1.2, D).astype(np.float32)
            w[p + ln + ".bias"] = rng.normal(0, 0.05, D).astype(np.float32)
        for n in ("query", "key", "value"):
            lin(p + "attention." + n, D, D)
        lin(p + "attention.output", D, D, std=0.5 / math.sqrt(D))
        lin(p + "intermediate", D, cfg.mlp)
        lin(p + "output", cfg.mlp, D, std=0.5 / math.sqrt(cfg.mlp))
    w["layernorm.weight"] = rng.uniform(0.8, 1.2, D).astype(np.float32)
    w["layernorm.bias"] = rng.normal(0, 0.05, D).astype(np.float32)
    w["classifier.weight"] = rng.normal(0, 1.0 / math.sqrt(D), (cfg.num_classes, D)).astype(np.float32)
    w["classifier.bias"] = rng.normal(0, 0.01, cfg.num_classes).astype(np.float32)
    return w


def build_onnx(cfg: ViTConfig = ViTConfig(), opset: int = 17) -> Tuple[bytes, Dict[str, np.ndarray]]:
    w = make_weights(cfg)
    g = GraphBuilder(name="vit")
    for k, v in w.items():
        g.init(k, v)
    D, H, P = cfg.dim, cfg.heads, cfg.patch
    hd = D // H
    x = g.input("pixel_values", ["batch", cfg.in_ch, cfg.image, cfg.image])
    e = g.node("Conv", [x, "embeddings.patch.weight", "embeddings.patch.bias"], name="patch_embed",
               kernel_shape=[P, P], strides=[P, P], pads=[0, 0, 0, 0])
    e = g.node("Reshape", [e, g.const(np.array([0, D, -1], np.int64), "shape")], name="patch_flatten")
    e = g.node("Transpose", [e], name="patch_transpose", perm=[0, 2, 1])
    shp = g.node("Shape", [x], name="input_shape")
    bdim = g.node("Gather", [shp, g.const(np.array([0], np.int64), "idx")], name="batch_dim", axis=0)
    eshape = g.node("Concat", [bdim, g.const(np.array([1, D], np.int64), "tail")], name="cls_shape", axis=0)
    cls = g.node("Expand", ["embeddings.cls_token", eshape], name="cls_expand")
    h = g.node("Concat", [cls, e], name="tokens", axis=1)
    h = g.node("Add", [h, "embeddings.position_embeddings"], name="add_pos")
    scale = g.const(np.array(math.sqrt(hd), np.float32), "sqrt_d")
    heads_shape = g.const(np.array([0, 0, H, hd], np.int64), "heads_shape")
    merge_shape = g.const(np.array([0, 0, D], np.int64), "merge_shape")
    sqrt2 = g.const(np.array(1.4142135381698608, np.float32), "sqrt2")
    one = g.const(np.array(1.0, np.float32), "one")
    half = g.const(np.array(0.5, np.float32), "half")

    def linear(inp, name):
        y = g.node("MatMul", [inp, name + ".weight"], name=name + "/MatMul")
        return g.node("Add", [y, name + ".bias"], name=name + "/Add")

    two = g.const(np.array(2.0, np.float32), "two")
    eps_c = g.const(np.array(cfg.eps, np.float32), "ln_eps")

    def layer_norm(inp, wname, name):
        if not cfg.decomposed_ln:
            return g.node("LayerNormalization", [inp, wname + ".weight", wname + ".bias"], name=name, axis=-1,
                          epsilon=cfg.eps)
        mu = g.node("ReduceMean", [inp], name=name + "/mean", axes=[-1], keepdims=1)
        d = g.node("Sub", [inp, mu], name=name + "/sub")
        var = g.node("ReduceMean", [g.node("Pow", [d, two], name=name + "/pow")], name=name + "/var", axes=[-1],
                     keepdims=1)
        sd = g.node("Sqrt", [g.node("Add", [var, eps_c], name=name + "/add_eps")], name=name + "/sqrt")
        y = g.node("Div", [d, sd], name=name + "/div")
        y = g.node("Mul", [y, wname + ".weight"], name=name + "/scale")
        return g.node("Add", [y, wname + ".bias"], name=name + "/shift")

    for i in range(cfg.depth):
        p = "encoder.layer.%d." % i
        a = layer_norm(h, p + "layernorm_before", p + "layernorm_before")
        q = linear(a, p + "attention.query")
        k = linear(a, p + "attention.key")
        v = linear(a, p + "attention.value")
        q = g.node("Transpose", [g.node("Reshape", [q, heads_shape], name=p + "q_heads")], name=p + "q_perm",
                   perm=[0, 2, 1, 3])
        k = g.node("Transpose", [g.node("Reshape", [k, heads_shape], name=p + "k_heads")], name=p + "k_perm",
                   perm=[0, 2, 3, 1])
        v = g.node("Transpose", [g.node("Reshape", [v, heads_shape], name=p + "v_heads")], name=p + "v_perm",
                   perm=[0, 2, 1, 3])
        s = g.node("MatMul", [q, k], name=p + "scores")
        s = g.node("Div", [s, scale], name=p + "scale")
        s = g.node("Softmax", [s], name=p + "softmax", axis=-1)
        c = g.node("MatMul", [s, v], name=p + "context")
        c = g.node("Transpose", [c], name=p + "ctx_perm", perm=[0, 2, 1, 3])
        c = g.node("Reshape", [c, merge_shape], name=p + "ctx_merge")
        o = linear(c, p + "attention.output")
        h = g.node("Add", [o, h], name=p + "residual1")
        a = layer_norm(h, p + "layernorm_after", p + "layernorm_after")
        m = linear(a, p + "intermediate")
        t = g.node("Div", [m, sqrt2], name=p + "gelu/div")
        t = g.node("Erf", [t], name=p + "gelu/erf")
        t = g.node("Add", [t, one], name=p + "gelu/add")
        t = g.node("Mul", [m, t], name=p + "gelu/mul")
        t = g.node("Mul", [t, half], name=p + "gelu/half")
        o = linear(t, p + "output")
        h = g.node("Add", [o, h], name=p + "residual2")
    h = layer_norm(h, "layernorm", "layernorm")
    if cfg.cls_slice:
        h = g.node("Slice", [h, g.const(np.array([0], np.int64), "s0"), g.const(np.array([1], np.int64), "s1"),
                             g.const(np.array([1], np.int64), "s_axis")], name="cls_slice")
        h = g.node("Reshape", [h, g.const(np.array([0, D], np.int64), "cls_shape2")], name="cls_flat")
    else:
        h = g.node("Gather", [h, g.const(np.array(0, np.int64), "cls_index")], name="cls_select", axis=1)
    y = g.node("Gemm", [h, "classifier.weight", "classifier.bias"], name="logits", transB=1)
    if cfg.softmax_head:
        y = g.node("Softmax", [y], name="prob", axis=-1)
    g.output(y, ["batch", cfg.num_classes])
    return g.model_proto(opset=opset, ir_version=8), w


def torch_forward(w, x, cfg: ViTConfig = ViTConfig(), device="cpu"):
    import torch
    import torch.nn.functional as F

    t = {k: torch.from_numpy(v).to(device) for k, v in w.items()}
    if not torch.is_tensor(x):
        x = torch.from_numpy(np.asarray(x, np.float32))
    x = x.to(device).float()
    B = x.shape[0]
    D, H = cfg.dim, cfg.heads
    hd = D // H
    e = F.conv2d(x, t["embeddings.patch.weight"], t["embeddings.patch.bias"], stride=cfg.patch)
    e = e.flatten(2).transpose(1, 2)
    h = torch.cat([t["embeddings.cls_token"].expand(B, 1, D), e], dim=1) + t["embeddings.position_embeddings"]
    S = h.shape[1]
    for i in range(cfg.depth):
        p = "encoder.layer.%d." % i
        a = F.layer_norm(h, (D,), t[p + "layernorm_before.weight"], t[p + "layernorm_before.bias"], cfg.eps)

        def lin(z, n):
            return z @ t[n + ".weight"] + t[n + ".bias"]

        q = lin(a, p + "attention.query").view(B, S, H, hd).transpose(1, 2)
        k = lin(a, p + "attention.key").view(B, S, H, hd).transpose(1, 2)
        v = lin(a, p + "attention.value").view(B, S, H, hd).transpose(1, 2)
        s = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(hd), dim=-1)
        c = (s @ v).transpose(1, 2).reshape(B, S, D)
        h = lin(c, p + "attention.output") + h
        a = F.layer_norm(h, (D,), t[p + "layernorm_after.weight"], t[p + "layernorm_after.bias"], cfg.eps)
        m = lin(a, p + "intermediate")
        m = 0.5 * m * (1.0 + torch.erf(m / 1.4142135381698608))
        h = lin(m, p + "output") + h
    h = F.layer_norm(h, (D,), t["layernorm.weight"], t["layernorm.bias"], cfg.eps)
    y = F.linear(h[:, 0], t["classifier.weight"], t["classifier.bias"])
    return torch.softmax(y, -1) if cfg.softmax_head else y


def synthetic_input(batch: int, cfg: ViTConfig = ViTConfig(), seed: int = 1) -> np.ndarray:
    rng = np.random.default_rng(seed)
    x = rng.random((batch, cfg.in_ch, cfg.image, cfg.image), dtype=np.float32) * 2 - 1
    return np.round(x, 4).astype(np.float32)
