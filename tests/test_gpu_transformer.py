"""Numerics of the transformer kernels (csrc/kernels/transformer.hip + the GELU/residual GEMM
epilogue) against plain PyTorch fp32 references, and the ViT models end to end on the HIP engine."""
import math

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def rel_l2(a, b):
    a = a.float() if hasattr(a, "float") else a
    b = b.float() if hasattr(b, "float") else b
    import torch

    return float(torch.linalg.norm((a - b).flatten()) / max(float(torch.linalg.norm(b.flatten())), 1e-12))


@pytest.fixture(scope="module")
def K():
    from die_amd.ops import kernels

    return kernels


@pytest.mark.parametrize("C", [128, 768, 1024])
def test_layernorm(K, C):
    import torch

    g = torch.Generator(device="cuda").manual_seed(C)
    x = (torch.randn(37, C, device="cuda", generator=g) * 3 + 1).bfloat16()
    gamma = torch.rand(C, device="cuda", generator=g) + 0.5
    beta = torch.randn(C, device="cuda", generator=g) * 0.1
    y = K.layernorm(x, gamma, beta, eps=1e-12)
    ref = torch.nn.functional.layer_norm(x.float(), (C,), gamma, beta, 1e-12)
    assert rel_l2(y, ref) < 8e-3


def test_tokens_and_gather(K):
    import torch

    B, S0, C = 3, 196, 768
    p = torch.randn(B, S0, C, device="cuda").bfloat16()
    cls = torch.randn(C, device="cuda")
    pos = torch.randn(S0 + 1, C, device="cuda")
    out = K.tokens_assemble(p, cls, pos)
    ref = torch.cat([cls.expand(B, 1, C), p.float()], 1) + pos
    assert rel_l2(out, ref) < 5e-3
    g = K.gather_rows(out, 0)
    assert torch.equal(g, out[:, 0, :])
    g5 = K.gather_rows(out, 5)
    assert torch.equal(g5, out[:, 5, :])


def _attn_ref(q, k, v, H, scale):
    B, S, C = q.shape
    D = C // H
    qh = q.float().view(B, S, H, D).transpose(1, 2)
    kh = k.float().view(B, S, H, D).transpose(1, 2)
    vh = v.float().view(B, S, H, D).transpose(1, 2)
    p = torch_softmax(qh @ kh.transpose(-1, -2) * scale)
    return (p @ vh).transpose(1, 2).reshape(B, S, C)


def torch_softmax(x):
    import torch

    return torch.softmax(x, dim=-1)


@pytest.mark.parametrize("S,H", [(17, 2), (64, 1), (65, 3), (128, 2), (197, 12), (256, 4)])
def test_attention(K, S, H):
    import torch

    B, D = 2, 64
    C = H * D
    g = torch.Generator(device="cuda").manual_seed(S * 31 + H)
    # fused QKV rows [B, S, 3C]; q/k/v are strided column slices (exactly how the engine calls it)
    qkv = (torch.randn(B, S, 3 * C, device="cuda", generator=g) * 1.5).bfloat16()
    q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    scale = 1.0 / math.sqrt(D)
    out = K.attention(q, k, v, H, scale)
    ref = _attn_ref(q, k, v, H, scale)
    assert torch.isfinite(out.float()).all()
    assert rel_l2(out, ref) < 2e-2, rel_l2(out, ref)


def test_attention_rejects_bad_shapes(K):
    import torch

    from die_amd import native

    x = torch.zeros(1, 64, 96, device="cuda", dtype=torch.bfloat16)  # 2 heads of 48: not a supported head dim
    with pytest.raises(native.NativeError):
        K.attention(x, x, x, 2)


@pytest.mark.parametrize("D", [32, 80, 96, 128])
@pytest.mark.parametrize("S", [17, 197, 300])
def test_attention_head_dims(K, D, S):
    """The streaming kernel takes head dims 32, 64, 80, 96 and 128 (HD/16 k-steps of K Q^T,
    ceil(HD/32) output accumulators): bf16 against torch, and fp32 (split) against float64 at rel 1e-5."""
    import torch

    g = torch.Generator(device="cuda").manual_seed(S * 7 + D)
    B, H = 2, 2
    C = H * D
    qkv = torch.randn(B, S, 3 * C, device="cuda", generator=g)
    qb = qkv.bfloat16()
    q, k, v = qb[..., :C], qb[..., C:2 * C], qb[..., 2 * C:]
    scale = 1.0 / math.sqrt(D)
    out = K.attention(q, k, v, H, scale)
    assert rel_l2(out, _attn_ref(q, k, v, H, scale)) < 2e-2
    got = K.attention_qkv_split(qkv, H, scale)
    qd, kd, vd = (qkv[..., i * C:(i + 1) * C].double().reshape(B, S, H, D).transpose(1, 2) for i in range(3))
    ref = (torch.softmax(qd @ kd.transpose(-1, -2) * scale, -1) @ vd).transpose(1, 2).reshape(B, S, C)
    err = float((got.double() - ref).norm() / ref.norm())
    assert err <= 1e-5, err


@pytest.mark.parametrize("D", [64, 128])
def test_attention_deep_variant_bitwise(K, D):
    """Variant 1 (K/V staged two tiles ahead) computes the same tiles in the same order."""
    import torch

    g = torch.Generator(device="cuda").manual_seed(D)
    B, S, H = 3, 197, 2
    C = H * D
    qkv = torch.randn(B, S, 3 * C, device="cuda", generator=g)
    try:
        K.set_attention_variant(0)
        a = K.attention_qkv_split(qkv, H)
        K.set_attention_variant(1)
        b = K.attention_qkv_split(qkv, H)
    finally:
        K.set_attention_variant(0)
    assert torch.equal(a, b)


@pytest.mark.parametrize("S", [300, 520])
def test_attention_long_sequences(K, S):
    """The streaming kernel takes any sequence length (K/V in 32-key tiles, 128 queries per block)."""
    import torch

    g = torch.Generator(device="cuda").manual_seed(S)
    B, H, D = 2, 2, 64
    C = H * D
    qkv = torch.randn(B, S, 3 * C, device="cuda", generator=g).bfloat16()
    q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    scale = 1.0 / math.sqrt(D)
    out = K.attention(q, k, v, H, scale)
    ref = _attn_ref(q, k, v, H, scale)
    assert torch.isfinite(out.float()).all()
    assert rel_l2(out, ref) < 2e-2, rel_l2(out, ref)


@pytest.mark.parametrize("act", [0, 1, 2])
def test_linear_epilogues(K, act):
    import torch

    g = torch.Generator(device="cuda").manual_seed(act)
    B, S, Kd, N = 4, 197, 768, 3072
    x = torch.randn(B, S, Kd, device="cuda", generator=g).bfloat16()
    w = torch.randn(N, Kd, device="cuda", generator=g) / math.sqrt(Kd)
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    y = K.linear(x, w, b, act=act)
    ref = x.float() @ w.bfloat16().float().t() + b
    if act == 1:
        ref = torch.relu(ref)
    elif act == 2:
        ref = torch.nn.functional.gelu(ref)
    assert rel_l2(y, ref) < 1e-2


def test_linear_residual(K):
    import torch

    B, S, Kd, N = 2, 197, 3072, 768
    x = torch.randn(B, S, Kd, device="cuda").bfloat16()
    w = torch.randn(N, Kd, device="cuda") / math.sqrt(Kd)
    b = torch.randn(N, device="cuda") * 0.1
    r = torch.randn(B, S, N, device="cuda").bfloat16()
    y = K.linear(x, w, b, res=r)
    ref = x.float() @ w.bfloat16().float().t() + b + r.float()
    assert rel_l2(y, ref) < 1e-2


def test_vit_tiny_engine_vs_torch(native, models):
    import torch

    from die_amd.models import vit

    path, w, cfg = models["get_vit"]("tiny")
    e = native.Engine(path, device="hip", max_batch=8)
    x = vit.synthetic_input(5, cfg)
    got = e.run(x.reshape(5, -1))
    with torch.no_grad():
        ref = vit.torch_forward(w, x, cfg).numpy()
    err = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
    assert err < 1e-4, err  # fp32 engine (default precision)
    assert (got.argmax(1) == ref.argmax(1)).all()
    one = e.run(x[:1].reshape(1, -1))
    assert float(np.linalg.norm(one[0] - got[0]) / np.linalg.norm(got[0])) < 1e-4
    e.close()


def test_vit_base_engine_vs_torch(native, models):
    import torch

    from die_amd.models import vit

    path, w, cfg = models["get_vit"]("base")
    e = native.Engine(path, device="hip", max_batch=32)
    info = e.refresh_info()
    assert info["hip_graphs"] is True
    x = vit.synthetic_input(4, cfg)
    got = e.run(x.reshape(4, -1))
    with torch.no_grad():
        ref = vit.torch_forward(w, x, cfg, device="cuda").cpu().numpy()
    err = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
    assert err < 1e-4, err  # fp32 engine (default precision)
    assert (got.argmax(1) == ref.argmax(1)).all()
    e.close()


@pytest.mark.parametrize("size,stats_epi", [("tiny", False), ("tiny", True), ("base", False), ("base", True)])
def test_vit_fold_layernorm_vs_torch(native, models, size, stats_epi):
    """EngineOptions::fold_layernorm: every pre-norm LayerNorm computes row statistics only and the
    QKV / first-MLP GEMMs read the residual rows with gamma folded into their weights, beta into
    their bias and (mean, rstd) applied in the epilogue -- same accuracy bar as the unfolded engine
    (fp32 rel-L2 <= 1e-4 against torch, same top-1), in the autotuned and untuned paths.
    stats_epi (EngineOptions::ln_stats_epilogue, default on): the statistics come as per-64-column
    (mean, M2) partials from the token assembly (block 0) and the attention-out / MLP2 GEMM
    epilogues -- covered in the fused split-K, two-kernel split-K and plain epilogues."""
    import torch

    from die_amd.models import vit

    path, w, cfg = models["get_vit"](size)
    s = native.plan_summary(path, 8, precision="fp32", fold_layernorm=True, ln_stats_epilogue=stats_epi)
    assert sum(1 for o in s["ops"] if o.get("stats_only")) == (0 if stats_epi else 2 * cfg.depth)
    assert sum(1 for o in s["ops"] if o.get("stats_out")) == (2 * cfg.depth if stats_epi else 0)
    assert sum(1 for o in s["ops"] if o.get("layernorm_folded")) == 2 * cfg.depth
    x = vit.synthetic_input(5, cfg)
    with torch.no_grad():
        ref = vit.torch_forward(w, x, cfg, device="cuda").cpu().numpy()
    runs = [dict(autotune=False)]
    if size == "tiny":
        runs += [dict(autotune=True), dict(autotune=True, splitk_two_kernel=True)]
    for kw in runs:
        e = native.Engine(path, device="hip", max_batch=8, fold_layernorm=True, ln_stats_epilogue=stats_epi, **kw)
        try:
            assert e.refresh_info()["options"]["fold_layernorm"] is True
            assert e.refresh_info()["options"]["ln_stats_epilogue"] is stats_epi
            got = e.run(x.reshape(5, -1))
            # the statistics hand-off merges in a fixed order: bitwise repeatable
            assert np.array_equal(got, e.run(x.reshape(5, -1)))
            err = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
            assert err < 1e-4, (kw, err)
            assert (got.argmax(1) == ref.argmax(1)).all()
        finally:
            e.close()
    # bf16 mode plans without folding (fp32 mode only)
    assert not any(o.get("stats_only") for o in native.plan_summary(path, 8, precision="bf16")["ops"])
