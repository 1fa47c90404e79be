"""fp32 mode of the HIP kernels (split hi/lo bf16 planes, csrc/kernels/common.h) vs plain PyTorch fp32.

Unlike test_gpu_kernels.py the operands are NOT rounded to bf16 first: the split kernels must
reproduce fp32 numerics (the reference's ORT fp32 path, /root/reference/src/inference_engine.cpp:
163-183), so the bars are ~1e-5 relative, three orders below the bf16 kernels'."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]

TOL = 2e-5  # one split layer: hi/lo representation 2^-18, dropped lo*lo term 2^-18, split output store


def _t():
    import torch

    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    return torch


def rel_err(a, b):
    t = _t()
    a = a.double()
    b = b.double()
    return (t.linalg.vector_norm(a - b) / t.linalg.vector_norm(b).clamp_min(1e-30)).item()


SPLIT_CONV_SHAPES = [
    # B, H, Cin, Cout, k, stride, pad
    (2, 56, 64, 64, 1, 1, 0),      # dense 1x1 (LDS-DMA mode 0)
    (2, 56, 64, 64, 3, 1, 1),      # implicit 3x3 (LDS-DMA mode 2)
    (2, 56, 256, 128, 1, 2, 0),    # strided 1x1
    (2, 28, 128, 128, 3, 2, 1),    # 3x3 stride 2
    (3, 14, 256, 1024, 1, 1, 0),
    (4, 7, 512, 2048, 1, 1, 0),
    (2, 64, 4, 64, 7, 2, 3),       # stem: 4 stored channels (register-staged, 4-wide loads)
    (2, 32, 16, 32, 3, 1, 1),      # Cin 16: register-staged, 8-wide loads
    (1, 9, 24, 40, 3, 1, 1),       # ragged K and N
    (5, 1, 2048, 1000, 1, 1, 0),   # FC head
    (2, 8, 16, 12, 1, 1, 0),       # N % 8 != 0: register epilogue
]


@pytest.mark.parametrize("shape", SPLIT_CONV_SHAPES)
def test_split_conv_matches_fp32(native, shape):
    torch = _t()
    from die_amd.ops import kernels as K

    B, H, Cin, Cout, k, s, p = shape
    g = torch.Generator(device="cuda").manual_seed(hash(shape) % 2**31)
    x = torch.randn(B, Cin, H, H, device="cuda", generator=g)
    w = torch.randn(Cout, Cin, k, k, device="cuda", generator=g) / (Cin * k * k) ** 0.5
    bias = torch.randn(Cout, device="cuda", generator=g)
    ref = torch.nn.functional.conv2d(x.double(), w.double(), bias.double(), stride=s, padding=p)
    xn = x.permute(0, 2, 3, 1).contiguous()
    out32, _ = K.conv2d_nhwc(xn, w, bias=bias, stride=s, pad=p, out_f32=True, split=True)
    out, _ = K.conv2d_nhwc(xn, w, bias=bias, stride=s, pad=p, split=True)
    torch.cuda.synchronize()
    assert rel_err(out32.permute(0, 3, 1, 2), ref) < TOL, rel_err(out32.permute(0, 3, 1, 2), ref)
    assert rel_err(out.permute(0, 3, 1, 2), ref) < TOL, rel_err(out.permute(0, 3, 1, 2), ref)
    # and it is really better than bf16: the bf16 kernel on the same fp32 data is ~100x worse
    ob, _ = K.conv2d_nhwc(xn.to(torch.bfloat16), w, bias=bias, stride=s, pad=p, out_f32=True)
    assert rel_err(ob.permute(0, 3, 1, 2), ref) > 20 * rel_err(out32.permute(0, 3, 1, 2), ref)


@pytest.mark.parametrize("shape", [(3, 28, 128, 256, 1, 1, 0), (2, 14, 256, 256, 3, 1, 1), (2, 14, 512, 1024, 1, 2, 0),
                                   (3, 11, 128, 64, 3, 1, 1)])
@pytest.mark.parametrize("splits,fused", [(1, True), (3, True), (3, False)])
def test_split_conv_every_variant_and_epilogue(native, shape, splits, fused):
    """Every launch config that fits (split stages are twice as large), split-K fused/unfused, with
    the full epilogue: bias + split residual + ReLU + dual store."""
    torch = _t()
    from die_amd.ops import kernels as K

    B, H, Cin, Cout, k, s, p = shape
    g = torch.Generator(device="cuda").manual_seed(17 + splits)
    x = torch.randn(B, Cin, H, H, device="cuda", generator=g)
    w = torch.randn(Cout, Cin, k, k, device="cuda", generator=g) / (Cin * k * k) ** 0.5
    bias = torch.randn(Cout, device="cuda", generator=g)
    Ho = (H + 2 * p - k) // s + 1
    res = torch.randn(B, Ho, Ho, Cout, device="cuda", generator=g)
    s2 = torch.rand(Cout, device="cuda", generator=g) + 0.5
    b2 = torch.randn(Cout, device="cuda", generator=g)
    v = torch.relu(torch.nn.functional.conv2d(x.double(), w.double(), bias.double(), stride=s, padding=p)
                   .permute(0, 2, 3, 1) + res.double())
    u = torch.relu(v * s2.double() + b2.double())
    pr = K.ConvProblem(x.permute(0, 2, 3, 1).contiguous(), w, bias=bias, stride=s, pad=p, relu=True, res=res,
                       scale2=s2, shift2=b2, relu2=True, max_splits=splits, split=True)
    ran = []
    for cfg in range(K.NUM_CFGS):
        rc = pr.launch(cfg, splits, fused)
        if rc == 1:
            continue
        assert rc == 0
        torch.cuda.synchronize()
        out, out2 = pr.results()
        assert rel_err(out, v) < TOL, (cfg, rel_err(out, v))
        assert rel_err(out2, u) < TOL, (cfg, rel_err(out2, u))
        ran.append(cfg)
    assert any(c < 4 for c in ran) and any(c >= 4 for c in ran), ran
    if k == 3 and s == 1:
        assert 27 in ran, ran  # spatially tiled 3x3 kernel (variant 6)
        assert 39 in ran, ran  # four-tile 3x3 kernel (variant 9)


def test_split_conv_repeatable_bitwise(native):
    torch = _t()
    from die_amd.ops import kernels as K

    x = torch.randn(4, 28, 28, 128, device="cuda")
    w = torch.randn(128, 128, 3, 3, device="cuda") * 0.05
    pr = K.ConvProblem(x, w, pad=1, max_splits=4, split=True)
    for cfg in range(K.NUM_CFGS):
        for splits in (1, 4):
            if pr.launch(cfg, splits) == 1:
                continue
            ref = pr.out.clone()
            for _ in range(4):
                assert pr.launch(cfg, splits) == 0
                assert torch.equal(ref.view(torch.int16), pr.out.view(torch.int16)), (cfg, splits)


def test_split_conv_tile_order_bitwise(native):
    """ConvArgs::order only remaps blocks to tiles (XCD placement): N-fastest, M-fastest and the
    heuristic give bit-identical outputs for every config, with and without split-K."""
    torch = _t()
    from die_amd.ops import kernels as K

    x = torch.randn(2, 28, 28, 128, device="cuda")
    w = torch.randn(256, 128, 3, 3, device="cuda") * 0.05
    pr = K.ConvProblem(x, w, pad=1, max_splits=4, split=True)
    for cfg in range(K.NUM_CFGS):
        for splits in (1, 4):
            if pr.launch(cfg, splits, True, 0) == 1:
                continue
            ref = pr.out.clone()
            for order in (1, 2, 3, 4):
                assert pr.launch(cfg, splits, True, order) == 0
                assert torch.equal(ref.view(torch.int16), pr.out.view(torch.int16)), (cfg, splits, order)


def test_split_memory_bound_kernels(native):
    torch = _t()
    from die_amd.ops import kernels as K

    g = torch.Generator(device="cuda").manual_seed(5)
    # input prep (BN folded) -> split planes
    x = torch.rand(2, 3, 40, 40, device="cuda", generator=g)
    sc = torch.rand(3, device="cuda", generator=g) + 0.5
    sh = torch.randn(3, device="cuda", generator=g)
    xp = K.input_prep(x, sc, sh, cp=4, split=True)
    ref_in = (x.double() * sc.double().view(1, 3, 1, 1) + sh.double().view(1, 3, 1, 1))
    assert rel_err(xp[..., :3].permute(0, 3, 1, 2), ref_in) < 1e-5
    assert xp[..., 3].abs().max().item() == 0
    # pools
    a = torch.randn(2, 30, 30, 64, device="cuda", generator=g)
    y = K.pool2d_nhwc(a, 3, 2, 1, is_max=True, split=True)
    ref = torch.nn.functional.max_pool2d(a.permute(0, 3, 1, 2).double(), 3, 2, 1).permute(0, 2, 3, 1)
    assert rel_err(y, ref) < 1e-5
    y = K.pool2d_nhwc(a, 2, 2, 0, is_max=False, split=True)
    ref = torch.nn.functional.avg_pool2d(a.permute(0, 3, 1, 2).double(), 2, 2, 0).permute(0, 2, 3, 1)
    assert rel_err(y, ref) < 1e-5
    # GAP with BN + ReLU
    h = torch.randn(6, 7, 7, 2048, device="cuda", generator=g)
    s = torch.rand(2048, device="cuda", generator=g) + 0.5
    b = torch.randn(2048, device="cuda", generator=g)
    out, out32 = K.global_avgpool_nhwc(h, s, b, relu=True, split=True)
    ref = torch.relu(h.double() * s.double() + b.double()).mean(dim=(1, 2))
    assert rel_err(out32, ref) < 1e-6 and rel_err(out, ref) < 1e-5
    # affine + residual + relu
    z = torch.randn_like(h)
    y = K.affine_act(h, s, b, z=z, relu=True, split=True)
    assert rel_err(y, torch.relu(h.double() * s.double() + b.double() + z.double())) < 1e-5
    # layernorm, token assembly, gather
    r = torch.randn(3, 197, 768, device="cuda", generator=g) * 3 + 1
    gam = torch.rand(768, device="cuda", generator=g) + 0.5
    bet = torch.randn(768, device="cuda", generator=g)
    y = K.layernorm(r, gam, bet, 1e-6, split=True)
    ref = torch.nn.functional.layer_norm(r.double(), (768,), gam.double(), bet.double(), 1e-6)
    assert rel_err(y, ref) < 1e-5
    patches = torch.randn(3, 196, 768, device="cuda", generator=g)
    cls = torch.randn(768, device="cuda", generator=g)
    pos = torch.randn(197, 768, device="cuda", generator=g)
    y = K.tokens_assemble(patches, cls, pos, split=True)
    ref = torch.cat([cls.double().expand(3, 1, 768), patches.double()], 1) + pos.double()
    assert rel_err(y, ref) < 1e-5
    y = K.gather_rows(r, 0, split=True)
    assert rel_err(y, r[:, 0].double()) < 1e-5
    torch.cuda.synchronize()


@pytest.mark.parametrize("B,S,H", [(2, 197, 12), (3, 50, 4), (1, 128, 2), (2, 224, 3)])
def test_split_attention_matches_fp32(native, B, S, H):
    torch = _t()
    from die_amd.ops import kernels as K

    g = torch.Generator(device="cuda").manual_seed(B * 1000 + S)
    C = H * 64
    qkv = torch.randn(B, S, 3 * C, device="cuda", generator=g)
    got = K.attention_qkv_split(qkv, H)
    q, k, v = [t.double().reshape(B, S, H, 64).transpose(1, 2) for t in qkv.split(C, dim=2)]
    ref = torch.softmax(q @ k.transpose(-1, -2) / 8.0, -1) @ v
    ref = ref.transpose(1, 2).reshape(B, S, C)
    torch.cuda.synchronize()
    assert rel_err(got, ref) < TOL, rel_err(got, ref)


def test_split_linear_gelu_residual(native):
    torch = _t()
    from die_amd.ops import kernels as K

    g = torch.Generator(device="cuda").manual_seed(9)
    x = torch.randn(2, 197, 768, device="cuda", generator=g)
    w = torch.randn(3072, 768, device="cuda", generator=g) / 768 ** 0.5
    b = torch.randn(3072, device="cuda", generator=g)
    got = K.linear(x, w, bias=b, act=2, split=True)
    ref = torch.nn.functional.gelu(x.double() @ w.double().T + b.double())
    assert rel_err(got, ref) < TOL
    w2 = torch.randn(768, 3072, device="cuda", generator=g) / 3072 ** 0.5
    res = torch.randn(2, 197, 768, device="cuda", generator=g)
    got2 = K.linear(ref.float(), w2, res=res, split=True)
    ref2 = ref @ w2.double().T + res.double()
    torch.cuda.synchronize()
    assert rel_err(got2, ref2) < TOL


def _margin_ok(got, ref, frac):
    """Top-1 must agree on every sample whose reference top-1/top-2 margin exceeds `frac` of the
    logit spread (a smaller margin is inside the numerical tolerance being tested)."""
    srt = np.sort(ref, axis=1)
    margin = srt[:, -1] - srt[:, -2]
    spread = ref.std(axis=1)
    clear = margin > frac * spread
    return bool((got.argmax(1) == ref.argmax(1))[clear].all()), int(clear.sum())


@pytest.mark.parametrize("arch", ["resnet50", "vit_b16"])
def test_engine_fp32_matches_torch(native, models, arch):
    """Whole-model fp32 engine (the default precision) vs torch fp32: rel-L2 <= 1e-4 and identical
    top-1 at B in {1, 7, 17, 32}; the bf16 engine on the same inputs stays within rel-L2 1e-2."""
    torch = _t()
    if arch == "resnet50":
        from die_amd.models import resnet_v2 as r

        path, w, cfg = models["get_rn50"]()
    else:
        from die_amd.models import vit as r

        path, w, cfg = models["get_vit"]("base")
    e32 = native.Engine(path, device="hip", max_batch=32, precision="fp32")
    e16 = native.Engine(path, device="hip", max_batch=32, precision="bf16")
    assert e32.refresh_info()["precision"] == "fp32" and e16.refresh_info()["precision"] == "bf16"
    try:
        for B in (1, 7, 17, 32):
            x = r.synthetic_input(B, cfg, seed=50 + B)
            with torch.no_grad():
                ref = r.torch_forward(w, x, cfg, device="cuda").double().cpu().numpy()
            got = e32.run(x.reshape(B, -1)).astype(np.float64)
            err = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
            assert err <= 1e-4, (B, err)
            assert (got.argmax(1) == ref.argmax(1)).all(), B
            g16 = e16.run(x.reshape(B, -1)).astype(np.float64)
            err16 = float(np.linalg.norm(g16 - ref) / np.linalg.norm(ref))
            assert err16 <= 1e-2, (B, err16)
            ok, n_clear = _margin_ok(g16, ref, 0.05)
            assert ok, (B, n_clear)
            print("%s B=%d rel-L2 fp32 %.2e bf16 %.2e" % (arch, B, err, err16))
    finally:
        e32.close()
        e16.close()


@pytest.mark.parametrize("B,H,W,relu", [(2, 224, 224, True), (1, 37, 45, False)])
def test_split_stem_kernel(native, B, H, W, relu):
    torch = _t()
    from die_amd.ops import kernels as K

    g = torch.Generator(device="cuda").manual_seed(B * 7 + H)
    x = torch.zeros(B, H, W, 4, device="cuda")
    x[..., :3] = torch.rand(B, H, W, 3, device="cuda", generator=g) * 2 - 1
    w = torch.randn(64, 3, 7, 7, device="cuda", generator=g) / 12.0
    bias = torch.randn(64, device="cuda", generator=g) * 0.1
    got = K.conv_stem7x7(x, w, bias, relu=relu, split=True)
    ref = torch.nn.functional.conv2d(x[..., :3].permute(0, 3, 1, 2).double(), w.double(), bias.double(), stride=2,
                                     padding=3)
    if relu:
        ref = torch.relu(ref)
    torch.cuda.synchronize()
    assert rel_err(got.permute(0, 3, 1, 2), ref) < TOL, rel_err(got.permute(0, 3, 1, 2), ref)


@pytest.mark.parametrize("B,H,W,relu,max_blocks", [(3, 224, 224, True, 0), (2, 37, 45, False, 5), (1, 64, 80, True, 1)])
@pytest.mark.parametrize("split", [True, False])
def test_fused_nchw_stem_kernel(native, B, H, W, relu, max_blocks, split):
    """Persistent stem reading the fp32 NCHW graph input with the input BN applied on load (replaces
    input_prep + stem) vs torch fp32; max_blocks forces every block to walk several tiles."""
    torch = _t()
    from die_amd.ops import kernels as K

    g = torch.Generator(device="cuda").manual_seed(B * 11 + H + int(split))
    x = torch.rand(B, 3, H, W, device="cuda", generator=g) * 255.0
    scale = torch.tensor([0.017, 0.018, 0.0175], device="cuda")
    shift = torch.tensor([-2.1, -2.0, -1.8], device="cuda")
    w = torch.randn(64, 3, 7, 7, device="cuda", generator=g) / 12.0
    bias = torch.randn(64, device="cuda", generator=g) * 0.1
    got = K.conv_stem7x7_nchw(x, w, bias, scale=scale, shift=shift, relu=relu, split=split, max_blocks=max_blocks)
    xn = x.double() * scale.double().view(1, 3, 1, 1) + shift.double().view(1, 3, 1, 1)
    ref = torch.nn.functional.conv2d(xn, w.double(), bias.double(), stride=2, padding=3)
    if relu:
        ref = torch.relu(ref)
    torch.cuda.synchronize()
    err = rel_err(got.permute(0, 3, 1, 2), ref)
    assert err < (TOL if split else 8e-3), err


@pytest.mark.parametrize("split", [True, False])
def test_patchify_conv_lds_dma_mode(native, split):
    """Patchify convs (stride == kernel, no padding: the ViT patch embedding) run the LDS-DMA loops
    with each 64-wide K-step read as a contiguous piece of one input row (MODE 3), 1- and 2-stage."""
    torch = _t()
    from die_amd.ops import kernels as K

    B, H, Cin, Cout, k = 3, 48, 4, 128, 16  # 3 x 3 patches per image, M = 27 (an M tail on every tile)
    g = torch.Generator(device="cuda").manual_seed(29)
    x = torch.randn(B, Cin, H, H, device="cuda", generator=g)
    w = torch.randn(Cout, Cin, k, k, device="cuda", generator=g) / (Cin * k * k) ** 0.5
    bias = torch.randn(Cout, device="cuda", generator=g)
    ref = torch.nn.functional.conv2d(x.double(), w.double(), bias.double(), stride=k).permute(0, 2, 3, 1)
    xn = x.permute(0, 2, 3, 1).contiguous()
    if not split:
        xn, w, ref = xn.to(torch.bfloat16), w.to(torch.bfloat16), torch.nn.functional.conv2d(
            x.to(torch.bfloat16).double(), w.to(torch.bfloat16).double(), bias.double(), stride=k).permute(0, 2, 3, 1)
    ran = []
    for cfg in range(K.NUM_CFGS):
        out, _ = K.conv2d_nhwc(xn, w.float(), bias=bias, stride=k, pad=0, tile=cfg, split=split, out_f32=False)
        if out is None:
            continue
        torch.cuda.synchronize()
        err = rel_err(out.double(), ref)
        assert err < (TOL if split else 5e-3), (cfg, err)
        ran.append(cfg)
    assert any(4 <= c < 8 for c in ran), ran    # 2-stage LDS-DMA ring
    assert any(20 <= c < 24 for c in ran), ran  # 1-stage LDS-DMA loop


@pytest.mark.parametrize("split", [True, False])
@pytest.mark.parametrize("M,K,N", [(1, 2048, 1000), (7, 2048, 1000), (20, 2048, 1000), (32, 512, 64), (24, 256, 1008)])
def test_skinny_gemm(native, M, K, N, split):
    """Variant 8 (cfg 32, conv_skinny.hip): <= 32 dense rows, 16 channels per block, K split over 8
    waves and summed in wave order.  fp32 (split) against float64 at the layer bar, bf16 against
    torch; with the residual / dual-store epilogue, a live batch, bitwise repeatable; shapes it
    does not take (33 rows, K not a multiple of 256, split-K) are refused."""
    torch = _t()
    from die_amd.ops import kernels as K_

    g = torch.Generator(device="cuda").manual_seed(M * 13 + K + N)
    x = torch.randn(M, 1, 1, K, device="cuda", generator=g)
    w = torch.randn(N, K, 1, 1, device="cuda", generator=g) / K ** 0.5
    bias = torch.randn(N, device="cuda", generator=g)
    res = torch.randn(M, 1, 1, N, device="cuda", generator=g)
    s2 = torch.rand(N, device="cuda", generator=g) + 0.5
    b2 = torch.randn(N, device="cuda", generator=g)
    if not split:
        x, res = x.to(torch.bfloat16), res.to(torch.bfloat16)
    v = torch.relu(x.double().reshape(M, K) @ w.double().reshape(N, K).T + bias.double() + res.double().reshape(M, N))
    u = torch.relu(v * s2.double() + b2.double())
    pr = K_.ConvProblem(x, w, bias=bias, relu=True, res=res, scale2=s2, shift2=b2, relu2=True, max_splits=2, split=split)
    assert pr.launch(32, 1, False) == 0
    torch.cuda.synchronize()
    out, out2 = pr.results()
    tol = TOL if split else 2e-2
    assert rel_err(out.reshape(M, N), v) < tol, rel_err(out.reshape(M, N), v)
    assert rel_err(out2.reshape(M, N), u) < tol
    first = out.clone()
    for _ in range(3):
        assert pr.launch(32, 1, False) == 0
        torch.cuda.synchronize()
        assert torch.equal(pr.results()[0], first)
    # live batch: rows past it keep what was there
    if M > 1:
        lv = torch.tensor([M // 2], dtype=torch.int64, device="cuda")
        pr.out.zero_()
        assert pr.launch(32, 1, False, extra={"live": lv.data_ptr()}) == 0
        torch.cuda.synchronize()
        got = pr.results()[0].reshape(M, N)
        assert torch.equal(got[: M // 2], first.reshape(M, N)[: M // 2])
        assert not got[M // 2:].any()
    assert pr.launch(32, 2, False) != 0  # no split-K
    for cfg in (33, 34, 35):
        assert pr.launch(cfg, 1, False) != 0  # tile 0 only


def test_skinny_gemm_refuses_other_shapes(native):
    torch = _t()
    from die_amd.ops import kernels as K_

    for M, K in ((33, 2048), (8, 2000)):
        x = torch.randn(M, 1, 1, K, device="cuda")
        w = torch.randn(64, K, 1, 1, device="cuda")
        pr = K_.ConvProblem(x, w, split=True)
        assert pr.launch(32, 1, False) != 0, (M, K)
    x = torch.randn(2, 4, 4, 256, device="cuda")  # not a dense row problem (3x3)
    pr = K_.ConvProblem(x, torch.randn(64, 256, 3, 3, device="cuda"), pad=1, split=True)
    assert pr.launch(32, 1, False) != 0
