"""Numerics of the hand-written gfx950 kernels vs a plain PyTorch fp32 reference of the same op.

Inputs/weights are rounded to bf16 first, so the reference differs from the kernel only by the
accumulation order (f32) and the bf16 rounding of the output."""
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def _t():
    import torch

    return torch


def rel_err(a, b):
    t = _t()
    a = a.float()
    b = b.float()
    return (t.linalg.vector_norm(a - b) / t.linalg.vector_norm(b).clamp_min(1e-12)).item()


CONV_SHAPES = [
    # B, H, Cin, Cout, k, stride, pad
    (2, 56, 64, 64, 1, 1, 0),
    (2, 56, 64, 64, 3, 1, 1),
    (2, 56, 64, 256, 1, 1, 0),
    (2, 56, 256, 128, 1, 2, 0),
    (2, 56, 128, 128, 3, 2, 1),
    (3, 28, 512, 256, 1, 1, 0),
    (3, 14, 256, 256, 3, 1, 1),
    (4, 7, 512, 2048, 1, 1, 0),
    (4, 7, 512, 512, 3, 1, 1),
    (1, 9, 24, 40, 3, 1, 1),      # ragged: K not a multiple of 64, N not of 64
    (5, 1, 2048, 1000, 1, 1, 0),  # FC head as a 1x1 "conv"
    (2, 8, 16, 12, 1, 1, 0),      # N % 8 != 0: register epilogue path
]


@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_matches_torch(native, shape):
    torch = _t()
    from die_amd.ops import kernels as K

    B, H, Cin, Cout, k, s, p = shape
    g = torch.Generator(device="cuda").manual_seed(hash(shape) % 2**31)
    x = torch.randn(B, Cin, H, H, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(Cout, Cin, k, k, device="cuda", generator=g) / (Cin * k * k) ** 0.5).to(torch.bfloat16)
    bias = torch.randn(Cout, device="cuda", generator=g)
    ref = torch.nn.functional.conv2d(x.float(), w.float(), bias, stride=s, padding=p)
    out, _ = K.conv2d_nhwc(x.permute(0, 2, 3, 1).contiguous(), w.float(), bias=bias, stride=s, pad=p, out_f32=True)
    torch.cuda.synchronize()
    got = out.permute(0, 3, 1, 2)
    assert rel_err(got, ref) < 2e-3, rel_err(got, ref)


@pytest.mark.parametrize("tile,splits,fused", [(0, 1, True), (1, 1, True), (2, 1, True), (3, 1, True), (0, 3, True),
                                               (3, 4, True), (1, 9, True), (7, 4, True), (11, 3, True),
                                               (0, 3, False), (7, 4, False)])
def test_conv_all_tiles_and_epilogue(native, tile, splits, fused):
    torch = _t()
    from die_amd.ops import kernels as K

    B, H, Cin, Cout = 2, 20, 64, 192
    g = torch.Generator(device="cuda").manual_seed(7 + tile)
    x = torch.randn(B, Cin, H, H, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(Cout, Cin, 3, 3, device="cuda", generator=g) / (Cin * 9) ** 0.5).to(torch.bfloat16)
    bias = torch.randn(Cout, device="cuda", generator=g)
    res = torch.randn(B, H, H, Cout, device="cuda", generator=g).to(torch.bfloat16)
    s2 = torch.rand(Cout, device="cuda", generator=g) + 0.5
    b2 = torch.randn(Cout, device="cuda", generator=g)
    out, out2 = K.conv2d_nhwc(x.permute(0, 2, 3, 1).contiguous(), w.float(), bias=bias, stride=1, pad=1, relu=True,
                              res=res, scale2=s2, shift2=b2, relu2=True, tile=tile, splits=splits,
                              fused_splitk=fused)
    torch.cuda.synchronize()
    assert out is not None, "config not applicable"
    v = torch.nn.functional.conv2d(x.float(), w.float(), bias, padding=1).permute(0, 2, 3, 1) + res.float()
    v = torch.relu(v)
    u = torch.relu(v * s2 + b2)
    assert rel_err(out, v) < 5e-3
    assert rel_err(out2, u) < 5e-3
    if splits > 1:  # fused reduction is deterministic and leaves the counters reset (bitwise repeat)
        again, _ = K.conv2d_nhwc(x.permute(0, 2, 3, 1).contiguous(), w.float(), bias=bias, stride=1, pad=1, relu=True,
                                 res=res, scale2=s2, shift2=b2, relu2=True, tile=tile, splits=splits,
                                 fused_splitk=fused)
        assert torch.equal(again, out)


@pytest.mark.parametrize("shape", [
    (3, 28, 128, 256, 1, 1, 0),   # dense 1x1, M tail (3*784 = 2352 not a multiple of 128)
    (2, 14, 256, 256, 3, 1, 1),   # implicit 3x3, padding
    (2, 28, 128, 128, 3, 2, 1),   # implicit 3x3 stride 2
    (2, 14, 512, 1024, 1, 2, 0),  # strided 1x1 (implicit path)
    (3, 13, 64, 128, 3, 1, 1),    # 3x3/s1 on a 13x13 image: spatial 8x8 tiles with ragged edges
])
@pytest.mark.parametrize("splits", [1, 2])
def test_conv_every_variant(native, shape, splits):
    """Every launch config (4 tiles x {register-staged, LDS-DMA ring of 2, 3, 4, 6 stages, 1 stage}, and the
    spatially tiled 3x3 kernel)."""
    torch = _t()
    from die_amd.ops import kernels as K

    B, H, Cin, Cout, k, s, p = shape
    g = torch.Generator(device="cuda").manual_seed(11 + splits)
    x = torch.randn(B, Cin, H, H, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(Cout, Cin, k, k, device="cuda", generator=g) / (Cin * k * k) ** 0.5).to(torch.bfloat16)
    bias = torch.randn(Cout, device="cuda", generator=g)
    res = torch.randn(B, (H + 2 * p - k) // s + 1, (H + 2 * p - k) // s + 1, Cout, device="cuda",
                      generator=g).to(torch.bfloat16)
    ref = torch.relu(torch.nn.functional.conv2d(x.float(), w.float(), bias, stride=s, padding=p).permute(0, 2, 3, 1)
                     + res.float())
    xn = x.permute(0, 2, 3, 1).contiguous()
    ran = []
    for cfg in range(K.NUM_CFGS):
        out, _ = K.conv2d_nhwc(xn, w.float(), bias=bias, stride=s, pad=p, relu=True, res=res, tile=cfg,
                               splits=splits)
        if out is None:
            continue
        torch.cuda.synchronize()
        assert rel_err(out, ref) < 5e-3, (cfg, rel_err(out, ref))
        ran.append(cfg)
    assert any(c >= 4 for c in ran), "LDS-DMA variants must apply to these shapes"
    assert any(c >= 8 for c in ran)
    assert any(c >= 12 for c in ran), "4-stage ring"
    assert any(c >= 16 for c in ran), "6-stage ring"
    if k == 3 and s == 1:
        assert 27 in ran, "spatially tiled 3x3 kernel (variant 6)"


def test_stem_conv_with_input_prep(native):
    torch = _t()
    from die_amd.ops import kernels as K

    B = 2
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.rand(B, 3, 224, 224, device="cuda", generator=g)
    sc = torch.rand(3, device="cuda", generator=g) + 0.5
    sh = torch.randn(3, device="cuda", generator=g)
    xp = K.input_prep(x, sc, sh, cp=4)
    ref_in = (x * sc.view(1, 3, 1, 1) + sh.view(1, 3, 1, 1))
    torch.cuda.synchronize()
    assert rel_err(xp[..., :3].permute(0, 3, 1, 2), ref_in) < 4e-3
    assert xp[..., 3].abs().max().item() == 0
    w = (torch.randn(64, 3, 7, 7, device="cuda", generator=g) / 12.0).to(torch.bfloat16)
    out, _ = K.conv2d_nhwc(xp, w.float(), stride=2, pad=3, out_f32=True)
    ref = torch.nn.functional.conv2d(xp[..., :3].permute(0, 3, 1, 2).float(), w.float(), stride=2, padding=3)
    torch.cuda.synchronize()
    assert rel_err(out.permute(0, 3, 1, 2), ref) < 2e-3


@pytest.mark.parametrize("B,H,W,relu", [(2, 224, 224, True), (3, 64, 64, False), (1, 37, 45, True)])
def test_stem_lds_kernel(native, B, H, W, relu):
    """7x7/2 LDS-patch stem kernel vs torch fp32 (odd sizes exercise the tile tails)."""
    torch = _t()
    from die_amd.ops import kernels as K

    g = torch.Generator(device="cuda").manual_seed(B * 100 + H)
    x = torch.rand(B, 3, H, W, device="cuda", generator=g) * 2 - 1
    xp = K.input_prep(x, torch.ones(3, device="cuda"), torch.zeros(3, device="cuda"), cp=4)
    w = (torch.randn(64, 3, 7, 7, device="cuda", generator=g) / 12.0).to(torch.bfloat16).float()
    bias = torch.randn(64, device="cuda", generator=g) * 0.1
    out = K.conv_stem7x7(xp, w, bias, relu=relu)
    ref = torch.nn.functional.conv2d(xp[..., :3].permute(0, 3, 1, 2).float(), w, bias, stride=2, padding=3)
    if relu:
        ref = torch.relu(ref)
    torch.cuda.synchronize()
    assert out.shape == (B, ref.shape[2], ref.shape[3], 64)
    assert rel_err(out.permute(0, 3, 1, 2).float(), ref) < 5e-3
    # bit-identical on repeat (race screen)
    again = K.conv_stem7x7(xp, w, bias, relu=relu)
    assert torch.equal(out, again)


def test_conv_repeatable_bitwise(native):
    """Race screen: repeated launches at several shapes must agree bit for bit."""
    torch = _t()
    from die_amd.ops import kernels as K

    for (B, H, Cin, Cout, k) in [(4, 28, 128, 128, 3), (8, 14, 256, 1024, 1)]:
        x = torch.randn(B, H, H, Cin, device="cuda").to(torch.bfloat16)
        w = torch.randn(Cout, Cin, k, k, device="cuda") * 0.05
        first, _ = K.conv2d_nhwc(x, w, pad=k // 2)
        for _ in range(10):
            again, _ = K.conv2d_nhwc(x, w, pad=k // 2)
            assert torch.equal(first.view(torch.int16), again.view(torch.int16))
        # every LDS-DMA ring depth (counted vmcnt per stage) and split-K, repeated
        pr = K.ConvProblem(x, w, pad=k // 2, max_splits=4)
        for cfg in range(4, K.NUM_CFGS):
            for splits in (1, 4):
                if pr.launch(cfg, splits) == 1:
                    continue
                ref = pr.out.clone()
                for _ in range(5):
                    assert pr.launch(cfg, splits) == 0
                    assert torch.equal(ref.view(torch.int16), pr.out.view(torch.int16)), (cfg, splits)
                if splits == 1 and cfg // 4 not in (6, 9):  # same K order (tap-major) per output element: bit-identical
                    assert torch.equal(ref.view(torch.int16), first.view(torch.int16)), cfg
                elif splits == 1:  # spatial / four-tile 3x3 kernels sum channel-slice-major: same value up to rounding
                    assert rel_err(ref.float(), first.float()) < 1e-2, cfg


@pytest.mark.parametrize("cfg", [(2, 112, 64, 3, 2, 1, True), (2, 14, 128, 2, 2, 0, False), (3, 9, 16, 3, 1, 1, False)])
def test_pool(native, cfg):
    torch = _t()
    from die_amd.ops import kernels as K

    B, H, C, k, s, p, is_max = cfg
    x = torch.randn(B, C, H, H, device="cuda").to(torch.bfloat16)
    y = K.pool2d_nhwc(x.permute(0, 2, 3, 1).contiguous(), k, s, p, is_max=is_max)
    if is_max:
        ref = torch.nn.functional.max_pool2d(x.float(), k, s, p)
    else:
        ref = torch.nn.functional.avg_pool2d(x.float(), k, s, p, count_include_pad=False)
    torch.cuda.synchronize()
    assert rel_err(y.permute(0, 3, 1, 2), ref) < 4e-3


def test_gap_and_affine(native):
    torch = _t()
    from die_amd.ops import kernels as K

    x = torch.randn(6, 7, 7, 2048, device="cuda").to(torch.bfloat16)
    sc = torch.rand(2048, device="cuda") + 0.5
    sh = torch.randn(2048, device="cuda")
    out, out32 = K.global_avgpool_nhwc(x, sc, sh, relu=True)
    ref = torch.relu(x.float() * sc + sh).mean(dim=(1, 2))
    torch.cuda.synchronize()
    assert rel_err(out32, ref) < 1e-5
    assert rel_err(out, ref) < 4e-3
    z = torch.randn_like(x)
    y = K.affine_act(x, sc, sh, z=z, relu=True)
    torch.cuda.synchronize()
    assert rel_err(y, torch.relu(x.float() * sc + sh + z.float())) < 4e-3
