"""128-pixel x 256-channel GEMM tile (kernels.h configs 28-30, conv_igemm_impl.h launch_wide_cfg):
each wave owns 64 x 128 outputs, so a K-step's LDS fragment reads feed twice the MFMAs of the
128x128 tile.  Checked against torch (float64) in fp32 (split) and bf16 mode on ViT-shaped GEMMs
and a 3x3 conv, bit-identical to the 128x128 LDS-DMA config (same K order), split-K fused ==
separate, and rejected where N % 256 != 0."""
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


CASES = [
    # B, H, Cin, Cout, k, pad: ViT MLP1 / MLP2 / QKV rows as 1x1 convs over [B, 197, 1] "images", a 3x3
    (4, 197, 768, 3072, 1, 0),
    (4, 197, 3072, 768, 1, 0),
    (3, 197, 768, 2304, 1, 0),
    (2, 14, 256, 256, 3, 1),
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("split", [True, False])
def test_wide_tile_matches_torch_and_128x128(native, case, split):
    import torch
    from die_amd.ops import kernels as K

    B, H, Cin, Cout, k, pad = case
    W = 1 if k == 1 else H
    g = torch.Generator(device="cuda").manual_seed(Cin + Cout)
    x = torch.randn(B, H, W, Cin, device="cuda", generator=g)
    w = torch.randn(Cout, Cin, k, k, device="cuda", generator=g) / (Cin * k * k) ** 0.5
    bias = torch.randn(Cout, device="cuda", generator=g)
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).double(), w.double(), bias.double(), padding=pad)
    ref = torch.relu(ref).permute(0, 2, 3, 1)
    if not split:
        x = x.to(torch.bfloat16)
    pr = K.ConvProblem(x, w, bias=bias, pad=pad, relu=True, max_splits=4, split=split)
    assert pr.launch(4, 1) == 0  # 128x128, 2-stage LDS-DMA ring: the same K order
    torch.cuda.synchronize()
    base = pr.results()[0].clone()
    ran = []
    for cfg in K.WIDE_CFGS:
        rc = pr.launch(cfg, 1)
        if rc == 1:
            continue
        assert rc == 0
        torch.cuda.synchronize()
        out = pr.results()[0]
        assert _rel(out.float(), ref) < (1e-5 if split else 1e-2), (cfg, _rel(out.float(), ref))
        assert torch.equal(out, base), cfg
        # split-K: the in-kernel reduction equals the two-kernel one bit for bit
        assert pr.launch(cfg, 4, False) == 0
        torch.cuda.synchronize()
        sep = pr.results()[0].clone()
        assert pr.launch(cfg, 4, True) == 0
        torch.cuda.synchronize()
        assert torch.equal(pr.results()[0], sep), cfg
        assert _rel(sep.float(), ref) < (1e-5 if split else 1e-2)
        ran.append(cfg)
    assert ran, "no wide-tile config ran"


def test_wide_tile_rejects_narrow_n(native):
    import torch
    from die_amd.ops import kernels as K

    x = torch.randn(2, 7, 7, 256, device="cuda")
    w = torch.randn(320, 256, 1, 1, device="cuda") * 0.05  # 320 % 256 != 0
    pr = K.ConvProblem(x, w, split=True)
    for cfg in K.WIDE_CFGS:
        assert pr.launch(cfg, 1) == 1
