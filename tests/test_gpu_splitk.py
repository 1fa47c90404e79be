"""Fused split-K reduction (conv_igemm_impl.h tile_epilogue): the last split block of a tile sums
the partials it reads back through write-through (sc1) loads, with no agent fences.  A hand-off
bug shows up as a stale partial in a few words of a few tiles, only sometimes, so every launch of
every case is compared bit for bit with the two-kernel reduction (same summation order) -- on the
ResNet50 stage-3/4 shapes the engine splits, repeatedly, with other work queued beside it."""
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]

CASES = [
    # B, H, Cin, Cout, k, stride, pad, tile cfg, splits  (cfg = tile + 4 * variant)
    (20, 14, 256, 256, 3, 1, 1, 2 + 4 * 5, 4),     # stage-3 3x3 at the serving batch: 64x128, 1 stage
    (20, 14, 256, 256, 3, 1, 1, 3 + 4 * 1, 2),     # 64x64, 2-stage ring
    (20, 7, 512, 512, 3, 1, 1, 2 + 4 * 5, 8),      # stage-4 3x3
    (20, 7, 2048, 512, 1, 1, 0, 3 + 4 * 3, 2),     # stage-4 reduce, 4-stage ring
    (32, 1, 2048, 1000, 1, 1, 0, 3 + 4 * 2, 8),    # FC head (ragged N tiles)
    (7, 14, 256, 256, 3, 1, 1, 3 + 4 * 6, 4),      # spatial 3x3 kernel, split over channel slices
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("split", [True, False])
def test_fused_splitk_bitwise_vs_two_kernels(native, case, split):
    import torch
    from die_amd.ops import kernels as K

    B, H, Cin, Cout, k, s, p, cfg, splits = case
    g = torch.Generator(device="cuda").manual_seed(Cin * 31 + Cout + k)
    x = torch.randn(B, H, H, Cin, device="cuda", generator=g)
    w = torch.randn(Cout, Cin, k, k, device="cuda", generator=g) / (Cin * k * k) ** 0.5
    bias = torch.randn(Cout, device="cuda", generator=g)
    if not split:
        x = x.to(torch.bfloat16)
    pr = K.ConvProblem(x, w, bias=bias, stride=s, pad=p, relu=True, max_splits=splits, split=split)
    assert pr.launch(cfg, splits, False) == 0
    torch.cuda.synchronize()
    ref = pr.results()[0].clone()
    # other work on a second stream while the fused launches run (uneven load on the CUs)
    side = torch.cuda.Stream()
    big = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
    for it in range(12):
        with torch.cuda.stream(side):
            big.add_(1)
        assert pr.launch(cfg, splits, True) == 0
        torch.cuda.synchronize()
        got = pr.results()[0]
        assert torch.equal(got, ref), (it, (got.float() - ref.float()).abs().max().item())
    assert int(pr.counters.abs().sum().item()) == 0  # every tile counter back at zero
