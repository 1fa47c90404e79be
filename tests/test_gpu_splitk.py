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


TAIL_CASES = [
    # B, H, Cin, Cout, k, stride, pad, tile cfg, splits, live B (0 = all)
    (22, 14, 256, 256, 3, 1, 1, 3 + 4 * 5, 4, 0),      # stage-3 3x3, 64x64 1-stage: 272 tiles, 16 in the tail
    (22, 14, 256, 256, 3, 1, 1, 3 + 4 * 5, 4, 21),     # the same launch at live batch 21: 260 tiles, 4 in the tail
    (24, 14, 256, 256, 3, 1, 1, 2 + 4 * 1, 2, 0),      # 64x128 2-stage ring: 148 tiles, all whole
    (22, 28, 128, 128, 3, 1, 1, 3 + 4 * 2, 2, 0),      # stage-2 3x3, 3-stage ring: 540 tiles, 28 in the tail
    (22, 28, 128, 128, 3, 1, 1, 3 + 4 * 2, 2, 20),     # ... live 20: 490 tiles, 234 in the tail
    (22, 14, 256, 1024, 1, 1, 0, 3 + 4 * 3, 2, 0),     # stage-3 1x1 expand, 4-stage ring: 1088 tiles, 64 in the tail
]


@pytest.mark.parametrize("case", TAIL_CASES)
@pytest.mark.parametrize("split", [True, False])
def test_tail_splitk(native, case, split):
    """ConvArgs::tail (tail split-K): the tiles of whole 256-tile rounds run the full K range (bit for
    bit the unsplit result) and only the last partial round's tiles are split and reduced in-kernel
    (bit for bit the uniform fused split-K result) -- every output word is one of the two, the mix
    stays fixed over repeated launches under side load, and every tile counter returns to zero.
    With a live batch the whole/split boundary moves with the live tile count."""
    import torch
    from die_amd.ops import kernels as K

    B, H, Cin, Cout, k, s, p, cfg, splits, live = case
    g = torch.Generator(device="cuda").manual_seed(Cin * 7 + Cout + k + B)
    x = torch.randn(B, H, H, Cin, device="cuda", generator=g)
    w = torch.randn(Cout, Cin, k, k, device="cuda", generator=g) / (Cin * k * k) ** 0.5
    bias = torch.randn(Cout, device="cuda", generator=g)
    if not split:
        x = x.to(torch.bfloat16)
    pr = K.ConvProblem(x, w, bias=bias, stride=s, pad=p, relu=True, max_splits=splits, split=split)
    extra = {}
    lv = None
    if live:
        lv = torch.tensor([live], dtype=torch.int64, device="cuda")
        extra["live"] = lv.data_ptr()
    rows = (live or B) * H * H  # live rows (stride 1, same padding)

    def run(sp, fused, tail):
        e = dict(extra, tail=tail) if tail else dict(extra)
        assert pr.launch(cfg, sp, fused, extra=e) == 0
        torch.cuda.synchronize()
        return pr.results()[0].reshape(-1, Cout)[:rows].clone()

    whole = run(1, False, 0)
    sliced = run(splits, True, 0)
    ref = run(splits, True, 256)
    is_whole = (ref == whole).all(1)
    is_split = (ref == sliced).all(1)
    assert bool((is_whole | is_split).all())
    side = torch.cuda.Stream()
    big = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
    for it in range(6):
        with torch.cuda.stream(side):
            big.add_(1)
        got = run(splits, True, 256)
        assert torch.equal(got, ref), (it, (got.float() - ref.float()).abs().max().item())
    assert int(pr.counters.abs().sum().item()) == 0
    # the tail launch needs the in-kernel reduction and an LDS-DMA config
    assert pr.launch(cfg, splits, False, extra=dict(extra, tail=256)) != 0
    assert pr.launch(3 + 4 * 6 if k == 3 else 0, splits, True, extra=dict(extra, tail=256)) != 0
