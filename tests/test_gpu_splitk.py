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
    (24, 14, 256, 256, 3, 1, 1, 3 + 4 * 9, 2),     # four-tile 3x3 kernel: one 14x14 image per block
    (22, 7, 512, 512, 3, 1, 1, 3 + 4 * 9, 4),      # ... four 7x7 images per block
    (5, 7, 512, 512, 3, 1, 1, 3 + 4 * 9, 8),       # ... a last block with one image
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


SK_CASES = [
    # B, H, Cin, Cout, k, stride, pad, tile cfg, P (stream-K blocks), live B (0 = all)
    (24, 14, 1024, 256, 1, 1, 0, 3 + 4 * 1, 512, 0),    # stage-3 reduce, 64x64 2-stage: 296 tiles x 16 K-steps
    (24, 14, 1024, 256, 1, 1, 0, 3 + 4 * 1, 256, 0),    # ... one block per CU
    (24, 14, 1024, 256, 1, 1, 0, 3 + 4 * 5, 1024, 21),  # 1-stage, live batch 21
    (24, 7, 2048, 512, 1, 1, 0, 3 + 4 * 1, 512, 0),     # stage-4 reduce: 152 tiles x 32
    (24, 14, 256, 256, 3, 1, 1, 2 + 4 * 1, 256, 0),     # stage-3 3x3 implicit (MODE 2), 64x128
    (24, 7, 512, 2048, 1, 1, 0, 0 + 4 * 1, 256, 0),     # stage-4 expand, 128x128: 80 tiles x 8
    (3, 7, 512, 512, 3, 1, 1, 3 + 4 * 5, 512, 0),       # fewer iterations than blocks (empty ranges)
]


def _fp64_conv(x, w, bias, s, p):
    import torch

    y = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).double(), w.double(), bias.double(), s, p)
    return torch.relu(y).permute(0, 2, 3, 1)


@pytest.mark.parametrize("case", SK_CASES)
@pytest.mark.parametrize("split", [True, False])
def test_streamk(native, case, split):
    """ConvArgs::sk (stream-K): P blocks split the tiles x K-steps iterations evenly; tiles cut
    between blocks are summed in-kernel by their last arriving contributor in block order.  Checked
    against an fp64 conv of the same (stored) inputs, bit for bit repeatable over launches under
    side load, every tile counter back at zero; with a live batch only live rows are defined."""
    import torch
    from die_amd.ops import kernels as K

    B, H, Cin, Cout, k, s, p, cfg, P, live = case
    g = torch.Generator(device="cuda").manual_seed(Cin * 13 + Cout + k + B)
    x = torch.randn(B, H, H, Cin, device="cuda", generator=g)
    w = torch.randn(Cout, Cin, k, k, device="cuda", generator=g) / (Cin * k * k) ** 0.5
    bias = torch.randn(Cout, device="cuda", generator=g)
    if not split:
        x = x.to(torch.bfloat16)
    Ho = (H + 2 * p - k) // s + 1
    ws_splits = max(16, -(-P * 2 * 128 * 128 // (B * Ho * Ho * Cout)))  # stream-K: 2 slabs per block
    pr = K.ConvProblem(x, w, bias=bias, stride=s, pad=p, relu=True, max_splits=ws_splits, split=split)
    extra = {}
    if live:
        lv = torch.tensor([live], dtype=torch.int64, device="cuda")
        extra["live"] = int(lv.data_ptr())
    rows = (live or B) * pr.geom["Ho"] * pr.geom["Wo"]
    assert pr.launch(cfg, 1, True, extra=extra, sk=P) == 0
    torch.cuda.synchronize()
    first = pr.results()[0].reshape(-1, Cout)[:rows].clone()
    xs = K.join_planes(K.split_planes(x)) if split else x.float()
    wq = K.join_planes(K.split_planes(w)) if split else w.to(torch.bfloat16).float()
    ref = _fp64_conv(xs, wq, bias, s, p).reshape(-1, Cout)[:rows]
    err = float((first.double() - ref).norm() / ref.norm())
    assert err < (2e-5 if split else 8e-3), err
    side = torch.cuda.Stream()
    big = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
    for it in range(8):
        with torch.cuda.stream(side):
            big.add_(1)
        assert pr.launch(cfg, 1, True, extra=extra, sk=P) == 0
        torch.cuda.synchronize()
        got = pr.results()[0].reshape(-1, Cout)[:rows]
        assert torch.equal(got, first), (it, (got.float() - first.float()).abs().max().item())
    assert int(pr.counters.abs().sum().item()) == 0


@pytest.mark.parametrize("B,H,C,live", [(24, 14, 256, 0), (24, 14, 256, 21), (22, 7, 512, 0), (22, 7, 512, 17),
                                        (3, 14, 128, 0)])
@pytest.mark.parametrize("split", [True, False])
def test_quad_3x3(native, B, H, C, live, split):
    """Variant 9 (conv_quad.hip): four 8x8 sub-tiles x 64 channels per block, the tap weights loaded
    once for all four.  Against an fp64 conv of the stored inputs at every split-K factor, with a
    residual + dual-store epilogue, and with a live batch whose last block holds 1-3 sub-tiles."""
    import torch
    from die_amd.ops import kernels as K

    g = torch.Generator(device="cuda").manual_seed(B * 7 + H + C + live)
    x = torch.randn(B, H, H, C, device="cuda", generator=g)
    w = torch.randn(C, C, 3, 3, device="cuda", generator=g) / (C * 9) ** 0.5
    bias = torch.randn(C, device="cuda", generator=g)
    res = torch.randn(B, H, H, C, device="cuda", generator=g)
    s2 = torch.rand(C, device="cuda", generator=g) + 0.5
    b2 = torch.randn(C, device="cuda", generator=g)
    if not split:
        x, res = x.to(torch.bfloat16), res.to(torch.bfloat16)
    pr = K.ConvProblem(x, w, bias=bias, pad=1, relu=True, res=res, scale2=s2, shift2=b2, relu2=True, max_splits=8,
                       split=split)
    xs = K.join_planes(K.split_planes(x)) if split else x.float()
    wq = K.join_planes(K.split_planes(w)) if split else w.to(torch.bfloat16).float()
    rq = K.join_planes(K.split_planes(res)) if split else res.float()
    v = torch.relu(torch.nn.functional.conv2d(xs.permute(0, 3, 1, 2).double(), wq.double(), bias.double(), padding=1)
                   .permute(0, 2, 3, 1) + rq.double())
    u = torch.relu(v * s2.double() + b2.double())
    rows = (live or B) * H * H
    extra = {}
    if live:
        lv = torch.tensor([live], dtype=torch.int64, device="cuda")
        extra["live"] = int(lv.data_ptr())
    tol = 2e-5 if split else 8e-3
    outs = {}
    for sp in (1, 2, 4, 8):
        for fused in ((True, False) if sp > 1 else (True,)):
            assert pr.launch(39, sp, fused, extra=extra) == 0, sp
            torch.cuda.synchronize()
            o, o2 = pr.results()
            o, o2 = o.reshape(-1, C)[:rows], o2.reshape(-1, C)[:rows]
            e1 = float((o.double() - v.reshape(-1, C)[:rows]).norm() / v.reshape(-1, C)[:rows].norm())
            e2 = float((o2.double() - u.reshape(-1, C)[:rows]).norm() / u.reshape(-1, C)[:rows].norm())
            assert e1 < tol and e2 < tol, (sp, fused, e1, e2)
            if sp in outs:  # fused and two-kernel reductions sum in the same order
                assert torch.equal(outs[sp], o), (sp, "fused != two-kernel")
            outs[sp] = o.clone()
    assert int(pr.counters.abs().sum().item()) == 0
