"""Fused expand + next-reduce 1x1 pair (csrc/kernels/conv_pair.hip) on the GPU.

Checks, per ResNet-50 stage shape (stage 1: K1 64 / N1 256 / N2 64; stage 2: 128 / 512 / 128):
  * fp32 (split) mode vs a float64 torch reference of the same two layers at rel <= 2e-5;
  * bit-exactness against the two unfused kernels it replaces (the dual-store expand conv and the
    reduce conv, both at the 64x64 tile, no split-K): same K order, same MFMA sequence, same epilogue
    rounding, so the engine's fused and unfused plans give identical logits;
  * M tails (rows not a multiple of 64), the optional raw-sum store, and the bf16 mode.
The whole-model checks (fused plan vs torch fp32, vs the unfused plan) are in test_gpu_fp32.py and
test_gpu_engine.py."""
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def _t():
    import torch

    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    return torch


def rel_err(a, b):
    t = _t()
    a, b = a.double(), b.double()
    return (t.linalg.vector_norm(a - b) / t.linalg.vector_norm(b).clamp_min(1e-30)).item()


def _problem(M, K1, N1, N2, seed):
    torch = _t()
    g = torch.Generator(device="cuda").manual_seed(seed)
    y = torch.relu(torch.randn(M, K1, device="cuda", generator=g))
    w1 = torch.randn(N1, K1, device="cuda", generator=g) / K1 ** 0.5
    b1 = torch.randn(N1, device="cuda", generator=g) * 0.1
    res = torch.randn(M, N1, device="cuda", generator=g)
    s2 = torch.rand(N1, device="cuda", generator=g) + 0.5
    h2 = torch.randn(N1, device="cuda", generator=g) * 0.1
    w2 = torch.randn(N2, N1, device="cuda", generator=g) / N1 ** 0.5
    b2 = torch.randn(N2, device="cuda", generator=g) * 0.1
    return y, w1, b1, res, s2, h2, w2, b2


def _reference(y, w1, b1, res, s2, h2, w2, b2):
    torch = _t()
    x = y.double() @ w1.double().T + b1.double() + res.double()
    a = torch.relu(x * s2.double() + h2.double())
    out = torch.relu(a @ w2.double().T + b2.double())
    return x, out


PAIR_SHAPES = [
    # M, K1, N1, N2
    (2 * 56 * 56, 64, 256, 64),      # stage 1 at batch 2
    (3 * 28 * 28, 128, 512, 128),    # stage 2 at batch 3 (2352: tail of 48 rows)
    (1000, 64, 256, 64),             # ragged M
    (130, 128, 512, 128),            # three blocks, two of them partial
    (512, 64, 128, 128),             # mixed combination
    (448, 128, 256, 64),
    (20 * 28 * 28 - 5, 128, 512, 256),  # the stage-2 -> stage-3 boundary (256 reduce channels)
    (700, 64, 256, 256),
]


@pytest.mark.parametrize("shape", PAIR_SHAPES)
def test_pair_split_matches_fp64(native, shape):
    from die_amd.ops import kernels as K

    M, K1, N1, N2 = shape
    prob = _problem(M, K1, N1, N2, seed=M * 7 + K1 + N2)
    x, out = K.conv_pair(*prob, split=True)
    xr, outr = _reference(*prob)
    assert rel_err(x, xr) <= 2e-5, rel_err(x, xr)
    assert rel_err(out, outr) <= 2e-5, rel_err(out, outr)


@pytest.mark.parametrize("shape", [(2 * 56 * 56, 64, 256, 64), (3 * 28 * 28 - 17, 128, 512, 128),
                                   (2 * 28 * 28 - 3, 128, 512, 256)])
def test_pair_bit_exact_vs_unfused_kernels(native, shape):
    """The fused launch must reproduce the two unfused launches bit for bit (split mode)."""
    torch = _t()
    from die_amd.ops import kernels as K

    M, K1, N1, N2 = shape
    y, w1, b1, res, s2, h2, w2, b2 = _problem(M, K1, N1, N2, seed=11)
    # the unfused path: 1x1 convs over a [1, M, 1, C] "image" with the 64x64 LDS-DMA tile, 1 stage
    cfg = 3 + 4 * 5  # TILE_64x64 + NUM_TILES * variant 5
    expand = K.ConvProblem(y.reshape(1, M, 1, K1), w1.reshape(N1, K1, 1, 1), bias=b1, res=res.reshape(1, M, 1, N1),
                           scale2=s2, shift2=h2, relu2=True, max_splits=1, split=True)
    assert expand.launch(cfg) == 0
    xo, _ = expand.results()
    reduce_ = K.ConvProblem(torch.zeros(1, M, 1, N1, device="cuda"), w2.reshape(N2, N1, 1, 1), bias=b2, relu=True,
                            max_splits=1, split=True)
    reduce_.x = expand.out2  # the stored hi/lo planes themselves (re-splitting hi + lo is not always exact)
    assert reduce_.launch(cfg) == 0
    o2, _ = reduce_.results()
    xf, of, af = K.conv_pair(y, w1, b1, res, s2, h2, w2, b2, split=True, store_a=True)
    assert torch.equal(xf, xo.reshape(M, N1)), (xf - xo.reshape(M, N1)).abs().max().item()
    # the stored pre-activation (a stage boundary's projection shortcut reads it) = the expand's out2
    ao = K.join_planes(expand.out2).reshape(M, N1)
    assert torch.equal(af, ao), (af - ao).abs().max().item()
    assert torch.equal(of, o2.reshape(M, N2)), (of - o2.reshape(M, N2)).abs().max().item()


@pytest.mark.parametrize("split", [True, False])
@pytest.mark.parametrize("shape", [(24 * 28 * 28 - 9, 128, 512, 128), (2 * 56 * 56 - 1, 64, 256, 64),
                                   (3 * 28 * 28, 128, 512, 64), (1000, 128, 512, 256)])
def test_pair_shared_w_bitwise(native, shape, split):
    """PairArgs::shared_w: the W1 chunk and the W2 slice loaded in turn through one LDS buffer (two
    blocks per CU in fp32 at K1 = 128) is the same arithmetic in the same order -- x, a and the output
    equal the separate-buffer launch bit for bit, also when repeated (race screen), in both modes;
    auto (-1) picks it only above one block per CU for the shapes it helps."""
    torch = _t()
    from die_amd.ops import kernels as K

    M, K1, N1, N2 = shape
    prob = list(_problem(M, K1, N1, N2, seed=M + N2))
    if not split:
        for i in (0, 3):
            prob[i] = prob[i].to(torch.bfloat16)
    ref = K.conv_pair(*prob, split=split, store_a=True, shared_w=0)
    for _ in range(3):
        got = K.conv_pair(*prob, split=split, store_a=True, shared_w=1)
        for g, r in zip(got, ref):
            assert torch.equal(g, r), (g.float() - r.float()).abs().max().item()
    auto = K.conv_pair(*prob, split=split, store_a=True)
    for g, r in zip(auto, ref):
        assert torch.equal(g, r)


def test_pair_without_raw_store_and_repeatable(native):
    torch = _t()
    from die_amd.ops import kernels as K

    prob = _problem(777, 64, 256, 64, seed=5)
    x, out = K.conv_pair(*prob, split=True, store_x=False)
    assert x is None
    _, outr = _reference(*prob)
    assert rel_err(out, outr) <= 2e-5
    for _ in range(3):  # race screen: bitwise identical relaunches
        _, again = K.conv_pair(*prob, split=True, store_x=False)
        assert torch.equal(again, out)


@pytest.mark.parametrize("shape", [(1000, 64, 256, 64), (600, 128, 512, 128)])
def test_pair_bf16(native, shape):
    torch = _t()
    from die_amd.ops import kernels as K

    M, K1, N1, N2 = shape
    prob = list(_problem(M, K1, N1, N2, seed=3))
    for i in (0, 3):  # activations enter as bf16 tensors in this mode
        prob[i] = prob[i].to(torch.bfloat16)
    x, out = K.conv_pair(*prob, split=False)
    xr, outr = _reference(*[p.float() for p in prob])
    assert rel_err(x.float(), xr) <= 1e-2
    assert rel_err(out.float(), outr) <= 2e-2


def test_engine_fused_pairs_match_unfused_plan(native, models):
    """ResNet50-v2 fp32: the default plan (6 expand+reduce pairs fused) vs the unfused plan and torch
    fp32, at a full and a partial batch bucket."""
    import numpy as np

    torch = _t()
    from die_amd.models import resnet_v2 as r

    path, w, cfg = models["get_rn50"]()
    ef = native.Engine(path, device="hip", max_batch=20, precision="fp32")
    eu = native.Engine(path, device="hip", max_batch=20, precision="fp32", fuse_pairs=False)
    try:
        ops = native.plan_summary(path, 20, precision="fp32")["ops"]
        kinds = [o["kind"] for o in ops]
        # 5 unit boundaries inside stages 1/2 + the stage-1 -> 2 boundary, whose pre-activation the
        # stage-2 projection shortcut also reads (stored by the pair kernel: store_preact).  The
        # stage-2 -> 3 boundary (256 reduce channels) stays unfused by default (hip_plan.cpp kMaxPairN2).
        assert kinds.count("conv_pair") == 6, kinds
        assert sum(1 for o in ops if o.get("store_preact")) == 1
        assert ef.refresh_info()["options"]["fuse_pairs"] is True
        for B in (20, 13):
            x = r.synthetic_input(B, cfg, seed=90 + B)
            with torch.no_grad():
                ref = r.torch_forward(w, x, cfg, device="cuda").double().cpu().numpy()
            gf = ef.run(x.reshape(B, -1)).astype(np.float64)
            gu = eu.run(x.reshape(B, -1)).astype(np.float64)
            assert float(np.linalg.norm(gf - ref) / np.linalg.norm(ref)) <= 1e-4
            assert float(np.linalg.norm(gf - gu) / np.linalg.norm(gu)) <= 2e-5
            assert (gf.argmax(1) == ref.argmax(1)).all()
    finally:
        ef.close()
        eu.close()
