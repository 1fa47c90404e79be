"""LayerNorm statistics through the GEMM epilogues (kernels.h ConvArgs::stats_out / row_parts), at
the kernel level, for every launch configuration (tile x main-loop variant) and split-K form:

* producer: a rows GEMM with the residual add writes (mean, M2) of each row's 64-column groups of
  its output -- checked against the same statistics computed in fp64 from the stored output;
* reader: a LayerNorm-folded GEMM that merges those groups itself (row_parts) matches the same
  GEMM given precomputed (mean, rstd) rows (row_stats), and both match a torch fp64 reference
  of LN(x) @ (gamma W)^T + (beta W + b).

Shapes: ViT-B/16 rows at batch 7 (M = 1379: M-tail tiles) with K = 768, N = 768 / 3072."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

M, C = 7 * 197, 768


def _torch():
    import torch

    torch.backends.cuda.matmul.allow_tf32 = False
    return torch


def _group_stats(y):
    """[M, N] fp64 -> [M, N/64, 2] (mean, M2) per 64-column group."""
    g = y.reshape(y.shape[0], -1, 64)
    mean = g.mean(-1)
    return np.stack([mean, ((g - mean[..., None]) ** 2).sum(-1)], -1)


def K_NUM_CFGS():
    from die_amd.ops import kernels as K

    return K.NUM_CFGS


def _configs(splits_list=(1, 2)):
    for tile in range(K_NUM_CFGS()):
        for splits in splits_list:
            for fused in ((True, False) if splits > 1 else (True,)):
                yield tile, splits, fused


def test_epilogue_stats_producer_all_configs(native):
    torch = _t = _torch()
    from die_amd.ops import kernels as K

    g = torch.Generator().manual_seed(3)
    x = (torch.randn(M, C, generator=g) * 0.5).cuda()
    w = (torch.randn(C, C, generator=g) / C ** 0.5).cuda()
    b = (torch.randn(C, generator=g) * 0.1).cuda()
    res = (torch.randn(M, C, generator=g) + 3.0).cuda()  # residual rows with a non-zero mean
    pr = K.ConvProblem(x.reshape(M, 1, 1, C), w.reshape(C, C, 1, 1), bias=b, res=res.reshape(M, 1, 1, C),
                       max_splits=2, split=True)
    st = torch.zeros(M, C // 64, 2, dtype=torch.float32, device="cuda")
    ran = 0
    for tile, splits, fused in _configs():
        st.fill_(float("nan"))
        rc = pr.launch(tile, splits, fused, extra={"stats_out": int(st.data_ptr())})
        if rc == 1:  # config not applicable
            continue
        assert rc == 0, (tile, splits, fused, rc)
        torch.cuda.synchronize()
        out = pr.results()[0].reshape(M, C).double().cpu().numpy()
        want = _group_stats(out)
        got = st.double().cpu().numpy()
        # mean: relative to the row scale; M2: relative
        assert np.abs(got[..., 0] - want[..., 0]).max() < 1e-5, (tile, splits, fused)
        assert (np.abs(got[..., 1] - want[..., 1]) / want[..., 1]).max() < 1e-4, (tile, splits, fused)
        ran += 1
    assert ran >= 20


@pytest.mark.parametrize("N,offset", [(768, 0.0), (3072, 0.0), (768, 10.0), (768, 30.0), (768, 100.0)])
def test_epilogue_stats_reader_all_configs(native, N, offset):
    """offset > 0: every row also carries a DC offset of `offset` row sigmas (0.7)
    with a random sign -- the fold's own error (against fp64 on the stored rows) stays at the fp32 bar."""
    torch = _torch()
    from die_amd.ops import kernels as K

    g = torch.Generator().manual_seed(5)
    xr = torch.randn(M, C, generator=g) * 0.7 + torch.randn(M, 1, generator=g) * 2.0  # row offsets
    if offset:
        sign = torch.where(torch.rand(M, 1, generator=g) < 0.5, -1.0, 1.0)
        xr = xr + sign * offset * 0.7
    gamma = 1.0 + 0.1 * torch.randn(C, generator=g)
    beta = 0.1 * torch.randn(C, generator=g)
    w = torch.randn(N, C, generator=g) / C ** 0.5
    bias = 0.1 * torch.randn(N, generator=g)
    eps = 1e-12
    # reference: LN(x) @ W^T + b in fp64
    xd = xr.double()
    ref = torch.nn.functional.layer_norm(xd, (C,), gamma.double(), beta.double(), eps) @ w.double().T + bias.double()
    # folded form the planner builds (hip_plan.cpp fold_layernorm)
    wg = (w.double() * gamma.double()).float()
    fb = (bias.double() + w.double() @ beta.double()).float()
    wgs = K.join_planes(K.split_planes(wg)).double()  # what the GEMM multiplies by
    colsum = torch.zeros((N + 7) // 8 * 8, dtype=torch.float32)
    colsum[:N] = wgs.sum(1).float()
    xs = K.join_planes(K.split_planes(xr)).double()  # the stored (split) rows
    mean = xs.mean(1)
    rstd = 1.0 / torch.sqrt(xs.var(1, unbiased=False) + eps)
    row_stats = torch.stack([mean, rstd], 1).float().contiguous().cuda()
    parts = torch.from_numpy(_group_stats(xs.numpy())).float().contiguous().cuda()
    colsum = colsum.cuda()
    pr = K.ConvProblem(xr.reshape(M, 1, 1, C).cuda(), wg.reshape(N, C, 1, 1).cuda(), bias=fb.cuda(), max_splits=2,
                       split=True)
    common = {"col_sum": int(colsum.data_ptr()), "ln_eps": eps}
    ran, bad = 0, []
    for tile, splits, fused in _configs():
        rc = pr.launch(tile, splits, fused, extra=dict(common, row_stats=int(row_stats.data_ptr())))
        if rc == 1:
            continue
        assert rc == 0, (tile, splits, fused, rc)
        torch.cuda.synchronize()
        a = pr.results()[0].reshape(M, N).double().cpu()
        assert pr.launch(tile, splits, fused, extra=dict(common, row_stats=int(row_stats.data_ptr()))) == 0
        torch.cuda.synchronize()
        a2 = pr.results()[0].reshape(M, N).double().cpu()
        rc = pr.launch(tile, splits, fused, extra=dict(common, row_parts=int(parts.data_ptr())))
        assert rc == 0, (tile, splits, fused, rc)
        torch.cuda.synchronize()
        bb = pr.results()[0].reshape(M, N).double().cpu()
        e_stats = float((a - ref).norm() / ref.norm())
        e_parts = float((bb - ref).norm() / ref.norm())
        rows = ((bb - a).abs().amax(1) / ref.abs().amax()).numpy()
        rep = float((a2 - a).abs().max())
        # the folded form's own error grows with |mean| / std of the rows (here ~3); the two ways of
        # delivering the statistics agree far more closely than that
        # (outputs are stored as hi + lo bf16 planes: ~2^-17 relative steps)
        # with a DC offset the fold's own error grows with |mean| / std: its GEMM accumulates x.W' at
        # the offset's magnitude in fp32 before rstd * (acc - mean * colsum) cancels it (measured on
        # MI355X: < 5e-5 at 10 sigma, 1.14e-4 at 30, 4.54e-4 at 100 -- ~4.5e-6 per sigma of offset,
        # profiles/r6_fold_layernorm_offsets.md); the bound asserted is that law with 20 % margin
        bar = 5e-5 + 5.5e-6 * offset
        if not (e_stats < bar and e_parts < bar and rows.max() < 3e-5 + 1e-6 * offset and rep == 0.0):
            top = np.argsort(rows)[-4:][::-1]
            bad.append((tile, splits, fused, "%.2e %.2e" % (e_stats, e_parts), "repeat %.2e" % rep,
                        [(int(r), "%.2e" % rows[r]) for r in top]))
        ran += 1
    for b in bad:
        print("BAD", b)
    assert not bad and ran >= 20
