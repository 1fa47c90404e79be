"""ViT-B/16 (BASELINE config 5) on the CPU: generator vs torch through the C++ CPU executor, and the
HIP planner's lowering of the transformer graph (runs without a GPU: planning is host code)."""
import numpy as np


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-12))


def test_vit_tiny_cpu_executor_matches_torch(native, models):
    import torch

    from die_amd.models import vit

    path, w, cfg = models["get_vit"]("tiny")
    x = vit.synthetic_input(3, cfg)
    got = native.cpu_run(path, x)
    with torch.no_grad():
        ref = vit.torch_forward(w, x, cfg).numpy()
    assert got.shape == (3, cfg.num_classes)
    assert rel_l2(got, ref) < 1e-4


def test_vit_tiny_plan_fusions(native, models):
    path, w, cfg = models["get_vit"]("tiny")
    p = native.plan_summary(path, 8)
    kinds = [o["kind"] for o in p["ops"]]
    assert p["output_shape"] == [1, cfg.num_classes]
    # per layer: LN, fused QKV GEMM, attention, proj(+residual), LN, fc1(+GELU), fc2(+residual)
    assert kinds.count("attention") == cfg.depth
    assert kinds.count("layernorm") == 2 * cfg.depth + 1
    assert kinds.count("tokens") == 1 and kinds.count("gather_rows") == 1
    gemms = [o for o in p["ops"] if o["kind"] == "conv"]
    qkv = [o for o in gemms if o["name"].endswith("+qkv")]
    assert len(qkv) == cfg.depth and all(o["N"] == 3 * cfg.dim for o in qkv)
    assert sum(o["act"] == 2 for o in gemms) == cfg.depth  # GELU folded into fc1
    assert sum(o["residual"] for o in gemms) == 2 * cfg.depth
    S = (cfg.image // cfg.patch) ** 2 + 1
    assert all(o["rows"] == S for o in gemms if "encoder" in o["name"])
    # no standalone elementwise kernels are left
    assert "affine" not in kinds


def test_vit_base_plan(native, models):
    path, w, cfg = models["get_vit"]("base")
    p = native.plan_summary(path, 32)
    kinds = [o["kind"] for o in p["ops"]]
    assert kinds.count("attention") == 12
    assert len(p["ops"]) == 90
    # 86M parameters in bf16 (+ fp32 biases / LN params)
    assert 160e6 < p["param_bytes"] < 190e6
    assert abs(p["gflop_per_sample"] - 35.1) < 0.5


def test_fold_layernorm_plan(native, tmp_path):
    """fold_layernorm (default on): ViT's pre-norm LayerNorms (each read only by a GEMM) become statistics ops and
    their GEMMs read the residual rows; BERT's post-norm LayerNorms also feed residual adds, so they
    stay (models/generic.py bert)."""
    from die_amd.models import generic, vit

    c = vit.tiny_vit_config()
    p = str(tmp_path / "vit.onnx")
    open(p, "wb").write(vit.build_onnx(c)[0])
    plain = native.plan_summary(p, 8, precision="fp32", fold_layernorm=False)
    folded = native.plan_summary(p, 8, precision="fp32", ln_stats_epilogue=False)
    stats = [o for o in folded["ops"] if o.get("stats_only")]
    assert len(stats) == 2 * c.depth and not any(o.get("stats_only") for o in plain["ops"])
    convs = [o for o in folded["ops"] if o.get("layernorm_folded")]
    assert len(convs) == 2 * c.depth and all(o["name"].startswith("encoder.layer.") for o in convs)
    assert not any(o.get("stats_out") for o in folded["ops"])
    # the statistics buffers are tiny: the folded arena is no larger
    assert folded["arena_bytes"] <= plain["arena_bytes"]
    # default: the statistics come from the ops that write the LayerNorm inputs -- the token assembly
    # (block 0) and the GEMMs with the residual add (attention-out, MLP2): no statistics op is left
    d = native.plan_summary(p, 8, precision="fp32")
    assert not any(o.get("stats_only") for o in d["ops"])
    prod = [o for o in d["ops"] if o.get("stats_out")]
    assert [o["kind"] for o in prod].count("tokens") == 1 and len(prod) == 2 * c.depth
    assert all(o["residual"] and o["N"] == c.dim for o in prod if o["kind"] == "conv")
    assert all("out_stats" in o["bufs"] for o in prod)
    assert len(d["ops"]) == len(folded["ops"]) - 2 * c.depth
    cons = [o for o in d["ops"] if o.get("stats_from_producer")]
    assert len(cons) == 2 * c.depth and all(o["layernorm_folded"] for o in cons)
    # each producer's partials are read (in3) by the next op, the QKV or MLP1 GEMM, which arena
    # planning keeps them live for
    idx = {o["name"]: i for i, o in enumerate(d["ops"])}
    for o in prod:
        nxt = d["ops"][idx[o["name"]] + 1]
        assert nxt.get("stats_from_producer") and nxt["bufs"]["in3"] == o["bufs"]["out_stats"], nxt["name"]
    b = str(tmp_path / "bert.onnx")
    open(b, "wb").write(generic.build_onnx("bert"))
    s = native.plan_summary(b, 8, precision="fp32", fold_layernorm=True)
    assert not any(o.get("stats_only") for o in s["ops"])
