"""HIP engine on graphs beyond ResNet50 / ViT-B: MobileNetV2-style (depthwise
convs on the grouped-conv kernel, Clip epilogues, asymmetric SAME pads, Softmax head) and a ViT with
decomposed LayerNorm + Slice cls token, vs the C++ CPU executor and torch fp32."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a GPU")]


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _model(tmp_path, mod, cfg, name):
    blob, w = mod.build_onnx(cfg)
    p = str(tmp_path / (name + ".onnx"))
    open(p, "wb").write(blob)
    return p, w


@pytest.mark.parametrize("which", ["mobilenet_tiny", "mobilenet_224", "vit_decomposed"])
def test_extra_models_on_hip(native, tmp_path, which):
    import torch

    from die_amd.models import mobilenet as mb
    from die_amd.models import vit as v

    if which == "mobilenet_tiny":
        mod, cfg = mb, mb.tiny_mobilenet_config()
    elif which == "mobilenet_224":
        mod, cfg = mb, mb.MobileNetConfig()
    else:
        mod, cfg = v, v.ViTConfig(image=64, patch=8, dim=192, depth=3, heads=3, mlp=384, num_classes=32,
                                  decomposed_ln=True, cls_slice=True, softmax_head=True)
    p, w = _model(tmp_path, mod, cfg, which)
    e32 = native.Engine(p, device="hip", max_batch=16, precision="fp32")
    e16 = native.Engine(p, device="hip", max_batch=16, precision="bf16")
    try:
        for B in (1, 5, 16):
            x = mod.synthetic_input(B, cfg, seed=B)
            with torch.no_grad():
                ref = mod.torch_forward(w, x, cfg, device="cuda").double().cpu().numpy()
            got = e32.run(x.reshape(B, -1)).astype(np.float64)
            assert rel_l2(got, ref) <= 1e-4, (which, B, rel_l2(got, ref))
            assert (got.argmax(1) == ref.argmax(1)).all()
            g16 = e16.run(x.reshape(B, -1)).astype(np.float64)
            assert rel_l2(g16, ref) <= 2e-2, (which, B, rel_l2(g16, ref))
        cpu = native.cpu_run(p, mod.synthetic_input(4, cfg, seed=9))
        hip = e32.run(mod.synthetic_input(4, cfg, seed=9).reshape(4, -1))
        assert rel_l2(hip, cpu) <= 1e-4
    finally:
        e32.close()
        e16.close()


@pytest.mark.parametrize("cfg", [(2, 28, 96, 96, 3, 1, [1, 1, 1, 1], 96), (3, 14, 64, 64, 3, 2, [0, 0, 1, 1], 64),
                                 (2, 9, 32, 64, 3, 1, [1, 1, 1, 1], 8)])
@pytest.mark.parametrize("split", [False, True])
def test_grouped_conv_kernel(native, cfg, split):
    """Depthwise and grouped conv vs torch (asymmetric pads via explicit F.pad)."""
    import torch

    from die_amd import native as nat
    from die_amd.ops import kernels as K

    B, H, Cin, Cout, k, s, pads, groups = cfg
    g = torch.Generator(device="cuda").manual_seed(H + Cin)
    x = torch.randn(B, Cin, H, H, device="cuda", generator=g)
    w = torch.randn(Cout, Cin // groups, k, k, device="cuda", generator=g) * 0.3
    b = torch.randn(Cout, device="cuda", generator=g)
    xp = torch.nn.functional.pad(x.double(), (pads[1], pads[3], pads[0], pads[2]))
    ref = torch.clamp(torch.nn.functional.conv2d(xp, w.double(), b.double(), stride=s, groups=groups), 0, 6)
    got = K.grouped_conv(x.permute(0, 2, 3, 1).contiguous(), w, b, stride=s, pads=pads, groups=groups, clip=(0, 6),
                         split=split)
    torch.cuda.synchronize()
    err = float((got.permute(0, 3, 1, 2).double() - ref).norm() / ref.norm())
    assert err < (2e-5 if split else 1e-2), err


@pytest.mark.parametrize("split", [False, True])
def test_softmax_rows_kernel(native, split):
    import torch

    from die_amd.ops import kernels as K

    x = torch.randn(37, 1000, device="cuda") * 4
    if not split:
        x = x.to(torch.bfloat16).float()  # the bf16 kernel reads bf16 inputs
    got16, got32 = K.softmax_rows(x, split=split)
    ref = torch.softmax(x.double(), -1)
    torch.cuda.synchronize()
    # split input carries ~17 significant bits (exp of |x| <= 16 magnifies that to ~1e-5 relative)
    assert float((got32.double() - ref).norm() / ref.norm()) < (2e-5 if split else 1e-6)
    assert float((got16.double() - ref).norm() / ref.norm()) < (2e-5 if split else 1e-2)
