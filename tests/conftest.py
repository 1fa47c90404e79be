import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

import die_amd  # noqa: E402,F401  (sets the HIP runtime environment before any test touches the GPU)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def _ensure_built():
    import die_amd
    from die_amd import native

    if not os.path.exists(native.lib_path()):
        subprocess.check_call(["make", "-j8"], cwd=REPO)
    return native


@pytest.fixture(scope="session")
def native():
    return _ensure_built()


@pytest.fixture(scope="session")
def models(tmp_path_factory):
    """Generated ONNX files (random weights): tiny ResNet-v2 and full ResNet50-v2."""
    _ensure_built()
    from die_amd.models import resnet_v2 as r

    d = tmp_path_factory.mktemp("models")
    out = {}
    cfg = r.tiny_config()
    b, w = r.build_onnx(cfg)
    p = str(d / "tiny.onnx")
    open(p, "wb").write(b)
    out["tiny"] = (p, w, cfg)

    def rn50():
        if "rn50" not in out:
            c = r.ResNetConfig()
            b2, w2 = r.build_onnx(c)
            p2 = str(d / "rn50.onnx")
            open(p2, "wb").write(b2)
            out["rn50"] = (p2, w2, c)
        return out["rn50"]

    out["get_rn50"] = rn50

    def vit(name):
        from die_amd.models import vit as v

        key = "vit_" + name
        if key not in out:
            c = v.tiny_vit_config() if name == "tiny" else v.ViTConfig()
            b3, w3 = v.build_onnx(c)
            p3 = str(d / (key + ".onnx"))
            open(p3, "wb").write(b3)
            out[key] = (p3, w3, c)
        return out[key]

    out["get_vit"] = vit
    return out


def gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False
