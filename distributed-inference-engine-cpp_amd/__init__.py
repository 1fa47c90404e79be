"""MI355X-native distributed inference engine (gateway / worker / HIP engine).

See README.md for the layout; the native runtime lives in `csrc/` and is loaded through
`die_amd.native`.
"""
import os as _os

PKG_DIR = _os.path.dirname(_os.path.abspath(__file__))
REPO_DIR = _os.path.dirname(PKG_DIR)
LIB_DIR = _os.path.join(PKG_DIR, "lib")
BIN_DIR = _os.path.join(PKG_DIR, "bin")

__version__ = "0.1.0"

# HIP hardware queues per process.  HIP maps every stream onto one of GPU_MAX_HW_QUEUES hardware
# queues (HIP's default, and the value the GPU boxes export: 4) and lets streams share a queue beyond
# that, which serialises them.  The engine uses up to 4 streams (compute, 2 copy, prep/side), and an
# RCCL communicator adds its own internal streams: with 4 queues a data-parallel rank's copy streams
# share queues with kernels and the serving path loses 13-23 % (profiles/r3_rccl_hw_queues.md).  So
# a value below 8 -- the platform default, not a choice made for this engine -- is raised to 8;
# DIE_HIP_HW_QUEUES sets it explicitly (e.g. 4 for an A/B).  Must be in the environment before the
# process's first HIP call.
HIP_HW_QUEUES = 8


def configure_hip_env(environ=None) -> None:
    env = _os.environ if environ is None else environ
    want = env.get("DIE_HIP_HW_QUEUES")
    if want:
        env["GPU_MAX_HW_QUEUES"] = want
    else:
        try:
            cur = int(env.get("GPU_MAX_HW_QUEUES", "0"))
        except ValueError:
            cur = 0
        if cur < HIP_HW_QUEUES:
            env["GPU_MAX_HW_QUEUES"] = str(HIP_HW_QUEUES)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts (RCCL, IPC handles)


configure_hip_env()
