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
# queues (default 4) and lets streams share a queue beyond that, which serialises them.  The engine
# uses up to 4 streams (compute, 2 copy, prep/side), and an RCCL communicator adds its own internal
# streams: with 4 queues a data-parallel rank's copy streams ended up sharing queues, and the
# serving path lost 13-15 % (12.1k vs 14.2-14.4k req/s, RCCL merge path at world=1, identical
# otherwise; the plain worker is unchanged within noise at 6, 8 and 16: profiles/r3_rccl_hw_queues.md).
# Must be in the environment before the process's first HIP call; an explicit setting wins.
HIP_HW_QUEUES = 8


def configure_hip_env(environ=None) -> None:
    env = _os.environ if environ is None else environ
    env.setdefault("GPU_MAX_HW_QUEUES", str(HIP_HW_QUEUES))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts (RCCL, IPC handles)


configure_hip_env()
