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
