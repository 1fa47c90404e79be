#!/usr/bin/env python3
"""Reference-compatible benchmark client at the reference's path (benchmark.py); the
implementation lives in tools/benchmark.py (same CLI: --gateway --requests --threads ...)."""
import os
import runpy
import sys

if __name__ == "__main__":
    sys.argv[0] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools", "benchmark.py")
    runpy.run_path(sys.argv[0], run_name="__main__")
