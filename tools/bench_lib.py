#!/usr/bin/env python3
"""bench.py against another build of the library (A/B of a compile-time variant at the
method level): python tools/bench_lib.py LIB.so [bench.py args...].  One GPU only."""
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"
_lib = importlib.import_module(PKG + "._lib")
_lib.LIB_NAME = os.path.relpath(os.path.abspath(sys.argv[1]), os.path.join(REPO, PKG))
sys.argv = [os.path.join(REPO, "bench.py")] + sys.argv[2:]
import bench  # noqa: E402

bench.main()
