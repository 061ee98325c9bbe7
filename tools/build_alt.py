#!/usr/bin/env python3
"""Build an A/B copy of the library with extra defines: python tools/build_alt.py OUT.so -DX=1 ...
(time it against the tree's build with tools/beam_ab.py --lib OUT.so / tools/ab_lib.py OUT.so)"""
import importlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
bld = importlib.import_module(
    "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd.build")
out, defs = os.path.abspath(sys.argv[1]), sys.argv[2:]
objs = [out + "." + os.path.basename(s) + ".o" for s in bld.SOURCES]
with ThreadPoolExecutor(4) as ex:
    list(ex.map(lambda so: subprocess.check_call(["/opt/rocm/bin/hipcc"] + bld._flags() + defs +
                                                 ["-c", so[0], "-o", so[1]]), zip(bld.SOURCES, objs)))
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs)
for o in objs:
    os.remove(o)
