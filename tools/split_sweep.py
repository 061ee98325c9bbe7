#!/usr/bin/env python3
"""Sweep split-V target grid x streaming variant for the small-row (beam) shapes."""
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
ops = importlib.import_module(
    "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd.ops")
from beam_ab import timed  # noqa: E402

VARIANTS = {5: "b256_u4", 1: "b512_u4", 3: "b1024_u2", 4: "b256_u8", 6: "b1024_u4", 7: "b512_u8"}
dev = torch.device("cuda:0")
torch.cuda.set_device(0)
SHAPES = {"c3": (256, 256000, 0.0), "c5": (512, 128256, 0.0), "c1": (16, 128256, 0.0),
          "rows2048": (2048, 128256, 0.0), "c3cap": (256, 256000, 30.0)}
TWS = (256, 512, 1024, 2048, 4096, 8192)
if len(sys.argv) > 1:
    SHAPES = {k: SHAPES[k] for k in sys.argv[1].split(",")}
if len(sys.argv) > 2:
    TWS = tuple(int(t) for t in sys.argv[2].split(","))
for name, (rows, V, cap) in SHAPES.items():
    g = torch.Generator(device=dev).manual_seed(1)
    x = (torch.randn(rows, V, generator=g, device=dev) * 3).to(torch.bfloat16)
    ws = ops.Workspace()
    for tw in TWS:
        os.environ["CS_TARGET_WGS"] = str(tw)
        res = {}
        for v, vn in VARIANTS.items():
            os.environ["CS_LSG_VARIANT"] = str(v)
            res[vn] = round(timed(lambda: ops.logsoftmax_gather(x, None, softcap=cap, workspace=ws, want_lse=True)), 1)
        print(json.dumps({"shape": name, "target_wgs": tw, "us": res,
                          "ideal_us": round(rows * V * 2 / 8e12 * 1e6, 1)}), flush=True)
os.environ.pop("CS_TARGET_WGS")
os.environ.pop("CS_LSG_VARIANT")
