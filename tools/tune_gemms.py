"""Measure the forward GEMMs' best hipBLASLt solutions on this MI355X (PyTorch TunableOp)
and write them to the package's read-only selection file (runtime.use_gemm_tuning).

Runs bench.py's forward legs (C2 end-to-end scoring, C1 / C3 / C5 method decode) once as
a child process with TunableOp tuning on: every GEMM shape the legs launch is timed over
the library's candidate solutions and the fastest recorded.  The parent never touches the
GPU.

    python tools/tune_gemms.py [--out gpurun_out/gemm_tuned.csv] [--install]

--install copies the result to <package>/tuned/gemm_mi355x.csv (commit it; the results
are valid for the PyTorch / ROCm / hipBLASLt versions recorded in its header).
"""
import argparse
import glob
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "gemm_tuned.csv"))
    ap.add_argument("--install", action="store_true")
    ap.add_argument("--method", default="c1,c3,c5")
    ap.add_argument("--iters", default="30")
    ap.add_argument("--ms", default="30")
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    env = dict(os.environ, PYTORCH_TUNABLEOP_ENABLED="1", PYTORCH_TUNABLEOP_TUNING="1",
               PYTORCH_TUNABLEOP_FILENAME=args.out, PYTORCH_TUNABLEOP_VERBOSE="1",
               PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=args.iters,
               PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=args.ms)
    cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--steps", "2", "--warmup", "1",
           "--beam", "", "--cpu-seconds", "0", "--method", args.method]
    rc = subprocess.call(cmd, env=env, cwd=REPO)
    outs = sorted(glob.glob(os.path.splitext(args.out)[0] + "*.csv"))
    print("tuning results:", outs, "rc", rc, flush=True)
    if rc == 0 and args.install and outs:
        dst = os.path.join(REPO, PKG, "tuned", "gemm_mi355x.csv")
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        shutil.copy(outs[0], dst)
        print("installed", dst, flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
