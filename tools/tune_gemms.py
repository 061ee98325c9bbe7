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
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "generating-fair-consensus-statements-with-social-choice-on-token-level-mdps_amd"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "gemm_tuned.csv"))
    ap.add_argument("--install", action="store_true")
    ap.add_argument("--resume", type=int, default=1)
    ap.add_argument("--legs", default="e2e,c1,c3,c5")
    ap.add_argument("--iters", default="10")
    ap.add_argument("--ms", default="20")
    ap.add_argument("--rotating-mb", default="1024")
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    # continue from the installed results (TunableOp reads its file at start and only tunes
    # the shapes it does not hold; device 0 writes <out stem>0.csv)
    installed = os.path.join(REPO, PKG, "tuned", "gemm_mi355x.csv")
    first = os.path.splitext(args.out)[0] + "0.csv"
    if args.resume and os.path.exists(installed) and not os.path.exists(first):
        # (--resume 0 re-measures every shape)
        shutil.copy(installed, first)
    env = dict(os.environ, PYTORCH_TUNABLEOP_ENABLED="1", PYTORCH_TUNABLEOP_TUNING="1",
               PYTORCH_TUNABLEOP_FILENAME=args.out, PYTORCH_TUNABLEOP_VERBOSE="1",
               PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=args.iters,
               PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=args.ms,
               # rotate the operands through more memory than the 256 MB Infinity Cache, so
               # each candidate is timed as the forward runs it: weights streamed from HBM
               PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE=args.rotating_mb)
    # one child per leg (each appends its new shapes to the same results file), a heartbeat
    # line every 30 s while a child tunes
    legs = [(m, ["--method", ""] if m == "e2e" else ["--e2e", "0", "--method", m])
            for m in args.legs.split(",") if m]
    rc = 0
    for name, extra in legs:
        cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--steps", "2", "--warmup",
               "1", "--beam", "", "--cpu-seconds", "0"] + extra
        t0 = time.time()
        p = subprocess.Popen(cmd, env=env, cwd=REPO)
        while p.poll() is None:
            time.sleep(30)
            print(f"tuning {name}: {time.time() - t0:.0f} s", flush=True)
        rc = rc or p.returncode
        print(f"leg {name}: rc {p.returncode}, {time.time() - t0:.0f} s", flush=True)
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
