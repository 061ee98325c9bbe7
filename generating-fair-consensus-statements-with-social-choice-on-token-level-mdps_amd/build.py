"""In-tree build of the gfx950 HIP library (no JIT cache: the .so travels with the repo).

Seven translation units (csrc/*.hip, sharing csrc/cs_kernels.cuh) compile in parallel to
objects, then link into libconsensus_scoring.so."""
from __future__ import annotations

import hashlib
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_HERE)
_CSRC = os.path.join(_HERE, "csrc")
SOURCES = [os.path.join(_CSRC, n) for n in ("stream.hip", "fold.hip", "proposer.hip", "beam.hip", "attn.hip", "norm.hip", "gemm.hip")]
HEADERS = [os.path.join(_CSRC, "cs_kernels.cuh"), os.path.join(_REPO, "include", "consensus_scoring.h")]
OUT = os.path.join(_HERE, "libconsensus_scoring.so")
ARCH = os.environ.get("CS_OFFLOAD_ARCH", "gfx950")


STAMP = OUT + ".srchash"


def source_hash() -> str:
    """sha256 over every source and header the library is built from (in a fixed order)."""
    h = hashlib.sha256()
    for p in SOURCES + HEADERS:
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode() + b"\0" + f.read())
    return h.hexdigest()


def built_hash() -> str:
    try:
        with open(STAMP) as f:
            return f.read().strip()
    except OSError:
        return ""


def needs_build() -> bool:
    return not os.path.exists(OUT) or built_hash() != source_hash()


def _flags():
    # -ffp-contract=off: every FMA in the kernels is an explicit fmaf, so kernels that
    # share a formula (lse, gather, soft-cap) round identically wherever they are inlined
    return ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-ffp-contract=off", "-fPIC",
            "-I", os.path.join(_REPO, "include"), "-I", _CSRC]


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objs = [OUT + "." + os.path.basename(s) + ".o" for s in SOURCES]
    if os.path.exists(STAMP):         # a failed build must not leave a stale stamp behind
        os.remove(STAMP)
    cmds = [[hipcc] + _flags() + ["-c", s, "-o", o] for s, o in zip(SOURCES, objs)]
    if verbose:
        for c in cmds:
            print(" ".join(c))
    jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with ThreadPoolExecutor(jobs) as ex:
        for r in ex.map(lambda c: subprocess.run(c, check=True), cmds):
            pass
    link = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT + ".tmp"] + objs
    if verbose:
        print(" ".join(link))
    subprocess.run(link, check=True)
    os.replace(OUT + ".tmp", OUT)
    for o in objs:
        os.remove(o)
    with open(STAMP, "w") as f:       # the sources this library was built from
        f.write(source_hash() + "\n")
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
