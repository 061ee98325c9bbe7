#!/usr/bin/env bash
# PMC HBM traffic of the beam decode launches (C1 / C3 / C5): FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 passes over a short bench run (beam configs only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT="$R/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $c -d "$OUT/pmc_beam_$c" -o run -f csv -- \
     python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-seconds 0 --beam-steps 10 --e2e 0 --method "" --method-bon 0 \
     > "$OUT/pmc_beam_$c.log" 2>&1) || exit $?
done
