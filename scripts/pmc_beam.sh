#!/usr/bin/env bash
# PMC HBM traffic of the beam decode launches: FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 passes over a short bench run, ONE beam config per run (the 1-GPU and per-rank
# shapes share kernel instantiations, so each run's beam_decode_kernel launches are its own).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT="$R/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in ${BEAMS:-c1 c3 c5 r8c3 r8c5}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $c -d "$OUT/pmc_beam_${cfg}_$c" -o run -f csv -- \
       python3 "$R/bench.py" --steps 1 --warmup 1 --cpu-seconds 0 --beam "$cfg" --beam-steps 10 \
       --e2e 0 --method "" --method-bon 0 > "$OUT/pmc_beam_${cfg}_$c.log" 2>&1) || exit $?
  done
done
