#!/bin/bash
# One GPU profiling session: bench line, rocprofv3 kernel trace + stats, separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) for the hot kernels, and (headline workload) the SQ passes of the
# render kernels.  Usage (GPU box, repo root): tools/profile_round.sh TAG [bench args...]
#   tools/profile_round.sh r2a                      # headline tracking bench
#   tools/profile_round.sh r2am --workload mapping  # mapping workload
set -e
TAG=${1:-r2}
shift || true
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 500 python bench.py "$@" > "$OUT/bench.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv \
    -- python "$ROOT/bench.py" "$@" --steps 40 --warmup 20 --cpu-baseline off --dropin off --fisher off --mapping off > "$OUT/trace.log" 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-include-regex 'render_|gauss_bwd|tile_sort|duplicate|preprocess|sh_|map_' -T \
      -d "$OUT/pmc_$C" -o run --output-format csv \
      -- python "$ROOT/bench.py" "$@" --steps 20 --warmup 20 --cpu-baseline off --dropin off --fisher off --mapping off > "$OUT/pmc_$C.log" 2>&1
done
cd "$ROOT"
if [ $# -eq 0 ]; then bash tools/pmc_sq.sh "gpurun_out/$TAG/sq"; fi
echo profile_round done
