#!/bin/bash
# One GPU session: GPU tests, default bench line, rocprofv3 kernel trace + stats,
# and separate PMC passes (FETCH_SIZE, WRITE_SIZE) for the hot kernels.
# Usage (on the GPU box, from the repo root): tools/profile_round.sh TAG [bench args...]
#   tools/profile_round.sh r1g                      # headline tracking bench (+ GPU tests)
#   tools/profile_round.sh r1m --workload mapping   # mapping workload (no tests)
set -e
TAG=${1:-r1}
shift || true
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
if [ $# -eq 0 ]; then
  timeout -k 10 600 python -m pytest tests -q -m gpu > "$OUT/gpu_tests.log" 2>&1
fi
timeout -k 10 500 python bench.py "$@" > "$OUT/bench.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv \
    -- python "$ROOT/bench.py" "$@" --steps 40 --warmup 20 --cpu-baseline off > "$OUT/trace.log" 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-include-regex 'render_|gauss_bwd|tile_sort|duplicate|preprocess|sh_|map_' -T \
      -d "$OUT/pmc_$C" -o run --output-format csv \
      -- python "$ROOT/bench.py" "$@" --steps 20 --warmup 20 --cpu-baseline off > "$OUT/pmc_$C.log" 2>&1
done
echo profile_round done
