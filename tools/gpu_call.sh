#!/bin/bash
# Generic GPU session used during round 2: GPU tests, headline bench, drop-in leg, SQ passes.
# Usage: tools/gpu_call.sh TAG [steps...]   steps: tests bench dropin map sq
TAG=${1:-x}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for s in "$@"; do
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo "tests failed rc=$?"; tail -30 "$OUT/tests.log"; exit 1; } ;;
    bench) timeout -k 10 300 python bench.py --dropin off > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -30 "$OUT/bench.log"; exit 1; } ;;
    dropin) timeout -k 10 300 python bench.py --cpu-baseline off > "$OUT/bench_dropin.log" 2>&1 || { echo "dropin failed"; tail -30 "$OUT/bench_dropin.log"; exit 1; } ;;
    map) timeout -k 10 300 python bench.py --workload mapping --cpu-baseline off > "$OUT/bench_map.log" 2>&1 || { echo "map failed"; tail -30 "$OUT/bench_map.log"; exit 1; } ;;
    sq) bash tools/pmc_sq.sh "$OUT/sq" || { echo "sq failed"; exit 1; } ;;
    *) echo "unknown step $s"; exit 1 ;;
  esac
  echo "step $s ok"
done
