#!/bin/bash
# Round-3 GPU check (GPU box, repo root): the -m gpu suite, smoke(), the driver's default bench line.
# Usage: tools/r3_check.sh TAG [notests]
TAG=${1:-chk}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
if [ "$2" != notests ]; then
  timeout -k 10 700 python -u -m pytest tests -x -v -m gpu -rA --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -60 "$OUT/tests.log"; exit 1; }
  tail -3 "$OUT/tests.log"
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
