#!/bin/bash
# Fisher path check (GPU box): the Fisher GPU tests, then the bench's fisher leg alone.
OUT=gpurun_out/${1:-fis}; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_fisher.py -x -v -s -m gpu --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; }
grep -E "rel L2|passed|failed" "$OUT/tests.log"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off --dropin off --mapping off > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
python - "$OUT/bench.log" <<'PY'
import json, sys
b = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print("tracking", b["value"], "fisher", b["fisher"])
PY
