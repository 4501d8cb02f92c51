#!/bin/bash
# Unchanged-caller path check (GPU box): GPU suite, raster-unit host/device profile, bench dropin leg.
OUT=gpurun_out/${1:-dropin}; mkdir -p "$OUT"
if [ "$2" != notests ]; then
  timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; }
  tail -1 "$OUT/tests.log"
fi
timeout -k 10 200 python tools/raster_unit_profile.py --n 200 > "$OUT/unit.log" 2>&1 || { echo "unit profile failed"; tail -20 "$OUT/unit.log"; exit 1; }
head -3 "$OUT/unit.log"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline off --fisher off --mapping off > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
python - "$OUT/bench.log" <<'PY'
import json, sys
b = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = b["dropin"]
print("tracking", b["value"], "| dropin", d["value"], "render_bwd", d["render_bwd"]["avg_us"], "raster_unit", d["raster_unit"]["value"], d["raster_unit"]["ms_per_step"])
PY
