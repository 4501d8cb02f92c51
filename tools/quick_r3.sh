#!/bin/bash
# Round-3 quick GPU check (GPU box, repo root): GPU tests, render_bwd phase breakdown, bench without the
# slow legs.  Usage: tools/quick_r3.sh TAG [notests]
TAG=${1:-q}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
if [ "$2" != notests ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; }
  tail -1 "$OUT/tests.log"
fi
if [ -f splatam_amd/_diag/libgsr_phase.so ]; then
  timeout -k 10 120 python tools/phase_bwd.py 3 10 > "$OUT/phase.log" 2>&1 || { echo "phase failed"; tail -20 "$OUT/phase.log"; exit 1; }
  grep config "$OUT/phase.log"
fi
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --cpu-baseline off --dropin off --fisher off > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
python - "$OUT/bench.log" <<'PY'
import json, sys
b = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print("tracking", b["value"], "render_bwd", b["roofline"]["avg_us"], "render_fwd", b["stages_us"]["render_fwd"],
      "| mapping", b["mapping"]["value"], "render_bwd", b["mapping"]["roofline"]["avg_us"], "render_fwd", b["mapping"]["stages_us"]["render_fwd"])
PY
