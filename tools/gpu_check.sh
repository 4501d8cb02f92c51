#!/bin/bash
# GPU suite + rocprof kernel stats of the headline bench + the full bench line (GPU box, repo root).
# Usage: tools/gpu_check.sh TAG
TAG=${1:-chk}; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python "$ROOT/bench.py" \
    --steps 40 --warmup 20 --cpu-baseline off --dropin off --fisher off --mapping off > "$OUT/prof.log" 2>&1 || exit 1
cd "$ROOT"
timeout -k 10 300 python bench.py --dropin off --cpu-baseline off --fisher off > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
python - "$OUT" <<'PY'
import csv, glob, json, sys
f = glob.glob(f"{sys.argv[1]}/prof/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:6]:
    print(r["Name"].split("(")[0][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
b = [json.loads(l) for l in open(f"{sys.argv[1]}/bench.log") if l.startswith("{")][-1]
print("value", b["value"], "render_bwd", b["roofline"]["avg_us"], "mapping", b["mapping"]["value"])
PY
tail -1 "$OUT/tests.log"
