#!/bin/bash
# One GPU session (GPU box, repo root): any of
#   tests    the GPU suite (pytest -m gpu)
#   bench    the default bench line (dropin / cpu baseline off)
#   full     the default bench line exactly as the driver runs it
#   prof     rocprofv3 kernel trace + stats of the headline bench
#   map      the mapping bench leg alone
#   lock     lockstep / padding statistics of render_bwd's row lists (configs 3, 4)
# Usage: tools/gpu_round.sh TAG step...   (stops at the first failing step)
TAG=${1:-x}; shift
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
for s in "$@"; do
  case $s in
    tests) timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 \
             || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; } ;;
    bench) timeout -k 10 300 python bench.py --dropin off --cpu-baseline off > "$OUT/bench.log" 2>&1 \
             || { echo "bench failed"; tail -30 "$OUT/bench.log"; exit 1; } ;;
    full) timeout -k 10 400 python bench.py > "$OUT/full.log" 2>&1 || { echo "full bench failed"; tail -30 "$OUT/full.log"; exit 1; } ;;
    prof) ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run \
             --output-format csv -- python "$ROOT/bench.py" --steps 40 --warmup 20 --cpu-baseline off --dropin off \
             --fisher off --mapping off > "$OUT/prof.log" 2>&1 ) || { echo "prof failed"; tail -20 "$OUT/prof.log"; exit 1; } ;;
    map) timeout -k 10 300 python bench.py --workload mapping --cpu-baseline off > "$OUT/map.log" 2>&1 \
             || { echo "map failed"; tail -30 "$OUT/map.log"; exit 1; } ;;
    stream) timeout -k 10 120 tools/micro/stream > "$OUT/stream.json" 2>&1 || { echo "stream failed"; exit 1; } ;;
    lock) timeout -k 10 200 python tools/lockstep_stats.py 3 128 > "$OUT/lockstep3.txt" 2>&1 && \
          timeout -k 10 200 python tools/lockstep_stats.py 4 128 > "$OUT/lockstep4.txt" 2>&1 || { echo "lock failed"; exit 1; } ;;
    *) echo "unknown step $s"; exit 1 ;;
  esac
  echo "step $s ok"
done
python - "$OUT" <<'PY'
import csv, glob, json, os, sys
out = sys.argv[1]
for f in glob.glob(f"{out}/prof/**/run_kernel_stats.csv", recursive=True)[:1]:
    for r in list(csv.DictReader(open(f)))[:8]:
        print(r["Name"].split("(")[0][:48], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
for name in ("bench.log", "full.log", "map.log"):
    p = os.path.join(out, name)
    if os.path.exists(p):
        ls = [l for l in open(p) if l.startswith("{")]
        if ls:
            b = json.loads(ls[-1])
            rf = b.get("roofline", {})
            print(name, "value", b["value"], b["unit"], "render_bwd", rf.get("avg_us"), "frac", rf.get("frac"))
for name in ("lockstep3.txt", "lockstep4.txt", "stream.json"):
    p = os.path.join(out, name)
    if os.path.exists(p):
        print(open(p).read())
t = os.path.join(out, "tests.log")
if os.path.exists(t):
    print(open(t).read().strip().split("\n")[-1])
PY
