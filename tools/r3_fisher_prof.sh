#!/bin/bash
# rocprofv3 kernel stats of the Fisher pipeline alone (GPU box, repo root).
OUT=$(pwd)/gpurun_out/${1:-fprof}; mkdir -p "$OUT"; ROOT=$(pwd)
timeout -k 10 120 python tools/fisher_bench.py > "$OUT/fisher.log" 2>&1 || { tail -20 "$OUT/fisher.log"; exit 1; }
cat "$OUT/fisher.log" | tail -1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python "$ROOT/tools/fisher_bench.py" --launches 10 > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
python - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/prof/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print(r["Name"].split("(")[0][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), round(float(r["Percentage"]), 1))
PY
