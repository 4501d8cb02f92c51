#!/bin/bash
# Same-box A/B of the drop-in leg with and without the geometry reuse (GSR_GEOM_CACHE).
OUT=${1:-gpurun_out/abdrop}
mkdir -p "$OUT"
for r in on off on2 off2; do
  v=1; case $r in off*) v=0;; esac
  GSR_GEOM_CACHE=$v timeout -k 10 300 python bench.py --cpu-baseline off --fisher off --steps 20 > "$OUT/$r.log" 2>&1 || { echo "$r failed"; tail -20 "$OUT/$r.log"; exit 1; }
  python - "$OUT/$r.log" "$r" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)["dropin"]
        print(sys.argv[2], "dropin", d["value"], "raster_unit", d["raster_unit"]["value"], "stages", d["stages_us"])
PY
done
