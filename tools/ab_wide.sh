#!/bin/bash
# A/B of the wide render_bwd variants (GPU box, repo root): the default bench (tracking, drop-in, mapping legs)
# with libgsr.so and each splatam_amd/_diag/libgsr_<tag>.so, interleaved twice.  Usage: tools/ab_wide.sh OUTDIR TAG...
OUT=$1; shift; TAGS="$*"
mkdir -p "$OUT"
for r in 1 2; do
  for v in base $TAGS; do
    L=splatam_amd/libgsr.so; [ $v != base ] && L=splatam_amd/_diag/libgsr_$v.so
    GSR_LIB=$L timeout -k 10 300 python bench.py --cpu-baseline off --fisher off --steps 20 > "$OUT/${v}_$r.log" 2>&1 \
        || { echo "$v failed"; tail -20 "$OUT/${v}_$r.log"; exit 1; }
    python - "$OUT/${v}_$r.log" "${v}_$r" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(sys.argv[2], "track", round(d["value"], 1), "bwd", d["roofline"]["avg_us"],
      "| dropin bwd", d["dropin"]["render_bwd"]["avg_us"], "unit", round(d["dropin"]["raster_unit"]["value"], 1),
      "| mapping", round(d["mapping"]["value"], 1), "bwd", d["mapping"]["roofline"]["avg_us"],
      "| dropin_map", round(d["mapping"]["dropin"]["value"], 1))
PY
  done
done
