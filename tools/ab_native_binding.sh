set -e
OUT=gpurun_out/r8d; mkdir -p $OUT
for r in 1 2; do for v in 0 1; do
  GSR_NATIVE_BINDING=$v timeout -k 10 400 python bench.py --cpu-baseline off --fisher off --mapping off --configs off --unfused-leg off > $OUT/nat_${v}_$r.log 2>&1
  python - $OUT/nat_${v}_$r.log $v $r <<'PY'
import json, sys
b = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = b["dropin"]
print("native", sys.argv[2], "round", sys.argv[3], "dropin", d["value"], "raster_unit", d["raster_unit"]["value"], "ms", d["raster_unit"]["ms_per_step"])
PY
done; done | tee $OUT/abnat.txt
