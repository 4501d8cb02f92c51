#!/bin/bash
# Raster-unit A/B of the host-path switches (GPU box): geometry reuse and camera-copy cache on/off,
# interleaved, then a cProfile of the default path.
OUT=gpurun_out/${1:-unitab}; mkdir -p "$OUT"
for r in 1 2; do
  for gc in 1 0; do
    for cc in 1 0; do
      GSR_GEOM_CACHE=$gc GSR_CAM_CACHE=$cc timeout -k 10 120 python tools/unit_cprofile.py --n 300 --no-profile > "$OUT/u_${gc}${cc}_$r.log" 2>&1 || { tail -5 "$OUT/u_${gc}${cc}_$r.log"; exit 1; }
      echo "geom_cache=$gc cam_cache=$cc: $(grep 'unit ' "$OUT/u_${gc}${cc}_$r.log")"
    done
  done
done
timeout -k 10 120 python tools/unit_cprofile.py --n 300 > "$OUT/cprof.log" 2>&1 || exit 1
