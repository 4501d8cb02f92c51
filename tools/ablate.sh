#!/bin/bash
# Timing ablations of render_bwd (GPU box, repo root): tools/raster_bench.py (config 3, tracking-style
# dual_lean rasterization) against each prebuilt splatam_amd/_diag/libgsr_<tag>.so
# (python -c 'from splatam_amd import build; build.build_variant(tag, defines)' on the CPU first).
# Usage: tools/ablate.sh OUTDIR tag...
OUT=$1; shift
mkdir -p "$OUT"
timeout -k 10 120 python tools/raster_bench.py --iters 40 > "$OUT/base.json" 2>&1 || exit 1
for t in "$@"; do
  GSR_LIB=splatam_amd/_diag/libgsr_$t.so timeout -k 10 120 python tools/raster_bench.py --iters 40 \
      > "$OUT/$t.json" 2>&1 || { echo "variant $t failed"; exit 1; }
done
echo ablate done
