#!/bin/bash
# Kernel iteration loop on the GPU box: rasterizer-only timing, then the parity tests that cover
# render_bwd.  Usage: tools/quick_bwd.sh OUTDIR [pytest -k expr]
OUT=$1; K=${2:-"parity or configs or slam"}
mkdir -p "$OUT"
timeout -k 10 120 python tools/raster_bench.py --iters 40 > "$OUT/raster.json" 2>&1 || { echo "raster_bench failed"; tail -20 "$OUT/raster.json"; exit 1; }
grep -v amdgpu "$OUT/raster.json"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "$K" --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
