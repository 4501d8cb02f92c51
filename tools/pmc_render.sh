#!/bin/bash
# Collect PMC counters for the render kernels, one rocprofv3 pass per counter group.
# Usage: tools/pmc_render.sh OUTDIR
set -e
OUT=${1:-gpurun_out/pmc}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex 'render|gauss_bwd|tile_sort|preprocess|duplicate|scan_counts' -T \
     -d "$ROOT/$OUT/p$i" -o run --output-format csv -- python "$ROOT/tools/raster_bench.py" --iters 4 --warmup 1 \
     > "$ROOT/$OUT/p$i.log" 2>&1
done < "$ROOT/tools/pmc_groups.txt"
