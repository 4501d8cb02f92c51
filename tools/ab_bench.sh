#!/bin/bash
# A/B of the headline (and mapping) bench between libgsr.so and a variant library built by
# splatam_amd.build.build_variant(TAG, defines).  Usage (GPU box): tools/ab_bench.sh OUTDIR TAG [notrk|nomap]
OUT=$1; TAG=$2; SKIP=${3:-}
mkdir -p "$OUT"
run_one() {  # name lib
  if [ "$SKIP" != notrk ]; then
    GSR_LIB=$2 timeout -k 10 200 python bench.py --cpu-baseline off --dropin off --fisher off > "$OUT/trk_$1.log" 2>&1 || { echo "tracking $1 failed"; tail -20 "$OUT/trk_$1.log"; return 1; }
  fi
  if [ "$SKIP" != nomap ]; then
    GSR_LIB=$2 timeout -k 10 200 python bench.py --workload mapping --cpu-baseline off > "$OUT/map_$1.log" 2>&1 || { echo "mapping $1 failed"; tail -20 "$OUT/map_$1.log"; return 1; }
  fi
}
BASE=splatam_amd/libgsr.so
VAR=splatam_amd/_diag/libgsr_$TAG.so
run_one base $BASE && run_one var $VAR && run_one base2 $BASE || exit 1
grep -o '"value": [0-9.]*\|"avg_us": [0-9.]*' "$OUT"/*.log
