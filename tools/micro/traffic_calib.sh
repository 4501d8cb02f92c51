#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes (GPU box, repo root): tools/micro/traffic_calib.sh OUTDIR
set -e
OUT=$(pwd)/${1:-gpurun_out/calib}
BIN=$(pwd)/tools/micro/traffic_calib
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 "$BIN" > "$OUT/bytes.json"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -T -d "$OUT/pmc_$C" -o run --output-format csv -- "$BIN" > "$OUT/pmc_$C.log" 2>&1
done
echo calib done
