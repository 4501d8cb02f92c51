#!/bin/bash
# GPU tests + tracking and mapping bench lines into gpurun_out/$1 (one gpurun call).
set -e
OUT=gpurun_out/${1:-q}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
timeout -k 10 200 python bench.py --cpu-baseline off > "$OUT/bench.log" 2>&1
timeout -k 10 200 python bench.py --workload mapping --cpu-baseline off > "$OUT/bench_map.log" 2>&1
