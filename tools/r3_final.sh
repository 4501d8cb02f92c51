#!/bin/bash
# Round-3 close on the GPU box (repo root): tools/r3_check.sh (GPU suite, smoke, default bench line), then the
# rocprofv3 kernel statistics of the same default bench command.  Usage: tools/r3_final.sh TAG
TAG=${1:-final}; ROOT=$(pwd)
bash tools/r3_check.sh "$TAG" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/$TAG/prof" -o run --output-format csv -- \
    python "$ROOT/bench.py" --steps 20 --warmup 5 > "$ROOT/gpurun_out/$TAG/prof_bench.log" 2>&1 || { echo "rocprof failed"; exit 1; }
f=$(ls "$ROOT"/gpurun_out/$TAG/prof/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find "$ROOT/gpurun_out/$TAG/prof" -name run_kernel_stats.csv | head -1)
head -12 "$f" | cut -c1-160
