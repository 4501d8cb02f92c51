#!/bin/bash
# SQ issue / wait / LDS counters of render_bwd_fisher_kernel (GPU box, repo root), one rocprofv3 pass per
# group (<= 8 SQ counters each), then the same for the tracking render_bwd for comparison.
# Usage: tools/pmc_fisher.sh OUTDIR
OUT=${1:-gpurun_out/sqf}
ROOT=$(pwd)
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
G2="SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
i=0
for G in "$G1" "$G2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G --kernel-include-regex 'render_bwd' -T \
     -d "$ROOT/$OUT/sq$i" -o run --output-format csv \
     -- python "$ROOT/tools/fisher_bench.py" --launches 4 > "$ROOT/$OUT/sq$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$ROOT/$OUT/sq$i.log"; exit 1; }
done
cd "$ROOT" && python tools/sq_summary.py "$OUT" > "$OUT/summary.json" && echo pmc_fisher done
