#!/bin/bash
# SQ issue / wait counters (two rocprofv3 passes, <= 8 SQ counters each) of the headline bench's kernels
# matching REGEX.  Usage (GPU box, repo root): tools/pmc_sq_kernel.sh REGEX OUTDIR [bench args...]
RX=$1; OUT=$2; shift 2
ROOT=$(pwd)
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
G2="SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
i=0
for G in "$G1" "$G2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex "$RX" -T -d "$ROOT/$OUT/sq$i" -o run --output-format csv \
     -- python "$ROOT/bench.py" --steps 20 --warmup 20 --cpu-baseline off --dropin off --fisher off --mapping off "$@" \
     > "$ROOT/$OUT/sq$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$ROOT/$OUT/sq$i.log"; exit 1; }
done
cd "$ROOT" && python tools/sq_summary.py "$OUT" > "$OUT/summary.json" && echo pmc_sq_kernel done
