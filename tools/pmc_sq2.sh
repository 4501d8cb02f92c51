#!/bin/bash
# Second set of SQ counters for the render kernels of the headline bench: LDS / VMEM pipeline pressure and
# latency levels, VALU lane utilisation.  One rocprofv3 pass per group (<= 8 SQ counters each).
# Usage (GPU box, repo root): tools/pmc_sq2.sh OUTDIR
OUT=${1:-gpurun_out/sq2}
ROOT=$(pwd)
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LEVEL_WAVES"
G2="SQ_WAVES SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM"
G3="SQ_WAVES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU"
i=0
for G in "$G1" "$G2" "$G3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G --kernel-include-regex 'render_' -T \
     -d "$ROOT/$OUT/sq$i" -o run --output-format csv \
     -- python "$ROOT/bench.py" --steps 20 --warmup 20 --cpu-baseline off --dropin off --fisher off --mapping off > "$ROOT/$OUT/sq$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$ROOT/$OUT/sq$i.log"; exit 1; }
done
cd "$ROOT" && python tools/sq_summary.py "$OUT" > "$OUT/summary.json" && echo pmc_sq2 done
