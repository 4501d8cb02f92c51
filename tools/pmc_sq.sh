#!/bin/bash
# SQ issue/wait counters for the render kernels of the headline bench (one rocprofv3 pass per group,
# at most 8 SQ counters each).  Usage (GPU box, repo root): tools/pmc_sq.sh OUTDIR [bench args...]
set -e
OUT=${1:-gpurun_out/sq}
shift || true
ROOT=$(pwd)
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
G2="SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
G3="SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for G in "$G1" "$G2" "$G3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex 'render_' -T \
     -d "$ROOT/$OUT/sq$i" -o run --output-format csv \
     -- python "$ROOT/bench.py" --steps 20 --warmup 20 --cpu-baseline off --dropin off --fisher off --mapping off "$@" > "$ROOT/$OUT/sq$i.log" 2>&1
done
echo pmc_sq done
