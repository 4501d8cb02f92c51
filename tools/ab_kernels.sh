#!/bin/bash
# Per-kernel A/B (GPU box, repo root): rocprofv3 kernel stats of the headline tracking bench with
# libgsr.so and with a variant built by splatam_amd.build.build_variant(TAG, defines).
# Usage: tools/ab_kernels.sh OUTDIR TAG [bench args...]
OUT=$1; TAG=$2; shift 2
ROOT=$(pwd)
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
for v in base var base2; do
  L=$ROOT/splatam_amd/libgsr.so
  [ $v = var ] && L=$ROOT/splatam_amd/_diag/libgsr_$TAG.so
  GSR_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/$v" -o run --output-format csv \
      -- python "$ROOT/bench.py" --steps 40 --warmup 20 --cpu-baseline off --dropin off --fisher off --mapping off "$@" \
      > "$ROOT/$OUT/$v.log" 2>&1 || { echo "$v failed"; tail -20 "$ROOT/$OUT/$v.log"; exit 1; }
done
cd "$ROOT"
python - "$OUT" <<'PY'
import csv, glob, sys
for v in ("base", "var", "base2"):
    f = glob.glob(f"{sys.argv[1]}/{v}/**/run_kernel_stats.csv", recursive=True)[0]
    rows = {r["Name"].split("(")[0][:40]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f))}
    print(v, {k: round(x, 2) for k, x in rows.items() if any(s in k for s in ("render", "gauss", "dupl", "prepro", "colscan", "sh_", "map_"))})
PY
