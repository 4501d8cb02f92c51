#!/bin/bash
# Per-kernel A/B of the mapping bench (GPU box, repo root): rocprofv3 kernel stats with libgsr.so and with
# each splatam_amd/_diag/libgsr_<tag>.so, then base again.  Usage: tools/ab_map_kernels.sh OUTDIR TAG...
OUT=$1; shift; TAGS="$*"; ROOT=$(pwd)
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
for v in base $TAGS base2; do
  L=$ROOT/splatam_amd/libgsr.so; [ $v != base ] && [ $v != base2 ] && L=$ROOT/splatam_amd/_diag/libgsr_$v.so
  GSR_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/$v" -o run --output-format csv \
      -- python "$ROOT/bench.py" --workload mapping --steps 40 --warmup 20 --cpu-baseline off > "$ROOT/$OUT/$v.log" 2>&1 \
      || { echo "$v failed"; tail -20 "$ROOT/$OUT/$v.log"; exit 1; }
done
cd "$ROOT"
python - "$OUT" base $TAGS base2 <<'PY'
import csv, glob, json, sys
for v in sys.argv[2:]:
    f = glob.glob(f"{sys.argv[1]}/{v}/**/run_kernel_stats.csv", recursive=True)[0]
    rows = {r["Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0][-28:]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f))}
    b = [json.loads(l) for l in open(f"{sys.argv[1]}/{v}.log") if l.startswith("{")][-1]
    print(v, round(b["value"], 1), {k: round(x, 1) for k, x in rows.items() if any(s in k for s in ("render", "gauss", "dupl", "prepro", "colscan", "sh_", "map_"))})
PY
