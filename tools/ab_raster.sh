#!/bin/bash
# Interleaved A/B of render stages (GPU box, repo root): tools/raster_bench.py on libgsr.so and on each
# splatam_amd/_diag/libgsr_<tag>.so, two rounds.  Usage: tools/ab_raster.sh OUTDIR "MODE:CONFIG ..." tag...
OUT=$1; CASES=$2; shift 2
mkdir -p "$OUT"
for r in 1 2; do
  for t in base "$@"; do
    L=splatam_amd/libgsr.so; [ $t != base ] && L=splatam_amd/_diag/libgsr_$t.so
    for c in $CASES; do
      m=${c%%:*}; cf=${c##*:}
      GSR_LIB=$L timeout -k 10 120 python tools/raster_bench.py --iters 60 --mode $m --config $cf > "$OUT/${t}_${m}_${cf}_$r.json" 2>&1 || { echo "$t $c failed"; tail -5 "$OUT/${t}_${m}_${cf}_$r.json"; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stages_us']; print(sys.argv[2], sys.argv[3], 'bwd', s['render_bwd'], 'fwd', s['render_fwd'], 'gauss', s['gauss_bwd'], 'ms', round(d['ms_per_frame'],4))" "$OUT/${t}_${m}_${cf}_$r.json" $t $c
    done
  done
done
