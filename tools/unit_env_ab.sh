# interleaved A/B of the drop-in legs (bench.py's dropin.value and dropin.raster_unit) with one environment
# setting on / off: tools/unit_env_ab.sh OUTDIR VAR=VALUE [ROUNDS]
out=$1; kv=$2; rounds=${3:-3}
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do for t in base var; do
  env=""; [ $t = var ] && env="$kv"
  env $env timeout -k 10 300 python bench.py --cpu-baseline off --fisher off --mapping off --configs off --unfused-leg off --stage-breakdown off --sequence off > "$out/d_${t}_$r.json" 2>&1 || exit 1
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])['dropin']; print('unit', sys.argv[2], sys.argv[3], d['raster_unit']['value'], d['value'])" "$out/d_${t}_$r.json" $t $r | tee -a "$out/ab.txt"
done; done
