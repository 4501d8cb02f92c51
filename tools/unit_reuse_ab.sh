# interleaved A/B of the drop-in unit (bench.py's dropin.raster_unit) with the geometry reuse on / off
mkdir -p gpurun_out/r10i
for r in 1 2; do for t in gated off; do
  env=""; [ $t = off ] && env="GSR_GEOM_CACHE=0"
  env $env timeout -k 10 300 python bench.py --cpu-baseline off --fisher off --mapping off --configs off --unfused-leg off --stage-breakdown off --sequence off > gpurun_out/r10i/d_${t}_$r.json 2>&1 || exit 1
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])['dropin']; print('unit', sys.argv[2], sys.argv[3], d['raster_unit']['value'], d['value'])" gpurun_out/r10i/d_${t}_$r.json $t $r | tee -a gpurun_out/r10i/ab.txt
done; done
