set -e
O=gpurun_out/wbb; mkdir -p $O
for v in base var base2; do
  L=splatam_amd/libgsr.so; [ $v = var ] && L=splatam_amd/_build_wbb96/libgsr_wbb96.so
  GSR_LIB=$L timeout -k 10 120 python tools/raster_bench.py --mode single --iters 40 > $O/single_$v.json 2>&1
  GSR_LIB=$L timeout -k 10 200 python bench.py --workload mapping --cpu-baseline off > $O/map_$v.log 2>&1
done
echo done
