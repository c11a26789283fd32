mkdir -p gpurun_out/${AB_TAG:-r5h}
for v in ${AB_VARIANTS:-default pipe3 tile_block cond_loads}; do
  if [ $v = default ]; then L=$PWD/flink_amd/libflinkgpu.so; else L=$PWD/flink_amd/var/lib_$v.so; fi
  FLINKGPU_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-records 0 --records 300000000 --steps 3 --warmup 1 > gpurun_out/${AB_TAG:-r5h}/b_$v.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/${AB_TAG:-r5h}/b_$v.log').read().strip().split(chr(10))[-1]); k=d['kernels_warmup']; print('$v', round(d['ms_per_step'],3), {n:round(x['avg_ms'],4) for n,x in k.items()})"
done
