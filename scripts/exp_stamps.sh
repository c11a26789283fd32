set -o pipefail
mkdir -p gpurun_out
for d in 0 2; do
  FG_STAGE_DROP=$d FG_MERGE_STAMPS=1 FLINKGPU_LIB=$PWD/flink_amd/libflinkgpu_stamps.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 1 --warmup 0 --records 200000000 > gpurun_out/stamps_drop$d.log 2>&1 || exit 1
done
echo done
