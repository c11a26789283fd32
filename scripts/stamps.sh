set -o pipefail
FG_STAMPS=1 FLINKGPU_LIB=$PWD/flink_amd/libflinkgpu_stamps.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 1 --warmup 0 --records 300000000 > gpurun_out/stamps.log 2>&1
grep "fg stamps" gpurun_out/stamps.log | head -8
