# Runs a subset of the GPU parity tests against variant libraries (experiment only)
# usage: bash scripts/test_variants.sh "<pytest -k expr>" lib1 lib2 ...
set -o pipefail
mkdir -p gpurun_out
K=$1; shift
for v in "$@"; do
  echo "== $v"
  LIB=$PWD/flink_amd/libflinkgpu_$v.so
  [ "$v" = main ] && LIB=$PWD/flink_amd/libflinkgpu.so
  FLINKGPU_LIB=$LIB timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 \
     --timeout-method thread -k "$K" > gpurun_out/tv_$v.log 2>&1
  tail -3 gpurun_out/tv_$v.log
done
