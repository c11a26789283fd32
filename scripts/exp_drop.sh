set -o pipefail
mkdir -p gpurun_out
for d in 0 1 2; do
  FG_STAGE_DROP=$d timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_drop$d.log 2>&1 || exit 1
done
echo done
