# Experiment: per-kernel time vs micro-batch size (does pass 2 read pass 1's output from the Infinity Cache?)
set -o pipefail
mkdir -p gpurun_out/batch_sweep
for B in 50000000 10000000 5000000 2500000; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --batch $B --h2d-records 0 \
      > gpurun_out/batch_sweep/b$B.log 2>&1 || { echo "batch $B failed"; exit 1; }
done
echo sweep-done
