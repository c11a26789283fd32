# The bench lines of round4_final.sh alone (the driver's default command, CPU leg included, then
# each workload), e.g. after the PMC summaries of the same build are committed. Usage: bash scripts/round4_benches.sh TAG
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 500 python bench.py > $O/bench_default.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_default.log; exit 1; }
tail -c 300 $O/bench_default.log
for W in hop cumulate zipf datastream strings; do
  timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --h2d-records 0 > $O/wl_$W.log 2>&1 || { echo "bench $W failed"; tail -5 $O/wl_$W.log; exit 1; }
done
echo benches-done
