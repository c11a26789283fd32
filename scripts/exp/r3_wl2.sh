# Round 3 late: HOP (33.3M-record batches) and STRING keys (100M) at their new defaults, + the headline again
set -o pipefail
O=gpurun_out/r03late2
mkdir -p $O
for w in hop strings; do
  timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --h2d-records 0 > $O/wl_$w.log 2>&1 || { tail -20 $O/wl_$w.log; exit 1; }
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --h2d-records 0 > $O/bench_headline.log 2>&1 || exit 1
echo done
