# Round 3: micro-batch sweep of the other workloads (HOP / CUMULATE / strings)
set -o pipefail
O=gpurun_out/r3s
mkdir -p $O
run() { timeout -k 10 200 python -u bench.py --workload $1 --steps 5 --warmup 2 --no-cpu-baseline --h2d-records 0 ${2:+--batch $2} $BENCH_X > $O/$1_${2:-def}${BENCH_X}.log 2>&1 || { echo "$1 $2 failed"; tail -5 $O/$1_${2:-def}.log; exit 1; }; }
run strings && run strings 100000000 && BENCH_X=--intern-serial run strings && run hop 33333334 && run hop 50000000 && run cumulate 33333334 && run cumulate 50000000 && run hop && run cumulate
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
echo done
