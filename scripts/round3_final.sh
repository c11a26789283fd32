# Round-3 final evidence (late build) on one GPU box.
#   A: every GPU test, the driver-style bench command (20 steps, CPU baseline, h2d leg), one line per
#      other workload;  B: the profile recipe (kernel trace + PMC passes) for TUMBLE/HOP/CUMULATE with
#      PMC traffic keyed by the library's sha256, and the 2-rank rehearsal of the N > 1 path.
# Usage: bash scripts/round3_final.sh A|B [out dir]
set -o pipefail
O=${2:-gpurun_out/r03late}
mkdir -p $O
if [ "$1" = A ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
      > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
  for w in hop cumulate zipf strings datastream; do
    timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --h2d-records 0 \
        > $O/wl_$w.log 2>&1 || { tail -20 $O/wl_$w.log; exit 1; }
  done
  echo part-A-done
else
  for w in tumble hop cumulate; do
    tag=r03late_$w
    if [ $w = tumble ]; then WL= bash scripts/profile.sh $tag 200000000 || exit 1
    else WL=$w bash scripts/profile.sh $tag 300000000 || exit 1; fi
    python3 profiles/pmc_summary.py "gpurun_out/prof_$tag/pmc*/run_counter_collection.csv" \
        gpurun_out/prof_$tag/pmc_traffic.json flink_amd/libflinkgpu.so > gpurun_out/prof_$tag/pmc_summary.txt || exit 1
  done
  REC=200000000 bash scripts/rehearse_2rank.sh > /dev/null || { echo rehearsal failed; exit 1; }
  cp gpurun_out/rehearse_2rank.log $O/rehearse_2rank.log
  echo part-B-done
fi
