# Round-6 evidence of the final build, in three GPU calls (each within one call's limit):
#   bash scripts/round6_final.sh suite TAG     every GPU test + smoke()
#   bash scripts/round6_final.sh bench TAG     the driver's default bench (CPU leg) + each workload + N=2 rehearsals
#   bash scripts/round6_final.sh prof TAG      kernel trace + PMC passes per workload (scripts/profile.sh)
set -o pipefail
O=gpurun_out/$2
mkdir -p $O
case $1 in
suite) bash scripts/gpu_suite.sh $2 ;;
bench)
  bash scripts/round6_bench.sh $2 || exit 1
  REC=200000000 BENCH_ARGS="" bash scripts/rehearse_2rank.sh > $O/rehearse_2rank_tumble.log 2>&1 || { echo "rehearsal failed"; tail -5 $O/rehearse_2rank_tumble.log; exit 1; }
  tail -c 300 $O/rehearse_2rank_tumble.log ;;
prof)
  for W in tumble hop cumulate zipf; do
    WL=$W timeout -k 10 560 bash scripts/profile.sh $2_$W 200000000 || { echo "profile $W failed"; exit 1; }
  done
  echo prof-done ;;
esac
