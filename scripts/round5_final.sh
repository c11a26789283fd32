# Round-5 evidence on one GPU box: every GPU test, smoke(), the driver's default bench command
# (CPU leg included), then each workload's bench line. Stops at the first failure.
# Usage: bash scripts/round5_final.sh TAG
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 500 python bench.py > $O/bench_default.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_default.log; exit 1; }
tail -c 400 $O/bench_default.log
for W in hop cumulate zipf datastream strings; do
  timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --h2d-records 0 > $O/wl_$W.log 2>&1 || { echo "bench $W failed"; tail -5 $O/wl_$W.log; exit 1; }
  python - $O/wl_$W.log $W <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("%-10s %.4g rec/s  %.2f ms/step  job %.3f  kernel %s %.3f" % (sys.argv[2], d["value"], d["ms_per_step"],
      d["job_roofline"]["frac"], d["roofline"]["kernel"], d["roofline"]["frac"]))
PY
done
echo final-done
