# Round-6 measurements on one GPU box: the driver's default bench command (CPU leg included), then
# each workload's bench line, then the N = 2 rehearsal of a workload's two-phase path on one device.
# Usage: bash scripts/round6_bench.sh TAG [rehearsal workload]
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 500 python bench.py > $O/bench_default.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_default.log; exit 1; }
tail -c 300 $O/bench_default.log; echo
for W in hop cumulate zipf datastream strings; do
  timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --h2d-records 0 > $O/wl_$W.log 2>&1 || { echo "bench $W failed"; tail -5 $O/wl_$W.log; exit 1; }
  python - $O/wl_$W.log $W <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ks = sorted(d["kernels_warmup"].items(), key=lambda kv: -kv[1]["total_ms"])[:3]
print("%-10s %.4g rec/s  %.2f ms/step  job %.3f  " % (sys.argv[2], d["value"], d["ms_per_step"], d["job_roofline"]["frac"])
      + "  ".join("%s %d x %.3f" % (k, v["launches"], v["avg_ms"]) for k, v in ks))
PY
done
if [ -n "$2" ]; then
  export BENCH_DIST_BACKEND=gloo BENCH_DEVICE=0 MASTER_ADDR=127.0.0.1
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
      bench.py --gpus 2 --workload $2 --records ${REC:-200000000} --steps 2 --warmup 1 --no-cpu-baseline \
      > $O/rehearse_2rank_$2.log 2>&1 || { echo "rehearsal failed"; tail -20 $O/rehearse_2rank_$2.log; exit 1; }
  tail -c 600 $O/rehearse_2rank_$2.log
fi
echo bench-done
