# Bench one workload with the shipped library and each libflinkgpu_<v>.so (experiment A/B).
# Usage: bash scripts/exp/wl_variants.sh TAG WORKLOAD [v1 v2 ...]
set -o pipefail
O=gpurun_out/$1; WL=$2; shift 2
mkdir -p $O
summ() {
python - $1 <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ks = sorted(d["kernels_warmup"].items(), key=lambda kv: -kv[1]["total_ms"])
r = d["roofline"]
print("  %.4g rec/s  %.2f ms/step  job %.3f  timed %s %.3f ms | " % (d["value"], d["ms_per_step"], d["job_roofline"]["frac"],
      r["kernel"], r["avg_launch_ms"]) +
      "  ".join("%s %.3f" % (k, v["avg_ms"]) for k, v in ks[:5]))
PY
}
echo "== $WL default"
timeout -k 10 300 python bench.py --workload $WL --steps 5 --warmup 2 --no-cpu-baseline --h2d-records 0 > $O/${WL}_default.log 2>&1 || { tail -5 $O/${WL}_default.log; exit 1; }
summ $O/${WL}_default.log
for v in "$@"; do
  echo "== $WL $v"
  FLINKGPU_LIB=$PWD/flink_amd/libflinkgpu_$v.so timeout -k 10 300 python bench.py --workload $WL --steps 5 --warmup 2 \
      --no-cpu-baseline --h2d-records 0 > $O/${WL}_$v.log 2>&1 || { tail -5 $O/${WL}_$v.log; exit 1; }
  summ $O/${WL}_$v.log
done
