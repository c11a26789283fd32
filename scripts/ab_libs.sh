# A/B of variant libraries on one box: the headline bench (or --workload W) per library, in
# rotation, printing ms/step and the dominant kernels' average launch times.
# Usage: bash scripts/ab_libs.sh TAG "bench args" lib1 lib2 ...   (lib: a dir under flink_amd/variants)
set -o pipefail
O=gpurun_out/$1; ARGS=$2; shift 2
mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    FLINKGPU_LIB=$PWD/flink_amd/variants/$v/libflinkgpu.so timeout -k 10 240 python bench.py --no-cpu-baseline --h2d-records 0 $ARGS \
      > $O/${v}_$rep.log 2>&1 || { echo "bench $v failed"; tail -5 $O/${v}_$rep.log; exit 1; }
    python - $O/${v}_$rep.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ks = sorted(d["kernels_warmup"].items(), key=lambda kv: -kv[1]["total_ms"])[:4]
print("%-10s %.2f ms/step  " % (sys.argv[2], d["ms_per_step"]) + "  ".join("%s %.3f" % (k, v["avg_ms"]) for k, v in ks))
PY
  done
done
