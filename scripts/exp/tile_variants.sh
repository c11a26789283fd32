# Bench the tile-staging variants (experiment): default library with FG_TILE=0 (two-pass
# partition) and =1, then each libflinkgpu_<v>.so. Usage: bash scripts/exp/tile_variants.sh TAG v1 v2 ...
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
summ() {
python - $1 <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ks = sorted(d["kernels_warmup"].items(), key=lambda kv: -kv[1]["total_ms"])
print("  %.4g rec/s  %.2f ms/step  job %.3f | " % (d["value"], d["ms_per_step"], d["job_roofline"]["frac"]) +
      "  ".join("%s %.3f" % (k, v["avg_ms"]) for k, v in ks[:4]))
PY
}
for t in 0 1; do
  echo "== default FG_TILE=$t"
  FG_TILE=$t timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --h2d-records 0 > $O/default_$t.log 2>&1 || { tail -5 $O/default_$t.log; exit 1; }
  summ $O/default_$t.log
done
for v in "$@"; do
  echo "== $v"
  FLINKGPU_LIB=$PWD/flink_amd/libflinkgpu_$v.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --h2d-records 0 > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  summ $O/$v.log
done
