# Times the default bench with each merge-buffering variant library (experiment only)
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  FLINKGPU_LIB=$PWD/flink_amd/libflinkgpu_$v.so timeout -k 10 240 python bench.py --no-cpu-baseline --steps 3 --warmup 1 \
     > gpurun_out/mv_$v.json 2> gpurun_out/mv_$v.err || exit 1
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/mv_{v}.json").read().strip().splitlines()[-1])
ks = {k: round(x["avg_ms"], 3) for k, x in d["kernels"].items()}
print(v, "ms/step", round(d["ms_per_step"], 2), ks, flush=True)
PY
done
