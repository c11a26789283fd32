# Times the default bench (all kernel classes from the warm-up step) with each variant library
# flink_amd/libflinkgpu_<v>.so ("base" = the shipped flink_amd/libflinkgpu.so). Experiment only.
set -o pipefail
mkdir -p gpurun_out/variants
for v in "$@"; do
  lib=$PWD/flink_amd/libflinkgpu_$v.so
  [ "$v" = base ] && lib=$PWD/flink_amd/libflinkgpu.so
  FLINKGPU_LIB=$lib timeout -k 10 180 python bench.py --no-cpu-baseline --h2d-records 0 --steps 3 --warmup 2 ${BENCH_ARGS} \
     > gpurun_out/variants/$v.json 2> gpurun_out/variants/$v.err || { echo "$v failed"; tail -5 gpurun_out/variants/$v.err; exit 1; }
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/variants/{v}.json").read().strip().splitlines()[-1])
ks = {k: round(x["avg_ms"], 4) for k, x in d["kernels_warmup"].items()}
print(v, "ms/step", round(d["ms_per_step"], 3), ks, flush=True)
PY
done
