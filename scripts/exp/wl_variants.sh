# hop / cumulate workloads with each variant library (experiment only)
set -o pipefail
mkdir -p gpurun_out/wlv
for v in "$@"; do
  lib=$PWD/flink_amd/libflinkgpu_$v.so
  [ "$v" = base ] && lib=$PWD/flink_amd/libflinkgpu.so
  for w in hop cumulate; do
    FLINKGPU_LIB=$lib timeout -k 10 200 python bench.py --workload $w --steps 2 --warmup 1 > gpurun_out/wlv/${w}_$v.json 2> gpurun_out/wlv/${w}_$v.err || { echo "$v $w failed"; tail -5 gpurun_out/wlv/${w}_$v.err; exit 1; }
    python - "$w" "$v" <<'PY'
import json, sys
w, v = sys.argv[1:3]
d = json.loads(open(f"gpurun_out/wlv/{w}_{v}.json").read().strip().splitlines()[-1])
ks = {k: round(x["avg_ms"], 4) for k, x in d["kernels_warmup"].items() if k.startswith("merge")}
print(w, v, "ms/step", round(d["ms_per_step"], 2), ks, flush=True)
PY
  done
done
