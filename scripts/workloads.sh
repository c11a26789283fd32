# Bench every BASELINE workload on one GPU (headline = tumble; the others are reported in DESIGN.md)
set -o pipefail
mkdir -p gpurun_out
for w in ${WORKLOADS:-hop cumulate zipf}; do
  timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-2} --warmup 1 > gpurun_out/wl_$w.json 2> gpurun_out/wl_$w.err || { echo "$w failed"; tail -20 gpurun_out/wl_$w.err; exit 1; }
  python - "$w" <<'PY'
import json, sys
w = sys.argv[1]
d = json.loads(open(f"gpurun_out/wl_{w}.json").read().strip().splitlines()[-1])
ks = {k: (x["launches"], round(x["avg_ms"], 3)) for k, x in d["kernels"].items()}
print(w, f"{d['value']/1e9:.2f} G rec/s", "ms/step", round(d["ms_per_step"], 2), "rows", d["rows_fired"], "late", d["late_dropped"], ks, flush=True)
PY
done
