# hop / cumulate at the default micro-batch and at one event-minute of records per batch
set -o pipefail
mkdir -p gpurun_out/hcb
for spec in "hop 25000000" "hop 33333334" "cumulate 12500000" "cumulate 16666667"; do
  set -- $spec
  timeout -k 10 200 python bench.py --workload $1 --batch $2 --steps 2 --warmup 1 > gpurun_out/hcb/$1_$2.json 2> gpurun_out/hcb/$1_$2.err || { echo "$1 $2 failed"; tail -5 gpurun_out/hcb/$1_$2.err; exit 1; }
  python - "$1" "$2" <<'PY'
import json, sys
w, b = sys.argv[1:3]
d = json.loads(open(f"gpurun_out/hcb/{w}_{b}.json").read().strip().splitlines()[-1])
ks = {k: (x["launches"], round(x["total_ms"], 2)) for k, x in d["kernels_warmup"].items()}
print(w, b, "ms/step", round(d["ms_per_step"], 2), "rows", d["rows_fired"], ks, flush=True)
PY
done
