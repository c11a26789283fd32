# Quick GPU check of a kernel change: the headline bench line, then the tile-path parity tests
# (tile split / spread fires, the configs at full key space, golden + stream cases).
# Usage: bash scripts/gpu_quick.sh TAG [pytest -k expression]
set -o pipefail
O=gpurun_out/$1; K=${2:-}
mkdir -p $O
timeout -k 10 240 python bench.py --no-cpu-baseline --h2d-records 0 --steps 3 --warmup 1 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
python - $O/bench.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ks = sorted(d["kernels_warmup"].items(), key=lambda kv: -kv[1]["total_ms"])[:4]
print("%.2f ms/step  " % d["ms_per_step"] + "  ".join("%s %.3f" % (k, v["avg_ms"]) for k, v in ks))
PY
timeout -k 10 900 python -u -m pytest tests/test_gpu_tile_split.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider ${K:+-k "$K"} > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
