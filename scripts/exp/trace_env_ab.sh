# Kernel trace + stats of one workload under several engine env settings (A/B of kernel times).
# Usage: bash scripts/exp/trace_env_ab.sh TAG WORKLOAD STEPS "ENV=V ..." ["ENV=V ..." ...]  ("-": none)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; WL=$2; ST=$3; shift 3
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for E in "$@"; do
  i=$((i+1))
  [ "$E" = "-" ] && E=""
  echo "variant $i: $E" > $OUT/v$i.env
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/v$i -o run -- \
      python3 $R/bench.py --workload $WL --steps $ST --warmup 1 --no-cpu-baseline --h2d-records 0 > $OUT/v$i.log 2>&1 \
      || { echo "variant $i failed"; exit 1; }
  python3 - $OUT/v$i <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print("  %-40s %6s calls %10.3f ms  avg %8.1f us" % (r["Name"][:40], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3))
PY
  tail -c 300 $OUT/v$i.log | grep -o '"ms_per_step": [0-9.]*'
done
echo trace-ab-done
