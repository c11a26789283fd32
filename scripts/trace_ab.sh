# Kernel traces of the default bench with an engine knob off and on (gap analysis: scripts/gaps.py)
set -o pipefail
VAR=${1:-FG_SPECULATE}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in 0 1; do
  env $VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace_$v -o run -- \
      python3 $R/bench.py --no-cpu-baseline --h2d-records 0 --steps 2 > $R/gpurun_out/trace_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
done
echo traced
