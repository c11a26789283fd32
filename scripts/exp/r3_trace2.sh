# Round 3: trace of the async-watermark bench + micro-batch A/B (50M vs 100M)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline --h2d-records 0 --steps 2 > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
cd $R
for B in 100000000 50000000 100000000 50000000; do
  timeout -k 10 180 python bench.py --no-cpu-baseline --h2d-records 0 --steps 10 --batch $B > $O/b$B.$RANDOM.log 2>&1 || { echo "batch $B failed"; exit 1; }
done
echo done
