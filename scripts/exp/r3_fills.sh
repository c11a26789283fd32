# Round 3: fewer fills per fire + no producer barrier on idle streams: GPU suite, then bench (50M, 100M batches)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3f
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_suite.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
for B in 100000000 50000000 100000000 50000000; do
  timeout -k 10 180 python bench.py --no-cpu-baseline --h2d-records 0 --steps 10 --batch $B > $O/b$B.$RANDOM.log 2>&1 || { echo "batch $B failed"; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline --h2d-records 0 --steps 2 > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
echo done
cd $R
for W in hop cumulate; do
  timeout -k 10 240 python bench.py --workload $W --steps 5 --warmup 2 > $O/wl_$W.log 2>&1 || { echo "workload $W failed"; exit 1; }
done
echo done2
