# Round 3: packet-carried timing events -- kernel trace + bench A/B of timing on/off
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline --h2d-records 0 --steps 2 > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
cd $R
for T in 1 0 1 0; do
  FG_KERNEL_TIMING=$T timeout -k 10 180 python bench.py --no-cpu-baseline --h2d-records 0 --steps 10 > $O/t$T.$RANDOM.log 2>&1 || { echo "timing $T failed"; exit 1; }
done
echo done
