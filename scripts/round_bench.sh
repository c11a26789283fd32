# Round artifacts (GPU box): default bench with the CPU baseline, then the profile recipe.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_full.log; exit 1; }
tail -c 1500 gpurun_out/bench_full.log
bash scripts/profile.sh ${1:-r01} 200000000
