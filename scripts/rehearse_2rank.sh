# Rehearse the N > 1 bench path on a one-GPU box: 2 ranks on device 0, collectives via gloo
set -o pipefail
mkdir -p gpurun_out
export BENCH_DIST_BACKEND=gloo BENCH_DEVICE=0 MASTER_ADDR=127.0.0.1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --records ${REC:-200000000} --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/rehearse_2rank.log 2>&1
rc=$?
tail -c 2500 gpurun_out/rehearse_2rank.log
exit $rc
