# Round 3: pass-1 shape sweep at 100M-record batches (variant libraries, experiment only)
set -o pipefail
O=gpurun_out/r3p
mkdir -p $O
for i in 1 2; do
for v in default p1t1024r4 p1t512r8 p1t768r4; do
  L=flink_amd/libflinkgpu.so; [ $v = default ] || L=flink_amd/libflinkgpu_$v.so
  FLINKGPU_LIB=$PWD/$L timeout -k 10 120 python -u bench.py --no-cpu-baseline --h2d-records 0 --steps 10 > $O/$v.$i.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.$i.log; exit 1; }
done
done
echo done
