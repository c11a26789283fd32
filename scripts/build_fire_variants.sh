# Diagnostic variant libraries of the tile fire: flink_amd/build_var/<name>/libflinkgpu.so
# Usage: bash scripts/build_fire_variants.sh name "defines" [name "defines" ...]
#        (then FLINKGPU_LIB=flink_amd/build_var/<name>/libflinkgpu.so python bench.py ...)
set -e
cd "$(dirname "$0")/../flink_amd"
make -s -j4 libflinkgpu.so
HIPCC=/opt/rocm/bin/hipcc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result"
build() {   # name, defines
    d=build_var/$1; mkdir -p $d
    for f in fg_keydict.hip fg_late.hip fg_comm.cpp; do cp build/$f.o $d/$f.o; done
    $HIPCC $F $2 -x hip -c csrc/fg_engine.cpp -o $d/fg_engine.cpp.o &
    $HIPCC $F $2 -x hip -c csrc/fg_kernels.hip -o $d/fg_kernels.hip.o
    wait
    $HIPCC --offload-arch=gfx950 -shared -fPIC -Wl,--version-script=csrc/libflinkgpu.map -o $d/libflinkgpu.so $d/*.o \
        -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
}
while [ $# -ge 2 ]; do build "$1" "$2" & shift 2; done
wait
mkdir -p variants
for d in build_var/*/; do n=$(basename $d); mkdir -p variants/$n; cp $d/libflinkgpu.so variants/$n/; done
ls -la variants/*/libflinkgpu.so
