# A/B variant libraries of the tile fire (round 5): flink_amd/build_var/<name>/libflinkgpu.so
# Usage: bash scripts/build_fire_variants.sh  (then FLINKGPU_LIB=... python bench.py)
set -e
cd "$(dirname "$0")/../flink_amd"
HIPCC=/opt/rocm/bin/hipcc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result"
build() {   # name, defines
    d=build_var/$1; mkdir -p $d
    for f in fg_engine.cpp fg_keydict.hip fg_late.hip fg_comm.cpp; do [ -f $d/$f.o ] || cp build/$f.o $d/$f.o; done
    $HIPCC $F $2 -x hip -c csrc/fg_kernels.hip -o $d/fg_kernels.hip.o
    $HIPCC --offload-arch=gfx950 -shared -fPIC -Wl,--version-script=csrc/libflinkgpu.map -o $d/libflinkgpu.so $d/*.o \
        -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
}
mkdir -p var
build shfl_scan "-DFG_EXP_SHFL_SCAN" &
build cond_loads "-DFG_EXP_COND_LOADS" &
build all_old "-DFG_EXP_SHFL_SCAN -DFG_EXP_COND_LOADS" &
build tile_block "-DFG_EXP_TILE_BLOCK" &
build pipe3 "-DFG_EXP_PIPE3" &
wait
ls -la build_var/*/libflinkgpu.so
