# Builds libflinkgpu_<name>.so variants of the kernels (experiment only; the shipped library
# is flink_amd/libflinkgpu.so). Arguments: name=-DFLAG=V,-DFLAG2=V ...
set -e
cd "$(dirname "$0")/../flink_amd"
make -s build/fg_engine.cpp.o build/fg_keydict.hip.o build/fg_late.hip.o
mkdir -p build_var
for v in "$@"; do
  name=${v%%=*}; flags=$(echo "${v#*=}" | tr ',' ' ')
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -x hip -c csrc/fg_kernels.hip -o build_var/k_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libflinkgpu_$name.so build_var/k_$name.o build/fg_engine.cpp.o build/fg_keydict.hip.o build/fg_late.hip.o
  echo built libflinkgpu_$name.so
done
