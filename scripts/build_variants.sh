# Experiment variants of the whole library (kernels + engine compiled with the flags): writes
# flink_amd/libflinkgpu_<name>.so (objects under flink_amd/build_var/<name>). The shipped library
# is flink_amd/libflinkgpu.so. Arguments: name=-DFLAG=V,-DFLAG2=V ...
set -e
cd "$(dirname "$0")/../flink_amd"
for v in "$@"; do
  name=${v%%=*}; flags=$(echo "${v#*=}" | tr ',' ' ')
  mkdir -p build_var/$name
  for f in fg_kernels.hip fg_engine.cpp fg_keydict.hip fg_late.hip; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -x hip -c csrc/$f -o build_var/$name/$f.o &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--version-script=csrc/libflinkgpu.map \
      -o libflinkgpu_$name.so build_var/$name/*.o
  echo built libflinkgpu_$name.so
done
