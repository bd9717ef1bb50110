# Builds an instrumented variant of the library in-tree: bash tools/build_variant.sh phases -DDSL_PHASES
set -e
cd /root/repo
V=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -Wno-unused-value -I include \
  -DDSL_WITH_RCCL=1 "$@" -o dslabs_amd/libdslabs_hip_$V.so dslabs_amd/csrc/engine.hip -L/opt/rocm/lib -lrccl
