#!/bin/bash
# dev only: libekfslam_<name>.so with ekf_kernels.hip built from <src> (a path, or git:<rev> for that
# revision's file) and extra defines; the other objects are the current build's.
# Usage: bash tools/build_variant.sh <name> <src> [-DFOO ...]
set -e
name=${1:?name}; src=${2:?src}; shift 2
cd "$(dirname "$0")/../ekf-slam_amd"
make -s libekfslam.so
tmp=build/var_${name}_kernels.hip
if [[ $src == git:* ]]; then git show "${src#git:}:ekf-slam_amd/csrc/ekf_kernels.hip" > $tmp; else cp "$src" $tmp; fi
HF="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -Wno-unused-value -I../include -Icsrc"
/opt/rocm/bin/hipcc $HF "$@" -x hip -c $tmp -o build/var_${name}_kernels.o
objs=$(ls build/*.o | grep -v -e '/diag_' -e 'var_' -e 'ekf_kernels.hip.o')
/opt/rocm/bin/hipcc $HF -shared -Wl,-rpath,/opt/rocm/lib -o libekfslam_${name}.so build/var_${name}_kernels.o $objs
echo built libekfslam_${name}.so
