#!/bin/bash
# Build an A/B variant of the library: tools/ab_build.sh <name> <source.hip> <-D flags...>
# Links the in-tree objects (build/) with <source> recompiled under the flags -> ab_libs/lib_<name>.so
set -eu
name=$1; src=$2; shift 2
cd "$(dirname "$0")/../mamba-clip_amd"
TORCH_LIB=$(python3 -c "import os,torch;print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
mkdir -p ../build_ab/$name ../ab_libs
base=$(basename $src)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c csrc/$base -o ../build_ab/$name/$base.o
objs=$(ls build/*.hip.o build/*.cpp.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -Wl,-rpath,$TORCH_LIB -Wl,--no-undefined $objs ../build_ab/$name/$base.o -o ../ab_libs/lib_$name.so
echo built ab_libs/lib_$name.so
