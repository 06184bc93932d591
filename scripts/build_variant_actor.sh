#!/bin/bash
# build ab/<name>.so with actor.hip compiled under extra flags
set -e
cd "$(dirname "$0")/../mopo_amd/csrc"
make -s -j8 >/dev/null
name=$1; shift
mkdir -p ../../ab ../../build/ab
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result "$@" -c actor.hip -o ../../build/ab/actor_$name.o
objs=$(ls ../../build/csrc/*.o | grep -v '/actor\.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../ab/$name.so ../../build/ab/actor_$name.o $objs
echo "built ab/$name.so"
