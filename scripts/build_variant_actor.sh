#!/bin/bash
# build abv/<name>.so with actor.hip compiled under extra flags
set -e
cd "$(dirname "$0")/../mopo_amd/csrc"
make -s -j8 >/dev/null
name=$1; shift
mkdir -p ../../abv ../../build/abv
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -mllvm -pragma-unroll-threshold=262144 "$@" -c actor.hip -o ../../build/abv/actor_$name.o
objs=$(ls ../../build/csrc/*.o | grep -v '/actor\.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../abv/$name.so ../../build/abv/actor_$name.o $objs
echo "built abv/$name.so"
