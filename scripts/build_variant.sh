#!/bin/bash
# Build abv/<name>.so: libmopo_hip.so with bnn.hip compiled under extra -D flags (for scripts/ab.sh).
# usage: scripts/build_variant.sh <name> [-DKNOB=V ...]
set -e
cd "$(dirname "$0")/../mopo_amd/csrc"
make -s -j8 >/dev/null
name=$1; shift
mkdir -p ../../abv ../../build/abv
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -mllvm -pragma-unroll-threshold=262144 "$@" -c bnn.hip -o ../../build/abv/bnn_$name.o
objs=$(ls ../../build/csrc/*.o | grep -v '/bnn\.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../abv/$name.so ../../build/abv/bnn_$name.o $objs
echo "built abv/$name.so"
