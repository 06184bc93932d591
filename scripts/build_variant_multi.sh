#!/bin/bash
# Build abv/<name>.so: libmopo_hip.so with bnn.hip AND actor.hip compiled under extra -D flags (knobs of the
# shared layer helpers in mlp_tile.h reach both).  usage: scripts/build_variant_multi.sh <name> [-DKNOB=V ...]
set -e
cd "$(dirname "$0")/../mopo_amd/csrc"
make -s -j8 >/dev/null
name=$1; shift
mkdir -p ../../abv ../../build/abv
for src in bnn actor; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -mllvm -pragma-unroll-threshold=262144 \
    "$@" -c $src.hip -o ../../build/abv/${src}_$name.o &
done
wait
objs=$(ls ../../build/csrc/*.o | grep -v -E '/(bnn|actor)\.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../abv/$name.so ../../build/abv/bnn_$name.o ../../build/abv/actor_$name.o $objs
echo "built abv/$name.so"
