#!/bin/bash
# Build abv/<name>.so: libmopo_hip.so with sac.hip compiled under extra -D flags (e.g. -DMOPO_SAC_STAMPS=1).
# usage: scripts/build_sac_variant.sh <name> [-DKNOB=V ...]
set -e
cd "$(dirname "$0")/../mopo_amd/csrc"
make -s -j8 >/dev/null
name=$1; shift
mkdir -p ../../abv ../../build/abv
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result "$@" -c sac.hip -o ../../build/abv/sac_$name.o
objs=$(ls ../../build/csrc/*.o | grep -v '/sac\.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../abv/$name.so ../../build/abv/sac_$name.o $objs
echo "built abv/$name.so"
