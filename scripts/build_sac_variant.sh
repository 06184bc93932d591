#!/bin/bash
# Build ab/<name>.so: libmopo_hip.so with sac.hip compiled under extra -D flags (e.g. -DMOPO_SAC_STAMPS=1).
# usage: scripts/build_sac_variant.sh <name> [-DKNOB=V ...]
set -e
cd "$(dirname "$0")/../mopo_amd/csrc"
make -s -j8 >/dev/null
name=$1; shift
mkdir -p ../../ab ../../build/ab
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result "$@" -c sac.hip -o ../../build/ab/sac_$name.o
objs=$(ls ../../build/csrc/*.o | grep -v '/sac\.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../ab/$name.so ../../build/ab/sac_$name.o $objs
echo "built ab/$name.so"
