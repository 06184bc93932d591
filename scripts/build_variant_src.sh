#!/bin/bash
# Build abv/<name>.so: libmopo_hip.so with ONE source file compiled under extra -D flags (for scripts/ab.sh
# and the training / SAC A/B scripts).  usage: scripts/build_variant_src.sh <name> <file.hip> [-DKNOB=V ...]
set -e
cd "$(dirname "$0")/../mopo_amd/csrc"
name=$1; src=$2; shift 2
base=${src%.hip}
mkdir -p ../../abv ../../build/abv
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result "$@" -c $src -o ../../build/abv/${base}_$name.o
objs=$(ls ../../build/csrc/*.o | grep -v "/${base}\.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../abv/$name.so ../../build/abv/${base}_$name.o $objs
echo "built abv/$name.so"
