#!/bin/bash
# Builds one bnn_knobs binary per knob (into scripts/micro/bin/, git-ignored):
# bin/bnn_<KNOB> (f32 ensemble) and bin/bnn16_<KNOB> (bf16 ensemble, KNOB_DTYPE=1).
cd "$(dirname "$0")"
mkdir -p bin
for k in BASE NOSWISH NOSTAGE NOBARRIER NOHEAD NOMFMA; do
  def=""; [ "$k" != BASE ] && def="-DBNN_KNOB_$k"
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include $def -DKNOB_NAME="\"$k\"" \
    bnn_knobs.hip ../../mopo_amd/csrc/errors.cpp -o bin/bnn_$k &
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include $def -DKNOB_DTYPE=1 \
    -DKNOB_NAME="\"bf16_$k\"" bnn_knobs.hip ../../mopo_amd/csrc/errors.cpp -o bin/bnn16_$k &
done
wait
ls bin
