#!/bin/bash
# Kernel-experiment builds of the engine library with the DCN core's staged-tile column pitch
# TP = TC + k (tools/exp_dcnp<k>.so): the row stride in 16-B LDS slots decides which random
# bilinear corner reads of a 16-lane group collide in the same bank group.
set -e
cd "$(dirname "$0")/../.."
for k in "$@"; do
  T=$(mktemp -d)
  cp -r Makefile include stif-continuous-video-representation_amd "$T"/
  rm -f "$T"/stif-continuous-video-representation_amd/*.so
  sed -i "s/  constexpr int TP = TC;  /  constexpr int TP = TC + $k;/" "$T"/stif-continuous-video-representation_amd/csrc/dcn.hip
  grep -q "TP = TC + $k;" "$T"/stif-continuous-video-representation_amd/csrc/dcn.hip
  make -C "$T" -j8 > "$T"/build.log 2>&1
  cp "$T"/stif-continuous-video-representation_amd/libstif_hip.so tools/exp_dcnp$k.so
  rm -rf "$T"
done
