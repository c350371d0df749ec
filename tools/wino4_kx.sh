#!/bin/bash
# Knock-out builds of the F(4x3) conv for timing decomposition (analysis aid; build host): tools/w4ko_<k>/libpcx.so
# with -DWINO4_KO=k (1: no input copies, 2: no weight copies, 4: no wait for the chunk copies (barrier kept); bits combine).
set -e
cd "$(dirname "$0")/.."
for k in ${KOS:-1 2 4 7}; do
  mkdir -p tools/w4ko_$k
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Iinclude -munsafe-fp-atomics -DWINO4_KO=$k \
      -fno-slp-vectorize -c phoneme_contrast_amd/csrc/conv_wino4.hip -o tools/w4ko_$k/conv_wino4.o
  objs=$(ls build/*.o | grep -v conv_wino4.o)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/w4ko_$k/libpcx.so $objs tools/w4ko_$k/conv_wino4.o
done
