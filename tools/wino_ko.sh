#!/bin/bash
# Knock-out builds of the Winograd conv for timing decomposition (analysis aid; run on the build
# host): tools/ko<k>/libpcx.so with -DWINO_KO=k (1: no operand copies, 2: no epilogue, 3: both).
# On the GPU box: LD_LIBRARY_PATH=tools/ko<k> tools/wino_bench ...
set -e
cd "$(dirname "$0")/.."
for k in ${KOS:-1 2 3}; do
  mkdir -p tools/ko$k
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Iinclude -munsafe-fp-atomics -DWINO_KO=$k \
      -fno-slp-vectorize -c phoneme_contrast_amd/csrc/conv_wino.hip -o tools/ko$k/conv_wino.o
  objs=$(ls build/*.o | grep -v conv_wino.o)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/ko$k/libpcx.so $objs tools/ko$k/conv_wino.o
done
