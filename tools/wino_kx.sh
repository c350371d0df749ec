#!/bin/bash
# Knock-out builds of the Winograd conv for timing decomposition (analysis aid; build host):
# tools/kx<k>/libpcx.so with -DWINO_KO=k (1: no operand copies, 2: no epilogue, 4: no chunk sync,
# 8: no BN + ReLU prologue; bits combine).  On the GPU box: tools/wino_kx_run.sh
set -e
cd "$(dirname "$0")/.."
for k in ${KOS:-1 2 4 8 3}; do
  mkdir -p tools/kx$k
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Iinclude -munsafe-fp-atomics -DWINO_KO=$k \
      -fno-slp-vectorize -c phoneme_contrast_amd/csrc/conv_wino.hip -o tools/kx$k/conv_wino.o
  objs=$(ls build/*.o | grep -v conv_wino.o)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/kx$k/libpcx.so $objs tools/kx$k/conv_wino.o
done
