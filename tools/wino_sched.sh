#!/bin/bash
# Scheduling-experiment builds of the Winograd conv (analysis aid; build host): tools/ws<k>/libpcx.so with
# -DWINO_SCHED=k (1: every LDS read of a K-step issued before its arithmetic).  GPU box: tools/wino_sched_run.sh
set -e
cd "$(dirname "$0")/.."
for k in ${KS:-1}; do
  mkdir -p tools/ws$k
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Iinclude -munsafe-fp-atomics -DWINO_SCHED=$k \
      -fno-slp-vectorize -c phoneme_contrast_amd/csrc/conv_wino.hip -o tools/ws$k/conv_wino.o
  objs=$(ls build/*.o | grep -v conv_wino.o)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/ws$k/libpcx.so $objs tools/ws$k/conv_wino.o
done
