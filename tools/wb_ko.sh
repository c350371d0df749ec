#!/bin/bash
# Knock-out builds of the fused layer-2 backward for timing decomposition (analysis aid; run on the
# build host): tools/wbko<k>/libpcx.so with -DWB_KO=k (1: no weight-gradient GEMM, 2: no data-gradient
# GEMM, 4: no epilogue, 8: no staging loads; bits combine).  On the GPU box: tools/wb_ko_run.sh
set -e
cd "$(dirname "$0")/.."
# EXTRA: more -D flags for every build (variant A/B builds: KOS=0 EXTRA=-DWB_LOADPOS=1 TAG=lp1)
for k in ${KOS:-1 2 4 8 3 7 12}; do
  mkdir -p tools/wbko$k${TAG}
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Iinclude -munsafe-fp-atomics -DWB_KO=$k $EXTRA \
      -fno-slp-vectorize -c phoneme_contrast_amd/csrc/wgbd_wino.hip -o tools/wbko$k${TAG}/wgbd_wino.o
  objs=$(ls build/*.o | grep -v wgbd_wino.o)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/wbko$k${TAG}/libpcx.so $objs tools/wbko$k${TAG}/wgbd_wino.o
done
