#!/bin/bash
# Build timing-decomposition variants of libpcx.so (conv_dma.hip compiled with -DPCX_CONV_EXPT=e)
# into phoneme_contrast_amd/expt/libpcx_e<e>.so; select one at run time with PCX_LIB=...
set -eo pipefail
cd "$(dirname "$0")/.."
make -s
mkdir -p build/expt phoneme_contrast_amd/expt
OBJS=$(ls build/*.o | grep -v conv_dma.o)
for e in "$@"; do (
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Iinclude -Wall -Wno-unused-result \
      -munsafe-fp-atomics -DPCX_CONV_EXPT=$e -c phoneme_contrast_amd/csrc/conv_dma.hip -o build/expt/conv_dma_e$e.o
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o phoneme_contrast_amd/expt/libpcx_e$e.so $OBJS build/expt/conv_dma_e$e.o) &
done
wait
