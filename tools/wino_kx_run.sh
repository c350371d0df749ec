#!/bin/bash
# knock-out timing decomposition of the Winograd conv (tools/wino_kx.sh builds; analysis aid)
cd "$(dirname "$0")"
for s in ${SHAPES:-"40 200 32 32 4096 5 0 1" "20 100 64 64 4096 5 0 1" "10 50 128 128 4096 5 0 1" "20 100 64 64 4096 5 1 0" "20 100 64 32 4096 5 4 0"}; do
  for k in 0 ${KOS:-1 2 4 8 3}; do
    if [ $k = 0 ]; then timeout -k 5 60 ./wino_bench $s | sed "s/^/kx0 /"; else LD_LIBRARY_PATH=$PWD/kx$k timeout -k 5 60 ./wino_bench $s | sed "s/^/kx$k /"; fi
  done
done
