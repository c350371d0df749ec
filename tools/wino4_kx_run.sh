#!/bin/bash
# knock-out timing decomposition of the F(4x3) conv (tools/wino4_kx.sh builds; analysis aid)
cd "$(dirname "$0")"
for s in ${SHAPES:-"40 200 32 32 4096 3 0 1" "10 50 128 128 4096 3 0 1" "10 50 128 128 24 3 0 1"}; do
  for k in 0 ${KOS:-1 2 4 7}; do
    if [ $k = 0 ]; then timeout -k 5 60 ./wino4_bench $s | sed "s/^/kx0 /"; else LD_LIBRARY_PATH=$PWD/w4ko_$k timeout -k 5 60 ./wino4_bench $s | sed "s/^/kx$k /"; fi
  done
done
