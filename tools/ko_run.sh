#!/bin/bash
# knock-out timing decomposition of the Winograd conv (needs tools/wino_ko.sh builds; analysis aid)
cd "$(dirname "$0")"
for s in ${SHAPES:-"40 200 32 32 4096 5 0 1" "40 200 32 32 4096 5 1 0" "10 50 128 128 4096 5 0 1"}; do
  for k in 0 ${KOS:-1 2 3}; do
    if [ $k = 0 ]; then timeout -k 5 60 ./wino_bench $s | sed "s/^/ko0 /"; else LD_LIBRARY_PATH=$PWD/ko$k timeout -k 5 60 ./wino_bench $s | sed "s/^/ko$k /"; fi
  done
done
