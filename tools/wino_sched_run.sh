#!/bin/bash
# A/B of the scheduling builds (tools/wino_sched.sh) on the cnn_small layer shapes (analysis aid)
cd "$(dirname "$0")"
for s in "40 200 32 32 4096 5 0 1" "20 100 64 64 4096 5 0 1" "10 50 128 128 4096 5 0 1" "20 100 64 64 4096 5 1 0" "20 100 64 32 4096 5 4 0"; do
  timeout -k 5 60 ./wino_bench $s | sed "s/^/base /" || exit 1
  for k in ${KS:-1}; do LD_LIBRARY_PATH=$PWD/ws$k timeout -k 5 60 ./wino_bench $s | sed "s/^/ws$k /" || exit 1; done
done
