#!/bin/bash
# knock-out timing decomposition of the fused layer-2 backward (needs tools/wb_ko.sh builds; analysis aid)
cd "$(dirname "$0")"
for k in 0 ${KOS:-1 2 4 8 3 7 12}; do
  if [ $k = 0 ]; then timeout -k 5 60 ./wb_bench 40 200 4096 5 | sed "s/^/ko0 /"
  else LD_LIBRARY_PATH=$PWD/wbko$k timeout -k 5 60 ./wb_bench 40 200 4096 5 | sed "s/^/ko$k /"; fi
  rc=$?; [ $rc -le 2 ] || exit 1
done
exit 0
