#!/bin/bash
# instruction mix / wait counters of the main cnn_small kernels at B = 4096 (tools/pmc_mix.sh)
set -o pipefail
cd "$(dirname "$0")/.."
tools/pmc_mix.sh wgrad_L6 wgrad_wino_kernel -- tools/ww_bench 10 50 128 128 4096 2 1 && \
tools/pmc_mix.sh wgrad_L4 wgrad_wino_kernel -- tools/ww_bench 20 100 64 64 4096 2 1 && \
tools/pmc_mix.sh fwd_L2 conv_wino_kernel -- tools/wino_bench 40 200 32 32 4096 2 0 1 && \
tools/pmc_mix.sh fwd_L6 conv_wino_kernel -- tools/wino_bench 10 50 128 128 4096 2 0 1 && \
tools/pmc_mix.sh dgrad_L4 conv_wino_kernel -- tools/wino_bench 20 100 64 64 4096 2 1 0 && \
tools/pmc_mix.sh wgbd_L2 wgbd_wino_kernel -- tools/wb_bench 40 200 4096 2 1 && echo mix-done
