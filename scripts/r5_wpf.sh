#!/bin/bash
# channel-last weight gradient prefetch depth: bf16 / conv tests, then the deep bf16 line with PF = 3 (default)
# and PF = 1 (the round-4 depth).  Output: gpurun_out/$1*
set -o pipefail
TESTS="tests/test_conv2d_gpu.py tests/test_deep_bf16_gpu.py tests/test_config5_gpu.py" bash scripts/r5_deep.sh ${1:-r5wpf} || exit 1
PCX_CONVN_WPF=1 NOTEST=1 bash scripts/r5_deep.sh ${1:-r5wpf}_pf1
