#!/bin/bash
# GPU suite, then the halo update fused into the kernel vs the separate halo_kernel, alternating.
set -o pipefail
OUT=gpurun_out/${1:-halo}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-other-configs > $OUT/fused_$i.json 2>/dev/null || exit 2
  FMRX_HALO_KERNEL=1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-other-configs > $OUT/sep_$i.json 2>/dev/null || exit 3
done
echo done
