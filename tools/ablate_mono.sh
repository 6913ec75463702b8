#!/bin/bash
# Time the fused kernel with phases removed (FMRX_ABLATE bitmask; results are wrong by design).
for rnd in 0 1; do
for a in ${ABL_LIST:-0 1 2 4 8 6 14 15}; do
  FMRX_MONO_VARIANT=6 FMRX_LIB_PATH=software-defined-radio-course-project_amd/build_ab/libfmrx.so FMRX_ABLATE=$a timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline \
    | python3 -c "import json,sys; j=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('ablate $a kernel_ms', j['roofline']['kernel_ms'])"
done
done
