#!/bin/bash
# One GPU session: bench line, kernel-trace stats, then HBM counters in separate passes.
# Usage (on the GPU box via gpurun): bash tools/gpu_bench_prof.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/kt -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-other-configs > $OUT/kt.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/pmc_fetch -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --min-warmup-seconds 0 --no-cpu-baseline --no-other-configs > $OUT/pmc_fetch.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/pmc_write -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --min-warmup-seconds 0 --no-cpu-baseline --no-other-configs > $OUT/pmc_write.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -T -d $OUT/pmc_grbm -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-other-configs > $OUT/pmc_grbm.log 2>&1 || exit 5
echo done
