#!/bin/bash
# Records of a round: the GPU test suite, smoke(), the bench line (with its configs[2..5] legs),
# and five more bench runs for the median.
set -o pipefail
TAG=${1:-record}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 2
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 3
bash tools/bench_median.sh $TAG/median || exit 4
echo done
