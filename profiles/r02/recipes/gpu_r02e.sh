#!/bin/bash
# Round-2 session of record after the lane-role PLL runner: GPU tests, the mono bench line with
# kernel trace and PMC passes (tools/gpu_bench_prof.sh), the stereo/RDS/CLI/config-5 benches and
# stereo kernel traces (tools/gpu_stereo_round.sh minus its duplicate bench line), runner SQ
# counters at one stream.
set -o pipefail
TAG=${1:-r02e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
bash tools/gpu_bench_prof.sh $TAG || exit 2
timeout -k 10 300 python tools/bench_stereo.py --streams 1 32 256 1024 2048 > $OUT/bench_stereo.json 2> $OUT/bench_stereo.err || exit 3
timeout -k 10 300 python tools/bench_stereo.py --gib > $OUT/bench_stereo_gib.json 2> $OUT/bench_stereo_gib.err || exit 4
timeout -k 10 300 python tools/bench_rds.py --streams 1,256 > $OUT/bench_rds.json 2> $OUT/bench_rds.err || exit 5
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29531 tools/bench_streams.py --streams 32 --seconds 10 --check > $OUT/bench_streams32.json 2> $OUT/bench_streams32.err || exit 6
timeout -k 10 300 python tools/bench_cli.py > $OUT/bench_cli.json 2> $OUT/bench_cli.err || exit 7
for ns in 1 256; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/kt_stereo$ns -o run --output-format csv -- \
      python3 tools/bench_stereo.py --streams $ns > $OUT/kt_stereo$ns.log 2>&1 || exit 8
done
bash tools/gpu_runner_sq.sh $TAG/runner_sq "1" "1 32" || exit 9
echo done
