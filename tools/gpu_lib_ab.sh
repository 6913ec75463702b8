#!/bin/bash
# A/B of two builds of libfmrx.so (package dir: libfmrx_<a>.so, libfmrx_<b>.so): kernel trace
# stats of the stereo bench at the given stream counts.
set -o pipefail
OUT=gpurun_out/${1:-lib_ab}
VARIANTS=${2:-"noslp slp"}
STREAMS=${3:-"1024"}
PKG=software-defined-radio-course-project_amd
mkdir -p $OUT
export TMPDIR=/tmp
for v in $VARIANTS; do
  cp $PKG/libfmrx_$v.so $PKG/libfmrx.so
  for ns in $STREAMS; do
    timeout -k 10 200 python tools/bench_stereo.py --streams $ns > $OUT/bench_${v}_$ns.json 2>> $OUT/bench.err || exit 2
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/kt_${v}_$ns -o run --output-format csv -- \
        python3 tools/bench_stereo.py --streams $ns > $OUT/kt_${v}_$ns.log 2>&1 || exit 3
  done
done
cp $PKG/libfmrx_${VARIANTS%% *}.so $PKG/libfmrx.so  # the first variant back in place
echo done
