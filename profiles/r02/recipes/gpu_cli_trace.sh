#!/bin/bash
# Kernel trace of the stereo CLI on 1 GiB from stdin (where the time goes beside the device work).
set -o pipefail
OUT=gpurun_out/${1:-cli_trace}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -c "
import sys; sys.path.insert(0, 'tests'); import iqgen
iq = iqgen.make('synth:0', (1 << 30) // 12800 * 12800)
iq.tofile('/tmp/cli_in.u8')" || exit 1
PKG=software-defined-radio-course-project_amd
s0=$(date +%s.%N); timeout -k 10 200 $PKG/bin/fmrx 0 2 --batch 2048 < /tmp/cli_in.u8 > /tmp/cli_out.s16 2> $OUT/plain.err || exit 2; s1=$(date +%s.%N); python3 -c "print('plain_seconds', $s1 - $s0)" > $OUT/time_plain.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -T -d $OUT/kt -o run --output-format csv -- \
    $PKG/bin/fmrx 0 2 --batch 2048 < /tmp/cli_in.u8 > /tmp/cli_out2.s16 2> $OUT/kt.log || exit 3
rm -f /tmp/cli_in.u8 /tmp/cli_out.s16 /tmp/cli_out2.s16
echo done
