set -o pipefail
mkdir -p gpurun_out/bal1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "mono or polyphase or stereo or rf_block or time_shard or window" > gpurun_out/bal1/pytest.log 2>&1 || exit 1
for i in 1 2; do
FMRX_MONO_BALANCE=0 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-other-configs > gpurun_out/bal1/bench_static_$i.json 2>/dev/null || exit 2
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-other-configs > gpurun_out/bal1/bench_bal_$i.json 2>/dev/null || exit 3
done
timeout -k 10 120 python tools/mono_stamps.py > gpurun_out/bal1/stamps_bal.json 2>gpurun_out/bal1/stamps.err || exit 4
FMRX_MONO_BALANCE=0 timeout -k 10 120 python tools/mono_stamps.py > gpurun_out/bal1/stamps_static.json 2>>gpurun_out/bal1/stamps.err || exit 5
echo ok
