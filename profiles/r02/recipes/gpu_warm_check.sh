set -o pipefail
mkdir -p gpurun_out/warm
for w in 3 1500 3; do
timeout -k 10 120 python bench.py --steps 20 --warmup $w --no-cpu-baseline --no-other-configs > gpurun_out/warm/b_w${w}_s20_$RANDOM.json 2>/dev/null || exit 1
done
timeout -k 10 120 python bench.py --steps 1500 --warmup 3 --no-cpu-baseline --no-other-configs > gpurun_out/warm/b_w3_s1500.json 2>/dev/null || exit 2
echo ok
