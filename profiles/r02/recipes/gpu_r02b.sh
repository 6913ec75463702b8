set -o pipefail
mkdir -p gpurun_out/r02b
python -c "import bench,json;print(json.dumps(bench.host_info()))" > gpurun_out/r02b/host.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02b/pytest_gpu.log 2>&1 || exit 1
bash tools/gpu_bench_prof.sh r02b || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/r02b/kt_stereo2048 -o run --output-format csv -- \
    python3 tools/bench_stereo.py --streams 2048 > gpurun_out/r02b/kt_stereo2048.log 2>&1 || exit 3
echo ALLDONE
