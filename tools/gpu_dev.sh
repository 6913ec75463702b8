#!/bin/bash
# tools/gpu_dev.sh <tag> [steps...] — development GPU call: each named step under its own time
# limit, stopping at the first failure.  Steps: tests (whole GPU suite), pll (PLL / stereo tests
# only), n2 (the N=2 bench line rehearsed with gloo, both ranks on device 0), mfma (tools/ubench_mfma_add), predict (tools/pll_predict.cpp on a 72 s GPU-made carrier, lookback 2), rprof22 (runner_prof of the forms at $TRIGS, default the 64-step forms from 2^21, 2^22, 2^23, with the profiling build), rprof (tools/runner_prof.py per form, with the FMRX_AB_PROF build), testsall (whole GPU suite, not stopping at a failure), idx (the index-runner tests), ubench (tools/ubench_idx), stages (tools/stage_times.py), stages1 (configs[4] with the serial engine), pipe (the pipelined-engine tests), s32 (configs[4]-length calls at 32 streams, serial vs 8 chunks), envab (configs[4] per value of $ENVVAR in $VALS, alternating, twice), libab (stage_times per A/B build in $LIBS, alternating, twice), redoc4 (configs[4] with the FMRX_AB_PROF build: runner cycles and redos per stream), ktrace (kernel trace of configs[4] calls + tools/trace_overlap.py), bench (bench.py, no CPU baseline), clitrace (rocprofv3 stats of `fmrx 0 2` over 1 GiB, per runner form), smoke.
set -o pipefail
TAG=${1:-dev}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
           tail -2 $OUT/tests.log ;;
    testsall) timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/testsall.log 2>&1; rc=$?
           tail -30 $OUT/testsall.log; [ $rc -le 1 ] || exit 1 ;;
    pll) timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pll or stereo or bench_config or trig_hint or refdata or cli" > $OUT/pll.log 2>&1 || { tail -40 $OUT/pll.log; exit 2; }
           tail -2 $OUT/pll.log ;;
    idx) timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "index" > $OUT/idx.log 2>&1 || { tail -40 $OUT/idx.log; exit 6; }
           tail -2 $OUT/idx.log ;;
    ubench) timeout -k 10 60 tools/ubench_idx > $OUT/ubench_idx.txt 2>&1 || { tail $OUT/ubench_idx.txt; exit 7; }
           cat $OUT/ubench_idx.txt ;;
    mfma) timeout -k 10 60 tools/ubench_mfma_add > $OUT/ubench_mfma_add.txt 2>&1 || { tail $OUT/ubench_mfma_add.txt; exit 8; }
           cat $OUT/ubench_mfma_add.txt ;;
    stages) timeout -k 10 300 python tools/stage_times.py > $OUT/stages.json 2> $OUT/stages.err || { tail $OUT/stages.err; exit 3; }
           cat $OUT/stages.json ;;
    stages1) FMRX_STEREO_CHUNKS=1 timeout -k 10 300 python tools/stage_times.py --no-gib --single 0 > $OUT/stages_serial.json 2> $OUT/stages1.err || { tail $OUT/stages1.err; exit 3; }
           cat $OUT/stages_serial.json ;;
    pipe) timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "pipelined or stereo_multistream or many_streams or bench_config or call_split" > $OUT/pipe.log 2>&1 || { tail -40 $OUT/pipe.log; exit 13; }
           tail -2 $OUT/pipe.log ;;
    bench) timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 4; }
           python -c "import json; j=json.load(open('$OUT/bench.json')); print(j['value'], j['roofline']['kernel_ms'], json.dumps(j.get('baseline_configs',{}))[:1500])" ;;
    n2) FMRX_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 3 --no-cpu-baseline \
          > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err || { tail $OUT/bench_n2_gloo.err; exit 9; }
          tail -c 3000 $OUT/bench_n2_gloo.json ;;
    rprof) TR="262144 524288 1048576 2097152 4194304"
           timeout -k 10 120 python tools/runner_prof.py --save /tmp/rp_states.npz $(for t in $TR; do echo --trig $t; done) \
               > $OUT/runner_prof.txt 2>&1 || { tail $OUT/runner_prof.txt; exit 10; }
           for tr in $TR; do
             FMRX_LIB_PATH=software-defined-radio-course-project_amd/build_ab/libfmrx.so timeout -k 10 120 \
               python tools/runner_prof.py --load /tmp/rp_states.npz --trig $tr >> $OUT/runner_prof.txt 2>&1 || { tail $OUT/runner_prof.txt; exit 10; }
           done
           timeout -k 10 120 python tools/runner_prof.py --load /tmp/rp_states.npz $(for t in $TR; do echo --trig $t; done) \
               >> $OUT/runner_prof.txt 2>&1 || { tail $OUT/runner_prof.txt; exit 10; }
           grep -v amdgpu.ids $OUT/runner_prof.txt ;;
    predict) timeout -k 10 300 python tools/make_carrier.py /tmp/carrier.f32 72 > $OUT/predict.txt 2>&1 || { tail $OUT/predict.txt; exit 11; }
             g++ -O2 -ffp-contract=off -o /tmp/pll_predict tools/pll_predict.cpp || exit 11
             timeout -k 10 600 /tmp/pll_predict /tmp/carrier.f32 2 >> $OUT/predict.txt 2>&1 || { tail $OUT/predict.txt; exit 11; }
             grep -A20 "extrapolated centre" $OUT/predict.txt | head -24
             tail -40 $OUT/predict.txt ;;
    ktrace) timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/kt_c4 -o run --output-format csv -- \
              python3 tools/stage_times.py --no-gib --single 0 > $OUT/kt_c4.log 2>&1 || { tail $OUT/kt_c4.log; exit 14; }
            f=$(ls $OUT/kt_c4/*/run_kernel_trace.csv $OUT/kt_c4/run_kernel_trace.csv 2>/dev/null | head -1)
            python tools/trace_overlap.py $f > $OUT/overlap_c4.json && cat $OUT/overlap_c4.json ;;
    redoc4) FMRX_LIB_PATH=software-defined-radio-course-project_amd/build_ab/libfmrx.so timeout -k 10 300 \
              python tools/stage_times.py --no-gib --single 0 > $OUT/redo_c4.json 2> $OUT/redo_c4.err || { tail $OUT/redo_c4.err; exit 15; }
            grep -v amdgpu.ids $OUT/redo_c4.err ;;
    libab) # stage_times with each A/B build named in $LIBS (package-relative .so paths), alternating, twice
            for r in 1 2; do for lib in ${LIBS:-libfmrx.so}; do
              tagl=$(echo $lib | tr / _)
              FMRX_LIB_PATH=software-defined-radio-course-project_amd/$lib timeout -k 10 300 python tools/stage_times.py \
                > $OUT/libab_${r}_$tagl.json 2>> $OUT/libab.err || { tail $OUT/libab.err; exit 16; }
              echo "$r $lib $(python -c "import json,sys; j=json.load(open(sys.argv[1])); print({k: v['wall_s'] for k, v in j.items()})" $OUT/libab_${r}_$tagl.json)"
            done; done ;;
    s32) for k in 1 8; do FMRX_STEREO_CHUNKS=$k timeout -k 10 300 python tools/stage_times.py --streams 32 --no-gib --single 0 \
            > $OUT/stages32_k$k.json 2>> $OUT/s32.err || { tail $OUT/s32.err; exit 17; }
          echo "k=$k $(python -c "import json,sys; j=json.load(open(sys.argv[1])); print({k: v['wall_s'] for k, v in j.items()})" $OUT/stages32_k$k.json)"; done ;;
    rprof22) TR=${TRIGS:-2097152 4194304 8388608}
           timeout -k 10 120 python tools/runner_prof.py --save /tmp/rp_states.npz $(for t in $TR; do echo --trig $t; done) \
               > $OUT/runner_prof22.txt 2>&1 || { tail $OUT/runner_prof22.txt; exit 10; }
           for tr in $TR; do
             FMRX_LIB_PATH=software-defined-radio-course-project_amd/build_ab/libfmrx.so timeout -k 10 120 \
               python tools/runner_prof.py --load /tmp/rp_states.npz --trig $tr >> $OUT/runner_prof22.txt 2>&1 || { tail $OUT/runner_prof22.txt; exit 10; }
           done
           grep -v amdgpu.ids $OUT/runner_prof22.txt ;;
    clitrace) # kernel stats of the CLI over 1 GiB of the bench stream (full kernel names: runner forms per range)
            timeout -k 10 200 python -c "import sys; sys.path.insert(0, 'tests'); import iqgen; fm = iqgen.load_fmrx(); f = open('/tmp/iq1g.u8', 'wb'); [f.write(fm.synth_host(5, 2400000, p, 1 << 25).tobytes()) for p in range(0, 1 << 29, 1 << 25)]; f.close()" || exit 19
            timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_cli -o run --output-format csv -- \
              software-defined-radio-course-project_amd/bin/fmrx 0 2 --batch 2048 < /tmp/iq1g.u8 > /tmp/cli.s16 2> $OUT/kt_cli.err || { tail $OUT/kt_cli.err; exit 19; }
            f=$(ls $OUT/kt_cli/*/run_kernel_stats.csv $OUT/kt_cli/run_kernel_stats.csv 2>/dev/null | head -1)
            python tools/kernel_stats_summary.py $f > $OUT/cli_kernel_classes.json && cat $OUT/cli_kernel_classes.json
            ls -la /tmp/cli.s16 ;;
    envab) # configs[4] calls with each value of $ENVVAR in $VALS, alternating, twice
            for r in 1 2; do for v in $VALS; do
              env $ENVVAR=$v timeout -k 10 300 python tools/stage_times.py --no-gib --single 0 \
                > $OUT/envab_${r}_$v.json 2>> $OUT/envab.err || { tail $OUT/envab.err; exit 18; }
              echo "$r $ENVVAR=$v $(python -c "import json,sys; j=json.load(open(sys.argv[1])); print({k: v['wall_s'] for k, v in j.items()}, {k: round(x['ms'],1) for k, x in j['configs[4]']['stages'].items() if 'runner' in k})" $OUT/envab_${r}_$v.json)"
            done; done ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 5; }
           tail -1 $OUT/smoke.log ;;
  esac
done
echo all done
