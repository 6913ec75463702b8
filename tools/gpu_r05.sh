#!/bin/bash
# tools/gpu_r05.sh <tag> [steps...] — round-5 GPU steps, each under its own time limit, stopping at
# the first failure.  Steps:
#   cnt       tools/ubench_cnt (chain forms' dependent latency per piece)
#   mode2     configs[3] (mode-2 mono, 1 GiB) profile of record: a warm (>= 1.5 s) kernel trace and
#             separate PMC passes FETCH_SIZE / WRITE_SIZE / GRBM (tools/bench_modes.py --modes 2)
#   tests     the whole GPU suite
#   pll       the PLL / stereo GPU tests
#   stages    tools/stage_times.py (one 10 s stream, configs[4], configs[2] stage times)
#   bench     bench.py without the CPU baseline
#   pllcnt    the PLL / stereo GPU tests with the count runner on the forms in $CNT (bitmask, default 31)
#   envab     stage_times per value of $ENVVAR in $VALS ($STARGS: its arguments), alternating, twice
#   seam      tools/bench_seam.py (per-block fmrx_rf_block + fmrx_audio_block, two contexts, the CLI at --batch 16)
#   rprof     tools/runner_prof.py per form ($TRIGS) and FMRX_PLL_CNT value ($CNTS), FMRX_AB_PROF build
#   n2        the N=2 bench line rehearsed with gloo (both ranks on device 0), chunked configs[4] gather
#   profmono  tools/gpu_bench_prof.sh (bench line, kernel trace, FETCH/WRITE/GRBM passes of the fused kernel)
#   libab     stage_times per library in $LIBS (A/B builds), alternating, twice
#   rec       the record: tests smoke, tools/gpu_bench_prof.sh (bench line, trace, PMC), mode2 stages seam
#   smoke     __graft_entry__.smoke()
set -o pipefail
TAG=${1:-r05}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
M2="python3 tools/bench_modes.py --modes 2 --steps 20 --warmup-seconds 1.5"
for step in "$@"; do
  case $step in
    cnt) timeout -k 10 120 tools/ubench_cnt > $OUT/ubench_cnt.txt 2>&1 || { tail $OUT/ubench_cnt.txt; exit 7; }
         cat $OUT/ubench_cnt.txt ;;
    mode2) timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/m2_kt -o run --output-format csv -- \
             $M2 > $OUT/m2_kt.log 2>&1 || { tail $OUT/m2_kt.log; exit 8; }
           timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/m2_fetch -o run --output-format csv -- \
             $M2 > $OUT/m2_fetch.log 2>&1 || { tail $OUT/m2_fetch.log; exit 8; }
           timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/m2_write -o run --output-format csv -- \
             $M2 > $OUT/m2_write.log 2>&1 || { tail $OUT/m2_write.log; exit 8; }
           timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/m2_grbm -o run --output-format csv -- \
             $M2 > $OUT/m2_grbm.log 2>&1 || { tail $OUT/m2_grbm.log; exit 8; }
           cat $OUT/m2_kt.log ;;
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
           tail -2 $OUT/tests.log ;;
    pll) timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pll or stereo or bench_config or trig_hint or refdata or cli or index" > $OUT/pll.log 2>&1 || { tail -40 $OUT/pll.log; exit 2; }
         tail -2 $OUT/pll.log ;;
    stages) timeout -k 10 300 python tools/stage_times.py > $OUT/stages.json 2> $OUT/stages.err || { tail $OUT/stages.err; exit 3; }
            cat $OUT/stages.json ;;
    bench) timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 4; }
           python -c "import json; j=json.load(open('$OUT/bench.json')); print(j['value'], j['roofline']['kernel_ms'], json.dumps(j.get('baseline_configs',{}))[:1500])" ;;
    pllcnt) FMRX_PLL_CNT=${CNT:-31} timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pll or stereo or index or bench_config or refdata or cli or pipe" > $OUT/pllcnt.log 2>&1 || { tail -40 $OUT/pllcnt.log; exit 12; }
         tail -2 $OUT/pllcnt.log ;;
    envab) # stage_times (configs[4], one 10 s stream, configs[2]) per value of $ENVVAR in $VALS, alternating, twice
         for r in 1 2; do for v in $VALS; do
           env $ENVVAR=$v timeout -k 10 300 python tools/stage_times.py $STARGS > $OUT/envab_${r}_$v.json 2>> $OUT/envab.err || { tail $OUT/envab.err; exit 18; }
           echo "$r $ENVVAR=$v $(python tools/stage_summary.py $OUT/envab_${r}_$v.json)"
         done; done ;;
    seam) timeout -k 10 400 python tools/bench_seam.py > $OUT/bench_seam.json 2> $OUT/bench_seam.err || { tail $OUT/bench_seam.err; exit 19; }
          cat $OUT/bench_seam.json ;;
    rprof) # per-form runner timing from the bench stream's real state at each trigOffset in $TRIGS, per
           # FMRX_PLL_CNT value in $CNTS, with the FMRX_AB_PROF build (chain / evaluator cycles an interval)
           TR=${TRIGS:-"131072 262144 524288 1048576 2097152"}
           timeout -k 10 120 python tools/runner_prof.py --save /tmp/rp_states.npz $(for t in $TR; do echo --trig $t; done) \
               > $OUT/rprof.txt 2>&1 || { tail $OUT/rprof.txt; exit 10; }
           for c in ${CNTS:-0 31}; do for tr in $TR; do
             echo "== FMRX_PLL_CNT=$c trig $tr" >> $OUT/rprof.txt
             FMRX_PLL_CNT=$c FMRX_LIB_PATH=software-defined-radio-course-project_amd/build_ab/libfmrx.so timeout -k 10 120 \
               python tools/runner_prof.py --load /tmp/rp_states.npz --trig $tr >> $OUT/rprof.txt 2>&1 || { tail $OUT/rprof.txt; exit 10; }
           done; done
           grep -v amdgpu.ids $OUT/rprof.txt ;;
    n2) FMRX_BENCH_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 3 --no-cpu-baseline \
          > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err || { tail $OUT/bench_n2_gloo.err; exit 9; }
        python -c "import json; j=json.load(open('$OUT/bench_n2_gloo.json')); c=j['baseline_configs']['configs[4]']; print(j['value'], {k: c.get(k) for k in ('seconds', 'seconds_process', 'seconds_gather', 'gather_chunks', 'gather_GBs_after_processing', 'bit_exact_vs_reference')})" ;;
    profmono) bash tools/gpu_bench_prof.sh $TAG/prof_mono || exit 20 ;;
    libab) # stage_times with each library in $LIBS (package-relative .so paths), alternating, twice
         for r in 1 2; do for lib in ${LIBS:-libfmrx.so}; do
           tagl=$(echo $lib | tr / _)
           FMRX_LIB_PATH=software-defined-radio-course-project_amd/$lib timeout -k 10 300 python tools/stage_times.py $STARGS \
             > $OUT/libab_${r}_$tagl.json 2>> $OUT/libab.err || { tail $OUT/libab.err; exit 16; }
           echo "$r $lib $(python tools/stage_summary.py $OUT/libab_${r}_$tagl.json)"
         done; done ;;
    rec) # the round's record at HEAD: GPU suite, smoke, bench line + kernel trace + PMC passes of the
         # fused kernel (tools/gpu_bench_prof.sh), configs[3]'s passes, stage times, the seam
         bash tools/gpu_r05.sh $TAG tests smoke && bash tools/gpu_bench_prof.sh $TAG/prof_mono && \
         bash tools/gpu_r05.sh $TAG mode2 stages seam || exit 21 ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 5; }
           tail -1 $OUT/smoke.log ;;
  esac
done
echo all done
