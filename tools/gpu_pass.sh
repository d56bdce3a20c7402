#!/bin/bash
# One GPU pass in priority order, inside one gpurun call (run from the repo root):
#   tools/gpu_pass.sh <tag> [budget_s] [steps...]
# steps (default: dpt bench ab prof phases decab tests): each GPU step runs under its own
# timeout; a step starts only while the call's time budget allows it; a timeout, abort or
# segfault (124/137/134/139) ends the pass, a failing test run (rc 1) does not.
TAG=${1:-r05x}; BUDGET=${2:-1100}; shift 2 || true
STEPS=${*:-dpt bench ab prof phases decab tests}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
T0=$(date +%s)
left() { echo $(( BUDGET - ($(date +%s) - T0) )); }
run() {   # run <name> <need_s> <timeout_s> <cmd...>
  local name=$1 need=$2 to=$3; shift 3
  if [ "$(left)" -lt "$need" ]; then echo "skip $name (budget)" >> "$OUT/pass.txt"; return 0; fi
  local t=$(date +%s)
  timeout -k 10 "$to" "$@"
  local rc=$?
  echo "$name rc=$rc $(( $(date +%s) - t ))s left=$(left)" >> "$OUT/pass.txt"
  echo "$name rc=$rc" >&2
  case $rc in 124|137|134|139) echo "stop after $name" >&2; cat "$OUT/pass.txt" >&2; exit $rc ;; esac
  return 0
}
lastms() { python -c "import json,sys;print(json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])['ms_per_step'])" "$1" 2>&1 | tail -1; }
for s in $STEPS; do
  case $s in
    dpt) run dpt 200 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_syncbn.py tests/test_gpu_norm.py \
           tests/test_gpu_overlap.py tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_gpu_metrics.py \
           -x -v --timeout 300 --timeout-method thread > "$OUT/dpt_tests.log" 2>&1 ;;
    bench) run bench 150 420 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    ab) for i in 1 2; do
          for e in TT2_WGRAD_OVERLAP=0 TT2_WGRAD_OVERLAP=1; do
            run "ab $e" 90 200 env $e python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-decode \
              > "$OUT/ab_run.json" 2> "$OUT/ab_run.err"
            echo "$e $(lastms "$OUT/ab_run.json")" >> "$OUT/ab.txt"
          done
        done ;;
    knobs) for e in ${KNOBS:-TT2_SIDE_WG=128 TT2_SIDE_SPLIT=2 TT2_SIDE_START=1 TT2_SIDE_START=3 TT2_WGRAD_OVERLAP=1}; do
             run "knob $e" 90 200 env ${e//,/ } python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-decode \
               > "$OUT/ab_run.json" 2> "$OUT/ab_run.err"
             echo "$e $(lastms "$OUT/ab_run.json")" >> "$OUT/knobs.txt"
           done ;;
    attn) for v in ${ATTN_VARIANTS:-3 4 5 3 4 5}; do
            run "attn $v" 60 120 env TT2_ATTN_VARIANT=$v python -u tools/attn_bench.py >> "$OUT/attn_v$v.txt" 2>&1
          done ;;
    attnab) for i in 1 2; do
              for lib in abl/${ATTNAB_OLD:-attn0}.so transformer-tacotron2_amd/tt2/libtt2.so; do
                echo "== $lib" >> "$OUT/attnab.txt"
                run "attnab $lib" 60 120 env TT2_LIB=$lib python -u tools/attn_bench.py >> "$OUT/attnab.txt" 2>&1
              done
            done ;;
    stepab) for i in 1 2; do
              for lib in abl/${STEPAB_OLD:-attn0}.so transformer-tacotron2_amd/tt2/libtt2.so; do
                run "stepab $lib" 90 200 env TT2_LIB=$lib python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline \
                  --no-decode > "$OUT/ab_run.json" 2> "$OUT/ab_run.err"
                echo "$lib $(lastms "$OUT/ab_run.json")" >> "$OUT/stepab.txt"
              done
            done ;;
    attnt) run attnt 60 300 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread \
             > "$OUT/attn_tests.log" 2>&1 ;;
    encg) run encg 60 200 python -u tools/enc_gemm_ab.py > "$OUT/enc_gemm.txt" 2>&1 ;;
    normab) for i in 1 2; do
              for lib in abl/norm0.so transformer-tacotron2_amd/tt2/libtt2.so; do
                run "normab $lib" 60 120 env TT2_LIB=$lib python -u tools/norm_ab.py >> "$OUT/normab.txt" 2>&1
              done
            done ;;
    decg) for i in 1 2; do
            for gs in 1 8 16; do
              run "decg $gs" 90 200 env TT2_DEC_GRAPH_STEPS=$gs python3 -u tools/decode_bench_only.py \
                > "$OUT/dec_run.json" 2> "$OUT/dec_run.err"
              echo "steps=$gs $(python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(d['decode']['value'], d.get('decode_longform',{}).get('value'))" "$OUT/dec_run.json" 2>&1 | tail -1)" >> "$OUT/decg.txt"
            done
          done ;;
    dect) run dect 60 300 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 200 --timeout-method thread \
            > "$OUT/dec_tests.log" 2>&1 ;;
    normt) run normt 60 300 python -u -m pytest tests/test_gpu_norm.py tests/test_gpu_syncbn.py tests/test_gpu_fullsize.py \
             -x -q --timeout 200 --timeout-method thread > "$OUT/norm_tests.log" 2>&1 ;;
    distt) run distt 60 300 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_syncbn.py -v --timeout 200 \
             --timeout-method thread > "$OUT/dist_tests.log" 2>&1 ;;
    otl) run otl 90 200 python -u tools/overlap_timeline.py > "$OUT/otl.txt" 2>&1 ;;
    prof) run prof 150 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- \
            python3 bench.py --profile-run --steps 10 --warmup 2 > "$OUT/bench_step.json" 2> "$OUT/bench_step.err" ;;
    phases) run phases 120 300 env TT2_LIB=abl/phase.so python -u tools/g7_phases.py --json "$OUT/phases.json" \
              > "$OUT/phases.txt" 2>&1 ;;
    decab) for i in 1 2; do
             for lib in abl/${DECAB_OLD:-dec0}.so transformer-tacotron2_amd/tt2/libtt2.so; do
               run "decab $lib" 90 240 env TT2_LIB=$lib python3 -u tools/decode_bench_only.py \
                 > "$OUT/dec_run.json" 2> "$OUT/dec_run.err"
               echo "$lib $(python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(d['decode']['value'], d['longform']['value'])" "$OUT/dec_run.json" 2>&1 | tail -1)" >> "$OUT/decab.txt"
             done
           done ;;
    pmc) run pmc_f 120 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
           python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-decode > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err"
         run pmc_w 120 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
           python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-decode > "$OUT/bench_write.json" 2> "$OUT/bench_write.err" ;;
    mfma) run mfma 120 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/mfma" -o run \
            --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-decode --no-cpu-baseline --no-ragged \
            > "$OUT/bench_mfma.json" 2> "$OUT/bench_mfma.err" ;;
    dpmc) run dpmc_f 120 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/dtr/fetch" -o run --output-format csv -- \
            python3 tools/decode_traffic.py --out="$OUT/dtr" > "$OUT/dtr_fetch.log" 2>&1
          run dpmc_w 120 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/dtr/write" -o run --output-format csv -- \
            python3 tools/decode_traffic.py --out="$OUT/dtr" > "$OUT/dtr_write.log" 2>&1 ;;
    lpmc) run lpmc_f 150 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/ltr/fetch" -o run --output-format csv -- \
            python3 tools/decode_traffic.py --longform --out="$OUT/ltr" > "$OUT/ltr_fetch.log" 2>&1
          run lpmc_w 150 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/ltr/write" -o run --output-format csv -- \
            python3 tools/decode_traffic.py --longform --out="$OUT/ltr" > "$OUT/ltr_write.log" 2>&1 ;;
    tests) run tests 300 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
             > "$OUT/gpu_tests.log" 2>&1
           run smoke 60 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    probe) # SyncBN + encoder overlap capture probes, least to most likely to crash (tools/capture_probe.py)
           for args in ${PROBES:-"--kind record --shape cfg2 --snap"}; do
             run "probe ${args//,/ }" 60 180 python -u tools/capture_probe.py ${args//,/ } >> "$OUT/probe.txt" 2>&1
           done ;;
    topo) for t in ${TOPOS:-simple nested2o nested2s refork reforks}; do
            run "topo $t" 30 60 python -u tools/capture_topo.py $t >> "$OUT/topo.txt" 2>&1
          done ;;
    pkgab) for i in 1 2 3; do   # host-schedule A/B: abl/pkg_<name>/tt2 (a copy of the package at an older commit)
             for pk in abl/pkg_${PKGAB_OLD:-head} ""; do
               run "pkgab $pk" 90 200 env TT2_PKG=$pk TT2_LIB=$PWD/transformer-tacotron2_amd/tt2/libtt2.so python -u \
                 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-decode > "$OUT/ab_run.json" 2> "$OUT/ab_run.err"
               echo "${pk:-current} $(lastms "$OUT/ab_run.json")" >> "$OUT/pkgab.txt"
             done
           done ;;
    dpab) for i in 1 2; do   # DP schedule on one GPU: no exchange / 1-rank RCCL in-graph / N-rank stand-in
            for m in "" "--force-dp" "--dp-standin"; do
              run "dpab $m" 90 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-decode --no-ragged \
                $m > "$OUT/ab_run.json" 2> "$OUT/ab_run.err"
              echo "${m:-plain} $(lastms "$OUT/ab_run.json")" >> "$OUT/dpab.txt"
            done
          done ;;
    bucketab) for i in 1 2; do   # bucket size under the stand-in (and the 1-rank RCCL path)
                for mb in ${BUCKETS:-25 12.5 8}; do
                  for m in ${BUCKET_MODES:---dp-standin}; do
                    run "bucketab $mb $m" 90 200 env TT2_BUCKET_MB=$mb python -u bench.py --steps 30 --warmup 5 \
                      --no-cpu-baseline --no-decode --no-ragged $m > "$OUT/ab_run.json" 2> "$OUT/ab_run.err"
                    echo "$mb $m $(lastms "$OUT/ab_run.json")" >> "$OUT/bucketab.txt"
                  done
                done
              done ;;
    modeab) for i in 1 2; do   # layer-aligned vs fixed-size DP buckets, no-DP step beside them
              run "modeab plain" 90 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-decode \
                --no-ragged > "$OUT/ab_run.json" 2> "$OUT/ab_run.err"
              echo "plain $(lastms "$OUT/ab_run.json")" >> "$OUT/modeab.txt"
              for mode in layers fixed; do
                for m in --dp-standin --force-dp; do
                  run "modeab $mode $m" 90 200 env TT2_BUCKET_MODE=$mode python -u bench.py --steps 30 --warmup 5 \
                    --no-cpu-baseline --no-decode --no-ragged $m > "$OUT/ab_run.json" 2> "$OUT/ab_run.err"
                  echo "$mode $m $(lastms "$OUT/ab_run.json")" >> "$OUT/modeab.txt"
                done
              done
            done ;;
    deferab) for i in 1 2; do   # bucket hand-off right after its side job (0) or after the next one (1)
               run "deferab plain" 90 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-decode \
                 --no-ragged > "$OUT/ab_run.json" 2> "$OUT/ab_run.err"
               echo "plain $(lastms "$OUT/ab_run.json")" >> "$OUT/deferab.txt"
               for dfr in 0 1; do
                 for m in --dp-standin --force-dp; do
                   run "deferab $dfr $m" 90 200 env TT2_DEFER_FORK=$dfr python -u bench.py --steps 30 --warmup 5 \
                     --no-cpu-baseline --no-decode --no-ragged $m > "$OUT/ab_run.json" 2> "$OUT/ab_run.err"
                   echo "defer=$dfr $m $(lastms "$OUT/ab_run.json")" >> "$OUT/deferab.txt"
                 done
               done
             done ;;
    encblas) run encblas 90 200 python -u tools/blas_cmp.py enc > "$OUT/encblas.txt" 2>&1
             run encblas_prof 90 300 rocprofv3 --kernel-trace --stats -d "$OUT/blas" -o run --output-format csv -- \
               python3 tools/blas_cmp.py enc > "$OUT/encblas_prof.txt" 2>&1 ;;
    libenc) for i in 1 2; do   # encoder shapes (tools/blas_cmp.py enc) against an A/B library
              for lib in abl/${LIBENC_OLD:-g8r8}.so transformer-tacotron2_amd/tt2/libtt2.so; do
                echo "== $lib" >> "$OUT/libenc.txt"
                run "libenc $lib" 60 150 env TT2_LIB=$lib python -u tools/blas_cmp.py enc >> "$OUT/libenc.txt" 2>&1
              done
            done ;;
    libab) for i in 1 2; do   # v7 / grouped-v7 shapes (tools/lib_ab.py) against an A/B library, outputs compared
             run "libab old" 60 150 env TT2_LIB=abl/${LIBAB_OLD:-prio0}.so python -u tools/lib_ab.py run /tmp/libab_old.pt \
               >> "$OUT/libab_old.txt" 2>&1
             run "libab new" 60 150 python -u tools/lib_ab.py run /tmp/libab_new.pt >> "$OUT/libab_new.txt" 2>&1
           done
           python tools/lib_ab.py compare /tmp/libab_old.pt /tmp/libab_new.pt > "$OUT/libab_cmp.txt" 2>&1 ;;
    encab) for lib in ${ENCAB_LIBS:-abl/g8lw8.so}; do   # forced v8 (15) vs auto on the encoder shapes, per library
             echo "== $lib" >> "$OUT/encab.txt"
             run "encab $lib" 60 150 env TT2_LIB=$lib python -u tools/gemm_ab.py 15 enc >> "$OUT/encab.txt" 2>&1
           done ;;
    otls) run otls 90 200 python -u tools/overlap_timeline.py --standin > "$OUT/otl_standin.txt" 2>&1 ;;
    det) run det 60 200 python -u tools/det_check.py > "$OUT/det.txt" 2>&1 ;;
    newt) run newt 120 600 python -u -m pytest ${NEWT:-tests/test_gpu_capture.py tests/test_gpu_dp_order.py} -x -v \
            --timeout 600 --timeout-method thread > "$OUT/new_tests.log" 2>&1 ;;
    decprof) run decprof 120 300 rocprofv3 --kernel-trace --stats -d "$OUT/dk" -o run --output-format csv -- \
               python3 tools/decode_prof.py > "$OUT/decprof.log" 2>&1 ;;
    *) echo "unknown step $s" ;;
  esac
done
cat "$OUT/pass.txt"
