#!/bin/bash
# One GPU-box driver for every measurement this repo takes (run through
# gpurun from the repo root).  Steps run in order and the script stops at the
# first failure; every GPU step has its own time limit.
#
#   tools/gpu/run.sh STEP [STEP ...]
#
#   test[:FILES]          pytest -m gpu (FILES comma-separated, default tests/)
#   bench[:CFG[:ENGINE]]  bench.py line -> gpurun_out/bench_cCFG_ENGINE.json
#   kstats[:CFG[:ENGINE]] rocprofv3 --kernel-trace --stats of the bench
#   pmc[:CFG[:ENGINE]]    FETCH_SIZE and WRITE_SIZE passes (one run each)
#   sq[:CFG[:ENGINE]]     two SQ counter passes (waves, VALU, LDS, waits)
#   flops[:CFG[:ENGINE]]  executed FP32 VALU flops (SQ_INSTS_VALU_FLOPS_FP32 + classes)
#   pmcx:CFG:ENGINE:NAME:C1,C2,..  one pass of the listed counters (mind the
#                         per-block limits: 8 SQ, 4 TCC, 4 TCP, 2 TA, 2 TD)
#   ablib[:L1,L2,..]      bench config 2 once per library tdoa/<L>.so (TDOA_LIB)
#   testlib:L[:FILES]     pytest -m gpu against tdoa/<L>.so
#   diagw64               phase stamps of k_p1k_w64 (needs the diag library)
#   diagf16[:CFG]         phase stamps of k_frame16 (config 3 or 4, diag library)
#   calib                 tools/hbm_copy (achievable HBM), plain and under rocprofv3
#   smoke                 __graft_entry__.smoke()
#
# Env: TAG (output subdirectory, default "cur"), STEPS (bench steps),
# BENCH_ARGS (extra bench.py arguments).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
TAG=${TAG:-cur}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ROOT=$GRAFT_REPO_ROOT

field() {  # field N of a colon-separated step, with a default
    local v
    v=$(echo "$1" | cut -d: -f"$2")
    [ "$v" = "$1" ] && [ "$2" != 1 ] && v=""
    echo "${v:-$3}"
}

prof() {  # prof NAME ROCPROF-ARGS... -- (bench args follow)
    local name=$1; shift
    (cd /tmp && timeout -s KILL 240 rocprofv3 "$@" -d "$ROOT/$OUT/$name" -o run --output-format csv \
        -- python3 "$ROOT/bench.py" $PARGS > "$ROOT/$OUT/$name.log" 2>&1)
}

for step in "$@"; do
    kind=$(field "$step" 1)
    case $kind in
    test)
        files=$(field "$step" 2 tests)
        files=${files//,/ }
        timeout -k 10 900 python -u -m pytest $files -m gpu -x -v --timeout 120 --timeout-method thread \
            -p no:cacheprovider > "$OUT/pytest.log" 2>&1
        rc=$?
        grep -E "passed|failed|error" "$OUT/pytest.log" | tail -3
        [ $rc -ne 0 ] && { tail -30 "$OUT/pytest.log"; exit $rc; }
        ;;
    ablib)
        # bench config 2 once per library variant (audio-triangulation_amd/tdoa/<name>.so)
        vs=$(field "$step" 2 "libtdoa,libtdoa_alt")
        for l in ${vs//,/ }; do
            TDOA_LIB=$ROOT/audio-triangulation_amd/tdoa/$l.so timeout -k 10 240 python bench.py --steps ${STEPS:-400} \
                --no-cpu $BENCH_ARGS > "$OUT/ablib_$l.log" 2>&1 || { echo "bench $l failed"; tail -5 "$OUT/ablib_$l.log"; exit 21; }
            tail -1 "$OUT/ablib_$l.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$l value %.4g kernel_ms %.4f frac %.4f' % (d['value'], r['kernel_ms'], r['frac']))"
        done
        ;;
    abenv)
        # bench (config 2 unless BENCH_ARGS) once per value of an env switch,
        # ROUNDS times interleaved: abenv:VAR:V1,V2
        var=$(field "$step" 2 TDOA_P1K); vs=$(field "$step" 3 "lean,w64")
        for r in $(seq 1 "${ROUNDS:-1}"); do
            for v in ${vs//,/ }; do
                env "$var=$v" timeout -k 10 240 python bench.py --steps ${STEPS:-400} --no-cpu --no-parity \
                    $BENCH_ARGS > "$OUT/abenv_${v}_$r.log" 2>&1 || { echo "bench $var=$v failed"; tail -5 "$OUT/abenv_${v}_$r.log"; exit 21; }
                tail -1 "$OUT/abenv_${v}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$var=$v value %.4g kernel_us %.2f frac %.4f' % (d['value'], r['kernel_ms']*1e3, r['frac']))"
            done
        done
        ;;
    testlib)
        # pytest -m gpu of FILES against library variant LIB: testlib:LIB:FILES
        l=$(field "$step" 2 libtdoa_alt); files=$(field "$step" 3 tests)
        files=${files//,/ }
        TDOA_LIB=$ROOT/audio-triangulation_amd/tdoa/$l.so timeout -k 10 900 python -u -m pytest $files -m gpu -x -q \
            --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_$l.log" 2>&1
        rc=$?
        grep -E "passed|failed|error" "$OUT/pytest_$l.log" | tail -3
        [ $rc -ne 0 ] && { tail -30 "$OUT/pytest_$l.log"; exit $rc; }
        ;;
    bench)
        c=$(field "$step" 2 2); e=$(field "$step" 3 gcc_phat)
        timeout -k 10 400 python bench.py --config $c --engine $e $BENCH_ARGS > "$OUT/bench_c${c}_$e.log" 2>&1 \
            || { echo "bench failed"; tail -5 "$OUT/bench_c${c}_$e.log"; exit 22; }
        tail -1 "$OUT/bench_c${c}_$e.log" > "$OUT/bench_c${c}_$e.json"
        cut -c1-400 "$OUT/bench_c${c}_$e.json"
        ;;
    kstats)
        c=$(field "$step" 2 2); e=$(field "$step" 3 gcc_phat)
        PARGS="--config $c --engine $e --steps ${STEPS:-50} --warmup 3 --no-cpu $BENCH_ARGS"
        prof "kt_c${c}_$e" --kernel-trace --stats || { echo "kstats failed"; tail -5 "$OUT/kt_c${c}_$e.log"; exit 23; }
        cut -d, -f1-4,6 "$OUT/kt_c${c}_$e/run_kernel_stats.csv" | cut -c1-160 | head -6
        ;;
    pmc)
        c=$(field "$step" 2 2); e=$(field "$step" 3 gcc_phat)
        PARGS="--config $c --engine $e --steps 24 --warmup 2 --no-cpu $BENCH_ARGS"
        prof "fetch_c${c}_$e" --pmc FETCH_SIZE || exit 24
        prof "write_c${c}_$e" --pmc WRITE_SIZE || exit 25
        echo "pmc c$c $e done"
        ;;
    sq)
        c=$(field "$step" 2 2); e=$(field "$step" 3 gcc_phat)
        PARGS="--config $c --engine $e --steps 24 --warmup 2 --no-cpu $BENCH_ARGS"
        prof "sq1_c${c}_$e" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
            SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit 26
        prof "sq2_c${c}_$e" --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU \
            SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA || exit 27
        echo "sq c$c $e done"
        ;;
    flops)
        # executed FP32 VALU work (SQ_INSTS_VALU_FLOPS_FP32 and the instruction
        # classes) of a bench launch: flops[:CFG[:ENGINE]]
        c=$(field "$step" 2 2); e=$(field "$step" 3 gcc_phat)
        PARGS="--config $c --engine $e --steps 24 --warmup 2 --no-cpu $BENCH_ARGS"
        prof "flops_c${c}_$e" --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 \
            SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU SQ_WAVES || exit 34
        echo "flops c$c $e done"
        ;;
    pmcx)
        c=$(field "$step" 2 2); e=$(field "$step" 3 gcc_phat); n=$(field "$step" 4 x)
        ctr=$(field "$step" 5 "")
        [ -z "$ctr" ] && { echo "pmcx needs counters"; exit 2; }
        PARGS="--config $c --engine $e --steps 24 --warmup 2 --no-cpu $BENCH_ARGS"
        prof "${n}_c${c}_$e" --pmc ${ctr//,/ } || exit 29
        echo "pmcx $n c$c $e done"
        ;;
    calib)
        # achievable HBM: tools/hbm_copy (16-B-per-lane copy + read sweeps, 1 GiB
        # buffers) plain, then under rocprofv3 --kernel-trace --stats
        timeout -k 10 120 "$ROOT/tools/hbm_copy" 1024 20 > "$OUT/calib.json" 2> "$OUT/calib.err" \
            || { cat "$OUT/calib.err"; exit 30; }
        cat "$OUT/calib.json"
        (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/calib_kt" -o run \
            --output-format csv -- "$ROOT/tools/hbm_copy" 1024 20 > "$ROOT/$OUT/calib_kt.log" 2>&1) \
            || { tail -5 "$OUT/calib_kt.log"; exit 31; }
        cut -d, -f1-4,6 "$OUT/calib_kt/run_kernel_stats.csv" | head -5
        ;;
    diagw64)
        # phase stamps of k_p1k_w64 (libtdoa_diag.so, make -C audio-triangulation_amd diag)
        timeout -k 10 120 python tools/diag_w64.py > "$OUT/diag_w64.txt" 2>&1 || { tail -5 "$OUT/diag_w64.txt"; exit 32; }
        cat "$OUT/diag_w64.txt"
        ;;
    diagf16)
        # phase stamps of k_frame16 (needs the diag library): diagf16:CFG
        c=$(field "$step" 2 4)
        timeout -k 10 120 python tools/diag_frame16.py $c 8192 > "$OUT/diag_f16_c$c.txt" 2>&1 \
            || { tail -5 "$OUT/diag_f16_c$c.txt"; exit 33; }
        cat "$OUT/diag_f16_c$c.txt"
        ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
            || { tail -20 "$OUT/smoke.log"; exit 28; }
        tail -2 "$OUT/smoke.log"
        ;;
    *)
        echo "unknown step $step"; exit 2 ;;
    esac
done
echo "run.sh done: $*"
