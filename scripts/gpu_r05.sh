#!/bin/bash
# Round-5 GPU steps; each under its own time limit, stop at the first failure.
#   scripts/gpu_r05.sh OUTDIR step [step ...]
# steps: pf (prefetch A/B, tools/tune_multi_pf), slice (scripts/slice_probe.py),
#        slice_prof (the same, rank 0 under rocprofv3 --kernel-trace),
#        va (tools/va_reuse_probe single-process modes), va_ipc (its 12-process mode),
#        tests:<pytest -k expr> (pytest -m gpu subset)
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
for step in "$@"; do
    echo "step $step $(date +%T)" >> $OUT/steps.log
    case $step in
    pf)
        for spec in "multi 8 24" "multi 4 24" "multi 16 24" "multi 8 26" "tree 8 24" "tree 3 24" "tree 12 24" "tree 6 24"; do
            tag=$(echo $spec | tr ' ' '_')
            timeout -k 10 150 tools/tune_multi_pf $spec 7 > $OUT/pf_$tag.txt 2>&1 || exit 1
        done ;;
    slice)
        timeout -k 10 500 python scripts/slice_probe.py $OUT/slice 4 2000 > $OUT/slice.txt 2>&1 || exit 1 ;;
    slice_extra)
        timeout -k 10 200 python scripts/slice_probe.py $OUT/slice 4 2000 mixed:none:all \
            freed:none:all shareable:none:one > $OUT/slice_extra.txt 2>&1 || exit 1 ;;
    slice_prof)
        SLICE_PROF_DIR=$OUT/slice_prof timeout -k 10 300 python scripts/slice_probe.py $OUT/slice_prof 4 2000 \
            shareable:read:all plain:read:all > $OUT/slice_prof.txt 2>&1 || exit 1 ;;
    slice_hsa)
        SLICE_PROF_DIR=$OUT/slice_hsa SLICE_PROF_TRACE=--hsa-trace timeout -k 10 300 \
            python scripts/slice_probe.py $OUT/slice_hsa 1 200 shareable:none:one plain:none:one \
            > $OUT/slice_hsa.txt 2>&1 || exit 1 ;;
    c4full)
        timeout -k 10 400 python -u -m pytest tests/test_group.py -m gpu -x -v -s --timeout 320 \
            --timeout-method thread -k c4_full_size > $OUT/c4full.log 2>&1 || exit 1 ;;
    pf2)
        for spec in "multi 8 24" "multi 8 26" "multi 16 24" "tree 8 24"; do
            tag=$(echo $spec | tr ' ' '_')
            timeout -k 10 200 tools/tune_multi_pf $spec 9 > $OUT/pf2_$tag.txt 2>&1 || exit 1
        done ;;
    pf3)
        for spec in "multi 8 24" "multi 8 26" "multi 16 24"; do
            tag=$(echo $spec | tr ' ' '_')
            timeout -k 10 200 tools/tune_multi_pf $spec 9 > $OUT/pf3_$tag.txt 2>&1 || exit 1
        done
        for c in FETCH_SIZE WRITE_SIZE; do
            timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv \
                -d $OUT/pf3_pmc/pmc_$c -o s -- tools/tune_multi_pf multi 8 24 1 \
                > $OUT/pf3_pmc_$c.txt 2>&1 || exit 1
        done
        python3 scripts/pmc_kernels.py $OUT/pf3_pmc > $OUT/pf3_pmc_by_kernel.txt 2>&1 ;;
    pf4)
        # prefetch distance: the tree fan-in's A/B, and the multi product at two tiles
        for spec in "tree 8 24" "tree 16 24" "tree 3 24" "tree 12 24" "tree 8 26" "multi 8 24" "multi 16 24"; do
            tag=$(echo $spec | tr ' ' '_')
            timeout -k 10 200 tools/tune_multi_pf $spec 9 > $OUT/pf4_$tag.txt 2>&1 || exit 1
        done ;;
    stagger)
        # do operands a power of two apart lose to HBM channel conflicts?
        for spec in "multi 8 26" "multi 8 24" "tree 8 26"; do
            for sg in 0 4352 2105600; do
                tag=$(echo $spec $sg | tr ' ' '_')
                timeout -k 10 200 tools/tune_multi_pf $spec 5 $sg > $OUT/stagger_$tag.txt 2>&1 || exit 1
            done
        done ;;
    pf_pmc)
        # one rocprofv3 pass per counter (FETCH_SIZE and WRITE_SIZE cannot share one)
        for spec in "multi 8 24" "tree 8 24" "tree 3 24"; do
            tag=$(echo $spec | tr ' ' '_')
            for c in FETCH_SIZE WRITE_SIZE; do
                timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv \
                    -d $OUT/pf_pmc_$tag/pmc_$c -o s -- tools/tune_multi_pf $spec 1 \
                    > $OUT/pf_pmc_${tag}_$c.txt 2>&1 || exit 1
            done
            python3 scripts/pmc_kernels.py $OUT/pf_pmc_$tag > $OUT/pf_pmc_${tag}_by_kernel.txt 2>&1
        done ;;
    gather_pmc)
        timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv \
            -d $OUT/gather_pmc/pmc_hit -o s -- tools/tune_misalign 1 > $OUT/gather_pmc_hit.txt 2>&1 || exit 1
        timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv \
            -d $OUT/gather_pmc/pmc_fetch -o s -- tools/tune_misalign 1 > $OUT/gather_pmc_fetch.txt 2>&1 || exit 1
        python3 scripts/pmc_kernels.py $OUT/gather_pmc > $OUT/gather_pmc_by_kernel.txt 2>&1 ;;
    va)
        timeout -k 10 300 tools/va_reuse_probe 200 6 > $OUT/va_reuse.txt 2>&1 || exit 1 ;;
    va_ipc)
        timeout -k 10 560 python scripts/va_reuse_ipc.py $OUT/va_ipc 12 100 6 close hold > $OUT/va_ipc.txt 2>&1 || exit 1 ;;
    tests:all)
        timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
            > $OUT/pytest_gpu.log 2>&1 || exit 1 ;;
    c3i)
        timeout -k 10 300 python scripts/c3_interleaved.py $OUT/c3_interleaved.json > $OUT/c3_interleaved.txt 2>&1 || exit 1 ;;
    prof)
        timeout -k 10 1000 scripts/profile_round.sh ${OUT#gpurun_out/}/prof > $OUT/profile_round.txt 2>&1 || exit 1 ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1 ;;
    c1ab)
        timeout -k 10 700 python scripts/c1_dev_ab.py $OUT/c1_dev_ab.json 2 r05 > $OUT/c1_dev_ab.log 2>&1 || exit 1 ;;
    bench)
        timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1 ;;
    tests:*)
        expr=${step#tests:}
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
            -k "$expr" > $OUT/pytest_$(echo "$expr" | tr -c 'a-zA-Z0-9_' '_' | cut -c1-40).log 2>&1 || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
echo "done $(date +%T)" >> $OUT/steps.log
