#!/bin/bash
# scripts/gpu_session.sh — one guarded GPU session on the box (used via gpurun).
# Each step runs under its own time limit; a crash-class exit (abort, segfault, timeout,
# kill) ends the session so nothing else touches a possibly faulted GPU. Assertion failures
# (exit 1) do not stop the later measurement steps.
#   scripts/gpu_session.sh <step> [<step> ...]   steps: info tests smoke tbo tbo-<OP> bench prof
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 5 "$OUT/$name.log"
    case $rc in 124|134|137|139) echo "crash-class exit $rc: stopping session"; exit $rc;; esac
    return 0
}
for step in "$@"; do
    case $step in
        info)  run info 60 bash -c 'lscpu | head -20; nproc; rocm-smi --showproductname; python -c "import torch;print(torch.cuda.get_device_name(0))"' ;;
        build) run build 600 python -c "import __graft_entry__ as g; g.build()" ;;
        tests) run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
        testsall) run testsall 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        tbo)   run tbo 900 env GGML_BACKEND_PATH=$PWD/ggml-gfx906_amd/libggml-hip-mi355x.so ./oracle/_ref/test-backend-ops test -o MUL_MAT -b MI355X0 ;;
        tboid) run tboid 900 env GGML_BACKEND_PATH=$PWD/ggml-gfx906_amd/libggml-hip-mi355x.so ./oracle/_ref/test-backend-ops test -o MUL_MAT_ID -b MI355X0 ;;
        tbogr) run tbogr 900 env GGML_BACKEND_PATH=$PWD/ggml-gfx906_amd/libggml-hip-mi355x.so ./oracle/_ref/test-backend-ops test -o GET_ROWS -b MI355X0 ;;
        tbocpy) run tbocpy 900 env GGML_BACKEND_PATH=$PWD/ggml-gfx906_amd/libggml-hip-mi355x.so ./oracle/_ref/test-backend-ops test -o CPY -b MI355X0 ;;
        tbo-*) op=${step#tbo-}; run "tbo_$op" 900 env GGML_BACKEND_PATH=$PWD/ggml-gfx906_amd/libggml-hip-mi355x.so ./oracle/_ref/test-backend-ops test -o "$op" -b MI355X0 ;;
        bench) run bench 600 python bench.py ;;
        ringpar) run ringpar 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "k11008 or k14336 or k14368 or k12288 or k9216 or k8192 or k131072 or k4096 or k1024" ;;
        ringb) run ringb 600 bash -c 'S="q4_0:14336:4096:1:1 q4_0:14336:4096:2:1 q4_0:14336:4096:3:1 q4_0:14336:4096:4:1 q4_0:14336:4096:5:1 q4_0:14336:4096:8:1 q4_K:14336:4096:1:1 q4_K:14336:4096:2:1 q4_K:14336:4096:4:1 q4_K:14336:4096:8:1 q5_K:14336:4096:8:1 q6_K:14336:4096:1:1 q6_K:14336:4096:8:1 q8_0:14336:4096:1:1 q8_0:14336:4096:8:1 q4_0:11008:4096:4:1 q4_0:11008:4096:8:1 q4_0:14336:4096:1:8 q4_0:14336:4096:8:8"; python scripts/mmvq_bench.py $S && GGML_MI355X_RING_DEPTH=2 python scripts/mmvq_bench.py $S && GGML_MI355X_RING_PRE=2 python scripts/mmvq_bench.py q4_0:14336:4096:2:1 q4_K:14336:4096:2:1 q6_K:14336:4096:2:1 q8_0:14336:4096:2:1' ;;
        mmatest) run mmatest 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_mmvq_mma.py ;;
        mmab) run mmab 600 bash -c 'S="q4_0:14336:4096:1:1 q4_0:14336:4096:2:1 q4_0:14336:4096:3:1 q4_0:14336:4096:4:1 q4_0:14336:4096:5:1 q4_0:14336:4096:8:1 q8_0:14336:4096:2:1 q8_0:14336:4096:8:1 q4_K:14336:4096:2:1 q4_K:14336:4096:8:1 q5_K:14336:4096:8:1 q6_K:14336:4096:2:1 q6_K:14336:4096:8:1 q4_0:4096:4096:1:1 q4_0:4096:4096:2:1 q4_0:4096:4096:8:1 q4_K:4096:11008:8:1 q4_0:14336:4096:1:8 q4_0:14336:4096:2:8 q4_0:14336:4096:8:8 q4_K:14336:4096:8:8"; GGML_MI355X_MMA=1 python scripts/mmvq_bench.py $S && GGML_MI355X_MMA=0 python scripts/mmvq_bench.py $S && python scripts/mmvq_bench.py $S' ;;
        profmma) run profmma 300 env GGML_MI355X_MMA=1 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profmma -o run -- python scripts/mmvq_bench.py q4_0:14336:4096:1:1 q4_0:14336:4096:8:1 q4_K:4096:11008:8:1 q4_0:4096:4096:8:1 \
                 && for t in $(find $OUT/profmma -name '*kernel_trace.csv'); do rm -f $t; done ;;
        profmma2) run profmma2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profmma2 -o run -- python scripts/mmvq_bench.py q4_0:14336:4096:8:1 q4_0:4096:11008:8:1 q8_0:4096:11008:8:1 q4_K:14336:4096:8:1 q4_K:4096:14336:8:1 q5_K:4096:11008:8:1 && find $OUT/profmma2 -name '*kernel_trace.csv' -delete ;;
        q8x) run q8x 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mmq8.py tests/test_gpu_parity.py -k "mmq8 or mm_1 or mmid or grouped or m512 or m2048" ;;
        q8xb) run q8xb 600 bash -c 'S="q8_0:4096:4096:512 q4_0:4096:4096:512 q4_K:4096:4096:512 q6_K:4096:11008:512 q8_0:4096:4096:2048 q4_K:4096:11008:512"; python scripts/mmq_bench.py $S' ;;
        rehearse) run rehearse 900 bash -c 'for n in 2 4; do BENCH_ONE_GPU_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 3 --warmup 1 --cpu-seconds 1 || exit 1; done' ;;
        mmaexp) run mmaexp 600 bash scripts/mma_exp.sh run base d4 d5 d6 ;;
        mmaprof) run mmaprof 600 bash scripts/mma_prof.sh $OUT/mmaprof base x1 x2 x3 ;;
        pmcmma) run pmcmma 600 bash -c "bash scripts/pmc_mma.sh mma q4_0:14336:4096:8:1 && MMA=0 bash scripts/pmc_mma.sh valu q4_0:14336:4096:8:1" ;;
        mmasweep) run mmasweep 900 bash -c 'S=" q4_0:4096:4096:4:1 q4_0:4096:4096:5:1 q4_0:4096:4096:6:1 q4_0:4096:4096:8:1 q4_0:4096:11008:4:1 q4_0:4096:11008:5:1 q4_0:4096:11008:6:1 q4_0:4096:11008:8:1 q4_0:11008:4096:4:1 q4_0:11008:4096:5:1 q4_0:11008:4096:6:1 q4_0:11008:4096:8:1 q4_0:14336:4096:4:1 q4_0:14336:4096:5:1 q4_0:14336:4096:6:1 q4_0:14336:4096:8:1 q4_0:4096:14336:4:1 q4_0:4096:14336:5:1 q4_0:4096:14336:6:1 q4_0:4096:14336:8:1 q8_0:4096:4096:4:1 q8_0:4096:4096:5:1 q8_0:4096:4096:6:1 q8_0:4096:4096:8:1 q8_0:4096:11008:4:1 q8_0:4096:11008:5:1 q8_0:4096:11008:6:1 q8_0:4096:11008:8:1 q8_0:11008:4096:4:1 q8_0:11008:4096:5:1 q8_0:11008:4096:6:1 q8_0:11008:4096:8:1 q8_0:14336:4096:4:1 q8_0:14336:4096:5:1 q8_0:14336:4096:6:1 q8_0:14336:4096:8:1 q8_0:4096:14336:4:1 q8_0:4096:14336:5:1 q8_0:4096:14336:6:1 q8_0:4096:14336:8:1 q4_K:4096:4096:4:1 q4_K:4096:4096:5:1 q4_K:4096:4096:6:1 q4_K:4096:4096:8:1 q4_K:4096:11008:4:1 q4_K:4096:11008:5:1 q4_K:4096:11008:6:1 q4_K:4096:11008:8:1 q4_K:11008:4096:4:1 q4_K:11008:4096:5:1 q4_K:11008:4096:6:1 q4_K:11008:4096:8:1 q4_K:14336:4096:4:1 q4_K:14336:4096:5:1 q4_K:14336:4096:6:1 q4_K:14336:4096:8:1 q4_K:4096:14336:4:1 q4_K:4096:14336:5:1 q4_K:4096:14336:6:1 q4_K:4096:14336:8:1 q5_K:4096:4096:4:1 q5_K:4096:4096:5:1 q5_K:4096:4096:6:1 q5_K:4096:4096:8:1 q5_K:4096:11008:4:1 q5_K:4096:11008:5:1 q5_K:4096:11008:6:1 q5_K:4096:11008:8:1 q5_K:11008:4096:4:1 q5_K:11008:4096:5:1 q5_K:11008:4096:6:1 q5_K:11008:4096:8:1 q5_K:14336:4096:4:1 q5_K:14336:4096:5:1 q5_K:14336:4096:6:1 q5_K:14336:4096:8:1 q5_K:4096:14336:4:1 q5_K:4096:14336:5:1 q5_K:4096:14336:6:1 q5_K:4096:14336:8:1"; GGML_MI355X_MMA=1 python scripts/mmvq_bench.py $S && GGML_MI355X_MMA=0 python scripts/mmvq_bench.py $S' ;;
        mmapair) run mmapair 600 bash -c 'S="q4_0:4096:4096:4:1 q4_0:4096:4096:8:1 q4_0:4096:11008:8:1 q4_0:11008:4096:8:1 q4_0:14336:4096:4:1 q4_0:14336:4096:8:1 q4_0:4096:14336:8:1 q8_0:4096:4096:8:1 q8_0:4096:11008:8:1 q8_0:14336:4096:8:1 q4_K:14336:4096:8:1 q4_K:4096:11008:8:1 q5_K:14336:4096:8:1"; GGML_MI355X_MMA=1 GGML_MI355X_MMA_PAIR=1 python scripts/mmvq_bench.py $S && GGML_MI355X_MMA=1 python scripts/mmvq_bench.py $S && GGML_MI355X_MMA=0 python scripts/mmvq_bench.py $S' ;;
        mmasweep2) run mmasweep2 1000 bash -c 'S1=" q4_0:4096:4096:3:1 q4_0:4096:4096:4:1 q4_0:4096:4096:5:1 q4_0:4096:4096:6:1 q4_0:4096:4096:8:1 q4_0:4096:11008:3:1 q4_0:4096:11008:4:1 q4_0:4096:11008:5:1 q4_0:4096:11008:6:1 q4_0:4096:11008:8:1 q4_0:11008:4096:3:1 q4_0:11008:4096:4:1 q4_0:11008:4096:5:1 q4_0:11008:4096:6:1 q4_0:11008:4096:8:1 q4_0:14336:4096:3:1 q4_0:14336:4096:4:1 q4_0:14336:4096:5:1 q4_0:14336:4096:6:1 q4_0:14336:4096:8:1 q4_0:4096:14336:3:1 q4_0:4096:14336:4:1 q4_0:4096:14336:5:1 q4_0:4096:14336:6:1 q4_0:4096:14336:8:1 q8_0:4096:4096:3:1 q8_0:4096:4096:4:1 q8_0:4096:4096:5:1 q8_0:4096:4096:6:1 q8_0:4096:4096:8:1 q8_0:4096:11008:3:1 q8_0:4096:11008:4:1 q8_0:4096:11008:5:1 q8_0:4096:11008:6:1 q8_0:4096:11008:8:1 q8_0:11008:4096:3:1 q8_0:11008:4096:4:1 q8_0:11008:4096:5:1 q8_0:11008:4096:6:1 q8_0:11008:4096:8:1 q8_0:14336:4096:3:1 q8_0:14336:4096:4:1 q8_0:14336:4096:5:1 q8_0:14336:4096:6:1 q8_0:14336:4096:8:1 q8_0:4096:14336:3:1 q8_0:4096:14336:4:1 q8_0:4096:14336:5:1 q8_0:4096:14336:6:1 q8_0:4096:14336:8:1"; S2=" q4_K:4096:4096:4:1 q4_K:4096:4096:5:1 q4_K:4096:4096:6:1 q4_K:4096:4096:8:1 q4_K:4096:11008:4:1 q4_K:4096:11008:5:1 q4_K:4096:11008:6:1 q4_K:4096:11008:8:1 q4_K:11008:4096:4:1 q4_K:11008:4096:5:1 q4_K:11008:4096:6:1 q4_K:11008:4096:8:1 q4_K:14336:4096:4:1 q4_K:14336:4096:5:1 q4_K:14336:4096:6:1 q4_K:14336:4096:8:1 q4_K:4096:14336:4:1 q4_K:4096:14336:5:1 q4_K:4096:14336:6:1 q4_K:4096:14336:8:1 q5_K:4096:4096:4:1 q5_K:4096:4096:5:1 q5_K:4096:4096:6:1 q5_K:4096:4096:8:1 q5_K:4096:11008:4:1 q5_K:4096:11008:5:1 q5_K:4096:11008:6:1 q5_K:4096:11008:8:1 q5_K:11008:4096:4:1 q5_K:11008:4096:5:1 q5_K:11008:4096:6:1 q5_K:11008:4096:8:1 q5_K:14336:4096:4:1 q5_K:14336:4096:5:1 q5_K:14336:4096:6:1 q5_K:14336:4096:8:1 q5_K:4096:14336:4:1 q5_K:4096:14336:5:1 q5_K:4096:14336:6:1 q5_K:4096:14336:8:1"; GGML_MI355X_MMA=1 GGML_MI355X_MMA_PAIR=1 python scripts/mmvq_bench.py $S1 && GGML_MI355X_MMA=1 python scripts/mmvq_bench.py $S1 $S2 && GGML_MI355X_MMA=0 python scripts/mmvq_bench.py $S1 $S2' ;;
        ringpar2) run ringpar2 600 env GGML_MI355X_RING_PRE=2 GGML_MI355X_MMA=0 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "k11008 or k14336 or k14368 or k12288 or k9216 or k8192 or k131072" ;;
        mmasweep3) run mmasweep3 900 bash -c 'S2=" q4_K:4096:4096:2:1 q4_K:4096:4096:3:1 q4_K:4096:4096:4:1 q4_K:4096:4096:5:1 q4_K:4096:4096:6:1 q4_K:4096:4096:8:1 q4_K:4096:11008:2:1 q4_K:4096:11008:3:1 q4_K:4096:11008:4:1 q4_K:4096:11008:5:1 q4_K:4096:11008:6:1 q4_K:4096:11008:8:1 q4_K:11008:4096:2:1 q4_K:11008:4096:3:1 q4_K:11008:4096:4:1 q4_K:11008:4096:5:1 q4_K:11008:4096:6:1 q4_K:11008:4096:8:1 q4_K:14336:4096:2:1 q4_K:14336:4096:3:1 q4_K:14336:4096:4:1 q4_K:14336:4096:5:1 q4_K:14336:4096:6:1 q4_K:14336:4096:8:1 q4_K:4096:14336:2:1 q4_K:4096:14336:3:1 q4_K:4096:14336:4:1 q4_K:4096:14336:5:1 q4_K:4096:14336:6:1 q4_K:4096:14336:8:1 q5_K:4096:4096:2:1 q5_K:4096:4096:3:1 q5_K:4096:4096:4:1 q5_K:4096:4096:5:1 q5_K:4096:4096:6:1 q5_K:4096:4096:8:1 q5_K:4096:11008:2:1 q5_K:4096:11008:3:1 q5_K:4096:11008:4:1 q5_K:4096:11008:5:1 q5_K:4096:11008:6:1 q5_K:4096:11008:8:1 q5_K:11008:4096:2:1 q5_K:11008:4096:3:1 q5_K:11008:4096:4:1 q5_K:11008:4096:5:1 q5_K:11008:4096:6:1 q5_K:11008:4096:8:1 q5_K:14336:4096:2:1 q5_K:14336:4096:3:1 q5_K:14336:4096:4:1 q5_K:14336:4096:5:1 q5_K:14336:4096:6:1 q5_K:14336:4096:8:1 q5_K:4096:14336:2:1 q5_K:4096:14336:3:1 q5_K:4096:14336:4:1 q5_K:4096:14336:5:1 q5_K:4096:14336:6:1 q5_K:4096:14336:8:1"; GGML_MI355X_MMA=1 python scripts/mmvq_bench.py $S2 && GGML_MI355X_MMA=0 python scripts/mmvq_bench.py $S2' ;;
        mmak4) run mmak4 900 bash -c 'S="q4_0:4096:4096:4:1 q4_0:4096:4096:5:1 q4_0:4096:4096:8:1 q4_0:4096:11008:4:1 q4_0:4096:11008:5:1 q4_0:4096:11008:8:1 q4_0:4096:14336:5:1 q4_0:4096:14336:8:1 q8_0:4096:4096:5:1 q8_0:4096:4096:8:1 q8_0:4096:11008:5:1 q8_0:4096:11008:8:1"; GGML_MI355X_MMA=1 GGML_MI355X_MMA_PAIR=1 GGML_MI355X_MMA_KH=1 GGML_MI355X_MMA_RT=1 python scripts/mmvq_bench.py $S && GGML_MI355X_MMA=1 GGML_MI355X_MMA_PAIR=1 GGML_MI355X_MMA_KH=1 python scripts/mmvq_bench.py $S && GGML_MI355X_MMA=1 python scripts/mmvq_bench.py $S && GGML_MI355X_MMA=0 python scripts/mmvq_bench.py $S' ;;
        skb) run skb 600 bash -c 'S="q8_0:4096:11008:512 q4_K:4096:11008:512 q6_K:4096:11008:512 q4_0:4096:14336:512 q8_0:4096:4096:768 q8_0:4096:4096:512"; GGML_MI355X_MMQ8_SK=1 python scripts/mmq_bench.py $S && GGML_MI355X_MMQ8_SK=0 python scripts/mmq_bench.py $S' ;;
        gpt2ab) run gpt2ab 600 bash scripts/gpt2_ab.sh r4blk head ;;
        stamps) run stamps 300 bash -c 'python scripts/stamps_probe.py q4_K 4096 4096 1 && python scripts/stamps_probe.py q4_0 4096 4096 1' ;;
        sktest) run sktest 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_mmq8.py -k "stream_k" ;;
        tboperf) run tboperf 900 env GGML_BACKEND_PATH=$PWD/ggml-gfx906_amd/libggml-hip-mi355x.so ./oracle/_ref/test-backend-ops perf -o MUL_MAT -b MI355X0 ;;
        cpychk) run cpychk 600 ./oracle/_ref/cpy_check $PWD/ggml-gfx906_amd/libggml-hip-mi355x.so 100 ;;
        repchk) run repchk 300 ./oracle/_ref/repack_check $PWD/ggml-gfx906_amd/libggml-hip-mi355x.so ;;
        prof)  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-extra --cpu-seconds 1 ;;
        pmc)   run pmc 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc -o pmc -- python bench.py --no-extra --cpu-seconds 1 --steps 5 --warmup 1 ;;
        pmcw)  run pmcw 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmcw -o pmcw -- python bench.py --no-extra --cpu-seconds 1 --steps 5 --warmup 1 ;;
        profsingles) run profsingles 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profsingles -o run -- python scripts/prof_singles.py ;;
        profgpt2) run profgpt2 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profgpt2 -o run -- python scripts/gpt2_bench.py 1 256 1 ;;
        gpt2b) run gpt2b 300 python scripts/gpt2_bench.py 1 256 1 ;;
        pmcfetch) run pmcfetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmcfetch -o pmc -- python scripts/mmvq_bench.py q4_0:14336:4096:1:1 q4_0:14336:4096:8:1 q8_0:14336:4096:1:1 q8_0:14336:4096:8:1 q4_K:14336:4096:1:1 q4_K:14336:4096:8:1 && python scripts/pmc_summary.py $OUT/pmcfetch > $OUT/pmcfetch_summary.txt && find $OUT/pmcfetch -name "*.csv" -size +2M -delete ;;
        gpt2tests) run gpt2tests 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpt2.py tests/test_gpt2_example.py tests/test_graph_fusion.py tests/test_gpt2_pipeline.py -m gpu ;;
        plugab) run plugab 600 bash scripts/plugin_gpt2_ab.sh ;;
        pmcring) run pmcring 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmcring -o pmc -- python scripts/mmvq_bench.py q4_0:14336:4096:1:8 q4_0:14336:4096:8:8 q4_K:14336:4096:8:8
                 python scripts/pmc_summary.py $OUT/pmcring > $OUT/pmcring_summary.txt; find $OUT/pmcring -name '*.csv' -size +2M -delete ;;
        floor) run floor_stream 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/floor_stream -o run -- scripts/hbm_probe s
               run floor_mv 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/floor_mv -o run -- python scripts/prof_singles.py 128 q4_K:4096:64
               for d in floor_stream floor_mv; do for t in $(find $OUT/$d -name '*kernel_trace.csv'); do python scripts/trace_summary.py $t 2 > $OUT/${d}_summary.txt; rm -f $t; done; done ;;
        mmq)   run mmq 300 python scripts/mmq_bench.py ;;
        profmmq) run profmmq 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profmmq -o run -- python scripts/mmq_bench.py q8_0:4096:4096:512 q4_K:4096:4096:512 ;;
        *) echo "unknown step $step" ;;
    esac
done
