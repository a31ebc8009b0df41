cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_real -o run -- python scripts/prof_singles.py 64 q4_0:4096:64 > gpurun_out/pmc_real.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_probe -o run -- scripts/gemv_probe > gpurun_out/pmc_probe.log 2>&1
