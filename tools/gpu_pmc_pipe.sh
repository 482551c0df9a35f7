#!/bin/bash
# Per-kernel PMC table of the bench pipeline (kernels serialized by the counter passes): SQ counters, then
# FETCH_SIZE and WRITE_SIZE in passes of their own; tools/pmc_kernels.py prints the table.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-latency --low-snr-db -1"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d gpurun_out/ppmc1 -o run --output-format csv -- $B > gpurun_out/ppmc1.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/ppmc_fetch -o run --output-format csv -- $B > gpurun_out/ppmc_fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/ppmc_write -o run --output-format csv -- $B > gpurun_out/ppmc_write.log 2>&1 || exit $?
python3 tools/pmc_kernels.py > gpurun_out/pmc_table.txt && cat gpurun_out/pmc_table.txt
