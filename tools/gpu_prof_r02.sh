#!/bin/bash
# Round-2 profiles: pipeline kernel trace, decoder HBM traffic (separate FETCH / WRITE passes), decoder VALU model.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency --low-snr-db -1"
set -o pipefail
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p2_trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-latency --low-snr-db -1 > gpurun_out/p2_trace.log 2>&1 || exit $?
echo trace done
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/p2_fetch -o run --output-format csv -- $B > gpurun_out/p2_fetch.log 2>&1 || exit $?
echo fetch done
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/p2_write -o run --output-format csv -- $B > gpurun_out/p2_write.log 2>&1 || exit $?
echo write done
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d gpurun_out/p2_sq -o run --output-format csv -- python3 tools/ldpc_hr_probe.py > gpurun_out/p2_sq.log 2>&1 || exit $?
echo sq done
