#!/bin/bash
# round-4: TB assembly and concatenation in one launch (asm_merged_kernel) -- decoder-chain parity suites, then the
# headline and one-cell graph with and without it (SRSRAN_AMD_ASM_MERGED=0).
set -o pipefail
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 700 python -u -m pytest -q -rf --timeout 240 --timeout-method thread tests/test_sch_gpu.py tests/test_sch_slot_gpu.py tests/test_pusch_processor_gpu.py tests/test_pipeline_gpu.py tests/test_integration_gpu.py tests/test_phy_plugins_gpu.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -le 1 ] || exit $rc
run() { local n=$1; shift; timeout -k 10 200 "$@" > $O/$n.log 2>&1 || exit $?; tail -1 $O/$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['value']/1e6,3), round(d['ms_per_step'],4))"; }
run pipe python bench.py --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
run pipe_old env SRSRAN_AMD_ASM_MERGED=0 python bench.py --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
run pipe2 python bench.py --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
run one python bench.py --graph --slots-pipeline 1 --steps 50 --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
run one_old env SRSRAN_AMD_ASM_MERGED=0 python bench.py --graph --slots-pipeline 1 --steps 50 --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1
run slot python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline
