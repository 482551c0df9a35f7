#!/bin/bash
# round-4: TB-assembly bytes per thread (ASM_TB_PER 32 / 16 / 8) -- assembly parity, headline, one-cell graph and the
# asm_tb_kernel time per variant (SRSRAN_AMD_LIB).
set -o pipefail
O=gpurun_out/r04asm
mkdir -p $O
export TMPDIR=/tmp
for v in libsrsran_amd var_asm16 var_asm8; do
  export SRSRAN_AMD_LIB=$PWD/srsran_project_amd/lib/$v.so
  timeout -k 10 300 python -u -m pytest -q -rf --timeout 240 --timeout-method thread tests/test_sch_gpu.py tests/test_sch_slot_gpu.py -k "decode or harq or roundtrip or slot" > $O/t_$v.log 2>&1; rc=$?
  echo "$v tests: $(tail -1 $O/t_$v.log)"; [ $rc -le 1 ] || exit $rc
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1 > $O/b_$v.log 2>&1 || exit $?
  tail -1 $O/b_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v headline', round(d['value']/1e6,3), round(d['ms_per_step'],4))"
  timeout -k 10 200 python bench.py --graph --slots-pipeline 1 --steps 50 --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1 > $O/o_$v.log 2>&1 || exit $?
  tail -1 $O/o_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v one-cell', round(d['ms_per_step'],4))"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/pa_$v -o p -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pinned --no-latency --low-snr-db -1 > $O/p_$v.log 2>&1 || exit $?
  python tools/rocpd_stats.py "$(find /tmp/pa_$v -name "*.db" -print -quit)" x | grep -E "asm_tb|assemble_kernel" | cut -c1-140
  rm -rf /tmp/pa_$v
done
