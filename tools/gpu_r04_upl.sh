#!/bin/bash
# round-4: descriptor uploads by a copy kernel -- slot / processor / modulator parity, then sch_slot in four
# processes (per-step intervals) and the slot pipeline.
set -o pipefail
O=gpurun_out/r04u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q -rf --timeout 240 --timeout-method thread tests/test_sch_slot_gpu.py tests/test_pusch_processor_gpu.py tests/test_pdsch_modulator_gpu.py tests/test_phy_plugins_gpu.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -le 1 ] || exit $rc
for r in 1 2 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/pu$r -o p -- python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline > $O/run$r.log 2>&1 || exit $?
  tail -1 $O/run$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('traced run $r', round(d['value']/1e6,3), round(d['ms_per_step'],3))"
  python tools/rocpd_timeline.py "$(find /tmp/pu$r -name "*.db" -print -quit)" pdsch_tb_crc -1 > $O/tl$r.txt; head -2 $O/tl$r.txt | tail -1 | cut -c1-160
  rm -rf /tmp/pu$r
done
for r in 1 2; do
  timeout -k 10 200 python bench.py --workload sch_slot --steps 20 --no-latency --no-cpu-baseline > $O/slot$r.log 2>&1 || exit $?
  tail -1 $O/slot$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('slot $r', round(d['value']/1e6,3), round(d['ms_per_step'],3))"
done
timeout -k 10 200 python bench.py --workload slot_pipeline --steps 10 --no-latency --no-cpu-baseline > $O/sp.log 2>&1 || exit $?
tail -1 $O/sp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('sp', round(d['value']/1e6,3), round(d['ms_per_step'],3))"
