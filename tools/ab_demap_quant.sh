#!/bin/bash
# A/B of the demapper quantizer (DEMAP_Q_CVT): demapper / equalizer / PUCCH / PUSCH GPU tests, then the slot pipeline
# with the in-tree library and tools/_build/libsrsran_amd_oldq.so (tools/build_variant.sh oldq pusch_demod.hip
# -DDEMAP_Q_CVT=0), alternately, twice, then one kernel-trace profile of each.
set -uo pipefail
out=gpurun_out/r06q
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pusch_demod_gpu.py \
  tests/test_equalizer_gpu.py tests/test_equalizer_mimo_gpu.py tests/test_modulation_gpu.py tests/test_pusch_tp_gpu.py \
  tests/test_pucch_gpu.py > $out/pytest.log 2>&1 || { echo "tests failed"; tail -5 $out/pytest.log; exit 3; }
tail -1 $out/pytest.log
for v in base oldq base oldq; do
  if [ $v = base ]; then unset SRSRAN_AMD_LIB; else export SRSRAN_AMD_LIB=$PWD/tools/_build/libsrsran_amd_$v.so; fi
  timeout -k 10 200 python3 bench.py --workload slot_pipeline --no-cpu-baseline > $out/slot_$v.json 2>$out/slot_$v.err || { echo "slot $v failed"; exit 3; }
  timeout -k 10 200 python3 bench.py --workload slot_pipeline --mixed --no-cpu-baseline > $out/mixed_$v.json 2>$out/mixed_$v.err || { echo "mixed $v failed"; exit 3; }
  echo "$v slot $(grep -o '"ms_per_step": [0-9.e+]*' $out/slot_$v.json | head -1) mixed $(grep -o '"ms_per_step": [0-9.e+]*' $out/mixed_$v.json | head -1)"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in base oldq; do
  if [ $v = base ]; then unset SRSRAN_AMD_LIB; else export SRSRAN_AMD_LIB=$PWD/tools/_build/libsrsran_amd_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$v -o run -- python3 bench.py --workload slot_pipeline --no-cpu-baseline --steps 10 > $out/prof_$v.log 2>&1 || { echo "prof $v failed"; exit 3; }
done
echo done
