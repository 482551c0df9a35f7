#!/bin/bash
# A/B of the decoders' barrier grouping (FR_GROUPS): decoder GPU tests, then configs[1], the mixed slot pipeline and
# sch_slot with the in-tree library and tools/_build/libsrsran_amd_nogroups.so (tools/build_variant.sh nogroups
# ldpc_decoder.hip -DFR_GROUPS=0), alternately, twice.
set -uo pipefail
out=gpurun_out/r06g
mkdir -p $out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ldpc_decoder_gpu.py > $out/pytest.log 2>&1 || { echo "tests failed"; tail -5 $out/pytest.log; exit 3; }
tail -1 $out/pytest.log
for v in base nogroups base nogroups; do
  if [ $v = base ]; then unset SRSRAN_AMD_LIB; else export SRSRAN_AMD_LIB=$PWD/tools/_build/libsrsran_amd_$v.so; fi
  timeout -k 10 200 python3 bench.py --workload ldpc --no-cpu-baseline > $out/ldpc_$v.json 2>$out/ldpc_$v.err || { echo "ldpc $v failed"; exit 3; }
  timeout -k 10 200 python3 bench.py --workload slot_pipeline --mixed --no-cpu-baseline > $out/mixed_$v.json 2>$out/mixed_$v.err || { echo "mixed $v failed"; exit 3; }
  timeout -k 10 200 python3 bench.py --workload sch_slot --no-cpu-baseline > $out/sch_$v.json 2>$out/sch_$v.err || { echo "sch $v failed"; exit 3; }
  echo "$v ldpc $(grep -o '"value": [0-9.e+]*' $out/ldpc_$v.json | head -1) mixed $(grep -o '"ms_per_step": [0-9.e+]*' $out/mixed_$v.json | head -1) sch_slot $(grep -o '"value": [0-9.e+]*' $out/sch_$v.json | head -1)"
done
