#!/bin/bash
# pmc_ab.sh <variant>... : SQ counters of the decoder kernel for each exp/<variant>.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM"; do
    tag=$(echo $set | cut -c1-8)
    SRSRAN_AMD_LIB=$PWD/exp/$v/libsrsran_amd.so timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmcab_${v}_$tag -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "$v rc=$rc"; exit $rc; fi
  done
  python3 - "$v" << 'PY'
import csv, glob, sys, collections
v=sys.argv[1]
agg=collections.defaultdict(list)
for f in glob.glob('gpurun_out/pmcab_%s_*/**/*counter_collection.csv' % v, recursive=True):
    for r in csv.DictReader(open(f)):
        if 'ldpc' in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
m={k: sum(x)/len(x) for k,x in agg.items()}
w=m.get('SQ_WAVES',1)
print(v, ' '.join('%s=%.4g' % (k, m[k]) for k in sorted(m)))
print(v, 'per-wave: valu %.0f salu %.0f lds %.0f smem %.0f vmem %.0f | wave_cycles %.0f wait_any %.2f wait_inst %.2f active_valu %.2f' % (
    m['SQ_INSTS_VALU']/w, m['SQ_INSTS_SALU']/w, m['SQ_INSTS_LDS']/w, m.get('SQ_INSTS_SMEM',0)/w, m.get('SQ_INSTS_VMEM',0)/w,
    m['SQ_WAVE_CYCLES']/w, m['SQ_WAIT_ANY']/m['SQ_WAVE_CYCLES'], m['SQ_WAIT_INST_ANY']/m['SQ_WAVE_CYCLES'], m['SQ_ACTIVE_INST_VALU']/m['SQ_WAVE_CYCLES']))
PY
done
