import re
import csv, collections, sys
def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        k = re.sub(r"srs_amd::|\(anonymous namespace\)::|void |at::native::", "", r["Kernel_Name"])[:40]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg
a = load("gpurun_out/ppmc1"); f = load("gpurun_out/ppmc_fetch"); w = load("gpurun_out/ppmc_write")
kt = collections.defaultdict(list)
for r in csv.DictReader(open("gpurun_out/ppmc1/run_kernel_trace.csv")):
    k = re.sub(r"srs_amd::|\(anonymous namespace\)::|void |at::native::", "", r["Kernel_Name"])[:40]
    kt[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))/1e3)
m = lambda x: sum(x)/len(x) if x else 0
print("%-40s %8s %8s %9s %8s %8s %7s %7s %8s" % ("kernel","us","waves","valu/wave","lds/w","wait%","MBread","MBwrite","GB/s"))
for k in sorted(a, key=lambda k: -m(kt[k])):
    c = a[k]
    waves = m(c["SQ_WAVES"]); 
    rd = 2*m(f[k]["FETCH_SIZE"])*1024/1e6 if k in f else 0
    wr = m(w[k]["WRITE_SIZE"])*1024/1e6 if k in w else 0
    us = m(kt[k])
    print("%-40s %8.1f %8.0f %9.0f %8.0f %7.1f %7.1f %7.1f %8.0f" % (k, us, waves, m(c["SQ_INSTS_VALU"])/max(waves,1), m(c["SQ_INSTS_LDS"])/max(waves,1),
          100*m(c["SQ_WAIT_ANY"])/max(m(c["SQ_WAVE_CYCLES"]),1), rd, wr, (rd+wr)*1e3/us if us else 0))
