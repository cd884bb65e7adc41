"""Summarise a rocprofv3 kernel trace: per-kernel stats and one step's timeline with gaps."""
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_c2"
r = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
calls = max(int(x["Calls"]) for x in r)
tot = 0.0
for x in r:
    print(f"{x['Name'][:60]:60s} {int(x['Calls']):6d} {float(x['AverageNs'])/1000:8.2f} {float(x['Percentage']):6.2f}")
    tot += float(x["TotalDurationNs"])
print("gpu us/step", tot / calls / 1000)
t = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
t.sort(key=lambda x: int(x["Start_Timestamp"]))
idx = [i for i, x in enumerate(t) if "k_budget" in x["Kernel_Name"]]
i0, i1 = idx[len(idx) // 2], idx[len(idx) // 2 + 1]
prev = None
for x in t[i0:i1]:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    print(f"  {x['Kernel_Name'][:44]:44s} dur {(e-s)/1000:7.2f} gap {((s-prev)/1000 if prev else 0):7.2f}")
    prev = e
print("step span", (int(t[i1]["Start_Timestamp"]) - int(t[i0]["Start_Timestamp"])) / 1000)
