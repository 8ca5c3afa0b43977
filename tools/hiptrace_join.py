"""Join rocprofv3 kernel-trace and hip-trace CSVs by correlation id: for the last C4 step,
each kernel's GPU start / duration / gap and the host time of its launch call (relative)."""
import csv
import glob
import os
import sys

d = sys.argv[1]


def rows(pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


ks = rows("*kernel_trace.csv")
hs = rows("*hip_api_trace.csv")
launch = {}
for h in hs:
    launch[h["Correlation_Id"]] = (int(h["Start_Timestamp"]), int(h["End_Timestamp"]), h["Function"])
ks.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(ks) if "k_filter<8" in r["Kernel_Name"] and
       int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) > 500000]
i0 = idx[-2] - 4   # the last TIMED step (the final one is the untimed level-2 phase split)
t0 = int(ks[i0]["Start_Timestamp"])
prev = None
print("   gpu_start     dur     gap   host_call(rel)  call_us  kernel")
for r in ks[i0:i0 + 28]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    prev = e
    hc = launch.get(r["Correlation_Id"])
    hrel = (hc[0] - t0) / 1e3 if hc else float("nan")
    hdur = (hc[1] - hc[0]) / 1e3 if hc else float("nan")
    print(f"{(s - t0) / 1e3:12.1f} {(e - s) / 1e3:7.1f} {gap:7.1f} {hrel:14.1f} {hdur:8.1f}  {r['Kernel_Name'][:70]}")
# host calls between the filter launch and the last kernel of the step
hs.sort(key=lambda h: int(h["Start_Timestamp"]))
print("\nhost API calls in the step window:")
tend = int(ks[min(i0 + 27, len(ks) - 1)]["End_Timestamp"])
for h in hs:
    s = int(h["Start_Timestamp"])
    if t0 - 200000 <= s <= tend:
        print(f"{(s - t0) / 1e3:12.1f} {(int(h['End_Timestamp']) - s) / 1e3:8.1f}  {h['Function']}")
