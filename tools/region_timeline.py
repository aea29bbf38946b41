"""Dev tool: the timed region of a bench run under rocprofv3 --kernel-trace --hip-trace, with the
host clocks bench.py prints under EKF_BENCH_TRACE=1 (CLOCK_MONOTONIC, the trace's clock domain).
Usage: python tools/region_timeline.py <trace dir> <bench stderr>"""
import csv
import glob
import json
import sys

d, errf = sys.argv[1], sys.argv[2]
clk = None
for line in open(errf):
    if "trace_clocks" in line:
        clk = {k: m for k, m, _ in json.loads(line)["trace_clocks"]}
t0, tq, t1 = clk["t0"], clk["enqueued"], clk["synced"]
ks = []
for r in csv.DictReader(open(glob.glob(d + "/*kernel_trace.csv")[0])):
    a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if b >= t0 and a <= t1:
        ks.append((a, b, r["Kernel_Name"].split("(")[0].split("::")[-1], r["Queue_Id"]))
ks.sort()
api = []
for r in (csv.DictReader(open(glob.glob(d + "/*hip_api_trace.csv")[0]))
          if glob.glob(d + "/*hip_api_trace.csv") else []):
    a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if b >= t0 and a <= t1:
        api.append((a, b, r["Function"]))
api.sort()
us = lambda t: (t - t0) / 1e3
print(f"host: enqueue returns {us(tq):.1f} us, synced {us(t1):.1f} us" +
      (f" (library streams synced {us(clk['lib_synced']):.1f} us)" if "lib_synced" in clk else ""))
first_api = api[0] if api else None
if first_api:
    print(f"first HIP API call {first_api[2]} at {us(first_api[0]):.1f} us")
from collections import Counter
print("API calls in region:", Counter(f for _, _, f in api).most_common(12))
for f in ("hipMemcpyAsync", "hipStreamSynchronize", "hipEventRecord", "hipStreamWaitEvent"):
    for a, b, g in api:
        if g == f:
            print(f"  {f} {us(a):.1f}-{us(b):.1f}")
            break
print(f"first kernel {ks[0][2]} q{ks[0][3]} starts {us(ks[0][0]):.1f}; last kernel {ks[-1][2]} ends {us(ks[-1][1]):.1f}")
for k in ks[:6] + ks[-8:]:
    a, b, n, q = k
    print(f"  {n:24s} q{q:>2s} {us(a):8.1f} {us(b):8.1f} dur {(b - a) / 1e3:6.1f}")
chains = [k for k in ks if k[2].startswith("k_chain")]
print("chain launches:", [(f"{us(a):.1f}", f"{(b - a) / 1e3:.1f}") for a, b, _, _ in chains])
for a, b, f in api:
    if f in ("hipMalloc", "hipFree", "hipHostMalloc", "hipStreamSynchronize", "hipMemcpyAsync"):
        print(f"  api {f:22s} {us(a):8.1f} {us(b):8.1f}")
