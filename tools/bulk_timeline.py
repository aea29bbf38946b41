"""Dev tool: the bulk stream's loop per chunk from a rocprofv3 kernel trace (rocpd database):
k_factors / k_sigma_pass / k_patch_stage start, end and the gaps between them, steady state of the
first chain launch of > 100 chunks (median over its chunks).  python tools/bulk_timeline.py <run_results.db> [launch]"""
import sqlite3
import sys

import numpy as np

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, [end] from kernels order by start").fetchall()
names = {"k_chain": "chain", "k_factors": "fac", "k_sigma_pass": "pass", "k_patch_stage": "stage"}
ev = []
for n, s, e in rows:
    for k, v in names.items():
        if k + "<" in n and "float" in n:
            ev.append((v, s, e))
chains = [x for x in ev if x[0] == "chain"]
# the chain launches with more than 100 chunks (bench.py --steps 200: the timed region is the first
# of them; argv[2] picks another)
longs = [ch for ch in chains if sum(1 for x in ev if x[0] == "fac" and ch[1] <= x[1] <= ch[2]) > 100]
big = longs[int(sys.argv[2]) if len(sys.argv) > 2 else 0]
inside = [x for x in ev if x[0] != "chain" and big[1] <= x[1] <= big[2]]
print(f"chain launch {(big[2] - big[1]) / 1e3:.1f} us, {len(inside)} bulk kernels inside")
fac = [x for x in inside if x[0] == "fac"]
out = {k: [] for k in ("fac_dur", "fac_to_pass", "pass_dur", "pass_to_stage", "stage_dur",
                       "stage_to_fac", "period")}
for i in range(5, len(fac) - 5):
    f0 = fac[i]
    p = next(x for x in inside if x[0] == "pass" and x[1] >= f0[2])
    s = next(x for x in inside if x[0] == "stage" and x[1] >= p[2])
    f1 = fac[i + 1]
    out["fac_dur"].append(f0[2] - f0[1])
    out["fac_to_pass"].append(p[1] - f0[2])
    out["pass_dur"].append(p[2] - p[1])
    out["pass_to_stage"].append(s[1] - p[2])
    out["stage_dur"].append(s[2] - s[1])
    out["stage_to_fac"].append(f1[1] - s[2])
    out["period"].append(f1[2] - f0[2])
for k, v in out.items():
    print(f"{k:14s} median {np.median(v) / 1e3:7.2f} us  (p10 {np.percentile(v, 10) / 1e3:.2f}, p90 {np.percentile(v, 90) / 1e3:.2f})")
