"""Dev tool: print a kernel timeline (start/end/gaps, µs) from a rocprofv3 kernel_trace.csv."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
want = sys.argv[2] if len(sys.argv) > 2 else "<float>"
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 200
cnt = int(sys.argv[4]) if len(sys.argv) > 4 else 24
ks = sorted([(r["Kernel_Name"].split("(")[0].split("::")[-1], int(r["Start_Timestamp"]),
              int(r["End_Timestamp"]), r.get("Queue_Id", "")) for r in rows
             if want in r["Kernel_Name"]], key=lambda x: x[1])
seg = ks[skip:skip + cnt]
t0 = seg[0][1]
prev_end = {}
for n, a, b, q in seg:
    print(f"{n:22s} q{q:>2s} {(a - t0) / 1e3:9.2f} {(b - t0) / 1e3:9.2f}  dur {(b - a) / 1e3:6.2f}")
chains = [k for k in ks[skip:] if k[0].startswith("k_chain")]
if len(chains) > 2:
    per = (chains[-1][1] - chains[0][1]) / (len(chains) - 1) / 1e3
    dur = sum(b - a for _, a, b, _ in chains) / len(chains) / 1e3
    print(f"chain period {per:.2f} us, chain duration {dur:.2f} us")
