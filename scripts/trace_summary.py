"""Per-(kernel, grid) launch-duration summary of a rocprofv3 kernel trace CSV."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gle::", "")
    key = (name[:40], int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), int(r["Grid_Size_Y"]))
    d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in d.values())
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v = sorted(v)
    print("%-40s grid %6d x %4d  n %5d  med %9.1f us  min %9.1f  total %10.1f us (%4.1f%%)"
          % (k[0], k[1], k[2], len(v), v[len(v) // 2], v[0], sum(v), 100 * sum(v) / tot))
