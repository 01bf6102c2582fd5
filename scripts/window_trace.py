"""Per-step timeline of the short (driver 20/5) and long windows from a rocprofv3 kernel trace of
scripts/exp_time.py: chain launches per step, kernel durations, gaps (which part of a short window
is slower than the steady state)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["n"] = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace("gle::", "").split("(")[0]
rows.sort(key=lambda r: r["s"])
A = [r for r in rows if r["n"].startswith("chain_kernel<0")]
BC = [r for r in rows if r["n"].startswith("chain_kernel<3")]
print("stage A launches", len(A), "BC", len(BC))
# the exp_time protocol: fill (2*256+5 = 517 steps), short (20), 64, long (512): step index = launch index
def window(i0, n, tag):
    a = A[i0:i0 + n]
    b = BC[i0:i0 + n]
    t0, t1 = a[0]["s"], b[-1]["e"]
    da = sorted((x["e"] - x["s"]) / 1e3 for x in a)
    db = sorted((x["e"] - x["s"]) / 1e3 for x in b)
    bg = [r for r in rows if r["s"] >= t0 and r["e"] <= t1 and not r["n"].startswith("chain")]
    busy = sum(r["e"] - r["s"] for r in bg) / 1e3
    print("%-6s steps %d  span %.1f us = %.2f us/step  A med %.2f max %.2f  BC med %.2f max %.2f  bg kernel-us %.0f (%d launches)"
          % (tag, n, (t1 - t0) / 1e3, (t1 - t0) / 1e3 / n, da[len(da) // 2], da[-1], db[len(db) // 2], db[-1], busy, len(bg)))
    gaps = [(a[i + 1]["s"] - b[i]["e"]) / 1e3 for i in range(n - 1)]
    inner = [(b[i]["s"] - a[i]["e"]) / 1e3 for i in range(n)]
    print("       gap BC->A med %.2f max %.2f   A->BC med %.2f max %.2f" % (sorted(gaps)[len(gaps) // 2], max(gaps),
                                                                          sorted(inner)[len(inner) // 2], max(inner)))
    return a, b

nfill = int(sys.argv[2]) if len(sys.argv) > 2 else 517
window(nfill, 20, "short")
window(nfill + 20 + 64, 512, "long")
for k in range(0, 20, 1):
    i = nfill + k
    print("  step %3d  A %.1f BC %.1f  A-start->BC-end %.1f" % (k, (A[i]["e"] - A[i]["s"]) / 1e3, (BC[i]["e"] - BC[i]["s"]) / 1e3,
                                                      (BC[i]["e"] - A[i]["s"]) / 1e3))
