"""Per-(kernel, grid) launch-duration summary of a rocprofv3 kernel trace CSV.

With --steps: steady-state per-step breakdown over the last N chain C launches, and the chain
kernels split by whether a background (other-queue) kernel overlapped them."""
import collections
import csv
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("gle::", "")
    return name.split("(")[0]


rows = list(csv.DictReader(open(sys.argv[1])))


def step_end_stage(rs):
    """The chain launch that closes a step: the composed step (chain_kernel<4, ...>, or <5, ...> with
    one-column VALU products, plans with GLE_PLAN_COMPOSED_STEP: one chain launch per step), the fused velocity stage (chain_kernel<3, ...>,
    plans with GLE_PLAN_FUSED_BC: 2 per step) or stage C (chain_kernel<2, ...>: 3 per step)."""
    for k in ("chain_kernel<5", "chain_kernel<4", "chain_kernel<3"):
        if any(r["n"].startswith(k) for r in rs):
            return k
    return "chain_kernel<2"


for r in rows:
    r["s"] = int(r["Start_Timestamp"])
    r["e"] = int(r["End_Timestamp"])
    r["n"] = short(r["Kernel_Name"])
    r["g"] = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
d = collections.defaultdict(list)
for r in rows:
    d[(r["n"][:40], r["g"], int(r["Grid_Size_Y"]))].append((r["e"] - r["s"]) / 1e3)
tot = sum(sum(v) for v in d.values())
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:30]:
    v = sorted(v)
    print("%-40s grid %6d x %4d  n %5d  med %9.1f us  min %9.1f  total %10.1f us (%4.1f%%)"
          % (k[0], k[1], k[2], len(v), v[len(v) // 2], v[0], sum(v), 100 * sum(v) / tot))

if "--last" in sys.argv:
    # average duration of the last N dispatches of a kernel (the bench's timed region)
    i = sys.argv.index("--last")
    kn, n = sys.argv[i + 1], int(sys.argv[i + 2])
    # --skip M: leave out the M newest dispatches (bench.py's third window, the chain stamps, follows
    # the far-field timing window)
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
    allk = sorted([r for r in rows if kn in r["n"]], key=lambda r: r["s"])
    ks = allk[len(allk) - n - skip:len(allk) - skip]
    if ks:
        print("\n%d dispatches of %s before the newest %d: avg %.2f us"
              % (len(ks), kn, skip, sum(r["e"] - r["s"] for r in ks) / len(ks) / 1e3))

if "--steps" in sys.argv:
    rows.sort(key=lambda r: r["s"])
    cs = [r for r in rows if r["n"].startswith(step_end_stage(rows))]
    n = min(100, len(cs) - 1)
    if n > 0:
        a, b = cs[-n - 1]["e"], cs[-1]["e"]
        win = [r for r in rows if r["s"] >= a and r["e"] <= b]
        per = collections.defaultdict(float)
        cnt = collections.Counter()
        for r in win:
            per[(r["n"][:32], r["g"])] += (r["e"] - r["s"]) / 1e3
            cnt[(r["n"][:32], r["g"])] += 1
        print("\nsteady state: %.2f us per step over %d steps" % ((b - a) / 1e3 / n, n))
        for k, v in sorted(per.items(), key=lambda kv: -kv[1]):
            print("  %-32s grid %6d  n %4d  per-step %8.2f us  avg %8.2f us" % (k[0], k[1], cnt[k], v / n, v / cnt[k]))
        chain = [r for r in win if r["n"].startswith("chain_kernel")]
        bg = [r for r in win if not r["n"].startswith("chain_kernel")]
        alone = collections.defaultdict(list)
        over = collections.defaultdict(list)
        for r in chain:
            ov = any(x["s"] < r["e"] and x["e"] > r["s"] for x in bg)
            (over if ov else alone)[r["n"]].append((r["e"] - r["s"]) / 1e3)
        for k in sorted(set(alone) | set(over)):
            fa = sorted(alone[k])
            fo = sorted(over[k])
            print("  %-18s alone n %4d med %6.1f us | beside background n %4d med %6.1f us"
                  % (k, len(fa), fa[len(fa) // 2] if fa else 0, len(fo), fo[len(fo) // 2] if fo else 0))
        gaps = []
        ch = sorted(chain, key=lambda r: r["s"])
        for x, y in zip(ch, ch[1:]):
            gaps.append((y["s"] - x["e"]) / 1e3)
        gaps.sort()
        if gaps:
            print("  chain launch gaps: med %.2f us  p90 %.2f us" % (gaps[len(gaps) // 2], gaps[int(len(gaps) * 0.9)]))

if "--gaps" in sys.argv:
    # idle time on the main stream between consecutive chain launches over the last 100 steps
    rows.sort(key=lambda r: r["s"])
    ch = [r for r in rows if r["n"].startswith("chain_kernel")][-301:]
    gaps = [(b["s"] - a["e"]) / 1e3 for a, b in zip(ch, ch[1:])]
    # the large-bath plan's fpot launch runs on the main stream between stage A and the fused stage:
    # main-stream idle time counts it as work
    fp = [r for r in rows if r["n"].startswith("fpot_kernel") and ch and r["s"] >= ch[0]["s"]]
    if fp:
        ms = sorted(ch + fp, key=lambda r: r["s"])
        idle = sum(max(0.0, (b["s"] - a["e"]) / 1e3) for a, b in zip(ms, ms[1:]))
    # steps in the window = its step-closing launches (1 chain launch per step in composed plans, 2 in
    # fused plans, 3 otherwise), not a fixed 3
    nsteps = sum(1 for r in ch[1:] if r["n"].startswith(step_end_stage(ch)))
    if gaps and nsteps:
        print("\nchain gaps over %d launches (%d steps): total %.1f us = %.2f us/step; largest %s"
              % (len(gaps), nsteps, sum(gaps), sum(gaps) / nsteps,
                 [round(x, 1) for x in sorted(gaps)[-8:]]))
        if fp:
            print("main-stream idle (chain and fpot launches as work): %.1f us = %.2f us/step; fpot %.2f us/step"
                  % (idle, idle / nsteps, sum((r["e"] - r["s"]) / 1e3 for r in fp) / nsteps))
