"""Per-step timeline of a rocprofv3 kernel trace (``--kernel-trace --output-format csv``):
splits the trace into train steps at the interpolation kernel, picks the median step
and reports, per hardware queue, busy time and the kernels by category, plus the time
when only one queue was busy (the serial part) and the idle gaps.

    python scripts/timeline.py gpurun_out/prof/..._kernel_trace.csv [--steps K]
"""
import csv
import re
import sys
from collections import defaultdict


def demangle(name):
    """Enough of the Itanium mangling for this library's kernel templates."""
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)", name)
    if not m:
        return name
    n = int(m.group(1))
    rest = name[m.end():]
    base, rest = rest[:n], rest[n:]
    if not rest.startswith("I"):
        return base
    args = re.findall(r"DF16b|Li(-?\d+)E|Lb([01])E|(?<=[IE])f(?=[LE])", rest[1:rest.find("EEv") + 1])
    out = []
    for tok in re.finditer(r"DF16b|Li(-?\d+)E|Lb([01])E|f", rest[1:rest.find("EEv") + 1]):
        t = tok.group(0)
        out.append("bf16" if t == "DF16b" else "float" if t == "f" else tok.group(1) if tok.group(1) is not None
                   else ("true" if tok.group(2) == "1" else "false"))
    return f"{base}<{', '.join(out)}>"


def cat(name):
    name = demangle(name)
    m = re.search(r"(\w+_kernel)", name)
    base = m.group(1) if m else name[:40]
    t = re.search(r"_kernel<([^>]*)>", name.replace("__bf16", "bf16"))
    return base + (f"<{t.group(1)}>" if t else "")


def main(path, start_kernel="interp_kernel"):
    rows = list(csv.DictReader(open(path)))
    ks = []
    for r in rows:
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?"), r["Kernel_Name"]))
    ks.sort()
    starts = [i for i, k in enumerate(ks) if start_kernel in k[3]]
    steps = []
    for a, b in zip(starts, starts[1:] + [len(ks)]):
        steps.append(ks[a:b])
    print("step walls (us):", [round((x[-1][1] - x[0][0]) / 1e3) for x in steps])
    rng = [a for a in sys.argv if a.startswith("--range=")]
    if rng:   # pick the timed graph replays by index
        a, b = map(int, rng[0][8:].split(":"))
        steps = steps[a:b]
    walls = sorted((s[-1][1] - s[0][0], i) for i, s in enumerate(steps))
    wall, idx = walls[len(walls) // 2]
    st = steps[idx]
    t0 = st[0][0]
    print(f"{len(steps)} steps analysed; median step wall {wall / 1e3:.1f} us, {len(st)} kernels")
    byq = defaultdict(list)
    for k in st:
        byq[k[2]].append(k)
    for q, kl in byq.items():
        busy = sum(e - s for s, e, _, _ in kl)
        print(f"queue {q}: {len(kl)} kernels, busy {busy / 1e3:.1f} us ({busy / wall:.2f} of wall)")
        agg = defaultdict(lambda: [0, 0])
        for s, e, _, n in kl:
            a = agg[cat(n)]
            a[0] += 1
            a[1] += e - s
        for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
            print(f"   {d / 1e3:8.1f} us  {c:3d}x  {n}")
    # busy-queue count over time
    ev = []
    for s, e, q, _ in st:
        ev.append((s, 1))
        ev.append((e, -1))
    ev.sort()
    cnt, last = 0, t0
    hist = defaultdict(int)
    for t, d in ev:
        hist[cnt] += t - last
        cnt += d
        last = t
    print("time with N kernels running:", {k: f"{v / 1e3:.1f} us" for k, v in sorted(hist.items())})
    # the sequence of the first queue (main) with gaps, coarse
    if "--seq" in sys.argv:
        for s, e, q, n in st:
            print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{q} {cat(n)}")


if __name__ == "__main__":
    main(sys.argv[1])
