"""Gaps on the GPU timeline of a rocprofv3 kernel trace (+ memory copies):
total busy time, idle time and the largest idle gaps with their neighbours.

  python tools/gap_report.py <dir>/<name>_kernel_trace.csv [<..>_memory_copy_trace.csv] [--last-ms N]
"""
import csv
import sys


def load(path, kind):
    out = []
    for r in csv.DictReader(open(path)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r.get("Kernel_Name") or r.get("Direction") or kind
        out.append((s, e, name[:70]))
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    last_ms = None
    if "--last-ms" in sys.argv:
        last_ms = float(sys.argv[sys.argv.index("--last-ms") + 1])
    ev = load(args[0], "kernel")
    if len(args) > 1:
        ev += load(args[1], "copy")
    ev.sort()
    if last_ms:
        t_end = max(e for _, e, _ in ev)
        ev = [x for x in ev if x[0] >= t_end - last_ms * 1e6]
    busy, gaps = 0, []
    cur_end = ev[0][1]
    prev = ev[0][2]
    busy += ev[0][1] - ev[0][0]
    for s, e, n in ev[1:]:
        if s > cur_end:
            gaps.append((s - cur_end, prev, n))
        busy += max(0, e - max(s, cur_end))
        if e > cur_end:
            cur_end, prev = e, n
    span = cur_end - ev[0][0]
    print(f"span {span/1e6:.3f} ms  busy {busy/1e6:.3f} ms  idle {(span-busy)/1e6:.3f} ms  events {len(ev)}")
    agg = {}
    for g, a, b in gaps:
        key = (a, b)
        agg.setdefault(key, [0, 0])
        agg[key][0] += g
        agg[key][1] += 1
    for (a, b), (g, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:25]:
        print(f"{g/1e6:8.3f} ms x{c:4d}  {a}  ->  {b}")


if __name__ == "__main__":
    main()
