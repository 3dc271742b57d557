"""Where a timed bench step goes: kernel time, GPU idle gaps, overlap.

    python tools/step_split.py <run_kernel_trace.csv> <steps> [label]

bench.py launches k_prof_mark (das_prof_mark) right before the synchronisation
that starts its timed steps and right after the one that ends them, so in a
rocprofv3 kernel trace every pair of marks brackets one leg's K timed steps.
Per bracket (per step, in microseconds):
  wall        first mark's end -> second mark's start
  busy        union of the kernel intervals inside (any stream)
  idle        wall - busy: the GPU runs nothing -- host lowering / launch
              turnaround / read-back spin with an empty queue
  kernel_sum  sum of kernel durations (exceeds busy where streams overlap)
  overlap     kernel_sum - busy
and the kernels by total time.  Prints one JSON object.
"""
import csv
import json
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n.replace("void ", "").replace("das::", "").strip()


def brackets(rows):
    marks = [i for i, r in enumerate(rows) if short(r[2]).endswith("k_prof_mark")]
    return [(marks[k], marks[k + 1]) for k in range(0, len(marks) - 1, 2)]


def split(rows, a, b, steps):
    t0, t1 = rows[a][1], rows[b][0]
    ks = [r for r in rows[a + 1:b]]
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in sorted(ks):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    ksum = sum(e - s for s, e, _ in ks)
    by = {}
    for s, e, n in ks:
        k = short(n)
        d = by.setdefault(k, [0, 0])
        d[0] += e - s
        d[1] += 1
    us = lambda ns: round(ns / 1e3 / steps, 2)  # noqa: E731
    wall = t1 - t0
    return {"steps": steps, "wall_us": us(wall), "busy_us": us(busy), "idle_us": us(wall - busy),
            "kernel_sum_us": us(ksum), "overlap_us": us(ksum - busy), "launches": round(len(ks) / steps, 1),
            "busy_frac": round(busy / wall, 4) if wall else None,
            "top_kernels_us": {k: [us(v[0]), round(v[1] / steps, 1)]
                               for k, v in sorted(by.items(), key=lambda kv: -kv[1][0])[:12]}}


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    label = sys.argv[3] if len(sys.argv) > 3 else path
    with open(path) as f:
        rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                      for r in csv.DictReader(f))
    out = {"trace": label, "regions": [split(rows, a, b, steps) for a, b in brackets(rows)]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
