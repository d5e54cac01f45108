"""Summarise rocprofv3 --pmc counter CSVs: per kernel and per run of consecutive dispatches of
that kernel (one benchmark shape), the mean of every counter over the run's dispatches."""
import collections
import csv
import re
import sys


def runs(paths, match):
    per = collections.OrderedDict()
    for p in paths:
        for r in csv.DictReader(open(p)):
            if match not in r["Kernel_Name"]:
                continue
            k = int(r["Dispatch_Id"])
            m = re.search(r"(\w+)(<[^>]*>)?\(", r["Kernel_Name"].replace("(anonymous namespace)::", ""))
            e = per.setdefault((p, k), {"name": m.group(1) + (m.group(2) or "") if m else r["Kernel_Name"][:40],
                                        "dur": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    out = collections.defaultdict(list)     # (path, name) -> list of runs (list of dicts)
    last = {}
    for (p, k), e in per.items():
        key = (p, e["name"])
        if key in last and last[key] == k - 1 or (key in last and k - last[key] < 3):
            out[key][-1].append(e)
        else:
            out[key].append([e])
        last[key] = k
    return out


if __name__ == "__main__":
    match = sys.argv[1]
    res = runs(sys.argv[2:], match)
    for (p, name), rl in res.items():
        for i, run in enumerate(rl):
            keys = [k for k in run[0] if k != "name"]
            mean = {k: sum(e[k] for e in run) / len(run) for k in keys}
            print(f"{p.split('/')[-2]} {name} run{i} n={len(run)} " +
                  " ".join(f"{k}={v:.4g}" for k, v in mean.items()))
