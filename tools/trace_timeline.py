"""Per-phase timelines from a rocprofv3 --kernel-trace CSV (the bench under rocprof):
one PPO minibatch (between two Adam launches), one env step (between two physics launches) and
the iteration boundaries (update end -> first physics, last rollout step -> first GEMM), with the
queue of every launch and the gaps between them.

Usage: python tools/trace_timeline.py gpurun_out/prof/run_kernel_trace.csv"""
import csv
import sys


def load(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def show(rows, a, b, t0, title):
    print(f"---- {title}")
    for r in rows[a:b]:
        s = (int(r["Start_Timestamp"]) - t0) / 1000
        e = (int(r["End_Timestamp"]) - t0) / 1000
        print(f"{s:9.1f} {e:9.1f} {e - s:7.1f} q{r['Queue_Id']} {r['Kernel_Name'][:80]}")


def main(path):
    rows = load(path)
    find = lambda key: [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
    adam, phys = find("adam_clip"), find("lgx_physics_kernel")
    if len(adam) >= 3:
        a, b = adam[-3], adam[-2]
        show(rows, a, b + 1, int(rows[a]["End_Timestamp"]), "one PPO minibatch (Adam to Adam)")
    if len(phys) >= 5:
        a, b = phys[-5], phys[-4]
        show(rows, a, b + 1, int(rows[a]["Start_Timestamp"]), "one env step (physics to physics)")
    if len(adam) >= 21:
        a = adam[-21]
        j = next(j for j in range(a, len(rows)) if "lgx_physics_kernel" in rows[j]["Kernel_Name"])
        show(rows, a, j + 1, int(rows[a]["End_Timestamp"]), "update end -> first physics of the next rollout")
    # GPU idle per iteration: wall between the first physics launches of consecutive rollouts vs
    # the union of all kernel intervals (any queue) inside it
    aset = set(adam)
    starts = [i for p, i in zip(phys, phys[1:]) if any(j in aset for j in range(p, i))]
    for a, b in zip(starts, starts[1:]):
        t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows[a:b])
        busy, cs, ce = 0, iv[0][0], iv[0][1]
        for s, e in iv[1:]:
            if s > ce:
                busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        print(f"iteration {t0}: wall {(t1 - t0) / 1e6:.3f} ms, GPU busy {busy / 1e6:.3f} ms, idle {(t1 - t0 - busy) / 1e3:.0f} us")
    if phys:
        b = phys[-1]
        j = next((j for j in range(b, len(rows)) if "gemm_nt_x3p" in rows[j]["Kernel_Name"]), None)
        if j is not None:
            show(rows, b, j + 1, int(rows[b]["End_Timestamp"]), "last rollout physics -> first update GEMM")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv")
