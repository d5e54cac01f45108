"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/<pass>/run_counter_collection.csv) into the
per-dispatch means JSON that bench.py reads (profiles/r02_pmc_env_kernels.json)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/r02_pmc_env_kernels.json"
what = sys.argv[3] if len(sys.argv) > 3 else None
out = {"what": what or "rocprofv3 --kernel-trace --pmc, per-dispatch means over tools/kbench.py physrun (go1_rough, "
               "4096 envs, 10 env steps); FETCH_SIZE/WRITE_SIZE in KB (gfx950: FETCH_SIZE reads half of wide "
               "coalesced bytes); SQ_* = wave-instruction totals per dispatch; passes *_sep ran with "
               "LGX_ACT_OVERLAP=0 (actuator net as its own launch)",
       "passes": {}}
# the workload the passes ran (bench.py uses a file's traffic / MFMA figures only for that workload)
out["workload"] = {"task": os.environ.get("LGX_PMC_TASK", "go1_rough"),
                   "num_envs": int(os.environ.get("LGX_PMC_ENVS", "4096"))}
for f in sorted(glob.glob(os.path.join(src, "*", "run_counter_collection.csv"))):
    name = os.path.basename(os.path.dirname(f))
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        k = re.sub(r"\(.*", "", k)
        if k.startswith(("at::", "rocprim", "Cijk", "__amd")) or not ("lgx_" in k or k.endswith("_kernel>") or
                                                                    "_kernel" in k):
            continue
        acc[k][r["Counter_Name"]].append((int(r.get("Dispatch_Id", 0)), float(r["Counter_Value"])))
    res = {}
    for k, cs in acc.items():
        res[k] = {}
        for c, vals in cs.items():
            per = defaultdict(float)   # a counter may come in several rows per dispatch (instances)
            for d, v in vals:
                per[d] += v
            res[k][c] = sum(per.values()) / len(per)
            res[k]["dispatches"] = len(per)
    out["passes"][name] = res
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out["passes"], indent=1)[:3000])
