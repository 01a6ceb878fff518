"""Summarise a profiles/profile.sh run (gpurun_out/prof_<tag>) into profiles/<round>/.

    python tools/summarize_profile.py <tag> <round_dir> [calls]

Writes <round_dir>/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats), <tag>_pmc.json
(SQ counters and HBM bytes per kernel) and profiles/traffic_latest.json (HBM bytes per
acoss_crp_align call, for bench.py's roofline.traffic). HBM bytes follow MI355X_MICROARCH.md
§HBM: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads half of a wide
streaming read, so it is doubled.
"""
import collections
import csv
import json
import os
import shutil
import sys

tag, rdir = sys.argv[1], sys.argv[2]
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 2
src = os.path.join("gpurun_out", "prof_" + tag)
os.makedirs(rdir, exist_ok=True)
shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"), os.path.join(rdir, tag + "_kernel_stats.csv"))
out = collections.defaultdict(dict)
for part in ("sq", "fetch", "write"):
    f = os.path.join(src, part, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "acoss" not in name:
            continue
        k = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("acoss::", "")
        out[k][r["Counter_Name"]] = out[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
tot = 0.0
for k, v in out.items():
    hbm = 1024.0 * (2.0 * v.get("FETCH_SIZE", 0.0) + v.get("WRITE_SIZE", 0.0))
    v["hbm_bytes_corrected"] = hbm
    tot += hbm
json.dump(out, open(os.path.join(rdir, tag + "_pmc.json"), "w"), indent=1, sort_keys=True)
json.dump({"source": os.path.join(rdir, tag + "_pmc.json"), "calls": calls, "frames": 2000,  # profile.sh: bench defaults
           "hbm_bytes_per_launch": tot / calls,
           "note": "sum over all acoss kernels of 1024*(2*FETCH_SIZE+WRITE_SIZE) / acoss_crp_align calls"},
          open(os.path.join("profiles", "traffic_latest.json"), "w"), indent=1)
print("HBM bytes per call: %.3e" % (tot / calls))
for k, v in sorted(out.items()):
    print("%-40s hbm=%.3e  valu=%.3e" % (k[:40], v["hbm_bytes_corrected"], v.get("SQ_INSTS_VALU", 0)))
