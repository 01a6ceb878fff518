"""Summarise a profiles/profile.sh run (gpurun_out/prof_<tag>) into profiles/<round>/.

    python tools/summarize_profile.py <tag> <round_dir> [calls] [corpus] [frames]

Writes <round_dir>/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats), <tag>_pmc.json
(SQ counters and HBM bytes per kernel), profiles/traffic_latest.json (HBM bytes per
acoss_crp_align call, bench.py's roofline.traffic) and profiles/valu_latest.json (per kernel:
average duration from the kernel trace, VALU wave-instructions per launch, and the VALU-issue
fraction = SQ_INSTS_VALU / (duration x 614.4 G wave-instructions/s: 256 CUs x 4 SIMDs x 2.4 GHz /
4 cycles per wave64 instruction), bench.py's roofline.valu_issue). HBM bytes follow
MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads half
of a wide streaming read, so it is doubled (the counters include Infinity-Cache hits).
"""
import collections
import csv
import json
import os
import shutil
import sys

tag, rdir = sys.argv[1], sys.argv[2]
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 2
corpus = sys.argv[4] if len(sys.argv) > 4 else "hard"
frames = int(sys.argv[5]) if len(sys.argv) > 5 else 2000
PEAK_WAVE_INSTR = 256 * 4 * 2.4e9 / 4
# the kernels acoss_crp_align launches (prep, OTI, roll, sweep + row select, column select, DP)
CRP_KERNEL = lambda n: any(s in n for s in ("k_track_", "k_pair_oti", "k_rotate_ref", "k_sweep_rows9", "k_sel_cols9",
                                            "k_crp_"))  # noqa: E731
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
        if "acoss" not in name or not CRP_KERNEL(name):
            continue
        k = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("acoss::", "")
        out[k][r["Counter_Name"]] = out[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
bfile = os.path.join(src, "build.json")
build = json.load(open(bfile)) if os.path.exists(bfile) else None
tot = 0.0
for k, v in out.items():
    hbm = 1024.0 * (2.0 * v.get("FETCH_SIZE", 0.0) + v.get("WRITE_SIZE", 0.0))
    v["hbm_bytes_corrected"] = hbm
    tot += hbm
json.dump(out, open(os.path.join(rdir, tag + "_pmc.json"), "w"), indent=1, sort_keys=True)
json.dump({"source": os.path.join(rdir, tag + "_pmc.json"), "calls": calls, "frames": frames, "corpus": corpus,
           "build": build, "hbm_bytes_per_launch": tot / calls,
           "note": "sum over all acoss kernels of 1024*(2*FETCH_SIZE+WRITE_SIZE) / acoss_crp_align calls"},
          open(os.path.join("profiles", "traffic_latest.json"), "w"), indent=1)
# per-kernel durations (kernel trace, one stream) and VALU-issue fractions
dur = {}
for r in csv.DictReader(open(os.path.join(src, "kt", "run_kernel_stats.csv"))):
    name = r["Name"]
    if "acoss" not in name or not CRP_KERNEL(name):
        continue
    k = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("acoss::", "")
    dur[k] = {"calls": int(r["Calls"]), "total_ms": float(r["TotalDurationNs"]) / 1e6,
              "avg_ms": float(r["AverageNs"]) / 1e6}
valu = {}
for k, d in dur.items():
    v = out.get(k, {})
    instr = v.get("SQ_INSTS_VALU", 0.0)
    valu[k] = dict(d, valu_instr_per_call=instr / calls, hbm_bytes_per_call=v.get("hbm_bytes_corrected", 0.0) / calls,
                   valu_issue_frac=(instr / (d["total_ms"] * 1e-3 * PEAK_WAVE_INSTR)) if d["total_ms"] > 0 else None)
ksum = sum(d["total_ms"] for d in dur.values()) / calls
json.dump({"source": os.path.join(rdir, tag + "_kernel_stats.csv") + " + " + os.path.join(rdir, tag + "_pmc.json"),
           "calls": calls, "frames": frames, "corpus": corpus, "streams": 1, "build": build,
           "kernel_ms_per_call": ksum, "kernels": valu,
           "peak_wave_instr_per_s": PEAK_WAVE_INSTR},
          open(os.path.join("profiles", "valu_latest.json"), "w"), indent=1)
print("kernel ms per call (one stream): %.3f" % ksum)
for k, v in sorted(valu.items(), key=lambda kv: -kv[1]["total_ms"]):
    print("  %-32s %9.3f ms/call  valu issue %s" % (k[:32], v["total_ms"] / calls,
                                                    "%.3f" % v["valu_issue_frac"] if v["valu_issue_frac"] else "-"))
print("HBM bytes per call: %.3e" % (tot / calls))
for k, v in sorted(out.items()):
    print("%-40s hbm=%.3e  valu=%.3e" % (k[:40], v["hbm_bytes_corrected"], v.get("SQ_INSTS_VALU", 0)))
