"""Summarise tools/pmc_detail.sh: python tools/pmc_detail_sum.py <tag>"""
import collections, csv, glob, sys
tag = sys.argv[1]
for d in sorted(glob.glob("gpurun_out/pmcd_%s_*" % tag)):
    if d.endswith(".log"):
        continue
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(d + "/*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if "acoss" not in n:
                continue
            k = n.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("acoss::", "")
            out[k][r["Counter_Name"]] += float(r["Counter_Value"])
    print("==", d)
    for k, v in out.items():
        if v.get("SQ_WAVE_CYCLES", 0) < 1e7:
            continue
        wc = v["SQ_WAVE_CYCLES"]
        print("  %s" % k)
        for c in sorted(v):
            print("     %-26s %12.4g  %6.3f of wave-cycles" % (c, v[c], v[c] / wc))
