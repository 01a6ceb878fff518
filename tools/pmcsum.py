"""Summarise tools/pmc2.sh output: python tools/pmcsum.py <tag>"""
import collections, csv, glob, sys
tag = sys.argv[1]
out = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob("gpurun_out/pmc_%s/*/run_counter_collection.csv" % tag):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "acoss" not in n:
            continue
        k = n.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("acoss::", "")
        out[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in out.items():
    if v.get("SQ_WAVE_CYCLES", 0) < 1e8:
        continue
    wc = v["SQ_WAVE_CYCLES"]
    print("%s  waves=%.0f" % (k, v.get("SQ_WAVES", 0)))
    for c in sorted(v):
        print("   %-26s %14.4g  %6.3f of wave-cycles" % (c, v[c], v[c] / wc))
