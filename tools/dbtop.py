"""Print the top kernels of a rocprofv3 results database: python tools/dbtop.py <dir> [n]."""
import glob
import sqlite3
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
db = sqlite3.connect(glob.glob(d + "/*.db")[0])
for name, calls, tot, avg, pct in db.execute("select * from top_kernels limit ?", (n,)):
    short = name.replace("acoss::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    print("%-46s %5d %10.1f us %9.1f us %5.1f%%" % (short[:46], calls, tot, avg, pct))
