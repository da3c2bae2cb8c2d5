"""Join tools/bench_fetch's printed byte counts with its FETCH_SIZE / WRITE_SIZE passes: counter bytes over the
known bytes per kernel (the correction a kernel of that access width needs).
usage: fetch_calib.py bench_stdout.csv FETCH_counter_collection.csv WRITE_counter_collection.csv"""
import collections
import csv
import re
import sys


def load(path, counter):
    d = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        k = re.sub(r"^void ", "", r["Kernel_Name"].split("(")[0]).strip()
        d[k] += float(r["Counter_Value"])
    return d


known = {}
for line in open(sys.argv[1]):
    if "," in line and not line.startswith("kernel"):
        k, b = line.strip().rsplit(",", 1)
        known[k] = float(b)
F, W = load(sys.argv[2], "FETCH_SIZE"), load(sys.argv[3], "WRITE_SIZE")


def find(d, k):
    for name, v in d.items():
        if name == k or name.startswith(k + "("):
            return v
    return None


print("%-22s %14s %14s %10s %14s %10s" % ("kernel", "bytes", "FETCH_SIZE B", "fetch/B", "WRITE_SIZE B", "write/B"))
for k, b in known.items():
    f, w = find(F, k), find(W, k)
    print("%-22s %14.0f %14s %10s %14s %10s" % (
        k, b, "%.0f" % (1024 * f) if f is not None else "-", "%.3f" % (1024 * f / b) if f is not None else "-",
        "%.0f" % (1024 * w) if w is not None else "-", "%.3f" % (1024 * w / b) if w is not None else "-"))
