"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate passes as the
MI355X guide prescribes) -> JSON summary.  FETCH_SIZE is doubled (gfx950 reports half the bytes of
wide coalesced reads, MI355X_MICROARCH.md "HBM"); counters are KB.

usage: python tools/pmc_summary.py FETCH.csv WRITE.csv out.json"""
import collections
import csv
import json
import sys


def load(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[r['Kernel_Name'].split('(')[0].replace('uvhp::', '')].append(float(r['Counter_Value']))
    return d


F, W = load(sys.argv[1]), load(sys.argv[2])
out = {"units": "bytes per launch", "fetch_correction": 2.0, "kernels": {}}
for k in sorted(set(F) | set(W)):
    f, w = F.get(k, [0.0]), W.get(k, [0.0])
    fb, wb = 1024 * sum(f) / len(f), 1024 * sum(w) / len(w)
    out["kernels"][k] = {"launches": len(f), "fetch": 2.0 * fb, "write": wb, "traffic": 2.0 * fb + wb}
grp = ["k_feature", "k_gemm_HPg", "k_gemm_HPg_tiled", "k_chi2"]
# per launch group (one k_feature each; the T GEMM is one of the two variants; the delayed-init groups run
# no chi2 kernel): the group kernels' total bytes over the number of groups
ngroups = out["kernels"]["k_feature"]["launches"]
out["feature_group_traffic"] = sum(out["kernels"][k]["traffic"] * out["kernels"][k]["launches"]
                                   for k in grp if k in out["kernels"]) / ngroups
json.dump(out, open(sys.argv[3], "w"), indent=1)
print("feature group traffic per launch: %.0f bytes" % out["feature_group_traffic"])
