"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate passes as the
MI355X guide prescribes) -> JSON summary.  FETCH_SIZE is doubled (gfx950 reports half the bytes of
wide coalesced reads, MI355X_MICROARCH.md "HBM"); counters are KB.

An optional third pass (MFMA.csv: SQ_INSTS_VALU_MFMA_MOPS_F64 and SQ_VALU_MFMA_BUSY_CYCLES) adds the FP64 MFMA
work per launch: flops = MOPS_F64 x 512 (rocprofv3's MfmaFlopsF64 expression) and the matrix-core busy
cycles.  Template instantiations of one kernel (k_ekf_fact<2>, ...) are merged under the kernel's name.

usage: python tools/pmc_summary.py FETCH.csv WRITE.csv out.json [MFMA.csv]"""
import collections
import csv
import json
import re
import sys


def kname(raw):
    n = raw.split('(')[0].replace('uvhp::', '').replace('void ', '').strip()
    return re.sub(r'<.*>', '', n)


def load(path, counter=None):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if counter and r.get('Counter_Name') != counter:
            continue
        d[kname(r['Kernel_Name'])].append(float(r['Counter_Value']))
    return d


F, W = load(sys.argv[1]), load(sys.argv[2])
out = {"units": "bytes per launch", "fetch_correction": 2.0, "kernels": {}}
for k in sorted(set(F) | set(W)):
    f, w = F.get(k, [0.0]), W.get(k, [0.0])
    fb, wb = 1024 * sum(f) / len(f), 1024 * sum(w) / len(w)
    out["kernels"][k] = {"launches": len(f), "fetch": 2.0 * fb, "write": wb, "traffic": 2.0 * fb + wb}
if len(sys.argv) > 4:
    M = load(sys.argv[4], "SQ_INSTS_VALU_MFMA_MOPS_F64")
    B = load(sys.argv[4], "SQ_VALU_MFMA_BUSY_CYCLES")
    for k, v in M.items():
        if k in out["kernels"]:
            out["kernels"][k]["mfma_f64_flops"] = 512.0 * sum(v) / len(v)
            b = B.get(k, [0.0])
            out["kernels"][k]["mfma_busy_cycles"] = sum(b) / len(b)
grp = ["k_feature", "k_gemm_HPg", "k_gemm_HPg_tiled", "k_chi2_S", "k_chi2_S2", "k_chi2"]
# per launch group (one k_feature each; the T GEMM is one of the two variants; the delayed-init groups run
# no chi2 kernel): the group kernels' total bytes over the number of groups
ngroups = out["kernels"]["k_feature"]["launches"]
out["feature_group_traffic"] = sum(out["kernels"][k]["traffic"] * out["kernels"][k]["launches"]
                                   for k in grp if k in out["kernels"]) / ngroups
json.dump(out, open(sys.argv[3], "w"), indent=1)
print("feature group traffic per launch: %.0f bytes" % out["feature_group_traffic"])
