import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

EUROC = os.path.join(ROOT, "configs", "euroc_mav", "estimator_config.yaml")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def euroc_yaml():
    return EUROC


# Rounding-tie steering accounting (tests/test_gpu_parity.py _check_steer): every lock-step test's steering events
# (count, cap, margins, features touched) are collected here and written at the end of the session to
# gpurun_out/steer/summary.json (kept by the GPU runs) and printed in the terminal summary.
STEER_RECORDS = {}


def record_steer(events, n_features, cap):
    test = os.environ.get("PYTEST_CURRENT_TEST", "unknown").split(" ")[0]
    rec = STEER_RECORDS.setdefault(test, {"events": 0, "found": 0, "features_updated": 0, "cap": 0,
                                          "max_margin": 0.0, "features": []})
    rec["events"] += len(events)
    rec["found"] += sum(1 for e in events if e["found"])
    rec["features_updated"] += int(n_features)
    rec["cap"] += int(cap) if cap is not None else 0
    for e in events:
        rec["max_margin"] = max(rec["max_margin"], float(e["margin"]))
        rec["features"].append({"kind": int(e["kind"]), "featid": int(e["featid"]), "stage": int(e["stage"]),
                                "cast": int(e["index"]), "margin": float(e["margin"]),
                                "before": float(e["before"]), "after": float(e["after"])})


def pytest_sessionfinish(session, exitstatus):
    if not STEER_RECORDS:
        return
    out = os.path.join(ROOT, "gpurun_out", "steer")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "summary.json"), "w") as f:
        json.dump(STEER_RECORDS, f, indent=1)


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    if not STEER_RECORDS:
        return
    terminalreporter.write_sep("-", "rounding-tie steering events per lock-step test (gpurun_out/steer/summary.json)")
    for test, r in sorted(STEER_RECORDS.items()):
        terminalreporter.write_line("%-90s events %3d / cap %3d  features updated %6d  max margin %.1e" %
                                    (test, r["events"], r["cap"], r["features_updated"], r["max_margin"]))
