"""Generate the committed golden fixtures (run from the repo root: python tests/golden/make_golden.py).

chi2_095.json: boost::math::quantile(chi_squared(dof), 0.95) for dof 1..999, the table the reference
builds in UpdaterMSCKF.cpp:52-55 / UpdaterSLAM.cpp:52-55 / StateHelper::initialize (boost is absent
here; scipy.stats.chi2.ppf computes the same quantile to ~1e-15 relative).
"""
import json
import os

from scipy.stats import chi2

HERE = os.path.dirname(os.path.abspath(__file__))

if __name__ == "__main__":
    table = {str(d): float(chi2.ppf(0.95, d)) for d in range(1, 1000)}
    with open(os.path.join(HERE, "chi2_095.json"), "w") as f:
        json.dump({"source": "scipy.stats.chi2.ppf(0.95, dof)", "table": table}, f, indent=0)
    print("wrote chi2_095.json")
