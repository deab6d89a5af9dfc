"""Every repository path DESIGN.md and INTEGRATION.md cite resolves (CPU only).

A cited path is a backticked token naming one of the repository's top-level directories (or a
package-relative `csrc/`, `mppi_solver/`, `robot/` path).  Tokens with a `:line` suffix are
citations of the REFERENCE's files and are skipped; `{a,b}` alternatives are expanded.
"""
import itertools
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "quadrotor_manipulator_mppi_amd")
REPO_DIRS = ("profiles/", "tests/", "tools/", "scripts/", "oracle/", "include/",
             "quadrotor_manipulator_mppi_amd/")
PKG_DIRS = ("csrc/", "mppi_solver/", "robot/")


def _expand(tok):
    parts = re.split(r"(\{[^}]*\})", tok)
    opts = [p[1:-1].split(",") if p.startswith("{") else [p] for p in parts]
    return ["".join(c) for c in itertools.product(*opts)]


def _cited(doc):
    text = open(os.path.join(ROOT, doc), encoding="utf-8").read()
    out = set()
    for tok in re.findall(r"`([^`\s]+)`", text):
        if re.search(r":\d", tok) or not tok.startswith(REPO_DIRS + PKG_DIRS):
            continue
        out.update(_expand(tok.rstrip(".,;")))
    return sorted(out)


@pytest.mark.parametrize("doc", ["DESIGN.md", "INTEGRATION.md"])
def test_cited_paths_resolve(doc):
    missing = []
    for p in _cited(doc):
        base = PKG if p.startswith(PKG_DIRS) else ROOT
        if not os.path.exists(os.path.join(base, p)):
            missing.append(p)
    assert not missing, f"{doc} cites paths that do not exist: {missing}"


def test_design_length():
    with open(os.path.join(ROOT, "DESIGN.md"), encoding="utf-8") as f:
        assert sum(1 for _ in f) <= 700


def _algorithmic_bytes(model, K, H, V):
    """Bytes one rollout launch must move (SURVEY §8d reduced count: the trajectory
    planes written + S; include/mppi_hip.h mppi_rollout_bytes with store_trajectory, device noise)."""
    C = {"drone": 3, "quadrotor": 6, "arm": 7 + 12, "wholebody": 10 + 12}[model]
    return V * K * H * C * 4 + V * K * 4


def test_design_traffic_table_matches_pmc_file():
    """every traffic row DESIGN.md §4a quotes -- algorithmic MB, PMC MB and their
    ratio -- agrees with profiles/pmc_rollout.json (ratio within 0.01), and every shape the PMC file
    holds is quoted."""
    import json
    with open(os.path.join(ROOT, "profiles", "pmc_rollout.json")) as f:
        pmc = json.load(f)
    text = open(os.path.join(ROOT, "DESIGN.md"), encoding="utf-8").read()
    rows = re.findall(r"^\| `(\w+_k\d+_h\d+(?:_v\d+)?)` \| ([\d.]+) \| ([\d.]+) \| ([\d.]+)× \|", text, re.M)
    assert rows, "no traffic table in DESIGN.md"
    quoted = set()
    for key, alg_mb, pmc_mb, ratio in rows:
        m = re.match(r"(\w+?)_k(\d+)_h(\d+)(?:_v(\d+))?$", key)
        model, K, H, V = m.group(1), int(m.group(2)), int(m.group(3)), int(m.group(4) or 1)
        alg = _algorithmic_bytes(model, K, H, V)
        got = pmc[key]["hbm_bytes_per_launch"]
        assert abs(float(alg_mb) - alg / 1e6) < 0.01, (key, alg_mb, alg)
        assert abs(float(pmc_mb) - got / 1e6) < 0.01, (key, pmc_mb, got)
        assert abs(float(ratio) - got / alg) < 0.01, (key, ratio, got / alg)
        quoted.add(key)
    shapes = {k for k, v in pmc.items() if isinstance(v, dict) and v.get("hbm_bytes_per_launch")}
    assert shapes <= quoted, f"PMC shapes DESIGN.md does not quote: {sorted(shapes - quoted)}"
