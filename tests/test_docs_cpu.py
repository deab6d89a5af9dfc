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
