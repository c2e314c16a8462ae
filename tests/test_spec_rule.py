"""The bracketed encoder's decision rule on the CPU (scripts/exp/spec_check.c, gcc).

qsgd_spec_quant writes a level without knowing the norm when ceil(fma(|x|, c_lo, -max(u, 2^-26)))
equals ceil(fma(|x|, c_hi, -u)) for the bracket's outward-rounded multipliers; the checker draws
brackets, norms inside them, inputs at and around the decision points j + u, sub-normal ratios and
u == 0, and compares every decided level with the reference's exact level
(src/omnifed/hybrid/compression/qsgd.py:50-63).  It must find no mismatch.
"""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "scripts", "exp", "spec_check.c")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_spec_decision_rule_has_no_mismatch(tmp_path):
    exe = str(tmp_path / "spec_check")
    subprocess.run(["gcc", "-O2", "-o", exe, SRC, "-lm"], check=True)
    out = subprocess.run([exe, "10000000"], check=False, capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "mismatches 0" in out.stdout, out.stdout
