"""CPU: the reciprocal + fma quotient the march kernel uses for (d - min) / (max - min)
(vr_kernels.hip div_by_range) equals IEEE division on the domain the host enables it for.
A bounded run of tools/div_check.c (the full 3.8e9-pair run is recorded in DESIGN.md)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reciprocal_fma_division_is_correctly_rounded(tmp_path):
    exe = tmp_path / "div_check"
    try:
        subprocess.run(["gcc", "-O2", "-mfma", "-ffp-contract=off",
                        os.path.join(ROOT, "tools", "div_check.c"), "-o", str(exe), "-lm"],
                       check=True, capture_output=True)
    except (OSError, subprocess.CalledProcessError) as e:
        pytest.skip(f"gcc -mfma unavailable: {e}")
    r = subprocess.run([str(exe), "4000", "5000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout
    assert r.stdout.strip().endswith("mismatches 0")
