"""The row Adam divides sqrt(v) by the step constant c_t with Markstein's correction instead of an
IEEE division (csrc/lgcn_rowadam.hip div_step). tools/markstein_check.c proves it equal to the IEEE
quotient for every normal s, one binade per constant (scale invariance); the full schedule of
beta2 = 0.999 (10,030 constants, ~4 CPU-minutes) is in profiles/r03x_adam/markstein_check.log.
Here: the first 64 constants, and that a perturbed formula is caught (the checker can fail)."""
import pathlib
import shutil
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    out = tmp_path_factory.mktemp("mk") / "markstein_check"
    subprocess.run(["gcc", "-O2", "-mfma", "-ffp-contract=off", str(ROOT / "tools" / "markstein_check.c"), "-lm",
                    "-o", str(out)], check=True)
    return out


def test_first_step_constants_exact(checker):
    r = subprocess.run([str(checker), "0.999", "64"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout
    assert "64 distinct step constants" in r.stdout and ", 0 mismatches" in r.stdout, r.stdout


def test_checker_catches_a_wrong_formula(tmp_path):
    """Without the correction step (q = s * rc alone) the quotient is not always correctly rounded:
    the checker must report mismatches."""
    src = (ROOT / "tools" / "markstein_check.c").read_text().replace(
        "const float q = fmaf(fmaf(-c, q0, s), rc, q0);", "const float q = q0;")
    assert "const float q = q0;" in src
    (tmp_path / "bad.c").write_text(src)
    exe = tmp_path / "bad"
    subprocess.run(["gcc", "-O2", "-mfma", "-ffp-contract=off", str(tmp_path / "bad.c"), "-lm", "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe), "0.999", "4"], capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "0 mismatches" not in r.stdout
