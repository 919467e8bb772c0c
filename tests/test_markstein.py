"""The fused kernel's shared-reciprocal division (bmfr_device.h div_by_recip)
must be the correctly rounded quotient: checked on the CPU, where glibc's
fmaf is exact, over every divisor mantissa of a binade and random pairs."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_markstein_division_is_correctly_rounded(tmp_path):
    exe = str(tmp_path / "markstein_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math",
                    os.path.join(HERE, "native", "markstein_check.c"), "-o", exe, "-lm"], check=True)
    out = subprocess.run([exe, "8", "20000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "bad 0" in out.stdout
