"""Tower-coordinate multiply tables, CPU only: builds
tests/cpp/tower_check.cpp against the library's host field code and runs it.
The check emulates the device multiply forms byte for byte (12-v_perm general
tables, 6-v_perm subfield tables) against the field of f2e16.hpp, and runs the
1024-point additive FFT / IFFT (additive_fft.hpp:99-141) at index 1024 q,
q = 0..3, in tower coordinates with the tower-image rule against the plain
transform."""
import pathlib
import subprocess

ROOT = pathlib.Path(__file__).resolve().parents[1]
CSRC = ROOT / "erasure-coding-crust_amd" / "csrc"


def test_tower_tables(tmp_path):
    exe = tmp_path / "tower_check"
    subprocess.run(["g++", "-std=c++17", "-O2", f"-I{CSRC}", str(ROOT / "tests" / "cpp" / "tower_check.cpp"),
                    str(CSRC / "gf_field.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "tower tables ok" in out.stdout
