"""The diagnostic-variant generators under scripts/variants/ patch copies of
the product kernels by exact string match; this checks that every variant
still applies to the current sources (two had gone stale) and that
the product sources carry none of their switches.  CPU only, no compile."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAR = os.path.join(ROOT, "scripts", "variants")


@pytest.mark.parametrize("kind", ["enc", "dec", "encw", "enc4", "dec4"])
def test_stamp_variant_applies(kind, tmp_path):
    out = tmp_path / "v.hip"
    r = subprocess.run([sys.executable, os.path.join(VAR, "stamps.py"), kind, str(out)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    src = out.read_text()
    assert "STAMP(" in src and "ECCR_DIAG_stamps" in src


@pytest.mark.parametrize("kind", ["nobar", "nbread", "nbstg", "static", "nobar+static", "cmp+static", "cmp+wdyn", "nobar+wdyn", "xnobar+xnogat+xnoout+xwdyn", "xnobar+xwdyn", "xnobar", "xnogat", "xnorv", "xnoout", "nost", "nold", "nostg", "stplain", "noprio", "notab", "cmp",
                                  "cmpt", "clk", "clk+nostg", "clk+cmp"])
def test_enc_diag_variant_applies(kind, tmp_path):
    r = subprocess.run([sys.executable, os.path.join(VAR, "enc_diag.py"), kind, str(tmp_path)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    assert (tmp_path / "enc_k256w.hip").exists() and (tmp_path / "cimg.hpp").exists()


def test_product_sources_have_no_diag_switches():
    csrc = os.path.join(ROOT, "erasure-coding-crust_amd", "csrc")
    for f in os.listdir(csrc):
        text = open(os.path.join(csrc, f)).read()
        assert "g_stamp" not in text and "ECCR_DIAG" not in text, f


@pytest.mark.parametrize("knobs", ["RB=5", "PRIO=1", "PRIO=2", "RB=7,PRIO=2"])
def test_n1024x_knob_variant_applies(knobs, tmp_path):
    """reconstruct_n1024x's tuning switches live in
    scripts/variants/n1024x_knobs.py, not in the product source."""
    out = tmp_path / "dec_n1024x.hip"
    r = subprocess.run([sys.executable, os.path.join(VAR, "n1024x_knobs.py"), knobs, str(out)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    src = out.read_text()
    assert ("prio3(wave_s, 3)" in src) == ("PRIO" in knobs)


def test_product_sources_have_no_tuning_macros():
    csrc = os.path.join(ROOT, "erasure-coding-crust_amd", "csrc")
    for f in os.listdir(csrc):
        text = open(os.path.join(csrc, f)).read()
        assert "N1024X_" not in text, f
