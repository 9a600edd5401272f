"""fmx_sincos (fmtuner-sdr_amd/csrc/fmx_math.h), the sin/cos every kernel's
NCOs and PLL phase rotations use in place of the reference's float sin/cos
(std::cos/std::sin at stereo_decoder.cpp:179-180, 219-220; std::polar
at redsea_port/dsp/liquid_wrappers.cpp:122 and liquid_wrappers.hh:104): built for the host
from the same header and checked against double-precision sin/cos over the
phase range the kernels feed it.  The bound is < 1 ulp (faithful rounding)."""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_sincos_within_one_ulp(tmp_path):
    exe = str(tmp_path / "math_test")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(ROOT, "tests", "cpp", "math_test.cpp")],
                   check=True, timeout=120)
    out = subprocess.run([exe, "2000000"], check=True, capture_output=True, text=True, timeout=120).stdout
    r = json.loads(out)
    assert r["max_ulp"] < 1.0, r
    assert r["max_abs"] < 1.2e-7, r
    assert r["nco_max_ulp"] < 1.0, r  # quadrant count from the NCO word (k_pll)


def test_near_clip_word_test_exhaustive(tmp_path):
    """fmx_word_near_clip over all 2^32 words (OpenMP, ~5 s on 8 cores)."""
    exe = str(tmp_path / "swar_test")
    subprocess.run(["g++", "-O2", "-fopenmp", "-std=c++17", "-o", exe,
                    os.path.join(ROOT, "tests", "cpp", "swar_test.cpp")], check=True, timeout=120)
    r = json.loads(subprocess.run([exe], check=True, capture_output=True, text=True, timeout=300).stdout)
    assert r == {"false_negatives": 0, "false_positives": 0}


def test_div_const_matches_ieee_division(tmp_path):
    """fmx_div_const (the kernels' division by a constant) is bit-identical
    to IEEE x / c for every normal numerator 1e-30 <= |x| <= 2^60 and zero,
    for the six divisors it is used with (blend target cR / cC / cP, PLL
    error 2 pi, RDS quad-phase 57000, RDS symsync scale 3).  Mismatches exist only below 1e-30
    (residual underflow), where the kernels' numerators never are.  The
    exhaustive sweep (stride 1) is committed in tests/golden/divconst_exhaustive.json;
    this runs every 7th bit pattern."""
    exe = str(tmp_path / "divconst_test")
    subprocess.run(["g++", "-O2", "-fopenmp", "-ffp-contract=off", "-std=c++17", "-o", exe,
                    os.path.join(ROOT, "tests", "cpp", "divconst_test.cpp")], check=True, timeout=120)
    r = json.loads(subprocess.run([exe, "7"], check=True, capture_output=True, text=True, timeout=600).stdout)
    for name in ("cR", "cC", "cP", "2pi", "57000", "3"):
        assert r[name]["bad_ge_1e-30"] == 0, (name, r[name])
    with open(os.path.join(ROOT, "tests", "golden", "divconst_exhaustive.json")) as f:
        ex = json.load(f)
    for name in ("cR", "cC", "cP", "2pi", "57000", "3"):
        assert ex[name]["bad_ge_1e-30"] == 0 and ex[name]["max_bad_abs"] < 1e-30
    assert ex["3"]["bad"] == 0  # division by 3: bit-identical for every normal numerator


def test_pll_chain_sine_error_bounds(tmp_path):
    """pll_sin_word (k_pll's feedback sine from the NCO word) against sin of
    the reference's float phase and of the exact phase.  Exhaustive over all
    2^32 words: tests/golden/pllsin_exhaustive.json (4.4e-7 vs the float
    phase, 1.3e-7 vs the exact phase; fmx_sincos_q on the float phase: 5e-8 /
    4.3e-7).  This runs every 61st word and checks the same bounds."""
    exe = str(tmp_path / "pllsin_test")
    subprocess.run(["g++", "-O2", "-fopenmp", "-ffp-contract=off", "-std=c++17", "-o", exe,
                    os.path.join(ROOT, "tests", "cpp", "pllsin_test.cpp")], check=True, timeout=120)
    r = json.loads(subprocess.run([exe, "61"], check=True, capture_output=True, text=True, timeout=600).stdout)
    assert r["pll_sin_word_vs_float_phase"] < 4.5e-7, r
    assert r["pll_sin_word_vs_exact"] < 1.4e-7, r
    assert r["sincos_q_vs_float_phase"] < 6e-8, r
    with open(os.path.join(ROOT, "tests", "golden", "pllsin_exhaustive.json")) as f:
        ex = json.load(f)
    assert ex["stride"] == 1 and ex["pll_sin_word_vs_float_phase"] < 4.5e-7 and ex["pll_sin_word_vs_exact"] < 1.4e-7


def test_discriminator_atan2_accuracy(tmp_path):
    """fmx_atan2f (the front end's FM discriminator) within 2 ulp of the exact
    atan2 and within 2.5e-7 of the C library's atan2f (the oracle's) over
    random IQ-product arguments spanning 15 decades, and on the axes."""
    exe = str(tmp_path / "atan2_test")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe,
                    os.path.join(ROOT, "tests", "cpp", "atan2_test.cpp")], check=True, timeout=120)
    r = json.loads(subprocess.run([exe, "1000000"], check=True, capture_output=True, text=True, timeout=300).stdout)
    assert r["max_ulp"] < 2.0, r
    assert r["max_abs_vs_atan2f"] < 2.5e-7, r
    assert r["zero_zero"] == 0.0, r


def test_nco_constrain_floor_form_is_exact(tmp_path):
    """fmx_nco_constrain (the kernels' NCO constrain: one floor instead of the
    reference's trunc / compare / double add) returns the reference form's
    word for every float, and fmx_nco_phase (the phase of a word in float
    arithmetic) the reference's double-rounded phase for every word.  Exhaustive over all 2^32 bit patterns:
    tests/golden/ncoconstrain_exhaustive.json; this runs every 13th."""
    exe = str(tmp_path / "ncoconstrain_test")
    subprocess.run(["g++", "-O2", "-fopenmp", "-ffp-contract=off", "-std=c++17", "-o", exe,
                    os.path.join(ROOT, "tests", "cpp", "ncoconstrain_test.cpp")], check=True, timeout=120)
    r = json.loads(subprocess.run([exe, "13"], check=True, capture_output=True, text=True, timeout=600).stdout)
    assert r["mismatches"] == 0 and r["phase_mismatches"] == 0 and r["checked"] > 3 * 10**8, r
    with open(os.path.join(ROOT, "tests", "golden", "ncoconstrain_exhaustive.json")) as f:
        ex = json.load(f)
    assert ex["stride"] == 1 and ex["checked"] == 2**32 and ex["mismatches"] == 0 and ex["phase_mismatches"] == 0
