"""Host-side exhaustive checks of the device math helpers in
fmtuner-sdr_amd/csrc/fmx_math.h that the kernels call (the near-clip byte
test of the RF level, division by a constant, the discriminator's atan2, the
NCO constrain / phase of k_rds and the block-end PLL state), each against the
reference's own arithmetic.  The stereo PLL chain's v_sin / truncating
converts are hardware arithmetic and are swept on the GPU instead
(tests/test_gpu_pllmath.py)."""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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
