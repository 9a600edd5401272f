"""The shipped stereo-PLL arithmetic of k_pll, pinned on the GPU (VERDICT r4
item 3).  k_pll calls fmx_chain_sin / fmx_chain_words (W0's feedback chain)
and fmx_word_sincos (the P waves' vcoI / vcoQ / cos 2 phase), all in
fmtuner-sdr_amd/csrc/fmx_math.h; tests/hip/pllmath_sweep.hip (test code,
built into tests/hip/libpllmath.so by __graft_entry__.build()) calls the same
functions on the GPU and sweeps:

  * every 2^32 NCO word: the chain sine and the word sine / cosine against
    sin / cos of the reference's float phase (float)(2 pi (float)theta / 2^32)
    -- what stereo_decoder.cpp:178-180 feeds std::sin / std::cos through
    liquid's nco_crcf_get_phase -- and against the exact phase, in double
    precision; plus the chain sine's mean signed error (its truncation bias);
  * every float pilot with 2^-30 <= |pilot| < 2, both signs, times eight vcoQ
    values: the chain's two pll_step words (round 6: the alpha word as the
    reference rounds it, 2^32 + x in f32 for e < 0; the beta word a
    truncating convert) against liquid's constrain of e alpha, e beta (e =
    pilot vcoQ in float), as fmx_nco_constrain_ref: maxima and, for e < 0,
    mean errors.

The maxima of the full sweep are committed in tests/golden/pllmath_gpu.json
(FMX_PLLMATH_OUT=path writes them); the sweep is deterministic hardware
arithmetic, so the live run must reproduce them exactly, and each stays under
the absolute bound written below."""
import ctypes as C
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# FMX_PLLMATH_LIB: a sweep built with other forms (A/B only, tests/hip variant)
LIB = os.environ.get("FMX_PLLMATH_LIB") or os.path.join(ROOT, "tests", "hip", "libpllmath.so")
GOLD = os.path.join(ROOT, "tests", "golden", "pllmath_gpu.json")
KEYS = ["chain_sin_vs_ref_phase", "chain_sin_vs_exact", "word_sin_vs_ref_phase", "word_cos_vs_ref_phase",
        "word_sin_vs_exact", "word_cos_vs_exact", "chain_sin_mean_err", "chain_sin_mean_abs_err", "words",
        "ca_max_pos", "cb_max_pos", "ca_max_neg", "cb_max_neg", "ca_rel_max", "cb_rel_max", "pairs",
        "chain_phase_bias", "form_chain", "form_word_sincos", "form_words", "ca_mean_abs_neg", "cb_mean_abs_neg"]
# absolute bounds (radian-free: sine units; words: units of 2^-32 turn)
BOUNDS = {
    # v_sin of the word's top 23 bits as a float in [1, 2): < 2^-23 turn of
    # truncation (7.5e-7 of sine) + the hardware sine + the reference
    # phase's own rounding
    "chain_sin_vs_ref_phase": 1.5e-6,
    "chain_sin_vs_exact": 1.5e-6,
    # the word as a 24-bit signed fraction of a turn
    "word_sin_vs_ref_phase": 6e-7,
    "word_cos_vs_ref_phase": 6e-7,
    "word_sin_vs_exact": 6e-7,
    "word_cos_vs_exact": 6e-7,
    # e >= 0: the float products' roundings (~2^-23 relative of words <=
    # 2^25 for alpha, 2^28 for beta); e < 0: the reference rounds 1 + frac
    # to 24 bits (256-word steps), the truncating convert does not
    "ca_max_pos": 64, "cb_max_pos": 512,
    "ca_max_neg": 512, "cb_max_neg": 1024,
}


def sweep():
    L = C.CDLL(LIB)
    L.pllmath_sweep.restype = C.c_int
    L.pllmath_sweep.argtypes = [C.c_float, C.c_float, C.POINTER(C.c_double), C.c_int]
    out = (C.c_double * len(KEYS))()
    # the design's PLL constants (fmx_design.cpp: bandwidth 0.01, beta = sqrt)
    alpha = np.float32(0.01)
    beta = np.sqrt(alpha, dtype=np.float32)
    rc = L.pllmath_sweep(C.c_float(alpha), C.c_float(beta), out, len(KEYS))
    assert rc == 0, rc
    return {k: out[i] for i, k in enumerate(KEYS)}


def test_pll_chain_math_exhaustive(torch_cuda):
    r = sweep()
    print(json.dumps(r))
    if os.environ.get("FMX_PLLMATH_OUT"):
        with open(os.environ["FMX_PLLMATH_OUT"], "w") as f:
            json.dump(r, f, indent=1)
    assert r["words"] == 2 ** 32
    for k, b in BOUNDS.items():
        assert r[k] <= b, (k, r[k], b)
    # the truncation biases the chain sine by < 2^-24 turn on average
    assert abs(r["chain_sin_mean_err"]) < 4e-7, r
    # the shipped forms (round 6, fmx_math.h): the chain sine of the word
    # rounded to 23 bits has no phase bias (the truncated one lagged by
    # 3.7e-7 rad), and the frequency (alpha) word follows the reference's
    # 256-word rounding for e < 0 -- a mean error well under a word, where
    # the truncating convert is off by ~64 on average
    assert r["form_chain"] == 1 and r["form_words"] == 3, r
    assert abs(r["chain_phase_bias"]) < 1e-8, r
    assert r["ca_mean_abs_neg"] < 2.0 and r["cb_mean_abs_neg"] < 128.0, r
    with open(GOLD) as f:
        g = json.load(f)
    for k in KEYS:
        assert r[k] == pytest.approx(g[k], rel=1e-9, abs=1e-12), (k, r[k], g[k])
