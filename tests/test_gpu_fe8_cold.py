"""k_fe8 takes every front end of a live receiver.

Round 4's fast front end (k_fe8) needed every channel's decimator history
full and the call a multiple of 2048 samples: one fmx_reset / fmx_retune of
ONE channel, or a reference-legal dsp_block_samples such as 1024 or 3000
(config.cpp:240 clamps to 1024..32768), sent the whole handle to the generic
k_frontend (1.78 ms against 0.47 ms at 4096 channels).  Round 5: k_fe8 reads
each channel's warmth (dec_valid) and, for a cold channel, enters the zeroed
window of a re-created firdecim (ComplexDecimator::reset,
liquid_primitives.cpp:405-420) as bytes 128 and takes the 127.5 centre of
those positions back out of the first outputs; a call runs as ceil(n / 2048)
chunks of one size, so any n >= 1024 (16-B aligned rows) stays on k_fe8.

  * 4096 channels pipelined as the bench runs them, one fmx_retune of channel
    5 before EVERY block (the reference's retune path main.cpp:1028-1042:
    reset + 40 ms mute): the retuned channel and its neighbours against the
    oracle (with the same retunes), and the kernel timers: every front end of
    the run was k_fe8 (FMX_K_FRONTEND), none the generic one;
  * block sizes 1024 and 3000 (and the first, cold, block of a handle) on
    k_fe8 against the oracle.
Bars as tests/test_gpu_parity.py."""
import pytest

import gpu_harness as H
from test_gpu_parity import check, make_iq, run_both

pytestmark = pytest.mark.gpu

MUTE = 32000 // 25  # kRetuneMuteSamples (main.cpp:696-697)


def test_retune_every_block_stays_on_k_fe8(fmx, oracle, torch_cuda):
    C, NBLK = 4096, 12
    keep = [4, 5, 6, 4095]
    cfg = fmx.make_config()
    scfg = fmx.make_synth(kind=2, n_bits=8192)
    retunes = {b: [(5, MUTE)] for b in range(1, NBLK)}
    g, iq_keep, _, _, kt = H.run_gpu_pipelined(fmx, torch_cuda, cfg, C, scfg, NBLK, keep, warmup=0, retunes=retunes)
    assert kt["frontend"][1] == NBLK and kt["frontend_generic"][1] == 0, kt
    assert kt["pilot"][1] == NBLK and kt["rs"][1] == NBLK, kt
    for j, c in enumerate(keep):
        ret = {b: MUTE for b in retunes} if c == 5 else None
        o = H.run_oracle_pipeline(oracle, oracle.make_cfg(), iq_keep[j], NBLK, retunes=ret)
        check(g, o, c, NBLK, "retune_every_block_fe8", gc=j)


@pytest.mark.parametrize("n", [1024, 3000])
def test_block_size_on_k_fe8(fmx, oracle, torch_cuda, n):
    C, nblk = 4, 10
    iq, _ = make_iq(fmx, 2, C, nblk, B=n)
    kt = {}
    g, outs = run_both(fmx, oracle, torch_cuda, dict(block=n), iq, nblk, ktimes=kt)
    assert kt["frontend"][1] == nblk and kt["frontend_generic"][1] == 0, kt  # the cold first block too
    for c in range(C):
        check(g, outs[c], c, nblk, tag=f"fe8_block_{n}")


@pytest.mark.parametrize("n", [1025, 1028, 3001])
def test_m8_block_sizes_front_end_choice(fmx, oracle, torch_cuda, n):
    """M = 8 (2.048 MS/s, the reference's own rate): every n passes k_fe8's
    IQ-row alignment test there, but its last chunk needs n % 4 == 0
    (ADVICE r5): 1028 runs on k_fe8 (a last chunk of 4 mod 8), 1025 and 3001
    on the generic k_frontend; all three against the oracle."""
    C, nblk = 3, 10
    kw = dict(iq_rate=2_048_000, dsp_rate=256_000, block=n)
    iq, _ = make_iq(fmx, 2, C, nblk, iq_rate=2_048_000, M=8, B=n)
    kt = {}
    g, outs = run_both(fmx, oracle, torch_cuda, kw, iq, nblk, ktimes=kt)
    if n % 4 == 0:
        assert kt["frontend"][1] == nblk and kt["frontend_generic"][1] == 0, kt
    else:
        assert kt["frontend_generic"][1] == nblk and kt["frontend"][1] == 0, kt
    for c in range(C):
        check(g, outs[c], c, nblk, tag=f"m8_block_{n}")
