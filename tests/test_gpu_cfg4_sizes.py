"""GPU parity at the per-GPU sizes of the Cfg4 strong-scaling curve
(BASELINE.json configs[3]: 16 384 channels over 1 / 2 / 4 / 8 GPUs, i.e.
16 384, 8 192, 4 096 and 2 048 channels in one handle).  4 096 is
test_gpu_pipelined.py's Cfg3 run and 2 048 its rank-1 shard; here the two
large handles, pipelined exactly as bench.py runs them:

  * sampled channels at the edges of every 4 096-channel quarter against the
    oracle (RDS groups bit-exact, PCM RMS < 1e-5, flags / pilot / counts
    exact: tests/test_gpu_parity.py's bars);
  * at 16 384 channels, every channel's error-free RDS groups against the
    transmitted group sequence (ground truth, size-independent), and stereo
    on > 99 % of the channels after acquisition."""
import os
import sys

import numpy as np
import pytest

import gpu_harness as H
from test_gpu_parity import check  # noqa: F401

pytestmark = pytest.mark.gpu

NBLK = 40


def _run(fmx, oracle, torch, C, keep, all_groups=None):
    cfg = fmx.make_config()
    scfg = fmx.make_synth(kind=2, n_bits=8192)
    g, iq_keep, tx, stereo_all, kt = H.run_gpu_pipelined(fmx, torch, cfg, C, scfg, NBLK, keep,
                                                         all_groups=all_groups)
    assert all(v[1] == NBLK - 5 for k, v in kt.items() if k != "frontend_generic") and kt["frontend_generic"][1] == 0, kt
    ngroups = 0
    for j, c in enumerate(keep):
        o = H.run_oracle_pipeline(oracle, oracle.make_cfg(), iq_keep[j], NBLK)
        st = check(g, o, c, NBLK, f"cfg4_{C}ch_pipelined", gc=j)
        ngroups += len(st["groups_oracle"])
    assert ngroups >= 2 * len(keep)
    assert stereo_all[-1] > 0.99
    return scfg


def test_cfg4_n1_16384_channels_pipelined(fmx, oracle, torch_cuda):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_oracle_pinning import groups_align
    C = 16384
    keep = [0, 4095, 4096, 8191, 12288, 16383]
    got = []
    scfg = _run(fmx, oracle, torch_cuda, C, keep, all_groups=got)
    _, tx = fmx.synth_rds_bits(scfg, 0, C)
    assert len(got) == C
    with_clean = [c for c in range(C) if any(x[4] == 0 for x in got[c])]
    bad = [c for c in with_clean if not groups_align(got[c], tx[c])]
    assert not bad, bad[:10]
    assert len(with_clean) > 0.99 * C, len(with_clean)


def test_cfg4_n2_8192_channels_pipelined(fmx, oracle, torch_cuda):
    _run(fmx, oracle, torch_cuda, 8192, [0, 1, 4095, 4096, 8191])
