"""GPU parity of the MEASURED mode: fmx_process_block back to back with no
host synchronisation between blocks, exactly as bench.py's timed loop runs
it (bench.py step(): four streams, three-deep intermediates, cross-step
events, the next step's resampler schedules uploaded speculatively, kernel
timing on, RF level on).  The other GPU parity tests synchronise after every
block; these compare the pipelined outputs with the oracle on the same IQ.

  * Cfg3 at full size (BASELINE.json configs[2]): 4096 channels, 36 blocks.
  * Cfg4's per-GPU shard (configs[3]): 16384 channels over 8 GPUs is 2048
    channels per GPU; rank 1's shard is channels [2048, 4096) of the
    synthetic plan (fmx_dist.shard(16384, 8, 1)), generated on the device
    with fmx_synth_device(ch0=2048), MPX output on.
  * SURVEY 8f row 3 end to end: the HIP-decoded groups through the product's
    XDR formatter (fmx_xdr_rds_lines) against the oracle's groups through the
    Python restatement of XDRServer::updateRDS (tests/xdr_ref.py), with PI
    changes (the groups of two stations fed to one server state in turn, as
    a retune does).

Bars as tests/test_gpu_parity.py (RDS groups bit-exact; PCM RMS < 1e-5;
flags, pilot level, counts exact; RF level as test_signal_level.py)."""
import numpy as np
import pytest

import gpu_harness as H
from test_gpu_parity import check, log_errors  # noqa: F401
from xdr_ref import PyXdr

pytestmark = pytest.mark.gpu

NBLK = 36


@pytest.fixture(scope="module")
def cfg3_pipelined(fmx, oracle, torch_cuda):
    C = 4096
    keep = [0, 1, 63, 64, 2047, 4095]
    cfg = fmx.make_config()
    scfg = fmx.make_synth(kind=2, n_bits=8192)
    g, iq_keep, tx, stereo_all, kt = H.run_gpu_pipelined(fmx, torch_cuda, cfg, C, scfg, NBLK, keep)
    outs = [H.run_oracle_pipeline(oracle, oracle.make_cfg(), iq_keep[j], NBLK) for j in range(len(keep))]
    return dict(g=g, outs=outs, keep=keep, iq_keep=iq_keep, tx=tx, stereo_all=stereo_all, kt=kt)


def test_cfg3_pipelined_bench_mode(cfg3_pipelined, oracle):
    r = cfg3_pipelined
    g, outs, keep = r["g"], r["outs"], r["keep"]
    # the run really was pipelined and timed like the bench
    assert all(v[1] == NBLK - 5 for k, v in r["kt"].items() if k != "frontend_generic"), r["kt"]
    assert r["kt"]["frontend_generic"][1] == 0, r["kt"]  # every front end on k_fe8
    ngroups = 0
    for j, c in enumerate(keep):
        st = check(g, outs[j], c, NBLK, "cfg3_pipelined", gc=j)
        ngroups += len(st["groups_oracle"])
        for b in range(NBLK):
            assert abs(float(g[b]["clip"][j]) - float(outs[j][b]["clip"])) < 1e-7, (c, b)
    assert ngroups >= 2 * len(keep)
    assert r["stereo_all"][-1] > 0.99


def test_cfg3_pipelined_signal_level(fmx, cfg3_pipelined):
    """The per-block RF level records (computeSignalLevel, the bench's scan
    reads) of the pipelined run against signal_level.cpp's formulas."""
    import oracle as O
    # the records were written into the per-block sig buffers; re-run the
    # checker on the same IQ
    r = cfg3_pipelined
    checker = O.ref_signal_level if O.ref_available() else O.signal_level
    n_iq = 4096 * 10
    for j in range(len(r["keep"])):
        sm = O.SignalSmoother()
        for b in range(NBLK):
            want = checker(r["iq_keep"][j, b * 2 * n_iq:(b + 1) * 2 * n_iq])
            got = r["g"][b]["sig"][j]
            assert abs(got.dbfs - want["dbfs"]) < 1e-9, (j, b, got.dbfs, want["dbfs"])
            assert abs(got.level120 - want["level120"]) <= 1e-4
            assert got.hard_clip_ratio == want["hard_clip_ratio"] and got.near_clip_ratio == want["near_clip_ratio"]
            assert abs(got.level120_smoothed - sm(want["level120"])) <= 1e-4


def test_cfg4_rank1_shard_pipelined(fmx, oracle, torch_cuda):
    """Cfg4's per-GPU shard at rank 1 of 8: 2048 channels starting at
    channel 2048 of the plan (the rank >= 1 offsets through fmx_synth_device
    and fmx_dist.shard), pipelined, MPX on."""
    import fmx_dist
    ch0, ch1 = fmx_dist.shard(16384, 8, 1)
    assert (ch0, ch1) == (2048, 4096)
    C = ch1 - ch0
    keep = [0, 1, 63, 64, 1023, 2047]
    cfg = fmx.make_config()
    scfg = fmx.make_synth(kind=2, n_bits=8192)
    g, iq_keep, tx, stereo_all, _ = H.run_gpu_pipelined(fmx, torch_cuda, cfg, C, scfg, NBLK, keep, ch0=ch0,
                                                        with_mpx=True)
    # the shard's rows are the plan's channels ch0 + j: a host synthesis of
    # the plan's channel (float libm vs device math: a few bytes may round the
    # other way) and not of the un-offset channel j
    bits1, _ = fmx.synth_rds_bits(scfg, ch0 + keep[-1], 1)
    host = fmx.synth_host(scfg, ch0 + keep[-1], 1, 0, 4096 * 10 * 4, bits1)[0].astype(np.int16)
    dev_row = iq_keep[-1, :host.size].astype(np.int16)
    assert np.max(np.abs(host - dev_row)) <= 1 and np.mean(host != dev_row) < 1e-3
    other = fmx.synth_host(scfg, keep[-1], 1, 0, 4096 * 10 * 4, fmx.synth_rds_bits(scfg, keep[-1], 1)[0])[0]
    assert np.mean(other.astype(np.int16) != dev_row) > 0.5
    ngroups = 0
    for j, c in enumerate(keep):
        o = H.run_oracle_pipeline(oracle, oracle.make_cfg(), iq_keep[j], NBLK)
        st = check(g, o, ch0 + c, NBLK, "cfg4_rank1_pipelined", gc=j)
        ngroups += len(st["groups_oracle"])
        # PI of the plan's channel (synthetic plan: PI = 0x1000 + channel)
        assert all(x[0] == (0x1000 + ch0 + c) & 0xFFFF for x in st["groups_oracle"] if (x[4] >> 6) == 0)
    assert ngroups >= 2 * len(keep)
    assert stereo_all[-1] > 0.99


def test_xdr_lines_from_gpu_groups(fmx, oracle, cfg3_pipelined):
    """8f row 3 on the GPU path: HIP-decoded groups -> fmx_xdr_rds_lines,
    byte for byte against the oracle's groups -> the restated updateRDS and
    against the HIP groups -> the reference's XDRServer (oracle/_ref), over
    36 blocks per station, stations switched (PI changes) as a retune would:
    channel 0's groups, then channel 1's, then channel 0's again, into one
    server state each side."""
    r = cfg3_pipelined
    g, outs = r["g"], r["outs"]
    gpu_x = fmx.XdrRds()
    ref_x = PyXdr()
    got, want = [], []
    n_pi = set()
    for j in (0, 1, 0):
        for b in range(NBLK):
            gg = g[b]["groups"][j]
            og = outs[j][b]["groups"]
            assert gg == og
            got += gpu_x.lines(gg)
            for grp in og:
                want += ref_x.update(*grp)
                if (grp[4] >> 6) == 0:
                    n_pi.add(grp[0])
    assert got == want
    # and the reference's own XDRServer (oracle/_ref, built in the build
    # container and shipped as a library) over the HIP groups
    if oracle.xdr_ref_available():
        hip_groups = [grp for j in (0, 1, 0) for b in range(NBLK) for grp in g[b]["groups"][j]]
        assert oracle.ref_xdr_session(hip_groups) == got
    # ~5 groups per station in 36 blocks (11.4 groups/s), three passes
    assert len(n_pi) == 2 and sum(1 for ln in got if ln.startswith("P")) >= 4
    assert sum(1 for ln in got if ln.startswith("R")) >= 10
