"""GPU parity: the HIP path (libfmx.so through its C ABI) against the oracle
on identical seeded IQ.  Contract (BASELINE.json north_star): RDS groups
bit-exact, PCM within 1e-4 RMS; stereo flag, XDR indicator, pilot level and
sample counts exact.  The numeric bars below sit 7-15x above the achieved
errors, which every comparison logs.

The XDR pilot level (stereo_decoder.cpp pilotLevelTenthsKHz, 0.1 kHz steps)
is exact wherever the pilot PLL is locked.  With a narrow IQ filter
(W0 / XDR bandwidth < 100 kHz) the 19 kHz pilot is attenuated, the PLL free-
runs, and the level becomes chaotic: the oracle against ITSELF moves by up to
13 tenths (4 channels x 12 blocks) when 1e-5 of noise is added to the MPX
(tests/test_oracle_pinning.py::test_unlocked_pilot_level_is_chaotic), and
the GPU (MPX within ~1e-6 RMS of the oracle) by up to 18 tenths, so those
blocks hold the level to PILOT_UNLOCKED_TOL instead; their stereo flag,
indicator, MPX and PCM keep the full bars.  Every test here runs on the GPU.
"""
import json
import os
import sys

import numpy as np
import pytest

import gpu_harness as H

pytestmark = pytest.mark.gpu

# Bars: the north_star's 1e-4 PCM RMS is the contract; the bars below are
# 7-15x the worst achieved values (every achieved error is logged to
# gpurun_out/parity_errors.jsonl; round 6, profiles/r06e_parity_errors.jsonl,
# 175 comparisons, summary in DESIGN.md section 3), so drift shows long
# before the contract is at risk.
PCM_RMS_TOL = 1e-5     # achieved <= 1.38e-6 (median 3.1e-7; round 5: 3.62e-6)
PCM_MAX_TOL = 2e-4     # achieved <= 1.9e-5
MPX_MAX_TOL = 3e-4     # achieved <= 1.0e-4 with the pilot inside the IQ filter (carrier at -40 dBFS)
MPX_RMS_TOL = 1e-5     # achieved <= 2.7e-6
# W0 / bandwidth < 100 kHz: the discriminator's atan2 sees a narrow-filtered
# (under noise: near-zero) IQ vector, where 1e-7 relative IQ differences move
# single MPX samples by up to 6e-4 (achieved, W0 = 9 kHz + AWGN) while the
# PCM stays within 3e-8 RMS
MPX_MAX_TOL_NARROW = 6e-3


def make_iq(fmx, kind, C, nblk, iq_rate=2_400_000, M=10, B=4096, noise=0.0, ch0=0, n=None):
    n = n or B
    scfg = fmx.make_synth(iq_rate=iq_rate, kind=kind, noise_std=noise, n_bits=8192)
    bits, groups = fmx.synth_rds_bits(scfg, ch0, C)
    iq = fmx.synth_host(scfg, ch0, C, 0, n * M * nblk, bits)
    return iq, groups


PILOT_UNLOCKED_TOL = 30   # tenths of kHz, free-running PLL only (see module doc)


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PARITY_LOG = os.environ.get("FMX_PARITY_LOG", os.path.join(ROOT, "gpurun_out", "parity_errors.jsonl"))


def log_errors(tag, c, st):
    """Achieved GPU-vs-oracle errors of every compared channel, one JSON line
    each (printed, and appended to FMX_PARITY_LOG / gpurun_out/)."""
    rec = {"test": tag, "channel": int(c)}
    rec.update({k: (float(v) if isinstance(v, float) else v) for k, v in st.items() if not k.startswith("groups")})
    rec["groups"] = len(st["groups_oracle"])
    line = json.dumps(rec)
    print("PARITY " + line)
    try:
        os.makedirs(os.path.dirname(PARITY_LOG), exist_ok=True)
        with open(PARITY_LOG, "a") as f:
            f.write(line + "\n")
    except OSError:
        pass


def check(g, o, c, nblk, tag="", pilot_tol=0, pcm_blocks=None, gc=None, narrow=False):
    """gc: channel index into the GPU result arrays (default c)."""
    st = H.compare(g, o, c if gc is None else gc, nblk, pcm_blocks=pcm_blocks)
    log_errors(tag, c, st)
    info = (tag, c, {k: v for k, v in st.items() if not k.startswith("groups")})
    assert st["count_mismatch"] == 0, info
    assert st["stereo_mismatch"] == 0, info
    assert st["indicator_mismatch"] == 0, info
    assert st["mpx_max"] < (MPX_MAX_TOL_NARROW if narrow else MPX_MAX_TOL), info
    assert st["mpx_rms"] < MPX_RMS_TOL, info
    assert st["pcm_rms"] < PCM_RMS_TOL, info
    assert st["pcm_max"] < PCM_MAX_TOL, info
    assert st["groups_gpu"] == st["groups_oracle"], (tag, c, st["groups_gpu"], st["groups_oracle"])
    assert st["pilot_maxdiff"] <= pilot_tol, info
    return st


def run_both(fmx, oracle, torch, cfgkw, iq, nblk, n=None, resets=None, params=None, per_channel_resets=None,
             ktimes=None):
    C = iq.shape[0]
    g = H.run_gpu_pipeline(fmx, torch, fmx.make_config(**cfgkw), iq, nblk, n=n, resets=resets, params=params,
                           ktimes=ktimes)
    outs = []
    for c in range(C):
        rs = None
        if resets:
            rs = {b: ch for b, ch in resets.items() if ch in (-1, c)}
        op = None
        if params:
            op = {b: [(k, v) for (k, v, ch) in lst if ch in (-1, c)] for b, lst in params.items()}
        outs.append(H.run_oracle_pipeline(oracle, oracle.make_cfg(**cfgkw), iq[c], nblk, n=n, resets=rs, params=op))
    return g, outs


def test_stereo_rds_parity_2m4(fmx, oracle, torch_cuda):
    """Cfg2/3 channel: 2.4 MS/s stereo FM + RDS, M=10 -> 240 kHz, 50 us."""
    C, nblk = 8, 40
    iq, _ = make_iq(fmx, 2, C, nblk)
    g, outs = run_both(fmx, oracle, torch_cuda, {}, iq, nblk)
    ngroups = 0
    for c in range(C):
        st = check(g, outs[c], c, nblk, "2m4")
        ngroups += len(st["groups_oracle"])
    assert ngroups >= 3 * C


def test_reference_native_rate_2m048(fmx, oracle, torch_cuda):
    """The reference's own configuration: 2.048 MS/s, M=8 -> 256 kHz."""
    C, nblk = 4, 30
    kw = dict(iq_rate=2_048_000, dsp_rate=256_000)
    iq, _ = make_iq(fmx, 2, C, nblk, iq_rate=2_048_000, M=8)
    g, outs = run_both(fmx, oracle, torch_cuda, kw, iq, nblk)
    for c in range(C):
        check(g, outs[c], c, nblk, "2m048")


def test_decimation_factor_4(fmx, oracle, torch_cuda):
    C, nblk = 2, 12
    kw = dict(iq_rate=1_024_000, dsp_rate=256_000)
    iq, _ = make_iq(fmx, 2, C, nblk, iq_rate=1_024_000, M=4)
    g, outs = run_both(fmx, oracle, torch_cuda, kw, iq, nblk)
    for c in range(C):
        check(g, outs[c], c, nblk, "m4")


def test_decimation_factor_2(fmx, oracle, torch_cuda):
    """M=2 (512 kS/s -> 256 kHz): the k_fe8<2, 12> instantiation."""
    C, nblk = 2, 12
    kw = dict(iq_rate=512_000, dsp_rate=256_000)
    iq, _ = make_iq(fmx, 2, C, nblk, iq_rate=512_000, M=2)
    g, outs = run_both(fmx, oracle, torch_cuda, kw, iq, nblk)
    for c in range(C):
        check(g, outs[c], c, nblk, "m2")


@pytest.mark.parametrize("B", [2048, 8192])
def test_block_sizes_front_end_chunks(fmx, oracle, torch_cuda, B):
    """Handle blocks of one and of four 2048-sample front-end chunks (the
    chunk loop of k_fe8: DMA split, halo and RDS-copy carries)."""
    C, nblk = 4, 10 if B == 2048 else 6
    kw = dict(block=B)
    iq, _ = make_iq(fmx, 2, C, nblk, B=B)
    g, outs = run_both(fmx, oracle, torch_cuda, kw, iq, nblk)
    for c in range(C):
        check(g, outs[c], c, nblk, f"B{B}")


def test_partial_lane_groups_65_channels(fmx, oracle, torch_cuda):
    """65 channels: k_pll / k_rds run one full 64-lane workgroup and one with
    a single live lane (rows past C read 0 through the buffer range check)."""
    C, nblk = 65, 6
    iq, _ = make_iq(fmx, 2, C, nblk)
    g, outs = run_both(fmx, oracle, torch_cuda, {}, iq, nblk)
    for c in (0, 1, 31, 63, 64):
        check(g, outs[c], c, nblk, "c65")


def test_iq_capture_replay_through_pipeline(fmx, oracle, torch_cuda, tmp_path):
    """writeIqCapture (main.cpp:742-747) block by block, then the capture
    replayed (fmx_iq_replay) as the input of the GPU pipeline and the oracle:
    the replayed bytes equal the captured ones and the outputs match."""
    C, nblk, B, M = 2, 12, 4096, 10
    iq, _ = make_iq(fmx, 2, C, nblk)
    blk = 2 * B * M
    replayed = np.zeros_like(iq)
    for c in range(C):
        path = str(tmp_path / f"ch{c}.iq")
        for b in range(nblk):
            fmx.iq_capture(path, iq[c, b * blk:(b + 1) * blk], append=b > 0)
        for b in range(nblk):
            replayed[c, b * blk:(b + 1) * blk] = fmx.iq_replay(path, b * B * M, B * M)
    assert np.array_equal(replayed, iq)
    g, outs = run_both(fmx, oracle, torch_cuda, {}, replayed, nblk)
    for c in range(C):
        check(g, outs[c], c, nblk, "replay")


def test_direct_u8_no_decimation(fmx, oracle, torch_cuda):
    """iq_rate == dsp_rate: FMDemod::processSplit on bytes (fm_demod.cpp:219-249)."""
    C, nblk = 2, 10
    kw = dict(iq_rate=256_000, dsp_rate=256_000)
    iq, _ = make_iq(fmx, 2, C, nblk, iq_rate=256_000, M=1)
    g, outs = run_both(fmx, oracle, torch_cuda, kw, iq, nblk)
    for c in range(C):
        check(g, outs[c], c, nblk, "m1")


def test_mono_config1(fmx, oracle, torch_cuda):
    """Config 1: mono FM (1 kHz + 3 kHz, no pilot), stereo=false path."""
    C, nblk = 2, 16
    kw = dict(stereo=0, rds=0)
    iq, _ = make_iq(fmx, 0, C, nblk)
    g, outs = run_both(fmx, oracle, torch_cuda, kw, iq, nblk)
    for c in range(C):
        check(g, outs[c], c, nblk, "mono")
        assert np.array_equal(g[-1]["pcm_l"][c], g[-1]["pcm_r"][c])


def test_weak_signal_agc_fast_soft_blend(fmx, oracle, torch_cuda):
    """Config 5 subset: AWGN, dsp_agc=fast, stereo_blend=soft."""
    C, nblk = 4, 24
    kw = dict(dsp_agc=1, blend=0)
    iq, _ = make_iq(fmx, 2, C, nblk, noise=0.25)
    g, outs = run_both(fmx, oracle, torch_cuda, kw, iq, nblk)
    for c in range(C):
        check(g, outs[c], c, nblk, "weak")


@pytest.mark.parametrize("w0", [309_000, 114_000, 42_000, 9_000])
def test_w0_bandwidth_sweep(fmx, oracle, torch_cuda, w0):
    C, nblk = 2, 10
    kw = dict(w0_bandwidth_hz=w0)
    iq, _ = make_iq(fmx, 2, C, nblk, ch0=20)
    g, outs = run_both(fmx, oracle, torch_cuda, kw, iq, nblk)
    for c in range(C):
        check(g, outs[c], c, nblk, f"w0={w0}", pilot_tol=0 if w0 >= 100_000 else PILOT_UNLOCKED_TOL,
              narrow=w0 < 100_000)


@pytest.mark.parametrize("bw", [114_000, 63_000])
def test_resets_and_runtime_setters(fmx, oracle, torch_cuda, bw):
    """Runtime::reset of one channel / all channels, XDR bandwidth change
    (re-created IQ FIR), de-emphasis change, force mono, AGC switch.
    At 63 kHz the pilot PLL free-runs while the blend is still open (stereo was
    acquired at the wide setting): the oracle's own L/R then moves by 1e-2 RMS
    under 1e-5 of MPX noise, so PCM and pilot level are compared outside the
    narrow-bandwidth blocks 10..15 (MPX, flags, counts, RDS everywhere)."""
    C, nblk = 3, 30
    iq, _ = make_iq(fmx, 2, C, nblk, ch0=40)
    resets = {8: 1, 16: -1}
    params = {10: [("bandwidth_hz", bw, -1)], 12: [("deemphasis", 1, -1)],
              14: [("force_mono", 1, 2)], 18: [("force_mono", 0, 2), ("bandwidth_hz", 0, -1)],
              20: [("dsp_agc", 2, 0), ("blend", 2, -1)], 24: [("deemphasis", 2, 1)]}
    g, outs = run_both(fmx, oracle, torch_cuda, {}, iq, nblk, resets=resets, params=params)
    for c in range(C):
        narrow = bw < 100_000
        blocks = [b for b in range(nblk) if not (10 <= b < 16)] if narrow else None
        check(g, outs[c], c, nblk, f"setters bw={bw}", pcm_blocks=blocks,
              pilot_tol=PILOT_UNLOCKED_TOL if narrow else 0, narrow=narrow)


def test_rds_after_staggered_resets(fmx, oracle, torch_cuda):
    """Channels 3, 17 and 18 of 20 reset at different blocks (Runtime::reset,
    main.cpp:686-691).  The reset clears their RDS decoders (NCO, symsync,
    block sync) but not the 240k -> 171k resampler's timing
    (SubcarrierSet::reset leaves it alone, subcarrier.cpp:108), so all
    channels keep one RDS schedule and k_rs's MFMA tiles (16 channels on one
    schedule) keep running for both workgroups; every channel against the
    oracle, RDS groups bit-exact.  (Audio resampler timing does split per
    channel: k_audio reads each channel's group.)"""
    C, nblk = 20, 20
    iq, _ = make_iq(fmx, 2, C, nblk, ch0=200)
    resets = {5: 3, 8: 17, 11: 18}
    g, outs = run_both(fmx, oracle, torch_cuda, {}, iq, nblk, resets=resets)
    ngroups = 0
    for c in range(C):
        ngroups += len(check(g, outs[c], c, nblk, "rds_staggered_resets")["groups_oracle"])
    assert ngroups >= C


def test_custom_deemphasis_and_deviation(fmx, oracle, torch_cuda):
    """setDeemphasis(tau_us) with any tau on both FMDemod and AFPostProcessor
    (fm_demod.cpp:50-62, af_post_processor.cpp:31-45: alpha = dt / (tau + dt),
    IIR re-created) and FMDemod::setDeviation (fm_demod.cpp:64-71: kf =
    deviation / Fs, discriminator re-created), mid-stream and per channel."""
    C, nblk = 3, 24
    iq, _ = make_iq(fmx, 2, C, nblk, ch0=120)
    params = {0: [("deemph_us", 60, -1)], 6: [("deviation_hz", 70000, 1)],
              10: [("deemph_us", 0, 0), ("deemph_us", 100, 2)], 16: [("deviation_hz", 75000, 1)]}
    g, outs = run_both(fmx, oracle, torch_cuda, {}, iq, nblk, params=params)
    for c in range(C):
        check(g, outs[c], c, nblk, "tau/deviation")


@pytest.mark.parametrize("n", [1500, 333])
def test_ragged_call_sizes(fmx, oracle, torch_cuda, n):
    """Calls of n < dsp_block samples that do not divide the kernel chunks."""
    C, nblk = 3, 60 if n == 1500 else 40
    iq, _ = make_iq(fmx, 2, C, nblk, n=n, ch0=60)
    g, outs = run_both(fmx, oracle, torch_cuda, {}, iq, nblk, n=n)
    for c in range(C):
        check(g, outs[c], c, nblk, f"n={n}")


def test_stage_entry_points(fmx, oracle, torch_cuda):
    """fmx_decimate / fmx_demod / fmx_stereo / fmx_afpost / fmx_rds against the
    individual oracle objects (ComplexDecimator, FMDemod, StereoDecoder,
    AFPostProcessor, RDSDecoder)."""
    import ctypes as Ct
    torch = torch_cuda
    L = oracle.lib()
    C, B, M, nblk = 2, 4096, 10, 14
    iq, _ = make_iq(fmx, 2, C, nblk, ch0=80)
    cfg = fmx.make_config(bandwidth_hz=-1, deemphasis=1)  # objects as constructed (75 us, ctor IQ filter)
    h = fmx.Handle(cfg, C)
    dev = torch.device("cuda")
    d_iq = torch.from_numpy(iq).to(dev)
    bb = torch.zeros((C, 2 * B), dtype=torch.float32, device=dev)
    mpx = torch.zeros((C, B), dtype=torch.float32, device=dev)
    mono = torch.zeros((C, B), dtype=torch.float32, device=dev)
    cnt = torch.zeros(C, dtype=torch.int32, device=dev)
    lf = torch.zeros((C, B), dtype=torch.float32, device=dev)
    rf = torch.zeros((C, B), dtype=torch.float32, device=dev)
    st = torch.zeros(C, dtype=torch.int32, device=dev)
    pil = torch.zeros(C, dtype=torch.int32, device=dev)
    ol = torch.zeros((C, B), dtype=torch.float32, device=dev)
    orr = torch.zeros((C, B), dtype=torch.float32, device=dev)
    acnt = torch.zeros(C, dtype=torch.int32, device=dev)
    grp = torch.zeros((C, 8, 4), dtype=torch.int32, device=dev)
    gcnt = torch.zeros(C, dtype=torch.int32, device=dev)
    od = [L.oracle_decim_create(M, 28, 80.0) for _ in range(C)]
    odm = [L.oracle_demod_create(240_000, 32_000) for _ in range(C)]
    ost = [L.oracle_stereo_create(240_000, 32_000) for _ in range(C)]
    oaf = [L.oracle_afpost_create(240_000, 32_000) for _ in range(C)]
    ords = [L.oracle_rds_create(240_000) for _ in range(C)]
    groups_g = [[] for _ in range(C)]
    groups_o = [[] for _ in range(C)]
    for b in range(nblk):
        h.decimate(d_iq.data_ptr() + b * 2 * B * M, iq.shape[1], B, bb.data_ptr(), 2 * B)
        h.demod(bb.data_ptr(), 2 * B, B, mpx.data_ptr(), B, mono.data_ptr(), B, cnt.data_ptr())
        h.stereo(mpx.data_ptr(), B, B, lf.data_ptr(), rf.data_ptr(), B, st.data_ptr(), pil.data_ptr())
        h.afpost(lf.data_ptr(), rf.data_ptr(), B, B, ol.data_ptr(), orr.data_ptr(), B, B, acnt.data_ptr())
        h.rds(mpx.data_ptr(), B, B, grp.data_ptr(), 8, gcnt.data_ptr())
        h.sync()
        G = {k: v.cpu().numpy() for k, v in dict(bb=bb, mpx=mpx, mono=mono, cnt=cnt, lf=lf, rf=rf, st=st, pil=pil,
                                                  ol=ol, orr=orr, acnt=acnt, gcnt=gcnt).items()}
        graw = grp.cpu().numpy().view(np.uint8).reshape(C, 8, 16)
        for c in range(C):
            x = np.ascontiguousarray(iq[c, b * 2 * B * M:(b + 1) * 2 * B * M])
            obb = np.zeros(2 * B, np.float32)
            L.oracle_decim_execute_complex(od[c], x.ctypes.data, B * M, obb.ctypes.data, B)
            assert np.max(np.abs(obb - G["bb"][c])) < 1e-5
            om = np.zeros(B, np.float32)
            omono = np.zeros(B, np.float32)
            k = L.oracle_demod_process_split_complex(odm[c], G["bb"][c].ctypes.data, om.ctypes.data,
                                                     omono.ctypes.data, B)
            assert k == G["cnt"][c]
            assert np.max(np.abs(om - G["mpx"][c])) < MPX_MAX_TOL
            assert np.sqrt(np.mean((omono[:k] - G["mono"][c][:k]) ** 2)) < PCM_RMS_TOL
            ol_, or_ = np.zeros(B, np.float32), np.zeros(B, np.float32)
            s_, p_ = Ct.c_int(), Ct.c_int()
            mpx_c = np.ascontiguousarray(G["mpx"][c])
            L.oracle_stereo_process(ost[c], mpx_c.ctypes.data, ol_.ctypes.data, or_.ctypes.data, B,
                                    Ct.byref(s_), Ct.byref(p_))
            assert s_.value == G["st"][c] and p_.value == G["pil"][c]
            assert np.sqrt(np.mean((ol_ - G["lf"][c]) ** 2)) < PCM_RMS_TOL
            assert np.sqrt(np.mean((or_ - G["rf"][c]) ** 2)) < PCM_RMS_TOL
            al, ar = np.zeros(B, np.float32), np.zeros(B, np.float32)
            lfc, rfc = np.ascontiguousarray(G["lf"][c]), np.ascontiguousarray(G["rf"][c])
            k = L.oracle_afpost_process(oaf[c], lfc.ctypes.data, rfc.ctypes.data, B, al.ctypes.data,
                                        ar.ctypes.data, B)
            assert k == G["acnt"][c]
            assert np.max(np.abs(al[:k] - G["ol"][c][:k])) < 1e-5
            gg = (oracle.OracleGroup * 16)()
            ng = L.oracle_rds_process(ords[c], mpx_c.ctypes.data, B, gg, 16, None, 0, None)
            groups_o[c] += oracle.groups_to_tuples(gg, ng)
            for q in range(int(G["gcnt"][c])):
                w = graw[c, q]
                a, bb_, cc, d = np.frombuffer(w[:8].tobytes(), dtype=np.uint16)
                groups_g[c].append((int(a), int(bb_), int(cc), int(d), int(w[8])))
    for c in range(C):
        assert groups_g[c] == groups_o[c]
    assert sum(len(x) for x in groups_o) >= 2
    h.close()


def _oracle_rows(oracle, cfgs, iq_keep, nblk, retunes=None, params=None):
    n = len(cfgs)
    return [H.run_oracle_pipeline(oracle, cfgs[j], iq_keep[j], nblk, retunes=(retunes or [None] * n)[j],
                                  params=(params or [None] * n)[j])
            for j in range(n)]


def test_cfg3_full_size_sampled_channels(fmx, oracle, torch_cuda):
    """Cfg3 at its real size: 4096 channels of stereo FM + RDS in one handle;
    channels 0, 1, 63, 64 (first two k_pll / k_rds workgroups), 2047 and
    4095 (last row of the last workgroup, largest C x stride offsets)
    compared with the oracle for MPX, PCM, stereo flag, indicator, pilot and
    RDS groups."""
    C, nblk = 4096, 36
    keep = [0, 1, 63, 64, 2047, 4095]
    cfg = fmx.make_config()
    scfg = fmx.make_synth(kind=2, n_bits=8192)
    g, iq_keep, _ = H.run_gpu_sampled(fmx, torch_cuda, cfg, C, scfg, nblk, keep)
    outs = _oracle_rows(oracle, [oracle.make_cfg()] * len(keep), iq_keep, nblk)
    ngroups = 0
    for j, c in enumerate(keep):
        st = check(g, outs[j], c, nblk, "cfg3_full", gc=j)
        ngroups += len(st["groups_oracle"])
    assert ngroups >= 2 * len(keep)
    assert g[-1]["stereo_all"] > 0.99


CFG5_W0 = [309_000, 194_000, 114_000, 42_000, 9_000]


def test_cfg5_weak_signal_w0_sweep_1024(fmx, oracle, torch_cuda):
    """Cfg5 at its real size: 1024 channels of noisy IQ (AWGN sigma 0.1 per
    component on amplitude 0.8: CNR ~15 dB), dsp_agc=fast, stereo_blend=soft,
    and a W0 sweep across the channels (channel c: W0 = CFG5_W0[c % 5] via
    setW0BandwidthHz + setBandwidthHz(0)).  Sampled channels cover every W0,
    both ends of the handle and a workgroup boundary."""
    C, nblk = 1024, 30
    keep = [0, 1, 2, 3, 4, 63, 64, 515, 1021, 1022, 1023]
    cfg = fmx.make_config(dsp_agc=1, blend=0)
    setup = []
    for c in range(C):
        setup.append(("w0_hz", CFG5_W0[c % 5], c))
    setup.append(("bandwidth_hz", 0, -1))
    scfg = fmx.make_synth(kind=2, noise_std=0.1, n_bits=8192)
    g, iq_keep, _ = H.run_gpu_sampled(fmx, torch_cuda, cfg, C, scfg, nblk, keep, setup=setup)
    # the same runtime sequence on the oracle: setW0BandwidthHz, then
    # setBandwidthHz(0) before the first block (so W0 = 309k re-designs the
    # filter from its table entry instead of keeping the ctor filter)
    cfgs = [oracle.make_cfg(dsp_agc=1, blend=0)] * len(keep)
    params = [{0: [("w0_hz", CFG5_W0[c % 5]), ("bandwidth_hz", 0)]} for c in keep]
    outs = _oracle_rows(oracle, cfgs, iq_keep, nblk, params=params)
    for j, c in enumerate(keep):
        w0 = CFG5_W0[c % 5]
        check(g, outs[j], c, nblk, f"cfg5_w0={w0}", gc=j, pilot_tol=0 if w0 >= 100_000 else PILOT_UNLOCKED_TOL,
              narrow=w0 < 100_000)


def test_cfg2_stereo_without_rds_256(fmx, oracle, torch_cuda):
    """Cfg2: 256 channels of stereo FM without an RDS subcarrier (kind=1);
    the RDS decoder still runs (as the reference always does) and must emit
    exactly what the oracle emits (nothing decodable)."""
    C, nblk = 256, 24
    keep = [0, 1, 63, 64, 127, 255]
    cfg = fmx.make_config()
    scfg = fmx.make_synth(kind=1, n_bits=8192)
    g, iq_keep, _ = H.run_gpu_sampled(fmx, torch_cuda, cfg, C, scfg, nblk, keep)
    outs = _oracle_rows(oracle, [oracle.make_cfg()] * len(keep), iq_keep, nblk)
    for j, c in enumerate(keep):
        st = check(g, outs[j], c, nblk, "cfg2", gc=j)
        assert all(e[4] != 0 for e in st["groups_oracle"])


def test_retune_fade_mute(fmx, oracle, torch_cuda):
    """a12: the retune path (main.cpp:1028-1042) -- reset fan-out plus the
    40 ms fade-out / mute / fade-in of the clamped PCM (main.cpp:1310-1337),
    including a retune while a mute is still running, a short custom mute
    and a cancelled one."""
    C, nblk = 4, 20
    keep = [0, 1, 2, 3]
    cfg = fmx.make_config()
    scfg = fmx.make_synth(kind=2, n_bits=8192)
    retunes = {8: (1, -1), 9: (1, -1), 12: (-1, 300), 15: (2, 2000), 16: (2, 0)}
    g, iq_keep, _ = H.run_gpu_sampled(fmx, torch_cuda, cfg, C, scfg, nblk, keep, retunes=retunes)
    orets = []
    for c in keep:
        orets.append({b: m for b, (ch, m) in retunes.items() if ch in (-1, c)})
    outs = _oracle_rows(oracle, [oracle.make_cfg()] * len(keep), iq_keep, nblk, retunes=orets)
    for j, c in enumerate(keep):
        check(g, outs[j], c, nblk, "retune", gc=j)
    # the mute really happened: block 10 of channel 1 is silent (muted region
    # 1280 samples from block 9), the fade-in at the end is not
    assert np.all(outs[1][10]["pcm_l"] == 0.0)
    assert np.array_equal(g[10]["pcm_l"][1][:len(outs[1][10]["pcm_l"])], outs[1][10]["pcm_l"])


def test_stereo_indicator_force_mono(fmx, oracle, torch_cuda):
    """a12: XDR stereo indicator = isStereo() || (forceMono && stereo &&
    pilot >= 20) (main.cpp:1298-1300).  With force mono from the start the
    pilot level passes 2.0 kHz before (and while) detection runs, so the
    indicator is 1 on blocks where isStereo() is 0."""
    C, nblk = 2, 16
    iq, _ = make_iq(fmx, 2, C, nblk, ch0=100)
    g, outs = run_both(fmx, oracle, torch_cuda, dict(force_mono=1), iq, nblk)
    for c in range(C):
        check(g, outs[c], c, nblk, "indicator")
    assert any(o["indicator"] == 1 and o["stereo"] == 0 for o in outs[0])


def test_full_size_properties(fmx, torch_cuda):
    """Bench size (4096 channels): no NaN, exact sample counts, stereo on
    every channel after acquisition, and every error-free RDS group equals
    the transmitted group sequence (ground truth, size-independent)."""
    torch = torch_cuda
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_oracle_pinning import groups_align
    C, B, M, nblk = 4096, 4096, 10, 40
    cfg = fmx.make_config()
    h = fmx.Handle(cfg, C)
    dev = torch.device("cuda")
    n_iq = B * M
    scfg = fmx.make_synth(kind=2, n_bits=int((nblk * n_iq + 4_800_000) * 1187.5 / 2.4e6) + 208)
    bits, tx = fmx.synth_rds_bits(scfg, 0, C)
    d_bits = torch.from_numpy(bits).to(dev)
    row = 2 * n_iq * nblk
    d_iq = torch.empty((C, row), dtype=torch.uint8, device=dev)
    h.synth_device(scfg, 0, C, 0, n_iq * nblk, d_bits.data_ptr(), d_iq.data_ptr(), row)
    pl = torch.zeros((C, B), dtype=torch.float32, device=dev)
    pr = torch.zeros((C, B), dtype=torch.float32, device=dev)
    cnt = torch.zeros(C, dtype=torch.int32, device=dev)
    st = torch.zeros(C, dtype=torch.int32, device=dev)
    grp = torch.zeros((C, 8, 4), dtype=torch.int32, device=dev)
    gcnt = torch.zeros(C, dtype=torch.int32, device=dev)
    out = fmx.BlockOut(None, 0, pl.data_ptr(), pr.data_ptr(), B, cnt.data_ptr(), st.data_ptr(), None, None,
                       grp.data_ptr(), 8, gcnt.data_ptr())
    got = [[] for _ in range(C)]
    total = 0
    for b in range(nblk):
        h.process_block(d_iq.data_ptr() + b * 2 * n_iq, row, B, out)
        h.sync()
        c_ = cnt.cpu().numpy()
        assert set(np.unique(c_)) <= {546, 547}
        assert torch.isfinite(pl).all() and torch.isfinite(pr).all()
        gc = gcnt.cpu().numpy()
        graw = grp.cpu().numpy().view(np.uint8).reshape(C, 8, 16)
        for c in np.nonzero(gc)[0]:
            for q in range(int(gc[c])):
                w = graw[c, q]
                a, bb_, cc, d = np.frombuffer(w[:8].tobytes(), dtype=np.uint16)
                got[c].append((int(a), int(bb_), int(cc), int(d), int(w[8])))
                total += 1
    assert st.float().mean().item() > 0.99
    assert total > 3 * C
    # some channels need > 40 blocks to acquire (oracle identical, see
    # DESIGN.md); every channel that produced an error-free group must align
    bad = [c for c in range(C) if any(g[4] == 0 for g in got[c]) and not groups_align(got[c], tx[c])]
    assert not bad, bad[:10]
    assert sum(1 for c in range(C) if any(g[4] == 0 for g in got[c])) > 0.99 * C
    h.close()


def test_graft_smoke(torch_cuda):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import __graft_entry__
    __graft_entry__.smoke()


def test_rds_resampler_inside_the_front_end_with_k_pilot(fmx, oracle, torch_cuda):
    """The process_block combination the Cfg runs never take: an
    RDS resampling step past k_rs's 64-sample tile window (rds_del > 2.1, here
    a 384 kHz DSP rate: 2.25) keeps the resampler inside k_fe8 (its RS=true
    instance) while the pilot BPF still runs as k_pilot -- k_fe8 then writes
    no pilot and the stereo history rows k_pilot starts from.  MPX, pilot
    level, PCM and RDS groups against the oracle at the full bars."""
    C, nblk = 4, 10
    iq, _ = make_iq(fmx, 2, C, nblk, iq_rate=3_072_000, M=8)
    kw = dict(iq_rate=3_072_000, dsp_rate=384_000)
    kt = {}
    g, outs = run_both(fmx, oracle, torch_cuda, kw, iq, nblk, ktimes=kt)
    assert kt["rs"][1] == 0, kt          # no k_rs launch: the resampler ran inside k_fe8
    assert kt["pilot"][1] >= nblk - 1, kt  # the pilot BPF as k_pilot (every block on k_fe8)
    for c in range(C):
        check(g, outs[c], c, nblk, tag="fe8_rs_with_k_pilot")
