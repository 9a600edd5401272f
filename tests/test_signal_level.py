"""RF signal level: computeSignalLevel / smoothSignalLevel
(src/signal_level.cpp:145-214) fused into the GPU front end.

CPU part: the oracle restatement against the reference's own compiled
signal_level.cpp (oracle/_ref), and the reference's own unit-test cases
(tests/test_signal_level.cpp:5-53) replayed on both.  GPU part: the
fmx_block_out.d_signal output of fmx_process_block against the reference."""
import numpy as np
import pytest

import oracle as O


def _cases():
    rng = np.random.default_rng(3)
    yield "random", rng.integers(0, 256, 2 * 4096, dtype=np.uint8)
    yield "quiet", np.clip(127.5 + rng.normal(0, 2, 2 * 3000), 0, 255).astype(np.uint8)
    yield "clipped", np.clip(127.5 + rng.normal(0, 140, 2 * 5000), 0, 255).astype(np.uint8)
    yield "silent", np.full(256, 127, np.uint8)
    yield "zeros", np.zeros(256, np.uint8)


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built")
@pytest.mark.parametrize("name,iq", list(_cases()))
@pytest.mark.parametrize("params", [(0, 0.5, -4.0, -55.0, -19.0), (20, 0.5, 3.0, -80.0, -12.0), (0, 0.5, 0.0, -20.0, -40.0)])
def test_oracle_signal_level_matches_reference(name, iq, params):
    a = O.signal_level(iq, *params)
    b = O.ref_signal_level(iq, *params)
    for k in a:
        assert a[k] == pytest.approx(b[k], rel=0, abs=1e-12), (name, k, a[k], b[k])


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built")
def test_reference_unit_cases_on_both():
    """tests/test_signal_level.cpp:5-53 of the reference."""
    for f in (O.signal_level, O.ref_signal_level):
        assert f(np.zeros(0, np.uint8), 0, 0.5, 0.0, -80.0, -12.0)["dbfs"] == -120.0
        r = f(np.full(256, 127, np.uint8), 0, 0.5, 0.0, -80.0, -12.0)
        assert r["dbfs"] < -60.0 and r["level120"] == 0.0
        assert f(np.zeros(256, np.uint8), 0, 0.5, 0.0, -80.0, -12.0)["hard_clip_ratio"] > 0.0
    sm = O.SignalSmoother()
    assert sm(50.0) == 50.0
    v = sm(60.0)
    assert 50.0 < v < 60.0
    import ctypes as C
    R = O.ref()
    ini, val = C.c_int(0), C.c_float(0.0)
    sm2 = O.SignalSmoother()
    for x in [50.0, 60.0, 10.0, 10.0, 119.0, 0.0]:
        assert R.ref_smooth_signal_level(x, C.byref(ini), C.byref(val)) == sm2(x)


def _run_gpu(fmx, torch, cfg, iq, nblk, n, params=None):
    C_ = iq.shape[0]
    M = cfg.iq_rate // cfg.dsp_rate
    h = fmx.Handle(cfg, C_)
    if params:
        h.set_signal_params(*params)
    dev = torch.device("cuda")
    d_iq = torch.from_numpy(np.ascontiguousarray(iq)).to(dev)
    B = cfg.block
    pl = torch.zeros((C_, B), dtype=torch.float32, device=dev)
    pr = torch.zeros((C_, B), dtype=torch.float32, device=dev)
    cnt = torch.zeros(C_, dtype=torch.int32, device=dev)
    sig = torch.zeros((C_, 40), dtype=torch.uint8, device=dev)
    out = fmx.BlockOut(None, 0, pl.data_ptr(), pr.data_ptr(), B, cnt.data_ptr(), None, None, None, None, 0, None,
                       sig.data_ptr())
    res = []
    for b in range(nblk):
        h.process_block(d_iq.data_ptr() + b * 2 * n * M, iq.shape[1], n, out)
        h.sync()
        raw = sig.cpu().numpy()
        res.append([fmx.SignalLevel.from_buffer_copy(raw[c].tobytes()) for c in range(C_)])
    h.close()
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("iq_rate,n,noise", [(2_400_000, 4096, 0.0), (2_400_000, 1500, 0.3), (256_000, 4096, 0.1),
                                             (2_400_000, 4096, 0.3), (2_048_000, 4096, 0.2), (2_400_000, 3000, 0.25)])
def test_gpu_signal_level(fmx, oracle, torch_cuda, iq_rate, n, noise):
    """k_fe8 (whole and ragged chunks; its decimator-fused byte sums with the
    near-clip counts in full waves and in the halo / partial waves' exact
    path, at M = 10 and 8) and the M = 1 direct path; reference
    signal_level.cpp as the checker."""
    C_, nblk = 3, 6
    M = iq_rate // (240_000 if iq_rate % 240_000 == 0 else 256_000)
    dsp = iq_rate // M
    scfg = fmx.make_synth(iq_rate=iq_rate, kind=2, noise_std=noise, n_bits=4096, amplitude=0.8)
    bits, _ = fmx.synth_rds_bits(scfg, 0, C_)
    iq = fmx.synth_host(scfg, 0, C_, 0, n * M * nblk, bits)
    cfg = fmx.make_config(iq_rate=iq_rate, dsp_rate=dsp)
    params = (12, 0.5, -2.0, -60.0, -15.0)
    g = _run_gpu(fmx, torch_cuda, cfg, iq, nblk, n, params)
    checker = O.ref_signal_level if O.ref_available() else O.signal_level
    for c in range(C_):
        sm = O.SignalSmoother()
        for b in range(nblk):
            seg = iq[c, b * 2 * n * M:(b + 1) * 2 * n * M]
            r = checker(seg, *params)
            got = g[b][c]
            assert abs(got.dbfs - r["dbfs"]) < 1e-9, (c, b, got.dbfs, r["dbfs"])
            assert abs(got.compensated_dbfs - r["compensated_dbfs"]) < 1e-9
            assert abs(got.level120 - r["level120"]) <= 1e-4
            assert got.hard_clip_ratio == r["hard_clip_ratio"] and got.near_clip_ratio == r["near_clip_ratio"]
            assert abs(got.level120_smoothed - sm(r["level120"])) <= 1e-4


@pytest.mark.gpu
def test_gpu_scan_line_three_reads(fmx, oracle, torch_cuda):
    """SURVEY 8f row 2, the multi-channel scan (main.cpp:1064-1121): every
    channel is one scan point; three process_block reads give three
    level120 values per point (computeSignalLevel of each read), averaged in
    double and formatted by fmx_xdr_scan_line.  The expected line applies the
    reference's signal_level.cpp (oracle/_ref) to the same IQ reads."""
    C_, nblk, n = 16, 3, 4096
    # a spread of signal strengths and noise over the points
    rows = []
    for c in range(C_):
        scfg = fmx.make_synth(kind=2, noise_std=0.02 * (c % 4), amplitude=0.05 + 0.06 * c, n_bits=4096)
        bits, _ = fmx.synth_rds_bits(scfg, c, 1)
        rows.append(fmx.synth_host(scfg, c, 1, 0, n * 10 * nblk, bits)[0])
    iq = np.stack(rows)
    cfg = fmx.make_config()
    params = (20, 0.5, -2.0, -60.0, -15.0)
    g = _run_gpu(fmx, torch_cuda, cfg, iq, nblk, n, params)
    freqs = [87500 + 100 * c for c in range(C_)]
    gpu_sum = [sum(float(g[b][c].level120) for b in range(nblk)) for c in range(C_)]
    checker = O.ref_signal_level if O.ref_available() else O.signal_level
    ref_sum = [sum(float(np.float32(checker(iq[c, b * 2 * n * 10:(b + 1) * 2 * n * 10], *params)["level120"]))
                   for b in range(nblk)) for c in range(C_)]
    line = fmx.xdr_scan_line(freqs, gpu_sum, [nblk] * C_)
    want = "U" + ",".join("%d=%.1f" % (f, float(np.float32(s / nblk))) for f, s in zip(freqs, ref_sum))
    print(line)
    print(want)
    assert line.startswith("U") and len(line[1:].split(",")) == C_
    for pg, pw, sg, sw in zip(line[1:].split(","), want[1:].split(","), gpu_sum, ref_sum):
        fg, vg = pg.split("=")
        fw, vw = pw.split("=")
        # per-read levels agree to 1e-4 (test_gpu_signal_level); the one-decimal
        # text can differ by one display step only at a rounding boundary
        assert fg == fw and abs(sg - sw) <= 3e-4 and abs(float(vg) - float(vw)) <= 0.1 + 1e-9, (pg, pw, sg, sw)
    assert len(set(v.split("=")[1] for v in line[1:].split(","))) > C_ // 2  # a spread of levels
