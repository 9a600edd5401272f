"""Host-side consumers of the GPU outputs (fmx_host.cpp):
XDR RDS lines with the server's PI debounce, the XDR scan line, the WAV sink
(header, volume ramp, S16 conversion) and IQ capture/replay.

Each test restates the reference routine in plain Python (the checker) and
compares the C-ABI result byte for byte.  CPU only: no GPU calls."""
import os
import struct

import numpy as np
import pytest


# ---- Python restatements of the reference (checkers) ----------------------
from xdr_ref import PyXdr  # noqa: E402,F401


def py_volume_s16(left, right, vol_percent, cur):
    """AudioOutput::write ramp (audio_output.cpp:1432-1467) in float32 +
    writeWAVData (:1379-1398)."""
    f = np.float32
    target = f(f(min(max(vol_percent, 0), 100)) / f(100)) * f(0.85)
    ramp = f(32000) * f(0.01)
    cur = f(cur)
    step = f(f(target - cur) / max(f(1), ramp))
    out = []
    for i in range(len(left)):
        if abs(f(target - cur)) > f(1e-6):
            cur = f(cur + step)
            if (step > 0 and cur > target) or (step < 0 and cur < target):
                cur = target
        for x in (left[i], right[i]):
            s = f(f(x) * cur)
            s = max(f(-1), min(f(1), s))
            out.append(int(np.trunc(f(s * f(32767)))))
    return np.array(out, dtype=np.int16), float(cur)


# ---- tests -----------------------------------------------------------------
def _random_groups(rng, n, pis):
    groups = []
    for _ in range(n):
        a = int(rng.choice(pis))
        e = int(rng.integers(0, 256))
        # mostly clean blocks, as a locked decoder produces
        if rng.random() < 0.6:
            e &= 0x0F
        groups.append((a, int(rng.integers(0, 65536)), int(rng.integers(0, 65536)),
                       int(rng.integers(0, 65536)), e))
    return groups


def test_xdr_rds_lines_match_server(fmx):
    rng = np.random.default_rng(7)
    for trial in range(4):
        groups = _random_groups(rng, 300, [0x1234, 0xC0DE, 0x9ABC][: trial % 3 + 1])
        ref = PyXdr()
        x = fmx.XdrRds()
        # feed in ragged batches: the state must carry across calls
        k = 0
        for m in (1, 7, 0, 64, 100, 128):
            batch = groups[k:k + m]
            k += m
            want = [ln for g in batch for ln in ref.update(*g)]
            assert x.lines(batch) == want


def _xdr_fixture():
    import json
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "xdr_server.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("stream", ["clean", "bursts", "retunes"])
def test_xdr_rds_lines_match_reference_fixture(fmx, stream):
    """fmx_xdr_rds_lines against the lines the REFERENCE's XDRServer sent a
    loopback client for the same groups (tests/golden/xdr_server.json, made by
    tools/gen_golden.py from oracle/_ref): byte for byte, in ragged batches,
    and the Python restatement (the GPU tests' checker) agrees as well."""
    fx = {s["name"]: s for s in _xdr_fixture()["streams"]}[stream]
    groups = [tuple(g) for g in fx["groups"]]
    x = fmx.XdrRds()
    got, k = [], 0
    for m in (1, 5, 0, 64, 111, 333, 1000):
        got += x.lines(groups[k:k + m])
        k += m
    assert k >= len(groups)
    assert got == fx["lines"]
    ref = PyXdr()
    assert [ln for g in groups for ln in ref.update(*g)] == fx["lines"]


def test_xdr_scan_line_framing_matches_reference_fixture(fmx):
    """XDRServer::pushScanLine's framing ("U" + the line) as the reference
    server sent it (fixture), against fmx_xdr_scan_line."""
    sc = _xdr_fixture()["scan"]
    for line, sent in zip(sc["lines"], sc["sent"]):
        pts = [p.split("=") for p in line.split(",")]
        freqs = [int(f) for f, _ in pts]
        sums = [float(v) for _, v in pts]
        assert fmx.xdr_scan_line(freqs, sums, [1] * len(pts)) == sent


def test_xdr_rds_lines_match_reference_live(fmx, oracle):
    """The same against the reference server compiled here (oracle/_ref),
    on fresh seeded streams: random error masks, missing A / B blocks, PI
    changes, and a long run past the server's 64-entry PI history."""
    if not oracle.xdr_ref_available():
        pytest.skip("oracle/_ref/libfmx_xdrref.so not built (no /root/reference here)")
    rng = np.random.default_rng(99)
    for trial in range(3):
        groups = _random_groups(rng, 700, [0x1234, 0xC0DE, 0x9ABC, 0x0001][: trial + 2])
        x = fmx.XdrRds()
        assert x.lines(groups) == oracle.ref_xdr_session(groups)


def test_xdr_pi_state_restatement_matches_reference(oracle):
    """evaluatePiState (xdr_server.cpp:189-213, the reference's own code in
    oracle/_ref) against the tests' restatement, on random histories."""
    if not oracle.xdr_ref_available():
        pytest.skip("oracle/_ref/libfmx_xdrref.so not built (no /root/reference here)")
    rng = np.random.default_rng(5)
    for _ in range(3000):
        x = PyXdr()
        x.fill = int(rng.integers(0, 65))
        vals = rng.choice([0x1111, 0x2222, 0x3333], size=64)
        x.buf = [int(v) for v in vals]
        x.err = [int(v) for v in rng.integers(0, 256, size=8)]
        v = int(rng.choice([0x1111, 0x2222, 0x3333, 0x4444]))
        assert x.state(v) == oracle.ref_xdr_pi_state(np.array(x.buf), np.array(x.err), x.fill, v)


def test_xdr_pi_debounce_known_answers(fmx):
    x = fmx.XdrRds()
    # first clean PI: one correct copy -> UNLIKELY, no P line; R line emitted
    assert x.lines([(0x1234, 1, 2, 3, 0x00)]) == ["R00010002000300"]
    # second clean copy -> CORRECT -> P line
    assert x.lines([(0x1234, 1, 2, 3, 0x00)]) == ["P1234", "R00010002000300"]
    # block A with error level 2 still printed with '??' once debounced
    assert x.lines([(0x1234, 1, 2, 3, 0x80)]) == ["P1234??", "R00010002000380"]
    # block A missing (err 3): no P line; block B error: no R line
    assert x.lines([(0x1234, 1, 2, 3, 0xD0)]) == []
    # a fresh PI needs its own confirmations
    assert x.lines([(0xBEEF, 4, 5, 6, 0x0C)]) == ["R0004000500060C"]


def test_xdr_rds_lines_small_buffer_keeps_state(fmx):
    import ctypes as C
    x = fmx.XdrRds()
    arr = (fmx.RdsGroup * 2)(fmx.RdsGroup(0x1234, 1, 2, 3, 0, 0, 0), fmx.RdsGroup(0x1234, 1, 2, 3, 0, 0, 0))
    buf = C.create_string_buffer(8)
    rc = fmx.lib().fmx_xdr_rds_lines(C.byref(x.st), C.cast(arr, C.c_void_p), 2, buf, 8)
    assert rc < 0 and -rc == len("R00010002000300\nP1234\nR00010002000300\n") + 1
    assert x.st.fill == 0 and x.st.pos == 63
    assert x.lines([(0x1234, 1, 2, 3, 0)] * 2) == ["R00010002000300", "P1234", "R00010002000300"]


def test_xdr_scan_line(fmx):
    freqs = [87500, 87600, 87700, 87800]
    sums = [3 * 41.26, 0.0, 2 * 10.04, 3 * 99.95]
    reads = [3, 0, 2, 3]
    want = []
    for f, s, r in zip(freqs, sums, reads):
        if r > 0:
            want.append("%d=%.1f" % (f, float(np.float32(s / r))))
    assert fmx.xdr_scan_line(freqs, sums, reads) == "U" + ",".join(want)
    assert fmx.xdr_scan_line([87500], [0.0], [0]) == ""
    assert fmx.xdr_scan_line([], [], []) == ""


def test_wav_header(fmx):
    h = fmx.wav_header(128000)
    want = (b"RIFF" + struct.pack("<I", 36 + 128000) + b"WAVE" + b"fmt " +
            struct.pack("<IHHIIHH", 16, 1, 2, 32000, 32000 * 4, 4, 16) + b"data" + struct.pack("<I", 128000))
    assert h == want and len(h) == 44


@pytest.mark.parametrize("vol,start", [(100, 0.85), (40, 0.85), (100, 0.0), (0, 0.85), (73, 0.5)])
def test_pcm_volume_ramp_s16(fmx, vol, start):
    rng = np.random.default_rng(vol)
    n = 700  # longer than the 320-sample ramp
    left = rng.uniform(-1.6, 1.6, n).astype(np.float32)
    right = rng.uniform(-1.6, 1.6, n).astype(np.float32)
    want, want_vs = py_volume_s16(left, right, vol, start)
    # two calls carrying the ramp state must equal one call
    a, vs = fmx.pcm_to_s16(left[:333], right[:333], vol, start)
    b, vs = fmx.pcm_to_s16(left[333:], right[333:], vol, vs)
    got = np.concatenate([a, b])
    want_a, vs_a = py_volume_s16(left[:333], right[:333], vol, start)
    want_b, vs_b = py_volume_s16(left[333:], right[333:], vol, vs_a)
    assert np.array_equal(got, np.concatenate([want_a, want_b]))
    assert vs == pytest.approx(vs_b, abs=0)
    if start == 0.85 and vol == 100:
        assert np.array_equal(got, want)


def test_iq_capture_replay_roundtrip(fmx, tmp_path):
    rng = np.random.default_rng(3)
    path = str(tmp_path / "cap.iq")
    blocks = [rng.integers(0, 256, 2 * n, dtype=np.uint8) for n in (1000, 0, 4096, 17)]
    fmx.iq_capture(path, blocks[0], append=False)
    for b in blocks[1:]:
        fmx.iq_capture(path, b, append=True)
    whole = np.concatenate(blocks)
    assert os.path.getsize(path) == whole.size
    assert np.array_equal(fmx.iq_replay(path, 0, whole.size // 2), whole)
    assert np.array_equal(fmx.iq_replay(path, 1000, 4096), whole[2000:2000 + 8192])
    # reading past the end returns the whole pairs that exist
    tail = fmx.iq_replay(path, 5100, 100)
    assert np.array_equal(tail, whole[10200:])
    # truncate on a fresh capture
    fmx.iq_capture(path, blocks[3], append=False)
    assert os.path.getsize(path) == blocks[3].size
