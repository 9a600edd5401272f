"""ASan + UBSan on the CPU build (the reference runs no
sanitizers).  tests/cpp/sanitize_main.cpp is built
from source with -fsanitize=address,undefined -fno-sanitize-recover=all
together with the CPU oracle (oracle/fmx_oracle.cpp), the product's host-side
design code (fmtuner-sdr_amd/csrc/fmx_design.cpp) and host formats
(fmx_host.cpp), and run on:
  * every design the product builds (4 rate configs x 5 W0 x 4 W) and the
    resampler timing simulation;
  * the XDR / scan / WAV / PCM / IQ-capture host formats;
  * the oracle regression fixture (tests/golden/oracle_regress.json): the
    sanitized oracle must reproduce it exactly as the normal build does;
  * the oracle's per-object entry points and its RDS block sync on the
    golden bit strings (tests/golden/blocksync.json);
  * the standalone C++ unit tests of tests/cpp (math, SWAR, division by a
    constant, PLL sine, atan2, NCO constrain) at reduced sweep sizes.
Any sanitizer report aborts the binary (non-zero exit) and fails the test.
The facade (fmx_blocks.cpp) calls the HIP library, so it runs on the GPU
(tests/test_facades.py), not here."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _run(cmd, timeout=600):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=ENV)
    assert r.returncode == 0, (cmd, r.returncode, r.stderr[-4000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    return r.stdout


@pytest.fixture(scope="module")
def san_exe(tmp_path_factory):
    d = tmp_path_factory.mktemp("san")
    exe = str(d / "sanitize_main")
    src = [os.path.join(ROOT, "tests", "cpp", "sanitize_main.cpp"),
           os.path.join(ROOT, "oracle", "fmx_oracle.cpp"),
           os.path.join(ROOT, "fmtuner-sdr_amd", "csrc", "fmx_design.cpp"),
           os.path.join(ROOT, "fmtuner-sdr_amd", "csrc", "fmx_host.cpp")]
    inc = ["-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "oracle"),
           "-I" + os.path.join(ROOT, "fmtuner-sdr_amd", "csrc")]
    _run(["g++", "-std=c++17", "-ffp-contract=off", *SAN, *inc, "-o", exe, *src, "-lpthread"], timeout=900)
    return exe, d


def test_design_and_schedules_sanitized(san_exe):
    exe, _ = san_exe
    r = json.loads(_run([exe, "design"]))
    assert r["designs"] == 4 * 5 * 4 and r["schedule_outputs"] > 0 and np.isfinite(r["tap_sum"])


def test_host_formats_sanitized(san_exe):
    exe, d = san_exe
    r = json.loads(_run([exe, "host", str(d)]))
    assert r["xdr_bytes"] > 0 and r["xdr_small"] < 0 and r["scan_bytes"] > 0
    assert r["wav"] == 44 and r["capture_rc"] == 10000 and r["replay"] == 10000 and r["replay_equal"]


def test_oracle_regression_fixture_sanitized(fmx, san_exe):
    """The sanitized oracle reproduces tests/golden/oracle_regress.json (the
    same fixture test_oracle_pinning.py checks against the normal build)."""
    exe, d = san_exe
    with open(os.path.join(ROOT, "tests", "golden", "oracle_regress.json")) as f:
        reg = json.load(f)
    for tag, kind, stereo in (("stereo_rds", 2, 1), ("mono", 0, 0)):
        B, M, nblk = 4096, 10, 12
        scfg = fmx.make_synth(kind=kind, n_bits=6000)
        bits, _ = fmx.synth_rds_bits(scfg, 3, 1)
        iq = fmx.synth_host(scfg, 3, 1, 0, B * M * nblk, bits)
        assert hashlib.sha256(iq.tobytes()).hexdigest() == reg[tag]["iq_sha256"]
        path = d / f"iq_{tag}.u8"
        iq[0].tofile(path)
        out = json.loads(_run([exe, "oracle", str(path), str(nblk), str(stereo)]))
        assert len(out) == len(reg[tag]["blocks"])
        for o, want in zip(out, reg[tag]["blocks"]):
            assert o["stereo"] == want["stereo"] and o["pilot"] == want["pilot"]
            assert o["n_pcm"] == want["n_pcm"]
            assert o["groups"] == want["groups"]
            np.testing.assert_allclose(o["pcm_l_head"], want["pcm_l_head"], rtol=0, atol=1e-6)
            np.testing.assert_allclose(o["mpx_head"], want["mpx_head"], rtol=0, atol=1e-6)


def test_oracle_stages_and_blocksync_sanitized(fmx, san_exe):
    exe, d = san_exe
    scfg = fmx.make_synth(kind=2, n_bits=4096)
    bits, _ = fmx.synth_rds_bits(scfg, 0, 1)
    iq = fmx.synth_host(scfg, 0, 1, 0, 40960, bits)
    path = d / "iq_stage.u8"
    iq[0].tofile(path)
    r = json.loads(_run([exe, "stages", str(path)]))
    assert r["decim"] == 4096 and r["demod"] > 500 and r["stereo"] > 500 and r["afpost"] > 500
    with open(os.path.join(ROOT, "tests", "golden", "blocksync.json")) as f:
        gold = json.load(f)
    streams = gold["streams"] if isinstance(gold, dict) and "streams" in gold else gold
    n = 0
    for s in (streams.values() if isinstance(streams, dict) else streams):
        b = s["bits"] if isinstance(s, dict) else s
        if isinstance(b, str):
            arr = np.frombuffer(b.encode(), dtype=np.uint8) - ord("0")
        else:
            arr = np.asarray(b, dtype=np.uint8)
        p = d / f"bits_{n}.u8"
        arr.astype(np.uint8).tofile(p)
        got = json.loads(_run([exe, "blocksync", str(p)]))
        if isinstance(s, dict) and "groups" in s:
            want = json.loads(s["groups"]) if isinstance(s["groups"], str) else s["groups"]
            assert got["groups"] == len(want), (s.get("name"), got, len(want))
        n += 1
    assert n > 0


@pytest.mark.parametrize("name,args,extra", [
    ("divconst_test", ["4099"], ["-fopenmp"]),
    ("atan2_test", ["20000"], ["-fopenmp"]),
    ("ncoconstrain_test", ["4099"], ["-fopenmp"]),
])
def test_cpp_unit_tests_sanitized(tmp_path, name, args, extra):
    exe = str(tmp_path / name)
    _run(["g++", "-std=c++17", "-ffp-contract=off", *SAN, *extra, "-o", exe,
          os.path.join(ROOT, "tests", "cpp", name + ".cpp")], timeout=600)
    json.loads(_run([exe, *args], timeout=900))
