"""The C++ facades of include/fmx_blocks.hpp (drop-in classes with the
reference's method signatures) against the oracle's reference objects:
tests/cpp/facade_test.cpp, built here and run on the GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_facades_match_oracle():
    subprocess.run(["make", "-C", os.path.join(ROOT, "fmtuner-sdr_amd"), "facade_test"], check=True,
                   capture_output=True)
    exe = os.path.join(ROOT, "fmtuner-sdr_amd", "build", "facade_test")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0 and "FACADES OK" in r.stdout, r.stdout + r.stderr


def test_facade_symbols_exported():
    """libfmx.so carries the C++ facade classes next to the C ABI."""
    lib = os.path.join(ROOT, "fmtuner-sdr_amd", "libfmx.so")
    out = subprocess.run(["nm", "-DC", lib], capture_output=True, text=True, check=True).stdout
    for sym in ("fmx::FMDemod::processSplitComplex", "fmx::StereoDecoder::processAudio",
                "fmx::AFPostProcessor::process", "fmx::RDSDecoder::process",
                "fmx::ComplexDecimator::executeComplex", "fmx::ComplexDecimator::execute",
                "fmx::FMDemod::process", "fmx::FMDemod::processComplex", "fmx::FMDemod::processNoDownsample",
                "fmx::FMDemod::setDeviation", "fmx::Receiver::processBlock"):
        assert sym in out, sym
