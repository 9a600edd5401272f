"""C-ABI boundary: libfmx.so loads and exports every function declared in
include/fmx.h; calls that need a GPU fail cleanly without one; the oracle
library exports its header too.  No compute calls on the GPU here."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions(path):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b((?:fmx|oracle)_[a-z0-9_]+)\s*\(", src)))


def test_fmx_exports_every_header_symbol(fmx):
    lib = ctypes.CDLL(fmx.LIB_PATH)
    names = header_functions(os.path.join(ROOT, "include", "fmx.h"))
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_oracle_exports_every_header_symbol(oracle):
    lib = ctypes.CDLL(oracle.ORACLE_LIB)
    names = header_functions(os.path.join(ROOT, "oracle", "fmx_oracle.h"))
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_create_without_gpu_fails_cleanly(fmx):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    assert fmx.lib().fmx_device_count() == 0
    with pytest.raises(fmx.FmxError):
        fmx.Handle(fmx.make_config(), 4)


def test_invalid_config_rejected_before_device(fmx):
    cfg = fmx.make_config(iq_rate=2_400_000, dsp_rate=250_000)  # not an integer ratio
    h = ctypes.c_void_p()
    rc = fmx.lib().fmx_create(ctypes.byref(cfg), 4, 0, ctypes.byref(h))
    assert rc != 0
    if h.value:
        fmx.lib().fmx_destroy(h)


def test_synth_host_deterministic_and_per_channel(fmx):
    scfg = fmx.make_synth(kind=2, n_bits=2000)
    bits, groups = fmx.synth_rds_bits(scfg, 5, 3)
    a = fmx.synth_host(scfg, 5, 3, 1000, 5000, bits)
    b = fmx.synth_host(scfg, 5, 3, 1000, 5000, bits, threads=1)
    assert np.array_equal(a, b)
    # channel 6 generated alone equals row 1 of the batch
    bits6, _ = fmx.synth_rds_bits(scfg, 6, 1)
    c = fmx.synth_host(scfg, 6, 1, 1000, 5000, bits6)
    assert np.array_equal(a[1], c[0])
    # continuity: a window starting later equals the tail of a longer run
    d = fmx.synth_host(scfg, 5, 1, 3000, 3000, bits[:1])
    assert np.array_equal(a[0, 2 * 2000:], d[0])
    assert groups.shape == (3, 2000 // 104, 4)
    assert (groups[:, :, 0] == (0x1000 + np.arange(5, 8))[:, None]).all()  # PI = 0x1000 + ch


def test_kernel_timer_ids_match_header_and_bench(fmx):
    """fmx_kernel_times ids (FMX_K_* in include/fmx.h) against fmx.py's
    KERNEL_NAMES order, and bench.py's per-kernel tables (design bytes per IQ
    sample, kernel names) cover every timer: a timer added to the ABI without
    them would break the bench line or mislabel a kernel."""
    src = open(os.path.join(ROOT, "include", "fmx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    ids = {m.group(1): int(m.group(2)) for m in re.finditer(r"FMX_K_([A-Z_]+)\s*=\s*(\d+)", src)}
    count = ids.pop("COUNT")
    assert count == len(ids) == len(fmx.KERNEL_NAMES)
    assert sorted(ids.values()) == list(range(count))
    for name, k in ids.items():
        assert fmx.KERNEL_NAMES[k] == name.lower(), (name, k)
        assert getattr(fmx, "K_" + name) == k
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert set(bench.PER_IQ) == set(fmx.KERNEL_NAMES) == set(bench.KNAME)
