"""ISA audit of the SHIPPED code object (CPU: disassembles the gfx950 code
object inside fmtuner-sdr_amd/libfmx.so).

Round 2's nondeterministic RDS groups came from k_fe8's RDS resampler in
packed-FP32 form.  The failing build had a packed-FP32
VALU op (v_pk_*_f32) directly followed by an LDS / vector-memory load whose
destination VGPRs are that op's sources ("load return over the sources of a
just-issued packed op", 56 times in that k_fe8).  No gfx950 hazard rule the
compiler knows pads this, and the mechanism is unproven.  The pattern is kept
OUT of every kernel of the product path -- k_fe8 (every instance: the kernel
that failed), k_pll, k_rs, k_rds and k_audio -- zero tolerance: where the
vectoriser made packed pairs next to LDS loads (k_audio's 32 kHz resampler,
k_fe8's cross-wave DC-blocker carry) the arithmetic is scalar asm in the
reference's mul-then-add order.  Only the fallback front end k_frontend
(call shapes k_fe8 does not take) still carries it; its count is pinned so
that it cannot grow unnoticed, and every output of two full-size pipelined
runs is bit-identical run to run (tests/test_gpu_determinism.py).
(tools/asm_war_scan.py runs the same scan
over a `hipcc -S` listing.)"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "fmtuner-sdr_amd", "libfmx.so")
LLVM = "/opt/rocm/lib/llvm/bin"

LOADS = ("ds_read", "ds_load", "buffer_load", "global_load", "flat_load", "scratch_load", "ds_bpermute",
         "ds_swizzle")


def _vregs(op):
    op = op.strip()
    m = re.match(r"v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)\b", op)
    return {int(m.group(1))} if m else set()


def war_pairs(lines):
    """(kernel, packed op, next load) where the load's destination VGPRs are
    sources of the packed-FP32 op right before it."""
    fn, out = None, []
    prev = None
    for ln in lines:
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", ln)
        if m:
            fn, prev = m.group(1), None
            continue
        t = ln.split("//")[0].strip()
        if not t or t.startswith(";") or t.endswith(":"):
            continue
        mnem = t.split()[0]
        if prev is not None and mnem.startswith(LOADS):
            ops = t.split(None, 1)[1].split(",") if " " in t else []
            if ops and (_vregs(ops[0]) & prev[1]):
                out.append((fn, prev[0], t))
        if mnem.startswith("v_pk_") and mnem.endswith("_f32"):
            ops = [o.strip() for o in t.split(None, 1)[1].split(",")]
            src = set().union(*[_vregs(o) for o in ops[1:4]])
            prev = (t, src)
        else:
            prev = None
    return out


def _disasm(tmp_path):
    if not os.path.exists(LIB):
        pytest.skip("libfmx.so not built")
    if not shutil.which("objcopy") or not os.path.exists(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("objcopy / llvm-objdump not available")
    fat, co = str(tmp_path / "fat.bin"), str(tmp_path / "k.co")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", LIB, fat], check=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--input=" + fat, "--output=" + co,
                    "--unbundle"], check=True)
    return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co], check=True,
                          capture_output=True, text=True).stdout.split("\n")


def test_scanner_finds_the_pattern():
    """The scanner itself, on a listing with one such pair and two near misses."""
    lst = ["0000000000001000 <_ZN3fmx1kE>:",
           "\tv_pk_add_f32 v[12:13], v[4:5], v[6:7]",
           "\tds_read2_b64 v[4:7], v1 offset1:1",      # overwrites the sources: a hit
           "\tv_pk_mul_f32 v[2:3], v[8:9], s[0:1]",
           "\tds_read_b64 v[10:11], v1",                # disjoint: no hit
           "\tv_pk_fma_f32 v[2:3], v[8:9], v[14:15], v[2:3]",
           "\tv_add_f32_e32 v0, v1, v2",
           "\tglobal_load_dwordx2 v[8:9], v[0:1], off"]  # not right after: no hit
    hits = war_pairs(lst)
    assert len(hits) == 1 and hits[0][2].startswith("ds_read2_b64")


# kernels that may still carry the pattern, with the count of the round-4
# build as the ceiling (per instantiation)
TRACKED = {r"10k_frontendILi": 25}


def test_shipped_kernels_have_no_load_over_packed_fp32_sources(tmp_path):
    lines = _disasm(tmp_path)
    kernels = [ln for ln in lines if re.match(r"^[0-9a-f]+ <_Z", ln)]
    assert len(kernels) >= 10, kernels
    assert any("5k_fe8" in k for k in kernels) and any("4k_rs" in k for k in kernels)
    per = {}
    for fn, a, b in war_pairs(lines):
        per.setdefault(fn, []).append((a, b))
    for fn, v in per.items():
        cap = next((n for pat, n in TRACKED.items() if re.search(pat, fn)), 0)
        assert len(v) <= cap, (fn, len(v), v[0])
