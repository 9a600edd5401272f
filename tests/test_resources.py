"""Register and LDS budgets of the built kernels (CPU: reads the gfx950 code
object's metadata out of fmtuner-sdr_amd/libfmx.so).

The pipelined step relies on co-residency: two k_fe8
workgroups per CU (one wave of each per SIMD) must leave a SIMD room for a
k_pll or k_rds wave, so k_fe8 stays within 168 VGPRs (2 x 168 + 176 = 512)
and k_pll within 88 (two of its waves beside the two front-end waves), with
no scratch spills.  A compiler-side change of a few lines once moved k_fe8
from 162 to 189 VGPRs (an s_setprio branch at kernel entry), which silently
cost the pipelined step 3 %: this test makes such a change fail loudly."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "fmtuner-sdr_amd", "libfmx.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _kernels(tmp_path):
    if not os.path.exists(LIB):
        pytest.skip("libfmx.so not built")
    if not shutil.which("objcopy") or not os.path.exists(os.path.join(LLVM, "clang-offload-bundler")):
        pytest.skip("objcopy / clang-offload-bundler not available")
    fat = str(tmp_path / "fatbin.bin")
    co = str(tmp_path / "k.co")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", LIB, fat], check=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--input=" + fat, "--output=" + co,
                    "--unbundle"], check=True)
    notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                           capture_output=True, text=True).stdout
    out = {}
    for blk in re.split(r"\n\s+- \.", notes):
        m = re.search(r"\.name:\s+(\S+)", blk)
        if not m:
            continue
        f = {}
        for key in ("vgpr_count", "agpr_count", "vgpr_spill_count", "sgpr_spill_count",
                    "group_segment_fixed_size", "private_segment_fixed_size"):
            mm = re.search(r"\." + key + r":\s+(\d+)", blk)
            if mm:
                f[key] = int(mm.group(1))
        out[m.group(1)] = f
    return out


def _find(ks, pat):
    hits = {k: v for k, v in ks.items() if re.search(pat, k)}
    assert hits, (pat, sorted(ks))
    return hits


def test_front_end_register_budget(tmp_path):
    ks = _kernels(tmp_path)
    for name, f in _find(ks, r"k_fe8ILi10ELi28").items():
        regs = f.get("vgpr_count", 0) + f.get("agpr_count", 0)
        # process_block's instance (RS = false, "Lb0"): 3 waves per SIMD; the
        # RS = true instance (stage calls, RDS steps past k_rs): 2
        assert regs <= (168 if "Lb0" in name else 256), (name, f)
        assert f.get("vgpr_spill_count", 0) == 0 and f.get("private_segment_fixed_size", 0) == 0, (name, f)


def test_pll_register_and_lds_budget(tmp_path):
    ks = _kernels(tmp_path)
    hits = _find(ks, r"k_pllILi(16|24)EEEvNS_7PllArgs")
    # two workgroup shapes (16 or 24 channels x 16-sample tiles, fmx_pll.inc)
    assert len(hits) == 2, sorted(hits)
    for name, f in hits.items():
        assert f.get("vgpr_count", 0) + f.get("agpr_count", 0) <= 80, (name, f)
        # LDS: the tile rings take 31.2 KB at 16 channels, 46.8 KB at 24: one
        # k_pll workgroup beside two k_fe8 (43.3 KB each in process_block's
        # instance) and a k_rs (16.5 KB) in 160 KB
        lds = 32 * 1024 if "ILi16E" in name else 47 * 1024
        assert f.get("group_segment_fixed_size", 0) <= lds, (name, f)
        assert f.get("vgpr_spill_count", 0) == 0 and f.get("private_segment_fixed_size", 0) == 0, (name, f)


def test_pilot_kernel_budget(tmp_path):
    """k_pilot (the pilot BPF after k_fe8, round 4): 18.1 KB of f16 images and
    (round 6) the 4.5 KB tap window.  It runs on the front end's stream, so it
    never shares a CU with k_fe8; beside the other streams' workgroups -- one
    24-channel k_pll (46.8 KB), k_audio (28.3 KB), k_rs (16.5 KB), k_rds
    (11.1 KB) -- two k_pilot workgroups fit in 160 KB; four accumulator
    chains without spills."""
    ks = _kernels(tmp_path)
    hits = _find(ks, r"7k_pilotENS_9PilotArgs")
    assert len(hits) == 1
    for name, f in hits.items():
        assert f.get("group_segment_fixed_size", 0) <= 24 * 1024, (name, f)
        assert 2 * f.get("group_segment_fixed_size", 0) + 47 * 1024 + 28944 + 16896 + 11392 <= 160 * 1024, (name, f)
        assert f.get("vgpr_count", 0) + f.get("agpr_count", 0) <= 64, (name, f)
        assert f.get("vgpr_spill_count", 0) == 0 and f.get("private_segment_fixed_size", 0) == 0, (name, f)


def test_rds_fits_beside_two_front_ends(tmp_path):
    ks = _kernels(tmp_path)
    for name, f in _find(ks, r"5k_rdsILb0E").items():
        assert f.get("vgpr_count", 0) + f.get("agpr_count", 0) <= 512 - 2 * 168, (name, f)
        assert f.get("vgpr_spill_count", 0) == 0, (name, f)


def test_rs_fits_beside_two_front_ends_and_pll(tmp_path):
    """k_rs shares a CU with two k_fe8 (53.7 KB each) and one k_pll (31.2 KB)
    workgroup: LDS <= 16 KB (dynamic since round 4: the launcher passes
    sizeof(RsLds)), and its wave fits a SIMD's registers beside two
    front-end waves and a k_pll wave (80)."""
    ks = _kernels(tmp_path)
    hits = _find(ks, r"4k_rsENS_6RsArgs")
    assert len(hits) == 1
    for name, f in hits.items():
        assert f.get("group_segment_fixed_size", 0) <= 16 * 1024, (name, f)
        assert f.get("vgpr_count", 0) + f.get("agpr_count", 0) <= 512 - 2 * 168 - 80, (name, f)
        assert f.get("vgpr_spill_count", 0) == 0 and f.get("private_segment_fixed_size", 0) == 0, (name, f)
