"""Diagnostic: per-stage clocks of k_frontend and k_rds on the bench workload.
Needs the diagnostics library (make -C fmtuner-sdr_amd diag; FMX_LIB=...
libfmx_diag.so); runs with FMX_STAMPS=1 (set here).  Prints
the share of each stage in thread 0's timeline."""
import ctypes as C
import os
import sys

os.environ["FMX_STAMPS"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fmtuner-sdr_amd"))
import torch  # noqa: E402
import fmx  # noqa: E402

NAMES = ["decim", "dc", "iqfir+agc", "discrim", "pilot", "rds_rs", "state_out", "setup+carry+dma_wait"]
if os.environ.get("DECIM"):  # a library built with -DFMX_STAMPS_DECIM
    NAMES = ["dec_staging", "rf_sums", "dec_mfma", "dc+iqfir+disc", "pilot", "rds_rs", "state_out", "setup+carry+dma_wait"]
L = fmx.lib()
L.fmx_debug_stamps.restype = C.c_int
L.fmx_debug_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_int]
Cn, B, M, nblk = int(os.environ.get("C", "4096")), 4096, 10, int(os.environ.get("NBLK", "4"))
# channels per k_pll workgroup (launch_pll: 16 up to 2 048 channels on 256 CUs, else 24)
PLL_CH = int(os.environ.get("PLL_CH", "16" if int(os.environ.get("C", "4096")) <= 2048 else "24"))
h = fmx.Handle(fmx.make_config(), Cn)
dev = torch.device("cuda")
scfg = fmx.make_synth(kind=2, n_bits=6000)
bits, _ = fmx.synth_rds_bits(scfg, 0, Cn)
d_bits = torch.from_numpy(bits).to(dev)
NW = 2  # warm-up blocks: the first block runs k_frontend (cold decimator), not k_fe8
row = 2 * B * M * (nblk + NW)
d_iq = torch.empty((Cn, row), dtype=torch.uint8, device=dev)
h.synth_device(scfg, 0, Cn, 0, B * M * (nblk + NW), d_bits.data_ptr(), d_iq.data_ptr(), row)
h.sync()
# the bench's outputs (groups, flags, RF level records) so that every stage runs as timed
pl = torch.empty((Cn, B), device=dev)
pr = torch.empty((Cn, B), device=dev)
i32 = [torch.empty(Cn, dtype=torch.int32, device=dev) for _ in range(5)]
clip = torch.empty(Cn, device=dev)
grp = torch.empty((Cn, 8, 4), dtype=torch.int32, device=dev)
sig = torch.zeros((Cn, 10), device=dev)
out = fmx.BlockOut(None, 0, pl.data_ptr(), pr.data_ptr(), B, i32[0].data_ptr(), i32[1].data_ptr(), i32[2].data_ptr(),
                   clip.data_ptr(), grp.data_ptr(), 8, i32[3].data_ptr(),
                   None if os.environ.get("NO_SIG") else sig.data_ptr(), i32[4].data_ptr())


def read():
    v = (C.c_ulonglong * 48)()
    assert L.fmx_debug_stamps(h.h, v, 48) == 0
    return list(v)


for b in range(NW):
    h.process_block(d_iq.data_ptr() + b * 2 * B * M, row, B, out)
v0 = read()
for b in range(NW, NW + nblk):
    h.process_block(d_iq.data_ptr() + b * 2 * B * M, row, B, out)
v1 = read()
v = [a - b for a, b in zip(v1, v0)]
tot = sum(v[:8])
print(f"k_fe8 (thread 0 of each workgroup; {nblk} blocks after {NW} warm-up blocks)")
for k in range(8):
    print(f"  {NAMES[k]:10s} {v[k] / tot * 100:6.1f} %  {v[k] / (Cn * nblk):10.0f} ticks/launch-WG")
print(f"  (of which DMA wait + barrier: first chunk {v[40] / (Cn * nblk):8.0f}, later chunks {v[41] / (Cn * nblk):8.0f} ticks/launch-WG)")
print("  setup split (ticks/launch-WG): " + ", ".join(f"{nm} {v[42 + i] / (Cn * nblk):.0f}" for i, nm in enumerate(
    ["images+iq_hist", "carry words", "st_hist images", "agc+rds setup", "rs bank+dma issue", "to first wait"])))
RN = ["setup+store", "dma_wait+ld", "mix", "fir", "sum+agc", "symsync", "psk+nco", "decode"]
tot = sum(v[8:16]) or 1
nwg = (Cn + 7) // 8
print("k_rds (lane 0 of each workgroup of 8 channels; per decimation period = ticks / 121.6 at 4096 samples)")
for k in range(8):
    print(f"  {RN[k]:12s} {v[8 + k] / tot * 100:6.1f} %  {v[8 + k] / (nwg * nblk):10.0f} ticks/launch-WG"
          f"  {v[8 + k] / (nwg * nblk) / (B * 0.7125 / 24):8.1f} per period")
nwg = (Cn + PLL_CH - 1) // PLL_CH
print(f"k_pll per wave (lane 0): work / barrier-wait ticks per launch-WG ({PLL_CH} channels per workgroup)")
for w, nm in enumerate(["W0 chain", "WB blend", "P0", "P1", "P2", "P3", "P4", "P5"]):
    wk, wt, vm = v[16 + 2 * w], v[17 + 2 * w], v[32 + w]
    print(f"  {nm:14s} work {wk / (nwg * nblk):10.0f}  wait {wt / (nwg * nblk):10.0f}  (P waves: move wait {vm / (nwg * nblk):9.0f})")
