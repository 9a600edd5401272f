"""GPU determinism: the same synthetic IQ through two fresh handles gives
bit-identical outputs (MPX, PCM, counts, stereo flag, pilot level, RDS groups),
pipelined as bench.py runs it, at the Cfg3 channel count where two k_fe8
workgroups share a CU beside the serial kernels.  A difference is a race or a
hardware hazard: the packed-FP32 RDS resampler gave wrong upper-half lanes
next to MFMA waves; the libm atan2f in the discriminator
did the same for lanes 48-63 (fmx_math.h fmx_atan2f)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

C, NBLK, B, M = 4096, 6, 4096, 10


def _run(fmx, torch, cfg, scfg, d_bits, d_iq, row):
    dev = torch.device("cuda")
    h = fmx.Handle(cfg, C)
    h.synth_device(scfg, 0, C, 0, B * M * NBLK, d_bits.data_ptr(), d_iq.data_ptr(), row)
    mpx = torch.zeros((NBLK, C, B), dtype=torch.float32, device=dev)
    pl = torch.zeros((NBLK, C, B), dtype=torch.float32, device=dev)
    pr = torch.zeros((NBLK, C, B), dtype=torch.float32, device=dev)
    ints = torch.zeros((4, NBLK, C), dtype=torch.int32, device=dev)  # count, stereo, pilot, group count
    grp = torch.zeros((NBLK, C, 8, 4), dtype=torch.int32, device=dev)
    for b in range(NBLK):
        out = fmx.BlockOut(mpx[b].data_ptr(), B, pl[b].data_ptr(), pr[b].data_ptr(), B, ints[0, b].data_ptr(),
                           ints[1, b].data_ptr(), ints[2, b].data_ptr(), None, grp[b].data_ptr(), 8,
                           ints[3, b].data_ptr())
        h.process_block(d_iq.data_ptr() + b * 2 * B * M, row, B, out)
    h.sync()
    torch.cuda.synchronize()
    res = {"mpx": mpx.cpu().numpy(), "pcm_l": pl.cpu().numpy(), "pcm_r": pr.cpu().numpy(),
           "ints": ints.cpu().numpy(), "groups": grp.cpu().numpy()}
    h.close()
    return res


def test_cfg3_outputs_bit_identical_across_runs(fmx, torch_cuda):
    torch = torch_cuda
    cfg = fmx.make_config()
    scfg = fmx.make_synth(kind=2, n_bits=8192)
    bits, _ = fmx.synth_rds_bits(scfg, 0, C)
    dev = torch.device("cuda")
    d_bits = torch.from_numpy(bits).to(dev)
    row = 2 * B * M * NBLK
    d_iq = torch.empty((C, row), dtype=torch.uint8, device=dev)
    a = _run(fmx, torch, cfg, scfg, d_bits, d_iq, row)
    b = _run(fmx, torch, cfg, scfg, d_bits, d_iq, row)
    diffs = {k: int(np.sum(a[k].view(np.uint32) != b[k].view(np.uint32))) for k in a}
    print("determinism:", diffs)
    assert all(v == 0 for v in diffs.values()), diffs
    # the run decoded something (the comparison is not vacuous)
    # (stereo detection needs 6 blocks of pilot presence: the level is checked instead)
    assert a["ints"][3].sum() > 300 and a["ints"][2][-1].mean() > 10, (a["ints"][3].sum(), a["ints"][2][-1].mean())
