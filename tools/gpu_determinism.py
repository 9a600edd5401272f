"""Determinism check: the same synthetic IQ through two fresh handles must
give bit-identical MPX / pilot-derived outputs; any difference is a race.
Prints every differing (block, channel, sample) with the two values.
usage: python tools/gpu_determinism.py [C] [NBLK] [RUNS]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fmtuner-sdr_amd"))
import torch  # noqa: E402
import fmx  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
NBLK = int(sys.argv[2]) if len(sys.argv) > 2 else 8
RUNS = int(sys.argv[3]) if len(sys.argv) > 3 else 3
B, M = 4096, 10
dev = torch.device("cuda")
ST = int(os.environ.get("STEREO", "1"))
RDS = int(os.environ.get("RDS", "1"))
cfg = fmx.make_config(iq_rate=2_400_000, dsp_rate=240_000, out_rate=32_000, block=B, w0_bandwidth_hz=194_000,
                      bandwidth_hz=0, dsp_agc=0, stereo=ST, blend=1, deemphasis=0, rds=RDS)
scfg = fmx.make_synth(iq_rate=2_400_000, kind=2, n_bits=8192)
bits, _ = fmx.synth_rds_bits(scfg, 0, C)
d_bits = torch.from_numpy(bits).to(dev)
row = 2 * B * M * NBLK
d_iq = torch.empty((C, row), dtype=torch.uint8, device=dev)


def run(pipelined):
    h = fmx.Handle(cfg, C)
    h.synth_device(scfg, 0, C, 0, B * M * NBLK, d_bits.data_ptr(), d_iq.data_ptr(), row)
    mpx = torch.zeros((NBLK, C, B), dtype=torch.float32, device=dev)
    pl = torch.zeros((NBLK, C, B), dtype=torch.float32, device=dev)
    pr = torch.zeros((NBLK, C, B), dtype=torch.float32, device=dev)
    cnt = torch.zeros((NBLK, C), dtype=torch.int32, device=dev)
    st = torch.zeros((NBLK, C), dtype=torch.int32, device=dev)
    pil = torch.zeros((NBLK, C), dtype=torch.int32, device=dev)
    grp = torch.zeros((NBLK, C, 8, 4), dtype=torch.int32, device=dev)
    gc = torch.zeros((NBLK, C), dtype=torch.int32, device=dev)
    for b in range(NBLK):
        out = fmx.BlockOut(mpx[b].data_ptr(), B, pl[b].data_ptr(), pr[b].data_ptr(), B, cnt[b].data_ptr(),
                           st[b].data_ptr(), pil[b].data_ptr(), None, grp[b].data_ptr(), 8, gc[b].data_ptr())
        h.process_block(d_iq.data_ptr() + b * 2 * B * M, row, B, out)
        if not pipelined:
            h.sync()
    h.sync()
    torch.cuda.synchronize()
    r = mpx.cpu().numpy()
    other = {"pcm": torch.cat([pl, pr]).cpu().numpy(), "count": cnt.cpu().numpy(), "stereo": st.cpu().numpy(),
             "pilot": pil.cpu().numpy(), "groups": grp.cpu().numpy(), "group_count": gc.cpu().numpy()}
    h.close()
    return r, other


ref, ref_other = run(False)
bad = 0
for k in range(RUNS):
    for mode in (False, True):
        x, other = run(mode)
        for key, v in other.items():
            nd = int(np.sum(v != ref_other[key]))
            if nd:
                idx = np.argwhere(v != ref_other[key])
                print(f"run {k} pipelined={mode}: {nd} differing {key} values; (block, channel) "
                      f"{sorted(set((int(i[0]), int(i[1])) for i in idx))[:12]}", flush=True)
                bad += nd
        d = np.argwhere(x != ref)
        print(f"run {k} pipelined={mode}: {len(d)} differing MPX samples", flush=True)
        for (b, c, j) in d[:20]:
            print(f"   block {b} channel {c} sample {j}: ref {ref[b, c, j]:.6f} got {x[b, c, j]:.6f}")
        # where do the wrong values come from?  search the ref for the first
        # differing 16-sample run (same block, any channel / offset)
        if len(d):
            b, c, j = d[0]
            j0 = j - j % 16
            seg = x[b, c, j0:j0 + 16]
            for bb in range(ref.shape[0]):
                hits = np.argwhere(np.all(np.abs(np.lib.stride_tricks.sliding_window_view(ref[bb], 16, axis=1) - seg) < 1e-6, axis=2))
                for (cc, jj) in hits[:5]:
                    print(f"   run [{b},{c},{j0}:+16] equals ref block {bb} channel {cc} samples {jj}:+16")
            print("   the differing samples per (block, channel):",
                  {(int(bb), int(cc)): int(k) for (bb, cc), k in zip(*np.unique(d[:, :2], axis=0, return_counts=True))} if False else "")
            u, cnts = np.unique(d[:, :2], axis=0, return_counts=True)
            print("   ", [(int(a), int(b_), int(k)) for (a, b_), k in zip(u[:30], cnts[:30])])
            print("   offsets mod 2048 of run starts:", sorted(set(int(v) for v in (d[:, 2] - d[:, 2] % 16)[:200] % 2048))[:40])
        bad += len(d)
# the RDS stage alone (fmx_rds: k_frontend's RDS resampler + k_rds) on the
# reference run's MPX, twice in fresh handles: separates the front end's RDS
# resampler in k_fe8 from k_rds
if os.environ.get("RDS_STAGE", "1") == "1":
    d_mpx = torch.from_numpy(ref).to(dev)
    outs = []
    for rep in range(2):
        h = fmx.Handle(cfg, C)
        g_all = torch.zeros((NBLK, C, 8, 4), dtype=torch.int32, device=dev)
        c_all = torch.zeros((NBLK, C), dtype=torch.int32, device=dev)
        for b in range(NBLK):
            h.rds(d_mpx[b].data_ptr(), B, B, g_all[b].data_ptr(), 8, c_all[b].data_ptr())
        h.sync()
        outs.append((g_all.cpu().numpy(), c_all.cpu().numpy()))
        h.close()
    nd_g = int(np.sum(outs[0][0] != outs[1][0]))
    nd_c = int(np.sum(outs[0][1] != outs[1][1]))
    nd_x = int(np.sum(outs[0][0] != ref_other["groups"]))
    print(f"rds stage twice: {nd_g} differing groups values, {nd_c} group counts; vs process_block: {nd_x}")
    bad += nd_g + nd_c
print("DETERMINISTIC" if bad == 0 else f"NONDETERMINISTIC ({bad} samples)")
