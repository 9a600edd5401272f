"""The RDS ring as checkpoints (round 6).

k_rds keeps the last 256 mixed RDS-rate samples of every channel (the
reference's 255-tap FIR window, which SubcarrierSet::reset keeps,
subcarrier.cpp:108) for the partial-sum rebuild after a reset moves the
decimation phase.  Round 5 wrote that ring every call: 2 KB per channel per
step, 8.4 of k_rds's 10.5 MB written per launch at 4096 channels.  Round 6:
a call of >= 256 samples writes per-round NCO checkpoints instead, and the
ring is refilled from them and the call's RDS-rate input (still in its
intermediate slot) where it is needed -- a reset's rebuild, a short call
after a long one, fmx_diag_rds_ring.

Checked here against the round-5 behaviour on the same handle shape
(fmx_diag_set(FMX_DIAG_RDS_RING_ALWAYS)): the refilled ring equals the ring
k_rds wrote, bit for bit, and every output of the two handles is identical
through resets and mixed long / short calls -- process_block (pipelined
streams) and the fmx_rds stage entry point; the groups also against the
oracle."""
import numpy as np
import pytest

import gpu_harness as H
from test_gpu_parity import make_iq

pytestmark = pytest.mark.gpu

RING_ALWAYS = 1


def _rings(hs, chans):
    return [[h.diag_rds_ring(c) for c in chans] for h in hs]


def _assert_rings_equal(hs, chans, tag):
    ra, rb = _rings(hs, chans)
    for c, a, b in zip(chans, ra, rb):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (tag, c, np.argwhere(a != b)[:5])
        assert np.any(a != 0.0), (tag, c)  # a ring of real samples, not the creation zeros


def test_ring_refill_matches_written_ring_process_block(fmx, oracle, torch_cuda):
    """20 channels (three k_rds workgroups, the last partial) through
    process_block on two handles, one writing the ring every call; resets of
    channels 3 and 17 before block 6 and of every channel before block 12
    (the rebuild reads the refilled ring); rings compared after blocks 3, 6,
    12 and 19, all outputs compared every block, groups against the oracle."""
    torch = torch_cuda
    C, nblk, B, M = 20, 20, 4096, 10
    iq, _ = make_iq(fmx, 2, C, nblk, ch0=300)
    cfg = fmx.make_config()
    dev = torch.device("cuda")
    d_iq = torch.from_numpy(np.ascontiguousarray(iq)).to(dev)
    hs = [fmx.Handle(cfg, C), fmx.Handle(cfg, C)]
    hs[1].diag_set(RING_ALWAYS, 1)
    GS = 8

    def bufs():
        return dict(mpx=torch.zeros((C, B), dtype=torch.float32, device=dev),
                    pl=torch.zeros((C, B), dtype=torch.float32, device=dev),
                    pr=torch.zeros((C, B), dtype=torch.float32, device=dev),
                    cnt=torch.zeros(C, dtype=torch.int32, device=dev),
                    st=torch.zeros(C, dtype=torch.int32, device=dev),
                    pil=torch.zeros(C, dtype=torch.int32, device=dev),
                    clip=torch.zeros(C, dtype=torch.float32, device=dev),
                    grp=torch.zeros((C, GS, 4), dtype=torch.int32, device=dev),
                    gcnt=torch.zeros(C, dtype=torch.int32, device=dev),
                    ind=torch.zeros(C, dtype=torch.int32, device=dev))

    bs = [bufs(), bufs()]
    outs = [fmx.BlockOut(b["mpx"].data_ptr(), B, b["pl"].data_ptr(), b["pr"].data_ptr(), B, b["cnt"].data_ptr(),
                         b["st"].data_ptr(), b["pil"].data_ptr(), b["clip"].data_ptr(), b["grp"].data_ptr(), GS,
                         b["gcnt"].data_ptr(), None, b["ind"].data_ptr()) for b in bs]
    resets = {6: [3, 17], 12: [-1]}
    groups = [[[] for _ in range(C)] for _ in range(2)]
    for blk in range(nblk):
        for h in hs:
            for ch in resets.get(blk, []):
                h.reset(ch)
        for h, o in zip(hs, outs):
            h.process_block(d_iq.data_ptr() + blk * 2 * B * M, iq.shape[1], B, o)
        for h in hs:
            h.sync()
        for k in ("mpx", "pl", "pr", "cnt", "st", "pil", "gcnt", "grp", "ind"):
            a, b = bs[0][k].cpu().numpy(), bs[1][k].cpu().numpy()
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), (blk, k)
        g = bs[0]["grp"].cpu().numpy().view(np.uint8).reshape(C, GS, 16)
        gc = bs[0]["gcnt"].cpu().numpy()
        for c in range(C):
            for q in range(min(int(gc[c]), GS)):
                w = g[c, q]
                a, bb, cc, d = np.frombuffer(w[:8].tobytes(), dtype=np.uint16)
                groups[0][c].append((int(a), int(bb), int(cc), int(d), int(w[8])))
        if blk in (3, 6, 12, 19):
            _assert_rings_equal(hs, [0, 3, 7, 8, 17, 19], f"block {blk}")
    for h in hs:
        h.close()
    ngroups = 0
    for c in (0, 3, 17):
        rs = {b: c for b, lst in resets.items() if c in lst or -1 in lst}
        o = H.run_oracle_pipeline(oracle, oracle.make_cfg(), iq[c], nblk, resets=rs)
        og = [tuple(x) for blk in o for x in blk["groups"]]
        assert groups[0][c] == og, c
        ngroups += len(og)
    assert ngroups >= 3


def test_ring_refill_short_and_long_rds_calls(fmx, torch_cuda):
    """fmx_rds (RDSDecoder::process) on two handles with calls of 4096, 300
    (213 RDS-rate samples: k_rds refills the ring before writing its own
    samples) and 1000 MPX samples in a mixed order, resets between some of
    them; rings compared after every call, groups identical."""
    torch = torch_cuda
    C, B = 12, 4096
    nblk = 6
    cfg = fmx.make_config()
    # MPX rows from the full pipeline (a real RDS subcarrier)
    iq, _ = make_iq(fmx, 2, C, nblk, ch0=500)
    g = H.run_gpu_pipeline(fmx, torch, cfg, iq, nblk)
    mpx = np.concatenate([blk["mpx"] for blk in g], axis=1)  # [C][nblk * B]
    dev = torch.device("cuda")
    d_mpx = torch.from_numpy(np.ascontiguousarray(mpx)).to(dev)
    row = mpx.shape[1]
    hs = [fmx.Handle(cfg, C), fmx.Handle(cfg, C)]
    hs[1].diag_set(RING_ALWAYS, 1)
    grp = [torch.zeros((C, 8, 4), dtype=torch.int32, device=dev) for _ in hs]
    gcnt = [torch.zeros(C, dtype=torch.int32, device=dev) for _ in hs]
    sizes = [4096, 4096, 300, 300, 4096, 1000, 300, 4096, 300, 4096, 4096, 1000]
    resets = {2: 5, 4: -1, 6: 11, 9: 0}
    pos = 0
    for i, n in enumerate(sizes):
        if pos + n > row:
            break
        for h in hs:
            if i in resets:
                h.reset(resets[i])
        for k, h in enumerate(hs):
            h.rds(d_mpx.data_ptr() + 4 * pos, row, n, grp[k].data_ptr(), 8, gcnt[k].data_ptr())
        for h in hs:
            h.sync()
        assert np.array_equal(gcnt[0].cpu().numpy(), gcnt[1].cpu().numpy()), i
        assert np.array_equal(grp[0].cpu().numpy(), grp[1].cpu().numpy()), i
        _assert_rings_equal(hs, [0, 5, 7, 11], f"call {i} (n={n})")
        pos += n
    for h in hs:
        h.close()
