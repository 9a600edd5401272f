"""Shared driver for the GPU parity tests and smoke(): runs the same
synthetic IQ through libfmx (GPU) and through the oracle (CPU) block by
block and returns both outputs."""
import numpy as np


def run_gpu_pipeline(fmx, torch, cfg, iq, nblk, n=None, resets=None, params=None, retunes=None, ktimes=None):
    """iq: uint8 [C][nblk * 2*B*M]. Returns per-block lists of numpy outputs.
    resets {block: channel}, retunes {block: (channel, mute_samples)},
    params {block: [(key, value, channel)]} are applied before that block.
    ktimes (a dict): filled with fmx_kernel_times ({kernel: (ms, launches)})
    of the whole run."""
    C = iq.shape[0]
    B = cfg.block
    M = cfg.iq_rate // cfg.dsp_rate
    n = n or B
    h = fmx.Handle(cfg, C)
    dev = torch.device("cuda")
    d_iq = torch.from_numpy(np.ascontiguousarray(iq)).to(dev)
    mpx = torch.zeros((C, B), dtype=torch.float32, device=dev)
    pl = torch.zeros((C, B), dtype=torch.float32, device=dev)
    pr = torch.zeros((C, B), dtype=torch.float32, device=dev)
    cnt = torch.zeros(C, dtype=torch.int32, device=dev)
    st = torch.zeros(C, dtype=torch.int32, device=dev)
    pil = torch.zeros(C, dtype=torch.int32, device=dev)
    clip = torch.zeros(C, dtype=torch.float32, device=dev)
    ind = torch.zeros(C, dtype=torch.int32, device=dev)
    GS = 8
    grp = torch.zeros((C, GS, 4), dtype=torch.int32, device=dev)  # 16-byte fmx_rds_group
    gcnt = torch.zeros(C, dtype=torch.int32, device=dev)
    out = fmx.BlockOut(mpx.data_ptr(), B, pl.data_ptr(), pr.data_ptr(), B, cnt.data_ptr(),
                       st.data_ptr(), pil.data_ptr(), clip.data_ptr(), grp.data_ptr(), GS,
                       gcnt.data_ptr(), None, ind.data_ptr())
    res = []
    row = iq.shape[1]
    if ktimes is not None:
        h.timing_enable(True)
    for b in range(nblk):
        if resets and b in resets:
            h.reset(resets[b])
        if retunes and b in retunes:
            h.retune(*retunes[b])
        if params and b in params:
            for (k, v, ch) in params[b]:
                h.set_param(k, v, ch)
        base = d_iq.data_ptr() + b * 2 * n * M
        h.process_block(base, row, n, out)
        h.sync()
        g = grp.cpu().numpy().view(np.uint8).reshape(C, GS, 16)
        gc = gcnt.cpu().numpy()
        groups = []
        for c in range(C):
            lst = []
            for k in range(min(int(gc[c]), GS)):
                w = g[c, k]
                a, bb, cc, d = np.frombuffer(w[:8].tobytes(), dtype=np.uint16)
                lst.append((int(a), int(bb), int(cc), int(d), int(w[8])))
            groups.append(lst)
        res.append(dict(mpx=mpx[:, :n].cpu().numpy().copy(), pcm_l=pl.cpu().numpy().copy(),
                        pcm_r=pr.cpu().numpy().copy(), count=cnt.cpu().numpy().copy(),
                        stereo=st.cpu().numpy().copy(), pilot=pil.cpu().numpy().copy(),
                        clip=clip.cpu().numpy().copy(), indicator=ind.cpu().numpy().copy(),
                        groups=groups))
    if ktimes is not None:
        ktimes.update(h.kernel_times())
    h.close()
    return res


def run_oracle_pipeline(oracle, ocfg, iq_row, nblk, n=None, resets=None, params=None, retunes=None):
    B = ocfg.block
    M = ocfg.iq_rate // ocfg.dsp_rate
    n = n or B
    p = oracle.Pipeline(ocfg)
    res = []
    for b in range(nblk):
        if resets and b in resets:
            p.reset()
        if retunes and b in retunes:
            p.retune(retunes[b])
        if params and b in params:
            for (k, v) in params[b]:
                p.set_param(k, v)
        res.append(p.block(iq_row[b * 2 * n * M:(b + 1) * 2 * n * M]))
    return res


def compare(gres, ores, c, nblk, pcm_blocks=None):
    """Per-channel comparison stats.  pcm_blocks (optional) restricts the PCM
    and pilot-level statistics to those blocks."""
    mpx_err = 0.0
    mpx_sq = 0.0
    mpx_n = 0
    pcm_sq = 0.0
    pcm_n = 0
    pcm_max = 0.0
    st_mismatch = 0
    pil_mismatch = 0
    pil_maxdiff = 0
    cnt_mismatch = 0
    ind_mismatch = 0
    g_gpu, g_ora = [], []
    mpx_where = None
    for b in range(nblk):
        o, g = ores[b], gres[b]
        if g["mpx"] is not None:  # None: a run without the MPX output (bench mode)
            dm = o["mpx"] - g["mpx"][c, :len(o["mpx"])]
            if dm.size and float(np.max(np.abs(dm))) > mpx_err:
                mpx_where = (b, int(np.argmax(np.abs(dm))))
            mpx_err = max(mpx_err, float(np.max(np.abs(dm))))
            mpx_sq += float(np.sum(dm.astype(np.float64) ** 2))
            mpx_n += dm.size
        k = len(o["pcm_l"])
        if int(g["count"][c]) != k:
            cnt_mismatch += 1
        st_mismatch += int(o["stereo"] != int(g["stereo"][c]))
        ind_mismatch += int(o["indicator"] != int(g["indicator"][c]))
        g_gpu += g["groups"][c]
        g_ora += o["groups"]
        if pcm_blocks is not None and b not in pcm_blocks:
            continue
        k = min(k, int(g["count"][c]))
        dl = o["pcm_l"][:k] - g["pcm_l"][c, :k]
        dr = o["pcm_r"][:k] - g["pcm_r"][c, :k]
        pcm_sq += float(np.sum(dl * dl) + np.sum(dr * dr))
        pcm_n += 2 * k
        pcm_max = max(pcm_max, float(np.max(np.abs(dl))) if k else 0.0, float(np.max(np.abs(dr))) if k else 0.0)
        pil_mismatch += int(o["pilot"] != int(g["pilot"][c]))
        pil_maxdiff = max(pil_maxdiff, abs(int(o["pilot"]) - int(g["pilot"][c])))
    return dict(mpx_max=mpx_err, mpx_where=mpx_where, mpx_rms=(mpx_sq / max(mpx_n, 1)) ** 0.5,
                pcm_rms=(pcm_sq / max(pcm_n, 1)) ** 0.5, pcm_max=pcm_max,
                stereo_mismatch=st_mismatch, indicator_mismatch=ind_mismatch, pilot_mismatch=pil_mismatch, pilot_maxdiff=pil_maxdiff, count_mismatch=cnt_mismatch,
                groups_gpu=g_gpu, groups_oracle=g_ora)


def _groups_of(grp_rows, gcnt_rows, GS):
    """grp_rows: int32 [K][GS][4] (16-byte fmx_rds_group records), gcnt_rows [K]."""
    g = grp_rows.view(np.uint8).reshape(len(gcnt_rows), GS, 16)
    out = []
    for j in range(len(gcnt_rows)):
        lst = []
        for k in range(min(int(gcnt_rows[j]), GS)):
            w = g[j, k]
            a, bb, cc, d = np.frombuffer(w[:8].tobytes(), dtype=np.uint16)
            lst.append((int(a), int(bb), int(cc), int(d), int(w[8])))
        out.append(lst)
    return out


def run_gpu_pipelined(fmx, torch, cfg, C, scfg, nblk, keep, ch0=0, with_mpx=False, warmup=5, all_groups=None,
                      retunes=None):
    """The bench's timed mode (bench.py step()): every block through
    fmx_process_block back to back, NO host synchronisation between blocks,
    kernel timing switched on after `warmup` blocks as the bench does, the
    RF-level output on, and the front end of step k overlapping steps k-1 /
    k-2 on the four streams.  Outputs go to per-block device buffers (the
    bench rotates three sets it never reads), so nothing is read back until
    the last block has been submitted.  Channels [ch0, ch0 + C) of the
    synthetic plan (a rank's fmx_dist shard).  Returns (per-block results
    indexed by position in keep, host IQ rows of keep, transmitted groups of
    keep, per-block stereo fraction over all C channels).  all_groups: a list
    that receives every channel's decoded groups over all blocks (full-size
    property checks).  retunes {block: [(channel, mute_samples), ...]}:
    fmx_retune calls queued before that block's fmx_process_block (no
    synchronisation, as a live receiver retunes)."""
    B = cfg.block
    M = cfg.iq_rate // cfg.dsp_rate
    n_iq = B * M
    h = fmx.Handle(cfg, C)
    dev = torch.device("cuda")
    bits, tx = fmx.synth_rds_bits(scfg, ch0, C)
    d_bits = torch.from_numpy(bits).to(dev)
    row = 2 * n_iq * nblk
    d_iq = torch.empty((C, row), dtype=torch.uint8, device=dev)
    h.synth_device(scfg, ch0, C, 0, n_iq * nblk, d_bits.data_ptr(), d_iq.data_ptr(), row)
    h.sync()  # the synth (stream sA) has read d_bits before torch may reuse its memory
    del d_bits
    GS = 8
    pl = torch.full((nblk, C, B), float("nan"), dtype=torch.float32, device=dev)
    pr = torch.full((nblk, C, B), float("nan"), dtype=torch.float32, device=dev)
    mpx = torch.full((nblk, C, B), float("nan"), dtype=torch.float32, device=dev) if with_mpx else None
    ints = torch.full((6, nblk, C), -1, dtype=torch.int32, device=dev)  # count, stereo, pilot, gcount, indicator
    clip = torch.zeros((nblk, C), dtype=torch.float32, device=dev)
    grp = torch.zeros((nblk, C, GS, 4), dtype=torch.int32, device=dev)
    sig = torch.zeros((nblk, C, 10), dtype=torch.float32, device=dev)
    h.sync()
    torch.cuda.synchronize()
    for b in range(nblk):
        if b == warmup:
            h.timing_enable(True)
        for (ch, mute) in (retunes or {}).get(b, []):
            h.retune(ch, mute)
        out = fmx.BlockOut(mpx[b].data_ptr() if with_mpx else None, B if with_mpx else 0,
                           pl[b].data_ptr(), pr[b].data_ptr(), B, ints[0, b].data_ptr(), ints[1, b].data_ptr(),
                           ints[2, b].data_ptr(), clip[b].data_ptr(), grp[b].data_ptr(), GS, ints[3, b].data_ptr(),
                           sig[b].data_ptr(), ints[4, b].data_ptr())
        h.process_block(d_iq.data_ptr() + b * 2 * n_iq, row, B, out)
    h.sync()
    torch.cuda.synchronize()
    kt = h.kernel_times()
    kidx = torch.tensor(keep, dtype=torch.long, device=dev)
    sel = lambda t: t.index_select(1, kidx).cpu().numpy()  # noqa: E731  [nblk][len(keep)]...
    PL, PR = sel(pl), sel(pr)
    MPX = sel(mpx) if with_mpx else None
    I = ints.index_select(2, kidx).cpu().numpy()  # [6][nblk][len(keep)]
    CL = sel(clip)
    G = sel(grp)
    SG = sel(sig)  # 40-byte fmx_signal_level records
    recs = [[fmx.SignalLevel.from_buffer_copy(SG[b, j].tobytes()) for j in range(len(keep))] for b in range(nblk)]
    stereo_all = ints[1].float().mean(dim=1).cpu().numpy()
    if all_groups is not None:
        ga = grp.cpu().numpy()  # [nblk][C][GS][4]
        gca = ints[3].cpu().numpy()
        per = [_groups_of(ga[b], gca[b], GS) for b in range(nblk)]
        all_groups.extend([g for b in range(nblk) for g in per[b][c]] for c in range(C))
        del ga
    res = []
    for b in range(nblk):
        d = dict(pcm_l=PL[b], pcm_r=PR[b], count=I[0, b], stereo=I[1, b], pilot=I[2, b], indicator=I[4, b],
                 clip=CL[b], groups=_groups_of(G[b], I[3, b], GS), sig=recs[b])
        d["mpx"] = MPX[b] if with_mpx else None
        res.append(d)
    iq_keep = d_iq.index_select(0, kidx).cpu().numpy()
    h.close()
    return res, iq_keep, tx[keep], stereo_all, kt


def run_gpu_sampled(fmx, torch, cfg, C, scfg, nblk, keep, setup=None, retunes=None, n_bits=None):
    """Full-size run: C channels of synthetic IQ generated in HBM
    (fmx_synth_device), every block through fmx_process_block, and only the
    rows of the channels in `keep` copied back.  setup: [(key, value,
    channel)] applied after creation; retunes: {block: (channel, mute)}.
    Returns (per-block results indexed by position in keep, host IQ rows of
    keep [len(keep)][nblk * 2*B*M], transmitted groups of keep)."""
    import numpy as np
    B = cfg.block
    M = cfg.iq_rate // cfg.dsp_rate
    n_iq = B * M
    h = fmx.Handle(cfg, C)
    for (k, v, ch) in (setup or []):
        h.set_param(k, v, ch)
    dev = torch.device("cuda")
    bits, tx = fmx.synth_rds_bits(scfg, 0, C)
    d_bits = torch.from_numpy(bits).to(dev)
    row = 2 * n_iq * nblk
    d_iq = torch.empty((C, row), dtype=torch.uint8, device=dev)
    h.synth_device(scfg, 0, C, 0, n_iq * nblk, d_bits.data_ptr(), d_iq.data_ptr(), row)
    kidx = torch.tensor(keep, dtype=torch.long, device=dev)
    mpx = torch.zeros((C, B), dtype=torch.float32, device=dev)
    pl = torch.zeros((C, B), dtype=torch.float32, device=dev)
    pr = torch.zeros((C, B), dtype=torch.float32, device=dev)
    cnt = torch.zeros(C, dtype=torch.int32, device=dev)
    st = torch.zeros(C, dtype=torch.int32, device=dev)
    pil = torch.zeros(C, dtype=torch.int32, device=dev)
    clip = torch.zeros(C, dtype=torch.float32, device=dev)
    ind = torch.zeros(C, dtype=torch.int32, device=dev)
    GS = 8
    grp = torch.zeros((C, GS, 4), dtype=torch.int32, device=dev)
    gcnt = torch.zeros(C, dtype=torch.int32, device=dev)
    out = fmx.BlockOut(mpx.data_ptr(), B, pl.data_ptr(), pr.data_ptr(), B, cnt.data_ptr(),
                       st.data_ptr(), pil.data_ptr(), clip.data_ptr(), grp.data_ptr(), GS,
                       gcnt.data_ptr(), None, ind.data_ptr())
    res = []
    for b in range(nblk):
        if retunes and b in retunes:
            h.retune(*retunes[b])
        h.process_block(d_iq.data_ptr() + b * 2 * n_iq, row, B, out)
        h.sync()
        sel = lambda t: t.index_select(0, kidx).cpu().numpy().copy()  # noqa: E731
        g = sel(grp).view(np.uint8).reshape(len(keep), GS, 16)
        gc = sel(gcnt)
        groups = []
        for j in range(len(keep)):
            lst = []
            for k in range(min(int(gc[j]), GS)):
                w = g[j, k]
                a, bb, cc, d = np.frombuffer(w[:8].tobytes(), dtype=np.uint16)
                lst.append((int(a), int(bb), int(cc), int(d), int(w[8])))
            groups.append(lst)
        res.append(dict(mpx=sel(mpx), pcm_l=sel(pl), pcm_r=sel(pr), count=sel(cnt), stereo=sel(st),
                        pilot=sel(pil), clip=sel(clip), indicator=sel(ind), groups=groups,
                        stereo_all=float(st.float().mean().item())))
    iq_keep = d_iq.index_select(0, kidx).cpu().numpy()
    h.close()
    return res, iq_keep, tx[keep]
