import sys, time, os
sys.path.insert(0, 'tests'); sys.path.insert(0, 'oracle'); sys.path.insert(0, 'fmtuner-sdr_amd')
import numpy as np, torch
import fmx, oracle, gpu_harness as H
C = int(os.environ.get('C', 4)); nblk = int(os.environ.get('NBLK', 30))
B, M = 4096, 10
scfg = fmx.make_synth(kind=2, n_bits=8192)
bits, groups = fmx.synth_rds_bits(scfg, 0, C)
if os.environ.get('SYNTH') == 'device':
    h0 = fmx.Handle(fmx.make_config(), 1)
    d_bits = torch.from_numpy(bits).cuda()
    d_iq = torch.empty((C, 2*B*M*nblk), dtype=torch.uint8, device='cuda')
    h0.synth_device(scfg, 0, C, 0, B*M*nblk, d_bits.data_ptr(), d_iq.data_ptr(), d_iq.shape[1])
    h0.sync(); iq = d_iq.cpu().numpy(); h0.close()
    ih = fmx.synth_host(scfg, 0, min(C, 2), 0, B*M*4, bits)
    print('device vs host synth bytes differing:', int(np.sum(ih != iq[:min(C,2), :ih.shape[1]])), 'of', ih.size)
else:
    iq = fmx.synth_host(scfg, 0, C, 0, B*M*nblk, bits)
cfg = fmx.make_config()
t = time.time()
g = H.run_gpu_pipeline(fmx, torch, cfg, iq, nblk)
print('gpu run', time.time()-t, flush=True)
for c in range(C):
    o = H.run_oracle_pipeline(oracle, oracle.make_cfg(), iq[c], nblk)
    st = H.compare(g, o, c, nblk)
    gg, go = st.pop('groups_gpu'), st.pop('groups_oracle')
    print(c, st, 'groups gpu/oracle', len(gg), len(go), 'equal', gg == go, flush=True)
    if c == 0:
        for b in [0, 1, 5, 10, 29]:
            if b < nblk:
                print('  blk', b, 'mpx[:4] gpu', g[b]['mpx'][0,:4], 'ora', o[b]['mpx'][:4])
                print('  blk', b, 'pcm[:4] gpu', g[b]['pcm_l'][0,:4], 'ora', o[b]['pcm_l'][:4], 'cnt', g[b]['count'][0], len(o[b]['pcm_l']))
                print('  st', g[b]['stereo'][0], o[b]['stereo'], 'pil', g[b]['pilot'][0], o[b]['pilot'], 'clip', g[b]['clip'][0], o[b]['clip'])
        print(gg[:4]); print(go[:4])
