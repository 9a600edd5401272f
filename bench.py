#!/usr/bin/env python3
"""bench.py -- IQ MS/s demodulated per GPU (2.4 MS/s FM channels, stereo+RDS).

Workload (BASELINE.json configs[2]): 4096 independent
2.4 MS/s channels per GPU, synthetic stereo FM (19 kHz pilot, L-R on 38 kHz,
57 kHz RDS carrying known groups), decimate-by-10 to 240 kHz, de-emphasis
50 us, dsp_block_samples = 4096.  One "step" = one reference block
(40960 IQ samples) for every channel: decimator -> discriminator -> stereo
PLL/blend -> 32 kHz audio -> RDS bits + block sync (fmx_process_block).
All step inputs are generated into HBM before the timed region (fresh,
phase-continuous IQ for every step).

Multi-GPU: one process per GPU (torchrun), channels sharded by rank with no
data-path collective (weak scaling); RCCL is used only for the barrier and
the max-over-ranks time.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fmtuner-sdr_amd"))

# per-unit algorithmic figures: bytes and FLOP per input
# IQ sample at M = 10 (stereo + RDS)
BYTES_PER_IQ_FRONTEND = 2.0 + 0.4 + 0.4 + 4.0 * 0.7125 / 10.0   # u8 IQ in; MPX, pilot, RDS-rate out
FLOP_PER_IQ_FRONTEND = 112.0 + 32.4 + 61.0 + 7.4                 # decim, IQ FIR, pilot BPF, RDS resampler
PER_IQ = {  # kernel: (algorithmic HBM bytes, FLOP) per IQ sample
    "frontend": (BYTES_PER_IQ_FRONTEND, FLOP_PER_IQ_FRONTEND),
    "stereo": (0.4 + 0.8 + 0.8, 20.0),      # pilot + MPX + delayed MPX in, raw L/R out
    "audio": (0.8 + 0.107, 48.0 + 3.0),     # raw L/R in, 32 kHz PCM out; L/R FIRs + AF
    "rds": (4.0 * 0.7125 / 10.0, 15.0),     # 171 kHz samples in (groups out ~0)
}
HBM_PEAK_GBS = 8000.0
FP32_PEAK_TFLOPS = 157.3


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--channels", type=int, default=4096, help="channels per GPU")
    ap.add_argument("--block", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sync-steps", action="store_true",
                    help="diagnostic: synchronize after every step (no cross-step overlap; not the reported mode)")
    ap.add_argument("--cpu-channels", type=int, default=256)
    ap.add_argument("--cpu-blocks", type=int, default=16)
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "r01_pmc_frontend.json"),
                    help="per-launch HBM bytes of the frontend kernel from rocprofv3 --pmc (optional)")
    return ap.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist
    import fmx

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # FMX_BENCH_BACKEND=gloo: rehearsal of the N-rank flow on fewer GPUs
    # (ranks share GPUs round-robin, the timing collectives go over gloo)
    backend = os.environ.get("FMX_BENCH_BACKEND", "nccl")
    gpu = local if backend == "nccl" else local % max(1, torch.cuda.device_count())
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", gpu if world > 1 else 0)
    cdev = dev if backend == "nccl" else torch.device("cpu")

    C = args.channels
    B = args.block
    M = 10
    nblk = args.warmup + args.steps
    cfg = fmx.make_config(iq_rate=2_400_000, dsp_rate=240_000, out_rate=32_000, block=B,
                          w0_bandwidth_hz=194_000, bandwidth_hz=0, dsp_agc=0, stereo=1, blend=1,
                          deemphasis=0, rds=1)
    h = fmx.Handle(cfg, C, device=gpu if world > 1 else 0)
    ch0 = rank * C
    # ---- inputs: synthetic stereo + RDS IQ for every step, resident in HBM ----
    n_iq = B * M
    n_bits = int((nblk * n_iq + 2 * 2_400_000) * 1187.5 / 2.4e6) + 208  # covers the per-channel RDS offset
    scfg = fmx.make_synth(iq_rate=2_400_000, kind=2, n_bits=n_bits)
    bits, _ = fmx.synth_rds_bits(scfg, ch0, C)
    d_bits = torch.from_numpy(bits).to(dev)
    row = 2 * n_iq * nblk
    d_iq = torch.empty((C, row), dtype=torch.uint8, device=dev)
    h.synth_device(scfg, ch0, C, 0, n_iq * nblk, d_bits.data_ptr(), d_iq.data_ptr(), row)
    # ---- outputs ----
    pl = torch.empty((C, B), dtype=torch.float32, device=dev)
    pr = torch.empty((C, B), dtype=torch.float32, device=dev)
    cnt = torch.empty(C, dtype=torch.int32, device=dev)
    st = torch.empty(C, dtype=torch.int32, device=dev)
    pil = torch.empty(C, dtype=torch.int32, device=dev)
    clip = torch.empty(C, dtype=torch.float32, device=dev)
    GS = 8
    grp = torch.empty((C, GS, 4), dtype=torch.int32, device=dev)
    gcnt = torch.empty(C, dtype=torch.int32, device=dev)
    out = fmx.BlockOut(None, 0, pl.data_ptr(), pr.data_ptr(), B, cnt.data_ptr(), st.data_ptr(),
                       pil.data_ptr(), clip.data_ptr(), grp.data_ptr(), GS, gcnt.data_ptr())
    h.sync()
    torch.cuda.synchronize()

    def step(b):
        h.process_block(d_iq.data_ptr() + b * 2 * n_iq, row, B, out)
        if args.sync_steps:
            h.sync()

    for b in range(args.warmup):
        step(b)
    h.sync()
    groups_warm = int(gcnt.sum().item())
    h.timing_enable(True)
    if world > 1:
        dist.barrier()
    h.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in range(args.warmup, nblk):
        step(b)
    h.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    ktimes = h.kernel_times()
    ngroups = int(gcnt.sum().item())
    stereo_frac = float(st.float().mean().item())
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    iq_samples = float(world) * C * args.steps * n_iq
    value = iq_samples / elapsed / 1e6  # MS/s, whole job
    ms_per_step = elapsed * 1e3 / args.steps

    # ---- roofline of the dominant kernel, from HIP events on its stream ----
    dom = max(ktimes, key=lambda k: ktimes[k][0])
    k_ms, k_n = ktimes["frontend"]
    fe_avg_s = (k_ms / max(k_n, 1)) * 1e-3
    units = C * n_iq
    fe_flops = FLOP_PER_IQ_FRONTEND * units
    fe_bytes = BYTES_PER_IQ_FRONTEND * units
    achieved_tf = fe_flops / fe_avg_s / 1e12
    traffic = None
    if os.path.exists(args.pmc_json):
        try:
            with open(args.pmc_json) as f:
                pm = json.load(f)
            if int(pm.get("channels", -1)) == C and int(pm.get("block", -1)) == B:
                traffic = float(pm["hbm_bytes_per_launch"])
        except Exception:
            traffic = None
    achieved_gbs = fe_bytes / fe_avg_s / 1e9
    roof = {"bound": "hbm", "kernel": "k_fe8 (frontend)", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved_gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
            "algorithmic_bytes_per_launch": fe_bytes, "avg_launch_ms": round(fe_avg_s * 1e3, 4),
            # the roof that binds this path (no MFMA: FIR/IIR/PLL work is FP32 VALU)
            "valu_view": {"achieved": round(achieved_tf, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": round(achieved_tf / FP32_PEAK_TFLOPS, 4),
                          "algorithmic_flop_per_launch": fe_flops}}
    kern = {}
    for k, v in ktimes.items():
        avg_s = v[0] / max(v[1], 1) * 1e-3
        bpi, fpi = PER_IQ[k]
        kern[k] = {"ms_total": round(v[0], 3), "launches": v[1], "avg_ms": round(avg_s * 1e3, 4),
                   # live in the pipelined timed region (co-running kernels included)
                   "hbm_gbs": round(bpi * units / max(avg_s, 1e-12) / 1e9, 1),
                   "fp32_tflops": round(fpi * units / max(avg_s, 1e-12) / 1e12, 3)}

    # ---- CPU baseline: the oracle on this box's host cores (rank 0, N=1) ----
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        cc = min(args.cpu_channels, C)
        nb = min(args.cpu_blocks, nblk)
        host = d_iq[:cc, : 2 * n_iq * nb].cpu().numpy().reshape(cc, nb, 2 * n_iq)
        threads = min(16, os.cpu_count() or 1)
        ocfg = oracle.make_cfg(block=B)
        secs, _ = oracle.run_many(ocfg, host, nb, threads)
        cpu = {"value": round(cc * nb * n_iq / secs / 1e6, 2), "unit": "MS/s", "cores": threads,
               "kind": "port",
               "sample": f"{cc} channels x {nb} blocks of 40960 IQ samples (stereo+RDS), oracle/fmx_oracle.cpp, "
                         f"one channel per thread, {secs:.2f} s wall"}

    res = {
        "metric": "IQ MS/s demodulated per GPU (2.4 MS/s FM channels, stereo+RDS) at 1/2/4/8 MI355X",
        "value": round(value, 1),
        "unit": "MS/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded stereo FM + RDS IQ generated in HBM)",
        "config": {"workload": "cfg3: 4096 ch x 2.4 MS/s stereo FM + 57 kHz RDS per GPU, M=10 -> 240 kHz, "
                               "dsp_block=4096, deemphasis 50 us",
                   "channels_per_gpu": C, "block": B, "iq_rate": 2_400_000, "parallelism": f"channels/{world}gpu"},
        "per_gpu_ms_s": round(value / world, 1),
        "realtime_channels_per_gpu": round(value / world / 2.4, 1),
        "roofline": roof,
        "kernels": kern,
        "dominant_kernel": dom,
        "cpu_baseline": cpu,
        "check": {"rds_groups_last_step": ngroups, "rds_groups_warmup": groups_warm,
                  "stereo_fraction": stereo_frac},
    }
    if rank == 0:
        print(json.dumps(res), flush=True)
    h.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
