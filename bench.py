#!/usr/bin/env python3
"""bench.py -- IQ MS/s demodulated per GPU (2.4 MS/s FM channels, stereo+RDS).

Workloads (BASELINE.json configs):
  cfg3 (default at N=1)  4096 channels PER GPU of synthetic stereo FM + 57 kHz
                  RDS (known groups), weak scaling over --gpus.
  cfg4 (default at N>1)  16384 channels IN TOTAL sharded over the ranks with
                  fmx_dist.shard (2048 per GPU at 8 GPUs), strong scaling: the
                  1/2/4/8-GPU curve BASELINE.json configs[3] names.
  --total-channels T overrides the total (sharded), --channels C the
  per-GPU count.
Every channel: 2.4 MS/s u8 IQ, decimate-by-10 to 240 kHz, de-emphasis 50 us,
dsp_block_samples = 4096.  One "step" = one reference block (40960 IQ
samples) for every channel: decimator -> discriminator -> stereo PLL/blend
-> 32 kHz audio -> RDS bits + block sync, plus the per-block RF level
(computeSignalLevel, main.cpp:1167) -- fmx_process_block.  All step inputs
are generated into HBM before the timed region (fresh, phase-continuous IQ
for every step), so `value` excludes PCIe.

Multi-GPU: one process per GPU.  `python bench.py --gpus N` with no
WORLD_SIZE in the environment re-launches itself under
torch.distributed.run (N ranks, 127.0.0.1) before touching the GPU; under a
launcher WORLD_SIZE must equal --gpus.  Channels are sharded by rank with no
data-path collective; RCCL carries only the barrier, the max-over-ranks time,
the summed channel count and the scan line's RF-level all_gather (the three
last timed blocks of every channel are the scan's 3 reads per point,
main.cpp:1064-1121).

Prints ONE JSON line (rank 0).
"""
import argparse
import glob
import json
import math
import os
import re
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fmtuner-sdr_amd"))

# algorithmic figures of the whole path per input IQ sample
# (stereo + RDS, M = 10): 2 B u8 IQ in + 8 B stereo PCM per 32 kHz frame
# (x 32000 / 2.4e6 = 0.107 B) = 2.107 B; 290 FLOP (decimator 112, IQ FIR
# 32.4, pilot BPF 61, L/R FIRs 48, RDS 15, AF 3, PLL/trig 20).
ALG_BYTES_PER_IQ = 2.107
ALG_FLOP_PER_IQ = 290.0
# per-kernel DESIGN figures: HBM bytes the design moves
# per IQ sample including its own intermediates (MPX, pilot, RDS-rate, raw
# L/R), and the kernel's share of the 290 FLOP
# The 240k -> 171k RDS resampler (k_rs: MPX in, RDS-rate samples out) runs on
# the RDS stream ahead of k_rds, which reads the RDS-rate samples.
PER_IQ = {
    "frontend": (2.0 + 0.4, 112.0 + 32.4),
    "stereo": (0.4 + 0.8 + 0.8, 20.0),
    "audio": (0.8 + 0.107, 48.0 + 3.0),
    "rds": (4.0 * 0.7125 / 10.0, 15.0),
    "rs": (0.4 + 4.0 * 0.7125 / 10.0, 7.4),
    "pilot": (0.4 + 0.4, 61.0),
    "frontend_generic": (2.0 + 0.4, 112.0 + 32.4),
    # k_bits: the PSK2 symbols (2 375 / s, f32) k_rds wrote; bit logic, no FLOP
    "bits": (4.0 * 2375.0 / 2.4e6, 0.0),
}
KNAME = {"frontend": "k_fe8", "stereo": "k_pll", "audio": "k_audio", "rds": "k_rds", "rs": "k_rs", "pilot": "k_pilot",
         "frontend_generic": "k_frontend", "bits": "k_bits"}


def pmc_bytes(pmc, k):
    """Counted HBM bytes per launch of the kernel(s) behind timer k, or None."""
    names = KNAME[k].split("+")
    if not pmc or not all(n in pmc for n in names):
        return None
    return sum(pmc[n]["hbm_bytes_per_launch"] for n in names)
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md
# per-unit peaks (MI355X_MICROARCH.md): 256 CUs x 4 SIMDs at ~2.4 GHz; a SIMD
# retires one wave64 VALU instruction per 2 cycles when several waves share it
CLOCK_HZ = 2.4e9
N_CU = 256
VALU_ISSUE_PEAK = N_CU * 4 * CLOCK_HZ / 2.0   # wave-instructions / s
MFMA_F16_PEAK = 2.5e15                        # dense FLOP / s
MFMA_F32_PEAK = 157.3e12
METRIC = "IQ MS/s demodulated per GPU (2.4 MS/s FM channels, stereo+RDS) at 1/2/4/8 MI355X"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (default: WORLD_SIZE or 1)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["cfg3", "cfg4"], default=None,
                    help="default: cfg3 on one GPU, cfg4 (BASELINE configs[3], the scaling curve) on N > 1")
    ap.add_argument("--channels", type=int, default=None, help="channels per GPU (cfg3 default 4096)")
    ap.add_argument("--total-channels", type=int, default=None, help="channels in total, sharded over ranks")
    ap.add_argument("--block", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="target wall time of the all-core CPU sample")
    ap.add_argument("--retune-per-step", action="store_true",
                    help="diagnostic: fmx_retune one channel before every step (main.cpp:1028-1042)")
    ap.add_argument("--sync-steps", action="store_true",
                    help="diagnostic: synchronize after every step (no cross-step overlap; not the reported mode)")
    ap.add_argument("--pmc-json", default=None,
                    help="per-kernel HBM bytes per launch from rocprofv3 --pmc (tools/pmc_traffic.py); "
                         "default: the newest profiles/r*_pmc*.json")
    ap.add_argument("--kernel-timing-every", type=int, default=1,
                    help="time the kernel launches of every N-th timed step (roofline / kernels figures)")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="diagnostic: no per-kernel HIP-event timing in the timed region (no roofline / kernels)")
    ap.add_argument("--no-signal-level", action="store_true",
                    help="diagnostic: skip the per-block RF level (computeSignalLevel) output")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: set up the ranks / shards / collectives and print the plan (tests)")
    return ap.parse_args(argv)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launcher_cmd(n, argv):
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)


def resolve_world(args):
    """(world, spawn): world size of this run, and whether this process must
    spawn the N ranks itself (no launcher in the environment)."""
    env = os.environ.get("WORLD_SIZE")
    if env is None:
        n = args.gpus or 1
        return n, n > 1
    w = int(env)
    if args.gpus is not None and args.gpus != w:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={w}")
    return w, False


def plan_channels(args, world, rank):
    """(ch0, C_local, total, scaling) for this rank."""
    from fmx_dist import shard
    total = args.total_channels
    if total is None and args.workload == "cfg4":
        total = 16384
    if total is not None:
        b, e = shard(total, world, rank)
        return b, e - b, total, "strong"
    c = args.channels or 4096
    return rank * c, c, c * world, "weak"


def tag_key(path):
    """Order of the profile tags r<round><letters>: r04z < r04aa < r04al."""
    m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
    return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")


def newest_pmc():
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc*.json")), key=tag_key)
    return files[-1] if files else None


def newest_units(channels, block):
    """The newest profiles/r*_units*.json (tools/gpu_units.sh) of this shape."""
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_units*.json")), key=tag_key, reverse=True):
        try:
            with open(f) as fh:
                u = json.load(fh)
        except (OSError, ValueError):
            continue
        if int(u.get("channels", -1)) == channels and int(u.get("block", -1)) == block:
            return f, u
    return None, None


def unit_fracs(u, t):
    """Fractions of each unit's peak that the counted work of one launch
    (units-file entry u) takes over t seconds."""
    out = {}
    if "valu_insts" in u:
        out["valu"] = u["valu_insts"] / t / VALU_ISSUE_PEAK
    if "mfma_flop_f16" in u or "mfma_flop_f32" in u:
        out["mfma"] = (u.get("mfma_flop_f16", 0.0) / MFMA_F16_PEAK + u.get("mfma_flop_f32", 0.0) / MFMA_F32_PEAK) / t
    if "lds_active_cycles" in u:
        out["lds"] = u["lds_active_cycles"] / (N_CU * CLOCK_HZ * t)
    if "hbm_bytes" in u:
        out["hbm"] = u["hbm_bytes"] / t / (HBM_PEAK_GBS * 1e9)
    return {k: round(v, 4) for k, v in out.items()}


def cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(math.ceil(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    usable = min(aff, quota) if quota else aff
    return {"cpu_model": model, "nproc": nproc, "affinity": aff, "cgroup_cpus": quota, "usable": usable}


def cpu_baseline(fmx, d_iq, C, nblk, n_iq, B, seconds):
    """The oracle (CPU restatement, kind "port") on this box's host cores:
    single-core rates for one Cfg3 channel and for Cfg1 (mono, 1 channel),
    then one channel per thread on every usable core, sized to ~`seconds`."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle
    info = cpu_info()
    threads = info["usable"]
    ocfg = oracle.make_cfg(block=B)
    # single core, one Cfg3 channel (stereo + RDS)
    nb1 = min(nblk, 40)
    one = d_iq[:1, : 2 * n_iq * nb1].cpu().numpy().reshape(1, nb1, 2 * n_iq)
    s1, _ = oracle.run_many(ocfg, one, nb1, 1)
    r1 = nb1 * n_iq / s1 / 1e6
    # single core, Cfg1: mono FM (1 kHz + 3 kHz), stereo=false path, no RDS
    mono = fmx.synth_host(fmx.make_synth(kind=0), 0, 1, 0, n_iq * nb1)
    sm, _ = oracle.run_many(oracle.make_cfg(block=B, stereo=0, rds=0), mono.reshape(1, nb1, 2 * n_iq), nb1, 1)
    rm = nb1 * n_iq / sm / 1e6
    # all usable cores: one channel per thread, enough blocks for ~`seconds`
    want_iq = seconds * threads * r1 * 1e6
    cc = min(C, max(threads, int(want_iq / (n_iq * nblk)) + 1))
    cc = max(threads, (cc // threads) * threads) if C >= threads else C
    nb = int(min(nblk, max(4, want_iq / (cc * n_iq))))
    host = d_iq[:cc, : 2 * n_iq * nb].cpu().numpy().reshape(cc, nb, 2 * n_iq)
    secs, _ = oracle.run_many(ocfg, host, nb, threads)
    # Cfg2 (BASELINE configs[1]): 256 stereo channels without RDS, all cores,
    # over the same IQ (stereo + pilot; the RDS subcarrier is just signal here)
    c2 = min(256, C)
    nb2 = int(min(nblk, max(2, (seconds / 2.0) * threads * r1 * 1.3e6 / (c2 * n_iq))))
    host2 = d_iq[:c2, : 2 * n_iq * nb2].cpu().numpy().reshape(c2, nb2, 2 * n_iq)
    secs2, _ = oracle.run_many(oracle.make_cfg(block=B, rds=0), host2, nb2, threads)
    return {"value": round(cc * nb * n_iq / secs / 1e6, 2), "unit": "MS/s", "cores": threads, "kind": "port",
            "sample": f"{cc} Cfg3 channels x {nb} blocks of 40960 IQ samples (stereo+RDS), oracle/fmx_oracle.cpp, "
                      f"one channel per thread on {threads} threads, {secs:.2f} s wall",
            "single_core": {"cfg3_one_channel_ms_s": round(r1, 3), "cfg1_mono_ms_s": round(rm, 3),
                            "blocks": nb1},
            "cfg2_all_core": {"value": round(c2 * nb2 * n_iq / secs2 / 1e6, 2), "unit": "MS/s", "cores": threads,
                              "sample": f"{c2} channels x {nb2} blocks, stereo without RDS, {secs2:.2f} s wall"},
            **{k: info[k] for k in ("cpu_model", "nproc", "affinity", "cgroup_cpus")}}


def _sha16(path):
    """First 16 hex digits of a file's SHA-256 (the bench line's library record)."""
    import hashlib
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def main():
    args = parse()
    world, spawn = resolve_world(args)
    if args.workload is None:
        args.workload = "cfg3" if world == 1 else "cfg4"
    if spawn:
        # no launcher: start the N ranks as children before any GPU call
        sys.exit(subprocess.run(launcher_cmd(world, sys.argv[1:])).returncode)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ch0, C, total, scaling = plan_channels(args, world, rank)
    import torch
    import torch.distributed as dist
    # FMX_BENCH_BACKEND=gloo: rehearsal of the N-rank flow on fewer GPUs (ranks
    # share GPUs round-robin, the collectives go over gloo); --dry-run: no GPU
    backend = "gloo" if args.dry_run else os.environ.get("FMX_BENCH_BACKEND", "nccl")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
        from fmx_dist import gather_levels
        lv = torch.full((C,), float(rank))
        allv = gather_levels(lv)
        tot = torch.tensor([float(C)])
        if world > 1:
            dist.all_reduce(tot)
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "world_reported": dist.get_world_size() if world > 1 else 1,
                              "backend": backend, "total_channels": total, "channels_summed": int(tot.item()),
                              "scaling": scaling, "ch0": ch0, "channels_rank0": C,
                              "gathered": int(allv.numel()),
                              "gathered_ranks": [int(x) for x in allv[:: max(1, C)].tolist()]}), flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    import numpy as np
    import fmx
    import fmx_dist
    gpu = local if backend == "nccl" else local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", gpu)
    cdev = dev if backend == "nccl" else torch.device("cpu")
    world_reported = dist.get_world_size() if world > 1 else 1

    B = args.block
    M = 10
    nblk = args.warmup + args.steps
    cfg = fmx.make_config(iq_rate=2_400_000, dsp_rate=240_000, out_rate=32_000, block=B,
                          w0_bandwidth_hz=194_000, bandwidth_hz=0, dsp_agc=0, stereo=1, blend=1,
                          deemphasis=0, rds=1)
    h = fmx.Handle(cfg, C, device=gpu)
    # ---- inputs: synthetic stereo + RDS IQ for every step, resident in HBM ----
    n_iq = B * M
    n_bits = int((nblk * n_iq + 2 * 2_400_000) * 1187.5 / 2.4e6) + 208  # covers the per-channel RDS offset
    # carrier levels spread over 24 dB (0.8 .. 0.05 of full scale, seeded per
    # channel): the scan line's RF levels span the 120-point scale instead of
    # saturating it; every channel still carries stereo + RDS
    scfg = fmx.make_synth(iq_rate=2_400_000, kind=2, n_bits=n_bits, level_spread_db=24.0)
    bits, _ = fmx.synth_rds_bits(scfg, ch0, C)
    d_bits = torch.from_numpy(bits).to(dev)
    row = 2 * n_iq * nblk
    d_iq = torch.empty((C, row), dtype=torch.uint8, device=dev)
    h.synth_device(scfg, ch0, C, 0, n_iq * nblk, d_bits.data_ptr(), d_iq.data_ptr(), row)
    h.sync()  # the synth (the handle's stream) has read d_bits before torch may reuse its memory
    del d_bits
    # ---- outputs ----
    pl = torch.empty((C, B), dtype=torch.float32, device=dev)
    pr = torch.empty((C, B), dtype=torch.float32, device=dev)
    cnt = torch.empty(C, dtype=torch.int32, device=dev)
    st = torch.empty(C, dtype=torch.int32, device=dev)
    pil = torch.empty(C, dtype=torch.int32, device=dev)
    ind = torch.empty(C, dtype=torch.int32, device=dev)
    clip = torch.empty(C, dtype=torch.float32, device=dev)
    GS = 8
    grp = torch.empty((C, GS, 4), dtype=torch.int32, device=dev)
    gcnt = torch.empty(C, dtype=torch.int32, device=dev)
    # fmx_signal_level records (40 B) of the last three steps: the scan's
    # three reads per point
    sig = torch.zeros((3, C, 10), dtype=torch.float32, device=dev)
    outs = [fmx.BlockOut(None, 0, pl.data_ptr(), pr.data_ptr(), B, cnt.data_ptr(), st.data_ptr(),
                         pil.data_ptr(), clip.data_ptr(), grp.data_ptr(), GS, gcnt.data_ptr(),
                         None if args.no_signal_level else sig[k].data_ptr(), ind.data_ptr()) for k in range(3)]
    h.sync()
    torch.cuda.synchronize()

    def step(b):
        if args.retune_per_step:  # diagnostic A/B: a live receiver retuning one channel per block
            h.retune((b * 7919) % C, -1)
        h.process_block(d_iq.data_ptr() + b * 2 * n_iq, row, B, outs[b % 3])
        if args.sync_steps:
            h.sync()

    # what runs between the warmup and the timed steps is made ready first:
    # the timing event pool (fmx_timing_enable creates 256 events), torch's
    # reduction kernel (its code object loads on first use) and, at N > 1,
    # the process group's first collective (RCCL sets up its communicator on
    # it).  Left to after the warmup they kept the GPU idle for ~100 ms there
    # (rocprofv3 trace), long enough for the timed steps to start from a cold GPU
    if world > 1:
        dist.barrier()
    if not args.no_kernel_timing:
        h.timing_enable(True, every=args.kernel_timing_every)
        h.timing_enable(False)
    int(gcnt.zero_().sum().item())
    for b in range(args.warmup):
        step(b)
    tw = time.perf_counter()
    h.sync()
    tw_sync = time.perf_counter()
    groups_warm = int(gcnt.sum().item())
    # per-kernel live times from HIP events around the launches of every
    # --kernel-timing-every-th timed step (default: all of them; timing off
    # altogether measured 0.772 against 0.782 ms, timing every 2nd step showed
    # no gain over the run-to-run spread: profiles/r03x_kernel_timing.txt)
    h.timing_enable(not args.no_kernel_timing, every=args.kernel_timing_every)
    if world > 1:
        dist.barrier()
    h.sync()
    torch.cuda.synchronize()
    h.host_stats()  # reset the counters: the timed region's waits only
    t0 = time.perf_counter()
    idle_before_ms = 1e3 * (t0 - tw)  # host time from the last warmup submission to the timed region
    host_call = []  # host time per process_block call (submission only): stalls show here
    for b in range(args.warmup, nblk):
        tc = time.perf_counter()
        step(b)
        host_call.append(time.perf_counter() - tc)
    h.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    ktimes = h.kernel_times()
    hstats = h.host_stats()
    ngroups = int(gcnt.sum().item())
    stereo_frac = float(st.float().mean().item())
    chans_all = float(C)
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        cc_ = torch.tensor([float(C)], dtype=torch.float64, device=cdev)
        dist.all_reduce(cc_, op=dist.ReduceOp.SUM)
        chans_all = float(cc_.item())
    iq_samples = chans_all * args.steps * n_iq
    value = iq_samples / elapsed / 1e6  # MS/s, whole job
    ms_per_step = elapsed * 1e3 / args.steps

    # ---- multi-channel scan line: every channel is a scan point; its level is
    # the mean of the last three blocks' computeSignalLevel (main.cpp:1078-1103),
    # gathered from all ranks (RCCL all_gather, fmx_dist.gather_levels) ----
    level_sum = (sig[0, :, 0] + sig[1, :, 0] + sig[2, :, 0]).to(torch.float64)
    tg0 = time.perf_counter()
    all_levels = fmx_dist.gather_levels(level_sum.to(cdev))
    gather_ms = (time.perf_counter() - tg0) * 1e3
    scan = None
    if rank == 0:
        lv = all_levels.cpu().numpy()
        freq = 87_500 + 50 * np.arange(lv.size, dtype=np.int64)  # synthetic channel plan, 50 kHz raster
        line = fmx.xdr_scan_line(freq.astype(np.int32), lv, np.full(lv.size, 3, np.int32))
        scan = {"points": int(lv.size), "reads_per_point": 3, "line_bytes": len(line),
                "gather_ms": round(gather_ms, 3), "mean_level120": round(float(lv.mean() / 3.0), 2),
                "head": line[:48]}

    # ---- roofline: the kernel with the longest live launch (HIP events on
    # its own stream over the timed region), against SURVEY 8(d)'s 2.107 B/IQ ----
    units_step = C * n_iq  # IQ samples one step processes on this rank
    # launches per timed step of each kernel (the front end may run as two
    # channel halves): a launch processes units_step / that many IQ samples
    timed = max(1, -(-args.steps // max(1, args.kernel_timing_every)))
    lps = {k: max(1, round(v[1] / timed)) for k, v in ktimes.items() if v[1] > 0}
    avg = {k: v[0] / max(v[1], 1) * 1e-3 for k, v in ktimes.items() if v[1] > 0}
    if not avg:  # --no-kernel-timing (diagnostic): no per-kernel figures
        avg = {k: float("nan") for k in ktimes}
    dom = max(avg, key=avg.get)
    dom_s = avg[dom]
    units_path, ucnt = newest_units(C, B)
    pmc_path = args.pmc_json or newest_pmc()
    pmc = None
    if ucnt and not args.pmc_json:
        # the units passes carry FETCH / WRITE too: one source for both
        pmc_path = units_path
        pmc = {k: {"hbm_bytes_per_launch": e["hbm_bytes"]} for k, e in ucnt["kernels"].items() if "hbm_bytes" in e}
    elif pmc_path and os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pm = json.load(f)
            if int(pm.get("channels", -1)) == C and int(pm.get("block", -1)) == B:
                pmc = pm.get("kernels", {})
        except (OSError, ValueError):
            pmc = None
    units = units_step // lps.get(dom, 1)  # IQ samples of one launch of the dominant kernel
    alg_bytes = ALG_BYTES_PER_IQ * units
    achieved = alg_bytes / dom_s / 1e9
    traffic = pmc_bytes(pmc, dom)
    step_traffic = None
    if all(pmc_bytes(pmc, k) is not None for k in avg):
        step_traffic = sum(pmc_bytes(pmc, k) * lps.get(k, 1) for k in avg)
    # measured per-unit utilisation (counters of tools/gpu_units.sh over the
    # live launch times of this run): the dominant kernel's and the step's
    unit_rec = None
    if ucnt:
        uk = ucnt["kernels"]
        dom_u = unit_fracs(uk.get(KNAME[dom], {}), dom_s)
        step_work = {}
        for k in avg:
            e = uk.get(KNAME[k])
            if e is None:
                continue
            for name in ("valu_insts", "mfma_flop_f16", "mfma_flop_f32", "lds_active_cycles", "hbm_bytes"):
                if name in e:
                    step_work[name] = step_work.get(name, 0.0) + e[name] * lps.get(k, 1)
        step_u = unit_fracs(step_work, ms_per_step * 1e-3)
        unit_rec = {"source": os.path.relpath(units_path, ROOT),
                    "source_library_sha256_16": ucnt.get("library_sha256_16"),
                    "source_matches_loaded_library": ucnt.get("library_sha256_16") == _sha16(fmx.LIB_PATH),
                    "peaks": {"valu": f"{VALU_ISSUE_PEAK:.4g} wave-instr/s (1024 SIMDs x 2.4 GHz / 2 cycles)",
                              "mfma": "2.5 PFLOP/s f16, 157.3 TFLOP/s f32 (dense)",
                              "lds": f"{N_CU} CUs x 2.4 GHz LDS-array cycles (SQ_LDS_IDX_ACTIVE)",
                              "hbm": f"{HBM_PEAK_GBS:.0f} GB/s"},
                    "dominant_kernel": {"kernel": KNAME[dom], "avg_launch_ms": round(dom_s * 1e3, 4), **dom_u},
                    "dominant_binding_unit": max(dom_u, key=dom_u.get) if dom_u else None,
                    "step": {"ms_per_step": round(ms_per_step, 4), **step_u},
                    "step_binding_unit": max(step_u, key=step_u.get) if step_u else None}
    # the contract's roof (hbm | mfma): whichever of the two the dominant
    # kernel's counters put closer to its peak (hbm when there are none);
    # achieved = the ALGORITHMIC bytes (or MFMA FLOP) of one launch over its
    # live time.  The unit that binds among all four is units.*_binding_unit.
    bound, r_ach, r_peak, r_unit = "hbm", round(achieved, 1), HBM_PEAK_GBS, "GB/s"
    du = unit_rec["dominant_kernel"] if unit_rec else {}
    if du.get("mfma", 0.0) > du.get("hbm", 0.0):
        alg_flop = PER_IQ[dom][1] * units
        bound, r_ach, r_peak, r_unit = "mfma", round(alg_flop / dom_s / 1e12, 2), MFMA_F16_PEAK / 1e12, "TFLOP/s"
    roof = {"bound": bound, "kernel": KNAME[dom], "achieved": r_ach, "peak": r_peak,
            "unit": r_unit, "frac": round(r_ach / r_peak, 4), "traffic": traffic,
            "traffic_source": os.path.relpath(pmc_path, ROOT) if pmc else None,
            "algorithmic_bytes_per_launch": alg_bytes, "bytes_per_iq": ALG_BYTES_PER_IQ,
            "avg_launch_ms": round(dom_s * 1e3, 4),
            # the whole step's counted HBM bytes (all four kernels) over the
            # path's algorithmic bytes: intermediates round-tripping HBM
            "step_traffic": step_traffic,
            "step_traffic_over_algorithmic": round(step_traffic / (ALG_BYTES_PER_IQ * units_step), 3) if step_traffic else None,
            # what the hardware units actually do: measured fractions of each
            # unit's peak (VALU issue, MFMA, LDS, HBM) for the dominant kernel
            # and the whole step; the FIRs run on f16 MFMA, the recursions on
            # the VALU, and none of the four is near its roof -- the path is
            # latency-bound
            "units": unit_rec}
    kern = {}
    for k, v in ktimes.items():
        if v[1] == 0:
            continue
        avg_s = avg[k]
        bpi, fpi = PER_IQ[k]
        units = units_step // lps[k]
        ent = {"kernel": KNAME[k], "ms_total": round(v[0], 3), "launches": v[1], "avg_ms": round(avg_s * 1e3, 4),
               "launches_per_step": lps[k],
               # live in the pipelined timed region (co-running kernels included)
               "design_bytes_per_launch": bpi * units,
               "design_hbm_gbs": round(bpi * units / avg_s / 1e9, 1),
               # the kernel's share of the path's 290 algorithmic FLOP/IQ (FIR MACs
               # as 2 FLOP; most of it runs on f16 hi/lo MFMA passes)
               "alg_tflops": round(fpi * units / avg_s / 1e12, 3)}
        if ucnt and KNAME[k] in ucnt["kernels"]:
            ent["units"] = unit_fracs(ucnt["kernels"][KNAME[k]], avg_s)
        pb = pmc_bytes(pmc, k)
        if pb is not None:
            ent["pmc_bytes_per_launch"] = pb
            ent["pmc_over_design"] = round(pb / (bpi * units), 3)
        kern[k] = ent

    # ---- CPU baseline: the oracle on this box's host cores (rank 0, N=1) ----
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(fmx, d_iq, C, nblk, n_iq, B, args.cpu_seconds)

    wl = {"cfg3": "cfg3: 4096 ch x 2.4 MS/s stereo FM + 57 kHz RDS per GPU",
          "cfg4": "cfg4: 16384 ch x 2.4 MS/s stereo FM + 57 kHz RDS sharded over the GPUs"}[args.workload]
    if args.total_channels is not None or args.channels is not None:
        wl += f" (channels overridden: {int(chans_all)} total)"
    res = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "MS/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f32 (FIR operands f16 hi+lo, f32 accumulate)",
        "data": "synthetic (seeded stereo FM + RDS IQ generated in HBM)",
        "config": {"workload": wl + ", M=10 -> 240 kHz, dsp_block=4096, deemphasis 50 us",
                   "total_channels": int(chans_all), "channels_rank0": C, "block": B, "iq_rate": 2_400_000,
                   "parallelism": f"channels/{world}gpu", "backend": backend if world > 1 else None,
                   "world_reported": world_reported,
                   **({"retune_per_step": True} if args.retune_per_step else {})},
        "per_gpu_ms_s": round(value / world, 1),
        "realtime_channels_per_gpu": round(value / world / 2.4, 1),
        "roofline": roof,
        "kernels": kern,
        "kernel_timing": None if args.no_kernel_timing else
        f"HIP events around the launches of every {max(1, args.kernel_timing_every)}. timed step",
        "dominant_kernel": dom,
        "cpu_baseline": cpu,
        "scan": scan,
        "warmup_to_timed_ms": {"total": round(idle_before_ms, 3), "warmup_drain": round(1e3 * (tw_sync - tw), 3)},
        "host_submit_ms": {"mean": round(1e3 * sum(host_call) / len(host_call), 4),
                           "max": round(1e3 * max(host_call), 4)},
        # waits of process_block on the pinned schedule images' last readers
        # (the host's only throttle): how many blocked, and for how long
        "host_image_waits": hstats,
        "check": {"rds_groups_last_step": ngroups, "rds_groups_warmup": groups_warm,
                  "stereo_fraction": stereo_frac},
        # the library this run loaded (fmx.LIB_PATH; FMX_LIB selects A/B builds)
        "library": {"path": os.path.relpath(fmx.LIB_PATH, ROOT), "sha256_16": _sha16(fmx.LIB_PATH),
                    "build_info": fmx.build_info()},
    }
    if rank == 0:
        print(json.dumps(res), flush=True)
    h.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
