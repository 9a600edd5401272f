#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

  blocksync.json  bit streams (clean groups, burst errors, random flips, bit
                  slips, noise) and the RDS groups the REFERENCE's own
                  BlockStream (src/redsea_port/block_sync.cpp + group.cpp,
                  compiled by oracle/Makefile into oracle/_ref/libfmx_ref.so)
                  emits for them.  Pins the oracle's and the GPU's block sync.
  xdr_server.json group streams (clean, burst errors, missing blocks, PI
                  changes as retunes make them) and scan lines, with the lines
                  the REFERENCE's own XDRServer (src/xdr_server.cpp, compiled
                  into oracle/_ref by refdrv/xdr_driver.cpp) sends a loopback
                  client for them (updateRDS / pushScanLine).  Pins
                  fmx_xdr_rds_lines and the tests' Python restatement.
  oracle_regress.json
                  hashes / excerpts of the oracle pipeline on seeded synthetic
                  IQ (pins the oracle restatement and the IQ generator against
                  unintended change; not a reference output -- see DESIGN.md).

Run in the build container (needs /root/reference to have built _ref):
    python tools/gen_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "fmtuner-sdr_amd"))
import fmx  # noqa: E402
import oracle  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")


def group_bits(scfg, ch, n_bits):
    """Undifferentiated (data) bits of the synthetic group sequence."""
    bits, groups = fmx.synth_rds_bits(scfg, ch, 1)
    enc = bits[0]
    data = np.empty_like(enc)
    prev = 0
    for i, e in enumerate(enc):  # differential decode
        data[i] = e ^ prev
        prev = e
    return data[:n_bits], groups[0]


def streams():
    rng = np.random.default_rng(0xB10C)
    scfg = fmx.make_synth(n_bits=104 * 40)
    out = {}
    clean, _ = group_bits(scfg, 7, 104 * 40)
    out["clean"] = clean
    out["offset_start"] = np.concatenate([rng.integers(0, 2, 37, dtype=np.uint8), clean])
    b = clean.copy()  # 1- and 2-bit bursts (correctable)
    for pos in rng.choice(np.arange(300, b.size - 2), 40, replace=False):
        b[pos] ^= 1
        if rng.random() < 0.5:
            b[pos + 1] ^= 1
    out["bursts"] = b
    b = clean.copy()  # random flips, BER 2e-2 (uncorrectable mixes)
    b ^= (rng.random(b.size) < 0.02).astype(np.uint8)
    out["flips_2e-2"] = b
    b = clean.copy()  # heavy errors: sync loss and re-acquisition
    b[1500:2300] ^= (rng.random(800) < 0.3).astype(np.uint8)
    out["sync_loss"] = b
    b = list(clean)  # bit slips
    del b[1200]
    b.insert(2500, 1)
    out["slips"] = np.array(b, dtype=np.uint8)
    out["noise"] = rng.integers(0, 2, 3000, dtype=np.uint8)
    scfg2 = fmx.make_synth(n_bits=104 * 30)
    other, _ = group_bits(scfg2, 4242, 104 * 30)
    out["two_stations"] = np.concatenate([clean[:1700], other])
    return out


def xdr_streams():
    """Seeded group streams for the XDR server fixture: (a, b, c, d, errors)."""
    rng = np.random.default_rng(2024)
    out = {}

    def grp(pi, emask):
        return (int(pi), int(rng.integers(0, 65536)), int(rng.integers(0, 65536)), int(rng.integers(0, 65536)),
                int(emask))

    # a locked station: clean groups, the odd corrected block
    out["clean"] = [grp(0x54A8, 0 if rng.random() < 0.9 else int(rng.choice([0x40, 0x10, 0x04, 0x01])))
                    for _ in range(300)]
    # burst errors: every error level on every block, missing blocks (3)
    out["bursts"] = [grp(int(rng.choice([0xC201, 0xC202])), int(rng.integers(0, 256))) for _ in range(400)]
    # retunes: the PI changes every 25-60 groups, a few noisy copies of the old one
    g, pis = [], [0x1000 + k for k in range(6)]
    while len(g) < 500:
        pi = int(rng.choice(pis))
        for _ in range(int(rng.integers(25, 60))):
            e = 0 if rng.random() < 0.7 else int(rng.integers(0, 256))
            g.append(grp(pi if rng.random() < 0.95 else pi ^ 0x0100, e))
    out["retunes"] = g[:500]
    return out


def xdr_scan_lines():
    return ["87500=41.3,87600=0.0,87700=10.0", "100000=120.0", "87500=-4.0,107900=99.9"]


def main():
    os.makedirs(GOLD, exist_ok=True)
    if not (oracle.ref_available() and oracle.xdr_ref_available()):
        sys.exit("oracle/_ref/libfmx_ref.so / libfmx_xdrref.so missing: build them with `make -C oracle` in the build container")
    fx = []
    for name, bits in streams().items():
        groups = oracle.ref_blocksync(bits)
        fx.append({"name": name, "bits": "".join("1" if x else "0" for x in bits),
                   "groups": [list(g) for g in groups]})
    with open(os.path.join(GOLD, "blocksync.json"), "w") as f:
        json.dump({"source": "reference BlockStream (src/redsea_port/block_sync.cpp, group.cpp) via "
                             "oracle/_ref/libfmx_ref.so; generated by tools/gen_golden.py",
                   "streams": fx}, f, indent=0)

    # the reference XDR server: one session per stream (a fresh server state)
    xs = []
    for name, groups in xdr_streams().items():
        xs.append({"name": name, "groups": [list(x) for x in groups], "lines": oracle.ref_xdr_session(groups)})
    scan = xdr_scan_lines()
    with open(os.path.join(GOLD, "xdr_server.json"), "w") as f:
        json.dump({"source": "reference XDRServer (src/xdr_server.cpp: updateRDS, pushScanLine) via "
                             "oracle/_ref/libfmx_ref.so (refdrv/xdr_driver.cpp, loopback client); "
                             "generated by tools/gen_golden.py",
                   "streams": xs, "scan": {"lines": scan, "sent": oracle.ref_xdr_session([], scan)}}, f, indent=0)

    # oracle regression pin (stereo+RDS at 2.4 MS/s, and mono cfg1)
    reg = {}
    for tag, kind, stereo in (("stereo_rds", 2, 1), ("mono", 0, 0)):
        B, M, nblk = 4096, 10, 12
        scfg = fmx.make_synth(kind=kind, n_bits=6000)
        bits, _ = fmx.synth_rds_bits(scfg, 3, 1)
        iq = fmx.synth_host(scfg, 3, 1, 0, B * M * nblk, bits)
        p = oracle.Pipeline(oracle.make_cfg(stereo=stereo, rds=1))
        blocks = []
        for b in range(nblk):
            o = p.block(iq[0, b * 2 * B * M:(b + 1) * 2 * B * M])
            blocks.append({"stereo": o["stereo"], "pilot": o["pilot"], "n_pcm": len(o["pcm_l"]),
                           "pcm_l_rms": float(np.sqrt(np.mean(o["pcm_l"] ** 2))) if len(o["pcm_l"]) else 0.0,
                           "pcm_l_head": [float(x) for x in o["pcm_l"][:4]],
                           "mpx_head": [float(x) for x in o["mpx"][:4]],
                           "groups": [list(g) for g in o["groups"]]})
        reg[tag] = {"iq_sha256": hashlib.sha256(iq.tobytes()).hexdigest(), "blocks": blocks}
    with open(os.path.join(GOLD, "oracle_regress.json"), "w") as f:
        json.dump(reg, f, indent=0)
    print("wrote", GOLD)


if __name__ == "__main__":
    main()
