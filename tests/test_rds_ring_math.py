"""CPU check of the RDS ring refill's sample -> round mapping (round 6).

rds_ring_fill (fmx_kernels.hip) finds, for each of a call's last
FMX_RDS_RING samples, the round of k_rds that mixed it and that round's
checkpoint slot.  Here k_rds's round construction is restated (rounds end on
the decimation instants: round 0 holds samples 0..o0, round r >= 1 the 24
samples from o0 + 1 + 24 (r - 1); the last round may end early, as the tail)
and, for every decimation phase o0 and every call length from FMX_RDS_RING to
a whole block, every ring sample must fall in one of the FMX_RDS_CK rounds
k_rds checkpoints -- so the kernel's clamp of the slot index never acts --
at the same period position k_rds gave it."""
import numpy as np

DECIM, RING, CK = 24, 256, 12  # FMX_RDS_DECIM, FMX_RDS_RING, FMX_RDS_CK (fmx_design.h)


def rounds_of_call(o0, count):
    """k_rds: R and, per round, (base, first sample, last sample)."""
    R = 0 if count <= 0 else (1 if o0 >= count else 1 + (count - o0 - 1 + DECIM - 1) // DECIM)
    out = []
    for r in range(R):
        base = o0 - (DECIM - 1) if r == 0 else o0 + 1 + DECIM * (r - 1)
        lo, hi = max(base, 0), min(base + DECIM - 1, count - 1)
        out.append((base, lo, hi))
    return R, out


def test_ring_samples_fall_in_checkpointed_rounds():
    for o0 in range(DECIM):
        for count in list(range(RING, RING + 3 * DECIM)) + [729, 1000, 2918, 2919, 4096]:
            R, rnd = rounds_of_call(o0, count)
            first = max(R - CK, 0)
            t = np.arange(count - RING, count)
            # rds_ring_fill's mapping
            r = np.where(t <= o0, 0, 1 + (t - o0 - 1) // DECIM)
            base = np.where(r == 0, o0 - (DECIM - 1), o0 + 1 + DECIM * (r - 1))
            i = r - first
            assert i.min() >= 0 and i.max() < CK, (o0, count, i.min(), i.max())
            for tt, rr, bb in zip(t, r, base):
                b, lo, hi = rnd[rr]
                assert b == bb and lo <= tt <= hi, (o0, count, tt, rr)
                assert 0 <= tt - bb < DECIM


def test_checkpoints_cover_the_ring():
    # the static_assert of fmx_kernels.hip: 24 (CK - 1) + 1 >= RING
    assert DECIM * (CK - 1) + 1 >= RING
