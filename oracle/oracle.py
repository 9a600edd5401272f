"""oracle.py -- TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU
restatement (oracle/libfmx_oracle.so) and of the reference's own compiled
block sync / signal level (oracle/_ref/libfmx_ref.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product (fmtuner-sdr_amd/) never does.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_LIB = os.path.join(_HERE, "libfmx_oracle.so")
REF_LIB = os.path.join(_HERE, "_ref", "libfmx_ref.so")
XDR_REF_LIB = os.path.join(_HERE, "_ref", "libfmx_xdrref.so")


class OracleCfg(C.Structure):
    _fields_ = [(n, C.c_int) for n in (
        "iq_rate", "dsp_rate", "out_rate", "block", "w0_bandwidth_hz",
        "bandwidth_hz", "dsp_agc", "stereo", "blend", "deemphasis",
        "force_mono", "force_stereo", "rds")]


class OracleGroup(C.Structure):
    _fields_ = [("a", C.c_uint16), ("b", C.c_uint16), ("c", C.c_uint16),
                ("d", C.c_uint16), ("errors", C.c_uint8), ("pad", C.c_uint8),
                ("block_index", C.c_uint32)]


class BlockInfo(C.Structure):
    _fields_ = [("n_mpx", C.c_int), ("n_pcm", C.c_int), ("stereo_detected", C.c_int),
                ("pilot_tenths_khz", C.c_int), ("clip_ratio", C.c_float),
                ("n_groups", C.c_int), ("stereo_indicator", C.c_int)]


_lib = None
_ref = None
_xref = None


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(ORACLE_LIB)
        vp, i, sz = C.c_void_p, C.c_int, C.c_size_t
        sigs = {
            "oracle_pipeline_create": (vp, [C.POINTER(OracleCfg)]),
            "oracle_pipeline_destroy": (None, [vp]),
            "oracle_pipeline_reset": (None, [vp]),
            "oracle_pipeline_retune": (None, [vp, i]),
            "oracle_pipeline_block": (i, [vp, vp, i, vp, vp, vp, i, vp, i, C.POINTER(BlockInfo)]),
            "oracle_pipeline_taps": (i, [vp, i, vp, i]),
            "oracle_pipeline_set": (None, [vp, i, i]),
            "oracle_decim_create": (vp, [C.c_uint32, C.c_uint32, C.c_float]),
            "oracle_decim_destroy": (None, [vp]),
            "oracle_decim_reset": (None, [vp]),
            "oracle_decim_execute_complex": (sz, [vp, vp, sz, vp, sz]),
            "oracle_decim_execute": (sz, [vp, vp, sz, vp, sz]),
            "oracle_demod_create": (vp, [i, i]),
            "oracle_demod_destroy": (None, [vp]),
            "oracle_demod_reset": (None, [vp]),
            "oracle_demod_set": (None, [vp, i, i]),
            "oracle_demod_process_split_complex": (sz, [vp, vp, vp, vp, sz]),
            "oracle_demod_process_split": (sz, [vp, vp, vp, vp, sz]),
            "oracle_demod_clip_ratio": (C.c_float, [vp]),
            "oracle_stereo_create": (vp, [i, i]),
            "oracle_stereo_destroy": (None, [vp]),
            "oracle_stereo_reset": (None, [vp]),
            "oracle_stereo_set": (None, [vp, i, i]),
            "oracle_stereo_process": (sz, [vp, vp, vp, vp, sz, C.POINTER(i), C.POINTER(i)]),
            "oracle_stereo_process_trace": (sz, [vp, vp, vp, vp, sz, vp, vp]),
            "oracle_afpost_create": (vp, [i, i]),
            "oracle_afpost_destroy": (None, [vp]),
            "oracle_afpost_reset": (None, [vp]),
            "oracle_afpost_set_deemphasis": (None, [vp, i]),
            "oracle_afpost_process": (sz, [vp, vp, vp, sz, vp, vp, sz]),
            "oracle_rds_create": (vp, [i]),
            "oracle_rds_destroy": (None, [vp]),
            "oracle_rds_reset": (None, [vp]),
            "oracle_rds_process": (i, [vp, vp, sz, vp, i, vp, i, C.POINTER(i)]),
            "oracle_blocksync_create": (vp, []),
            "oracle_blocksync_destroy": (None, [vp]),
            "oracle_blocksync_push": (i, [vp, vp, i, vp, i]),
            "oracle_run_many": (C.c_double, [C.POINTER(OracleCfg), i, vp, i, i, C.POINTER(C.c_double)]),
        }
        for k, (r, a) in sigs.items():
            f = getattr(L, k)
            f.restype = r
            f.argtypes = a
        _lib = L
    return _lib


def ref_available():
    return os.path.exists(REF_LIB)


def xdr_ref_available():
    return os.path.exists(XDR_REF_LIB)


def ref():
    """The reference's own block_sync/group/util + signal_level, compiled by
    oracle/Makefile from /root/reference (travels as a built .so)."""
    global _ref
    if _ref is None:
        L = C.CDLL(REF_LIB)
        vp, i = C.c_void_p, C.c_int
        L.ref_blocksync_create.restype = vp
        L.ref_blocksync_create.argtypes = []
        L.ref_blocksync_destroy.restype = None
        L.ref_blocksync_destroy.argtypes = [vp]
        L.ref_blocksync_push.restype = i
        L.ref_blocksync_push.argtypes = [vp, vp, i, vp, i]
        L.ref_signal_level.restype = None
        L.ref_signal_level.argtypes = [vp, C.c_size_t, i, C.c_double, C.c_double, C.c_double,
                                       C.c_double, C.POINTER(C.c_double)]
        L.ref_smooth_signal_level.restype = C.c_float
        L.ref_smooth_signal_level.argtypes = [C.c_float, C.POINTER(i), C.POINTER(C.c_float)]
        _ref = L
    return _ref


def xref():
    """The reference's XDRServer (src/xdr_server.cpp) behind refdrv/xdr_driver.cpp."""
    global _xref
    if _xref is None:
        L = C.CDLL(XDR_REF_LIB)
        vp, i = C.c_void_p, C.c_int
        L.ref_xdr_pi_state.restype = i
        L.ref_xdr_pi_state.argtypes = [vp, vp, i, C.c_uint16]
        L.ref_xdr_session.restype = i
        L.ref_xdr_session.argtypes = [vp, vp, i, C.c_char_p, i, i, C.c_char_p, i]
        _xref = L
    return _xref


def make_cfg(iq_rate=2_400_000, dsp_rate=240_000, out_rate=32_000, block=4096,
             w0_bandwidth_hz=194_000, bandwidth_hz=0, dsp_agc=0, stereo=1, blend=1,
             deemphasis=0, force_mono=0, force_stereo=0, rds=1):
    return OracleCfg(iq_rate, dsp_rate, out_rate, block, w0_bandwidth_hz, bandwidth_hz,
                     dsp_agc, stereo, blend, deemphasis, force_mono, force_stereo, rds)


def groups_to_tuples(arr, n):
    return [(arr[k].a, arr[k].b, arr[k].c, arr[k].d, arr[k].errors) for k in range(n)]


class Pipeline:
    """One channel of the reference per-block body (main.cpp:1232-1308)."""

    def __init__(self, cfg):
        self.L = lib()
        self.cfg = cfg
        self.p = self.L.oracle_pipeline_create(C.byref(cfg))
        if not self.p:
            raise RuntimeError("oracle_pipeline_create failed")
        self.M = cfg.iq_rate // cfg.dsp_rate

    def __del__(self):
        if getattr(self, "p", None):
            self.L.oracle_pipeline_destroy(self.p)
            self.p = None

    def reset(self):
        self.L.oracle_pipeline_reset(self.p)

    def retune(self, mute_samples=-1):
        self.L.oracle_pipeline_retune(self.p, mute_samples)

    PARAM = dict(bandwidth_hz=1, w0_hz=2, deemphasis=3, dsp_agc=4, blend=5,
                 force_mono=6, force_stereo=7, bandwidth_mode=8, deemph_us=9, deviation_hz=10)

    def set_param(self, key, value):
        k = self.PARAM[key] if isinstance(key, str) else key
        self.L.oracle_pipeline_set(self.p, k, value)

    def block(self, iq):
        """iq: uint8 array of 2*n*M bytes (n <= block) -> dict of outputs."""
        iq = np.ascontiguousarray(iq, dtype=np.uint8)
        B = self.cfg.block
        mpx = np.zeros(B, np.float32)
        pl = np.zeros(B, np.float32)
        pr = np.zeros(B, np.float32)
        g = (OracleGroup * 64)()
        info = BlockInfo()
        n = self.L.oracle_pipeline_block(self.p, iq.ctypes.data, iq.size // 2, mpx.ctypes.data,
                                         pl.ctypes.data, pr.ctypes.data, B, g, 64, C.byref(info))
        return dict(mpx=mpx[:info.n_mpx], pcm_l=pl[:n], pcm_r=pr[:n],
                    stereo=info.stereo_detected, pilot=info.pilot_tenths_khz,
                    indicator=info.stereo_indicator,
                    clip=info.clip_ratio, groups=groups_to_tuples(g, min(info.n_groups, 64)))

    def taps(self, which):
        n = self.L.oracle_pipeline_taps(self.p, which, None, 0)
        if n < 0:
            return None
        buf = np.zeros(n, np.float32)
        self.L.oracle_pipeline_taps(self.p, which, buf.ctypes.data, n)
        return buf


def blocksync(bits):
    L = lib()
    p = L.oracle_blocksync_create()
    bits = np.ascontiguousarray(bits, dtype=np.uint8)
    cap = bits.size // 26 + 8
    g = (OracleGroup * cap)()
    n = L.oracle_blocksync_push(p, bits.ctypes.data, bits.size, g, cap)
    L.oracle_blocksync_destroy(p)
    return groups_to_tuples(g, min(n, cap))


def ref_blocksync(bits):
    R = ref()
    p = R.ref_blocksync_create()
    bits = np.ascontiguousarray(bits, dtype=np.uint8)
    cap = bits.size // 26 + 8
    g = (OracleGroup * cap)()
    n = R.ref_blocksync_push(p, bits.ctypes.data, bits.size, g, cap)
    R.ref_blocksync_destroy(p)
    return groups_to_tuples(g, min(n, cap))


def ref_xdr_pi_state(buf64, err8, fill, value):
    """The reference's evaluatePiState (xdr_server.cpp:189-213), oracle/_ref/libfmx_xdrref.so."""
    b = np.ascontiguousarray(buf64, dtype=np.uint16)
    e = np.ascontiguousarray(err8, dtype=np.uint8)
    return xref().ref_xdr_pi_state(b.ctypes.data, e.ctypes.data, int(fill), int(value))


def ref_xdr_session(groups, scan_lines=(), port=None):
    """The lines the reference's started XDRServer sends one authenticated
    loopback client when `groups` ((a, b, c, d, errors) each) go through
    updateRDS and `scan_lines` through pushScanLine (oracle/_ref,
    refdrv/xdr_driver.cpp).  Returns the list of lines."""
    import random
    g = np.array([x[:4] for x in groups], dtype=np.uint16).reshape(-1, 4) if groups else np.zeros((0, 4), np.uint16)
    e = np.array([x[4] for x in groups], dtype=np.uint8) if groups else np.zeros(0, np.uint8)
    scan = b"".join(ln.encode() + b"\0" for ln in scan_lines)
    cap = 40 * (len(groups) + 1) + sum(len(x) + 2 for x in scan_lines) + 64
    out = C.create_string_buffer(cap)
    for attempt in range(8):  # a busy port: another one
        pt = port or random.randint(20000, 60000)
        rc = xref().ref_xdr_session(g.ctypes.data, e.ctypes.data, len(groups), scan or None, len(scan_lines), pt,
                                   out, cap)
        if rc != -1 or port:
            break
    if rc < 0:
        raise RuntimeError(f"ref_xdr_session failed ({rc})")
    return out.value.decode().splitlines()


def run_many(cfg, iq, n_blocks, threads):
    """CPU baseline: iq [C][n_blocks][2*B*M] uint8, one channel per thread."""
    iq = np.ascontiguousarray(iq, dtype=np.uint8)
    chk = C.c_double()
    secs = lib().oracle_run_many(C.byref(cfg), iq.shape[0], iq.ctypes.data, n_blocks,
                                 threads, C.byref(chk))
    return secs, chk.value


# ---- RF signal level (restates src/signal_level.cpp:145-214) ----
def signal_level(iq, gain_db=0, comp=0.5, bias=-4.0, floor_db=-55.0, ceil_db=-19.0):
    """computeSignalLevel on interleaved u8 IQ (numpy restatement, sequential
    double accumulation as the reference's scalar loop)."""
    iq = np.ascontiguousarray(iq, dtype=np.uint8)
    n = iq.size // 2
    out = dict(level120=0.0, dbfs=-120.0, compensated_dbfs=-120.0, hard_clip_ratio=0.0, near_clip_ratio=0.0)
    if n == 0:
        return out
    i = iq[0::2].astype(np.float64)
    q = iq[1::2].astype(np.float64)
    inorm = (i - 127.5) * (1.0 / 127.5)
    qnorm = (q - 127.5) * (1.0 / 127.5)
    # sequential sums (np.cumsum adds left to right in double)
    sumI = float(np.cumsum(inorm)[-1])
    sumQ = float(np.cumsum(qnorm)[-1])
    sumII = float(np.cumsum(inorm * inorm)[-1])
    sumQQ = float(np.cumsum(qnorm * qnorm)[-1])
    ib, qb = iq[0::2], iq[1::2]
    hard = int(np.count_nonzero((ib <= 1) | (ib >= 254) | (qb <= 1) | (qb >= 254))) * 2
    near = int(np.count_nonzero((ib <= 8) | (ib >= 247) | (qb <= 8) | (qb >= 247))) * 2
    nn = float(n)
    meanI, meanQ = sumI / nn, sumQ / nn
    varI = max(0.0, (sumII / nn) - meanI * meanI)
    varQ = max(0.0, (sumQQ / nn) - meanQ * meanQ)
    rms = np.sqrt(max(1e-15, 0.5 * (varI + varQ)))
    dbfs = 20.0 * np.log10(rms + 1e-12)
    comp_db = dbfs - (float(gain_db) * comp) + bias
    safe_ceil = max(ceil_db, floor_db + 1.0)
    norm = (comp_db - floor_db) / (safe_ceil - floor_db)
    out.update(level120=float(np.clip(np.float32(norm * 120.0), np.float32(0.0), np.float32(120.0))),
               dbfs=float(dbfs), compensated_dbfs=float(comp_db), hard_clip_ratio=hard / (2.0 * nn),
               near_clip_ratio=near / (2.0 * nn))
    return out


class SignalSmoother:
    """smoothSignalLevel (signal_level.cpp:206-214), float arithmetic."""

    def __init__(self):
        self.initialized = False
        self.value = np.float32(0.0)

    def __call__(self, x):
        x = np.float32(x)
        if not self.initialized:
            self.value = x
            self.initialized = True
            return float(self.value)
        alpha = np.float32(0.42) if x > self.value else np.float32(0.18)
        self.value = np.float32(self.value + np.float32(np.float32(x - self.value) * alpha))
        return float(self.value)


def ref_signal_level(iq, gain_db=0, comp=0.5, bias=-4.0, floor_db=-55.0, ceil_db=-19.0):
    """The reference's own computeSignalLevel (oracle/_ref)."""
    R = ref()
    iq = np.ascontiguousarray(iq, dtype=np.uint8)
    out = (C.c_double * 5)()
    R.ref_signal_level(iq.ctypes.data if iq.size else None, iq.size // 2, gain_db, comp, bias, floor_db, ceil_db, out)
    return dict(level120=out[0], dbfs=out[1], compensated_dbfs=out[2], hard_clip_ratio=out[3],
                near_clip_ratio=out[4])
